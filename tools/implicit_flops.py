#!/usr/bin/env python3
"""Algorithmic fp32 flops per problem of the DiLQR implicit backward as the HIP
kernels compute it (k_implicit_backward / k_implicit_backward_group: the
O(T d^3) reformulation of DESIGN.md §4, four passes over the horizon).

Counted, not measured: an FMA is 2 flops, add/sub/mul/div 1, a transcendental
or reciprocal 1.  The model terms are counted from the code that evaluates
them — the sympy-generated second derivatives (csrc/dilqr_models_gen.h: the
arithmetic operators of each CSE'd function body) — and the small linear
algebra of each pass from its loop nest (below, one line per product).  The
Jacobian of each model is counted the same way from its closed form (a
constant per model, stated below).  Writes profiles/implicit_flops.json, which
bench.py reads for the implicit backward's flop roofline.

  python tools/implicit_flops.py
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "differentiable-ilqr_amd", "csrc", "dilqr_models_gen.h")

# Jacobian (get_linear_dyn) flops per evaluation, counted from dilqr_models.h:
# pendulum: angle_step (sincos polynomial 14, rsqrt + normalise 7, rotate 6) +
#   12 for the partials and 8 products for D; cartpole: jacobian_sc 62 + the
#   angle_step 27 (jacobian() recomputes it); rocket: jac_row over the 13 rows
#   (69 structural nonzeros, 3-7 ops each: 236)
JAC = {"pendulum": 47, "cartpole": 89, "rocket": 236}
SHAPES = {"pendulum": (3, 1, 3), "cartpole": (5, 1, 4), "rocket": (13, 3, 5)}
TAGS = {"pendulum": "PendulumD2", "cartpole": "CartpoleD2", "rocket": "RocketD2"}


def struct_body(src, name):
    i = src.index(f"struct {name} {{")
    j = src.index("\n};", i)
    return src[i:j]


def fn_ops(body, fn):
    """Arithmetic operators in function `fn` of a generated struct (binary + - * /
    and libm calls; unary minus and the array indexing are not counted)."""
    i = body.index(f"static DEV void {fn}(")
    j = body.index("\n  }", i)
    code = body[body.index("{", i) + 1:j]
    code = "\n".join(line for line in code.split("\n") if "[[maybe_unused]]" not in line and "pragma" not in line)
    code = re.sub(r"\[[^\]]*\]", "", code)                  # indices
    code = re.sub(r"\b\d+\.\d*(e[-+]?\d+)?f\b", "1", code)  # literals
    ops = len(re.findall(r"(?<=[\w\)\s])\s*[-+*/]\s*(?=[\w\(\s])", code))
    calls = len(re.findall(r"\b(sinf|cosf|sqrtf|atan2f|powf|expf)\(", code))
    return ops + calls


def model_terms(model):
    src = open(GEN).read()
    body = struct_body(src, TAGS[model])
    if model == "rocket":
        # per-lane switch functions: a wave runs every case, the algorithm needs each once
        return {"lag_hess": fn_ops(body, "mcol"), "lag_dparam": fn_ops(body, "mp_row"),
                "f_theta": fn_ops(body, "xth_row")}
    return {"lag_hess": fn_ops(body, "lag_hess"), "lag_dparam": fn_ops(body, "lag_dparam"),
            "f_theta": fn_ops(body, "f_theta")}


def per_step(model):
    n, m, p = SHAPES[model]
    d = n + m
    g = model_terms(model)
    J = JAC[model]
    A = {   # pass A: closed-loop d x_t / d theta
        "jacobian": J, "f_theta": g["f_theta"],
        "D_x + D_u K": 2 * n * n * m,
        "f_theta + (D_x + D_u K) gradx": 2 * n * n * p + n * p,
    }
    B = {   # pass B: costates, Lagrangian Hessian, Riccati of C + M^T (u_zero_I engine)
        "jacobian": J, "lag_hess": g["lag_hess"], "C + M^T": d * d,
        "F^T V": 2 * d * n * n, "(F^T V) F + C": 2 * d * d * n + d * d, "q": 2 * d * n + d,
        "gain solve": (2 * n + 4) if m == 1 else (2 * m ** 3 // 3 + 2 * m * m * (n + 1)),
        "V, v update": 2 * n * m * m + n * n * (6 * m + 3) + n * (6 * m + 3),
        "lambda": 2 * n * (2 * n + m) + 3 * n,
    }
    C = {   # pass C: rollout of y
        "K y + k": 2 * m * n + m, "D y": 2 * n * d,
        "jacobian": J,
    }
    D = {   # pass D: w, dlam, dC, dc, dtheta
        "jacobian": J, "lag_hess": g["lag_hess"], "lag_dparam": g["lag_dparam"],
        "dC": 4 * d * d, "w": 2 * n * d + n, "y^T Mp": 2 * p * d,
        "h_x": n * (d * 2 * m + 2 * d + n * 2 * m + 2 * n) + n, "dtheta": p * (4 * n + 1),
        "dlam": 2 * n * (2 * n + m) + 3 * n,
    }
    return {"A": A, "B": B, "C": C, "D": D}


def main():
    out = {"what": "counted fp32 flops per problem per horizon step of the DiLQR implicit backward "
                   "(FMA = 2); tools/implicit_flops.py", "models": {}}
    for model in SHAPES:
        ps = per_step(model)
        tot = sum(sum(v.values()) for v in ps.values())
        out["models"][model] = {"per_step": tot, "passes": {k: sum(v.values()) for k, v in ps.items()},
                                "terms": ps, "model_terms": model_terms(model)}
    path = os.path.join(ROOT, "profiles", "implicit_flops.json")
    json.dump(out, open(path, "w"), indent=1)
    for k, v in out["models"].items():
        print(f"{k}: {v['per_step']} flops per step {v['passes']} (model terms {v['model_terms']})")


if __name__ == "__main__":
    main()
