#!/usr/bin/env python3
"""Generate csrc/dilqr_models_gen.h: second-order model terms for the implicit
(DiLQR) backward, as CSE'd straight-line fp32 device code.

For the one-lane-per-problem models (pendulum, cartpole) this emits
  lag_hess(th, x, u, lam, M)    M[j][k]  = sum_i lam_i d D[i][j] / d tau_k      (d x d)
  lag_dparam(th, x, u, lam, Mp) Mp[j][k] = sum_i lam_i D_grad_params[i][j][k]   (d x p)
  f_theta(th, x, u, ft)         ft[i][k] = d f_i / d theta_k                     (n x p)
where D = df/dtau.  D_grad_params uses the reference's closed forms where they
differ from the derivative (cartpole.py matrix_2_part_2/3 row 4).

For the rocket (16 lanes per problem, dilqr_group.h) it emits per-lane pieces,
built from the reference's build_batched_* tables (rocket.py:541-820) rather
than from derivatives, since those are what its implicit backward uses:
  mcol(r, th, ith, ..., lam, o)   o[k] = sum_i lam_i Dtau[i][k][r]   (column r of M, d)
  mp_row(j, ..., lam, o) o[k] = sum_i lam_i D_params[i][j][k]                (p)
  xx_row(r, ..., o)      row r of x_grad_xtm1                                (n)
  xth_row(r, ..., o)     row r of x_grad_theta = d f_r / d theta             (p)

The equations come from tools/model_sym.py (not from oracle/, which is test
infrastructure); tests/test_models_gen.py checks the output against the oracle.

Usage: python tools/gen_model_derivs.py   (rewrites the header; commit the result)
"""
import os
import sys

import sympy as sp
from sympy.printing.c import C99CodePrinter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import model_sym as ms  # noqa: E402

OUT = os.path.join(ROOT, "differentiable-ilqr_amd", "csrc", "dilqr_models_gen.h")


class F32Printer(C99CodePrinter):
    def _print_Float(self, e):
        return repr(float(e)) + "f"

    def _print_Rational(self, e):
        return f"({float(e.p)!r}f/{float(e.q)!r}f)"

    def _print_Integer(self, e):
        return f"{int(e)}.0f"

    def _print_Pow(self, e):
        b, ex = e.base, e.exp
        bs = self.parenthesize(b, 100)
        if ex.is_Integer:
            k = int(ex)
            if 1 <= k <= 6:
                return "(" + "*".join([bs] * k) + ")"
            if -6 <= k <= -1:
                return "(1.0f/(" + "*".join([bs] * (-k)) + "))"
        if ex == sp.Rational(1, 2):
            return f"sqrtf({self._print(b)})"
        if ex == sp.Rational(-1, 2):
            return f"(1.0f/sqrtf({self._print(b)}))"
        return f"powf({self._print(b)}, {self._print(ex)})"

    def _print_Function(self, e):
        name = {"sin": "sinf", "cos": "cosf", "atan2": "atan2f", "sqrt": "sqrtf", "exp": "expf",
                "vrcp": "vrcp"}.get(e.func.__name__)
        if name:
            return f"{name}({', '.join(self._print(a) for a in e.args)})"
        return super()._print_Function(e)


P = F32Printer()


def _f32_calls(txt):
    import re
    for fn in ("sin", "cos", "atan2", "sqrt", "exp", "pow"):
        txt = re.sub(r"\b%s\(" % fn, fn + "f(", txt)
    return txt


VRCP = sp.Function("vrcp")


def hw_rcp(e):
    """Every division by a state-dependent (or parameter) expression as the
    hardware reciprocal, 1/b^k -> vrcp(b^k) (v_rcp_f32, 1 ulp; an IEEE f32
    division is ~10 instructions on gfx950), so the C printer emits no `/`
    but constant rationals."""
    return sp.sympify(e).replace(lambda z: z.is_Pow and z.exp.is_Integer and z.exp < 0,
                                 lambda z: VRCP(z.base ** (-z.exp)))


def cse_rcp(exprs):
    repl, red = sp.cse(exprs, symbols=sp.numbered_symbols("s"), optimizations="basic")
    return [(v, hw_rcp(e)) for v, e in repl], [hw_rcp(e) for e in red]


def emit(name, args_sig, outputs, out_decl, syms):
    """outputs: list of (lvalue string, expr)."""
    exprs = [e for _, e in outputs]
    repl, red = cse_rcp(exprs)
    lines = [f"  static DEV void {name}({args_sig}, {out_decl}) {{"]
    lines += [f"    const float {s[0]} = {P.doprint(s[1])};" for s in repl]
    for (lv, _), e in zip(outputs, red):
        lines.append(f"    {lv} = {P.doprint(e)};")
    lines.append("  }")
    return _f32_calls("\n".join(lines))


def unpack_lines(xs, us, ps, lam=None):
    s = "    " + " ".join(f"[[maybe_unused]] const float {v} = x[{i}];" for i, v in enumerate(xs)) + "\n    " + \
        " ".join(f"[[maybe_unused]] const float {v} = u[{i}];" for i, v in enumerate(us)) + "\n    " + \
        " ".join(f"[[maybe_unused]] const float {v} = th[{i}];" for i, v in enumerate(ps))
    if lam is not None:
        s += "\n    " + " ".join(f"[[maybe_unused]] const float {v} = lam[{i}];" for i, v in enumerate(lam))
    return s


def emit_ptr(name, sig, outputs, unpack):
    """A function writing the nonzero entries `outputs` [(lvalue, expr)] through
    pointers (get_matrices; the caller zero-fills the rest), CSE'd."""
    nz = [(lv, e) for lv, e in outputs if e != 0]
    repl, red = cse_rcp([e for _, e in nz])
    lines = [f"  static DEV void {name}({sig}) {{", unpack]
    lines += [f"    const float {v} = {P.doprint(e)};" for v, e in repl]
    lines += [f"    {lv} = {P.doprint(e)};" for (lv, _), e in zip(nz, red)]
    lines.append("  }")
    return _f32_calls("\n".join(lines))


MAT_SIG = ("float* __restrict__ Dp, float* __restrict__ Dx, float* __restrict__ Du, "
           "float* __restrict__ xth, float* __restrict__ xx")


def model_block(M, cls_name):
    n, m, p = M.n, M.m, M.p
    d = n + m
    xs, us, ps = ms.symbols(n, m, p)
    lam = sp.symbols(f"lam0:{n}", real=True)
    dp_overrides = M.dp_overrides()
    f = sp.Matrix(M.next_state(xs, us, ps))
    tau = list(xs) + list(us)
    D = f.jacobian(tau)
    Dp = [[[sp.diff(D[i, j], ps[k]) for k in range(p)] for j in range(d)] for i in range(n)]
    if dp_overrides:
        for (i, j, k), fn in dp_overrides.items():
            Dp[i][j][k] = fn(xs, us, ps)
    Mh = [[sum(lam[i] * sp.diff(D[i, j], tau[k]) for i in range(n)) for k in range(d)] for j in range(d)]
    Mp = [[sum(lam[i] * Dp[i][j][k] for i in range(n)) for k in range(p)] for j in range(d)]
    ft = [[sp.diff(f[i], ps[k]) for k in range(p)] for i in range(n)]

    unpack = unpack_lines(xs, us, ps)
    unpack_l = unpack_lines(xs, us, ps, lam)[len(unpack):]
    sig = f"const float* __restrict__ th, const float (&x)[{n}], const float (&u)[{m}]"

    # The angle models' second-order terms hold cos and sin of ONE angle: the
    # integrated angle atan2(sin, cos) + dt * (...) of the next state.  The
    # device computes that pair once per step through the model's angle_step
    # (Model::next_cs, the Jacobian's own cos/sin), so the functions the
    # implicit backward calls take it as (cn, sn) instead of re-evaluating
    # atan2f, cosf and sinf in each of them; next_cs here evaluates the symbolic
    # expression (the host test's reference for the pair).
    trig = set()
    for e in [x for row in Mh for x in row] + [x for row in Mp for x in row] + [x for row in ft for x in row]:
        trig |= {a.args[0] for a in sp.sympify(e).atoms(sp.sin, sp.cos)}
    assert len(trig) <= 1, trig
    cn_, sn_ = sp.symbols("cn sn", real=True)
    if trig:
        A = trig.pop()
        sub = lambda e: sp.sympify(e).subs({sp.cos(A): cn_, sp.sin(A): sn_})  # noqa: E731
    else:
        A, sub = None, (lambda e: e)
    sig_cs = ", float cn, float sn"

    def fn(name, extra_sig, outs, out_decl, with_lam):
        body = emit(name, sig + extra_sig, outs, out_decl, None)
        head, rest = body.split("{", 1)
        return head + "{\n" + unpack + (unpack_l if with_lam else "") + rest

    if A is not None:
        nc = emit("next_cs", sig, [("cn", sp.cos(A)), ("sn", sp.sin(A))], "float& cn, float& sn", None)
        head, rest = nc.split("{", 1)
        next_cs = head + "{\n" + unpack + rest
    else:
        next_cs = ("  static DEV void next_cs(" + sig + ", float& cn, float& sn) { cn = 0.f; sn = 0.f; }")

    # get_matrices (cartpole.py:105-716, pendulum.py:152-382): D_grad_params
    # [n][d][p] (with the reference's overrides), D_grad_x [n][d][n], D_grad_u
    # [n][d][m], x_grad_theta [n][p], x_grad_xtm1 [n][n] = D[:, :n] (cartpole:
    # its [0][0] written 0, cartpole.py:666)
    mats = []
    for i in range(n):
        for j in range(d):
            for k in range(p):
                mats.append((f"Dp[{(i * d + j) * p + k}]", Dp[i][j][k]))
            for k in range(n):
                mats.append((f"Dx[{(i * d + j) * n + k}]", sp.diff(D[i, j], xs[k])))
            for k in range(m):
                mats.append((f"Du[{(i * d + j) * m + k}]", sp.diff(D[i, j], us[k])))
    for i in range(n):
        for k in range(p):
            mats.append((f"xth[{i * p + k}]", ft[i][k]))
        for k in range(n):
            zero = M.xx00_zero and i == 0 and k == 0
            mats.append((f"xx[{i * n + k}]", sp.Integer(0) if zero else D[i, k]))
    parts = [f"struct {cls_name} {{",
             f"  static constexpr int N = {n}, M = {m}, P = {p}, D = {d};",
             emit_ptr("matrices", sig + ", " + MAT_SIG, mats, unpack),
             next_cs,
             fn("lag_hess", f", const float (&lam)[{n}]" + sig_cs,
                [(f"Mo[{j}][{k}]", sub(Mh[j][k])) for j in range(d) for k in range(d)], f"float (&Mo)[{d}][{d}]",
                True),
             fn("lag_dparam", f", const float (&lam)[{n}]" + sig_cs,
                [(f"Mo[{j}][{k}]", sub(Mp[j][k])) for j in range(d) for k in range(p)], f"float (&Mo)[{d}][{p}]",
                True),
             fn("f_theta", "", [(f"Fo[{i}][{k}]", ft[i][k]) for i in range(n) for k in range(p)],
                f"float (&Fo)[{n}][{p}]", False),
             fn("f_theta_cs", sig_cs, [(f"Fo[{i}][{k}]", sub(ft[i][k])) for i in range(n) for k in range(p)],
                f"float (&Fo)[{n}][{p}]", False),
             "};"]
    return "\n".join(parts)


def emit_switch(name, sig, sel, n_out, cases, unpack):
    """A per-lane function: switch on `sel`, each case a CSE'd list of outputs
    (cases: {value: [expr] * n_out}); outputs not written are zero."""
    lines = [f"  static DEV void {name}(int {sel}, {sig}, float (&o)[{n_out}]) {{", unpack,
             f"#pragma unroll\n    for (int k = 0; k < {n_out}; ++k) o[k] = 0.f;", f"    switch ({sel}) {{"]
    for val in sorted(cases):
        exprs = cases[val]
        nz = [(k, e) for k, e in enumerate(exprs) if e != 0]
        if not nz:
            continue
        repl, red = cse_rcp([e for _, e in nz])
        lines.append(f"      case {val}: {{")
        lines += [f"        const float {v} = {P.doprint(e)};" for v, e in repl]
        lines += [f"        o[{k}] = {P.doprint(e)};" for (k, _), e in zip(nz, red)]
        lines.append("        break;\n      }")
    lines += ["      default: break;", "    }", "  }"]
    return _f32_calls("\n".join(lines))


def emit_select(name, sig, sel, n_out, cases, unpack):
    """The same per-lane function as emit_switch, without divergence: every
    lane evaluates every case's outputs (one CSE over all cases) and keeps its
    own case's by selects.  A switch on the lane's row makes a wave execute
    every case anyway, each behind an exec-mask branch, and merge the whole
    output array after each case (measured: ~24 register moves per case)."""
    items = [(val, k, e) for val in sorted(cases) for k, e in enumerate(cases[val]) if e != 0]
    repl, red = cse_rcp([e for _, _, e in items])
    lines = [f"  static DEV void {name}(int {sel}, {sig}, float (&o)[{n_out}]) {{", unpack,
             f"#pragma unroll\n    for (int k = 0; k < {n_out}; ++k) o[k] = 0.f;"]
    lines += [f"    const float {v} = {P.doprint(e)};" for v, e in repl]
    for (val, k, _), e in zip(items, red):
        lines.append(f"    o[{k}] = {sel} == {val} ? {P.doprint(e)} : o[{k}];")
    lines.append("  }")
    return _f32_calls("\n".join(lines))


def rocket_block():
    M = ms.Rocket
    n, m, p = M.n, M.m, M.p
    d = n + m
    xs, us, ps = ms.symbols(n, m, p)
    lam = sp.symbols(f"lam0:{n}", real=True)
    f = M.next_state(xs, us, ps)
    xx, Du, Dx, Dp = M.builders(xs, us, ps)
    # Dtau[i][j][k] = [D_x | D_u][i][j][k]
    Dtau = {}
    for (i, j, k), e in Dx.items():
        Dtau[(i, j, k)] = e
    for (i, j, a), e in Du.items():
        Dtau[(i, j, n + a)] = e
    mcol = {r: [sum((lam[i] * Dtau.get((i, k, r), 0) for i in range(n)), sp.Integer(0)) for k in range(d)]
            for r in range(d)}
    mp = {j: [sum((lam[i] * Dp.get((i, j, k), 0) for i in range(n)), sp.Integer(0)) for k in range(p)]
          for j in range(d)}
    xxr = {r: [xx.get((r, l), sp.Integer(0)) for l in range(n)] for r in range(n)}
    xth = {r: [sp.diff(f[r], ps[k]) for k in range(p)] for r in range(n)}
    sig = f"const float* __restrict__ th, const float (&x)[{n}], const float (&u)[{m}]"
    sig_l = sig + f", const float (&lam)[{n}]"
    up, upl = unpack_lines(xs, us, ps), unpack_lines(xs, us, ps, lam)
    # the per-lane pieces of the implicit backward divide only by parameters
    # (mass, inertias): the caller holds their reciprocals (ith[k] = 1/th[k],
    # wave-uniform, formed once per launch), so a division becomes a product
    ips = sp.symbols(f"ith0:{p}", real=True)

    def rcp(e):
        return sp.sympify(e).replace(lambda z: z.is_Pow and z.base in ps and z.exp.is_negative,
                                     lambda z: ips[ps.index(z.base)] ** (-z.exp))
    rc = lambda cases: {k: [rcp(e) for e in v] for k, v in cases.items()}  # noqa: E731
    sig_r = f"const float* __restrict__ th, const float (&ith)[{p}], const float (&x)[{n}], const float (&u)[{m}]"
    sig_rl = sig_r + f", const float (&lam)[{n}]"
    iun = "\n    " + " ".join(f"[[maybe_unused]] const float {v} = ith[{i}];" for i, v in enumerate(ips))
    upr, uplr = up + iun, upl + iun
    # get_matrices (rocket.py:258-261 with the build_batched_* tables)
    mats = [(f"Dp[{(i * d + j) * p + k}]", e) for (i, j, k), e in sorted(Dp.items())]
    mats += [(f"Dx[{(i * d + j) * n + k}]", e) for (i, j, k), e in sorted(Dx.items())]
    mats += [(f"Du[{(i * d + j) * m + k}]", e) for (i, j, k), e in sorted(Du.items())]
    mats += [(f"xth[{i * p + k}]", sp.diff(f[i], ps[k])) for i in range(n) for k in range(p)]
    mats += [(f"xx[{i * n + k}]", e) for (i, k), e in sorted(xx.items())]
    parts = ["struct RocketD2 {",
             f"  static constexpr int N = {n}, M = {m}, P = {p}, D = {d};",
             emit_ptr("matrices", sig + ", " + MAT_SIG, mats, up),
             emit_select("mcol", sig_rl, "r", d, rc(mcol), uplr),
             emit_select("mp_row", sig_rl, "j", p, rc(mp), uplr),
             emit_select("xx_row", sig_r, "r", n, rc(xxr), upr),
             emit_select("xth_row", sig_r, "r", p, rc(xth), upr),
             "};"]
    return "\n".join(parts)


def main():
    blocks = [model_block(ms.Pendulum, "PendulumD2"), model_block(ms.Cartpole, "CartpoleD2"), rocket_block()]
    hdr = ["// dilqr_models_gen.h — GENERATED by tools/gen_model_derivs.py; do not edit.",
           "// Second-order model terms for the implicit (DiLQR) backward; see the generator.",
           "#pragma once",
           "#ifdef __HIPCC__",
           '#include "dilqr_device.h"',
           "#else  // host build (tests/test_models_gen.py compiles this header with g++)",
           "#include <cmath>",
           "#define DEV inline",
           "inline float vrcp(float x) { return 1.0f / x; }",
           "#endif", "", "namespace dilqr {", "namespace gen {", ""]
    src = "\n".join(hdr) + "\n\n".join(blocks) + "\n\n}  // namespace gen\n}  // namespace dilqr\n"
    with open(OUT, "w") as fh:
        fh.write(src)
    print(f"wrote {OUT} ({len(src.splitlines())} lines)")


if __name__ == "__main__":
    main()
