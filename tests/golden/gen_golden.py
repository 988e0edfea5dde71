#!/usr/bin/env python3
"""Generate the golden input/output vectors under tests/golden/ from the reference.

TEST INFRASTRUCTURE ONLY.  This script imports the reference implementation
(josef-w/Differentiable-iLQR, mounted read-only at /root/reference) in the BUILD
container and writes small .npz fixtures (inputs + the reference's outputs).
It never runs on the GPU box; only the .npz files travel.  Nothing from the
reference is copied: the fixtures are data.

Recipes follow SURVEY.md §8(c):
  * flat imports with PYTHONDONTWRITEBYTECODE (the tree is read-only);
  * rocket.py does `from casadi import *` only for its animation code
    (rocket.py:6, 959, 1006) -> an empty stand-in module named `casadi`;
  * the Riccati sweep is reached through the LQRStepFn.forward closure;
  * the DiLQR implicit backward is driven through LQRStep(no_op_forward=True)
    (backward through mpc_explicit.MPC itself raises under torch 2.10);
  * data/*.pkl are NOT unpickled: their opcode stream is parsed statically
    with pickletools and only the embedded tensor storages are loaded, with
    torch.load(weights_only=True).

Usage:  python tests/golden/gen_golden.py   (takes ~1-2 minutes on 8 cores)
"""
import contextlib
import io
import os
import pickletools
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.set_num_threads(8)


def _import_reference():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    sys.modules.setdefault("casadi", types.ModuleType("casadi"))
    import util
    import pnqp
    import mpc            # before lqr_step: mpc.py <-> lqr_step.py import each other
    import lqr_step
    import mpc_backup     # likewise for lqr_step_backup.py
    import lqr_step_backup
    import lqr_step_explicit
    import mpc_explicit
    from env_dx import cartpole, pendulum, rocket
    return types.SimpleNamespace(
        util=util, pnqp=pnqp, lqr_step_explicit=lqr_step_explicit, lqr_step_backup=lqr_step_backup,
        lqr_step=lqr_step, mpc_explicit=mpc_explicit, mpc=mpc,
        cartpole=cartpole, pendulum=pendulum, rocket=rocket)


R = _import_reference()


@contextlib.contextmanager
def default_dtype(dt):
    old = torch.get_default_dtype()
    torch.set_default_dtype(dt)
    try:
        yield
    finally:
        torch.set_default_dtype(old)


def np_(t):
    if isinstance(t, (list, tuple)):
        return np.stack([np_(x) for x in t])
    if isinstance(t, torch.Tensor):
        return t.detach().cpu().numpy()
    return np.asarray(t)


def save(name, **arrs):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print(f"  wrote {name}.npz ({os.path.getsize(path)/1024:.1f} KiB)")


def model(name):
    return {"pendulum": R.pendulum.PendulumDx, "cartpole": R.cartpole.CartpoleDx,
            "rocket": R.rocket.RocketDx}[name]()


def tname(dt):
    return "f64" if dt == torch.float64 else "f32"


# --------------------------------------------------------------------------
# random inputs (numpy RandomState so the oracle tests can regenerate them)
# --------------------------------------------------------------------------
def sample_states(name, N, rng, wide=True):
    if name == "pendulum":
        th = rng.uniform(-np.pi, np.pi, N)
        dth = rng.uniform(-8, 8, N)
        x = np.stack([np.cos(th), np.sin(th), dth], 1)
        u = rng.uniform(-3, 3, (N, 1))       # beyond the +-2 clamp
    elif name == "cartpole":
        th = rng.uniform(-np.pi, np.pi, N)
        x = np.stack([rng.uniform(-1, 1, N), rng.uniform(-2, 2, N), np.cos(th), np.sin(th),
                      rng.uniform(-3, 3, N)], 1)
        u = rng.uniform(-150, 150, (N, 1)) if wide else rng.uniform(-5, 5, (N, 1))
    elif name == "rocket":
        r = rng.uniform([0, -4, -2.5], [10, 4, 2.5], (N, 3))
        v = rng.normal(0, 1.0, (N, 3))
        q = np.array([1., 0, 0, 0]) + 0.3 * rng.normal(size=(N, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        w = rng.normal(0, 0.5, (N, 3))
        x = np.concatenate([r, v, q, w], 1)
        u = rng.uniform(-30, 30, (N, 3))
    return x, u


def random_lqr(n, m, T, B, rng):
    """SURVEY.md §8(d) Riccati workload: C=LL^T+0.1I, c~N, F=[I+0.05N | 0.1N]."""
    d = n + m
    L = rng.normal(size=(T, B, d, d)) * 0.5 / np.sqrt(d)
    C = L @ np.swapaxes(L, -1, -2) + 0.1 * np.eye(d)
    c = rng.normal(size=(T, B, d))
    F = np.concatenate([np.eye(n) + 0.05 * rng.normal(size=(T - 1, B, n, n)),
                        0.1 * rng.normal(size=(T - 1, B, n, m))], -1)
    f = 0.1 * rng.normal(size=(T - 1, B, n))
    return C, c, F, f


def riccati_closure(step_mod, n, m, T, **kw):
    fn = step_mod.LQRStep(n, m, T, **kw).__self__.forward
    cells = dict(zip(fn.__code__.co_freevars, [c.cell_contents for c in fn.__closure__]))
    return cells["lqr_backward"]


# --------------------------------------------------------------------------
# A. dynamics models: forward, get_linear_dyn, get_matrices, grad_input
# --------------------------------------------------------------------------
def case_models():
    print("A. models")
    for dt in (torch.float64, torch.float32):
        with default_dtype(dt):
            out = {}
            for name in ("pendulum", "cartpole", "rocket"):
                rng = np.random.RandomState(100)
                N = 64
                x, u = sample_states(name, N, rng)
                dx = model(name)
                X, U = torch.tensor(x, dtype=dt), torch.tensor(u, dtype=dt)
                with torch.no_grad():
                    out[f"{name}_x"] = x
                    out[f"{name}_u"] = u
                    out[f"{name}_fwd"] = np_(dx(X, U))
                    out[f"{name}_D"] = np_(dx.get_linear_dyn(X, U))
                    Ns = 16
                    mats = dx.get_matrices(X[:Ns], U[:Ns])
                    for k, v in zip(("D", "D_params", "D_x", "D_u", "x_theta", "x_xtm1", "x_utm1"), mats):
                        out[f"{name}_gm_{k}"] = np_(v)
                    # grad_input over a short random closed-loop trajectory
                    T, B = 6, 3
                    rng2 = np.random.RandomState(7)
                    xs, us = sample_states(name, T * B, rng2, wide=False)
                    Xs = torch.tensor(xs.reshape(T, B, -1), dtype=dt)
                    Us = torch.tensor(us.reshape(T, B, -1), dtype=dt)
                    K = torch.tensor(rng2.normal(size=(T, B, dx.n_ctrl, dx.n_state)) * 0.3, dtype=dt)
                    gi = dx.grad_input(Xs, Us, K)
                    out[f"{name}_gi_X"], out[f"{name}_gi_U"], out[f"{name}_gi_K"] = np_(Xs), np_(Us), np_(K)
                    for k, v in zip(("grad_D", "grad_d", "D_x", "D_u", "D", "d_x", "d_u"), gi):
                        out[f"{name}_gi_{k}"] = np_(v)
            save(f"models_{tname(dt)}", **out)


# --------------------------------------------------------------------------
# B. Riccati sweep (lqr_backward) unconstrained / bounded / Cholesky variant
# --------------------------------------------------------------------------
def case_riccati():
    print("B. riccati")
    shapes = {"pendulum": (3, 1, 10, 16), "cartpole": (5, 1, 25, 16), "rocket": (13, 3, 30, 8)}
    for dt in (torch.float64, torch.float32):
        with default_dtype(dt):
            out = {}
            for name, (n, m, T, B) in shapes.items():
                rng = np.random.RandomState(0)
                C, c, F, _ = random_lqr(n, m, T, B, rng)
                u = rng.uniform(-0.5, 0.5, (T, B, m))
                Ct, ct, Ft, ut = (torch.tensor(a, dtype=dt) for a in (C, c, F, u))
                out[f"{name}_C"], out[f"{name}_c"], out[f"{name}_F"], out[f"{name}_u"] = C, c, F, u
                ctx = types.SimpleNamespace(current_u=ut)
                with torch.no_grad():
                    lb = riccati_closure(R.lqr_step_explicit, n, m, T)
                    Ks, ks, _ = lb(ctx, Ct, ct, Ft, None)
                    out[f"{name}_K"], out[f"{name}_k"] = np_(Ks[::-1]), np_(ks[::-1])
                    lo, hi = -1.0, 1.0
                    lb = riccati_closure(R.lqr_step_explicit, n, m, T, u_lower=lo, u_upper=hi)
                    Ks, ks, nqp = lb(ctx, Ct, ct, Ft, None)
                    out[f"{name}_box_K"], out[f"{name}_box_k"] = np_(Ks[::-1]), np_(ks[::-1])
                    out[f"{name}_box_nqp"] = np.array(nqp)
                    # adjoint engine (lqr_step_backup: Cholesky + 1e-6 I for m>1)
                    lb = riccati_closure(R.lqr_step_backup, n, m, T)
                    Ks, ks, _ = lb(ctx, Ct, ct, Ft, None)
                    out[f"{name}_chol_K"], out[f"{name}_chol_k"] = np_(Ks[::-1]), np_(ks[::-1])
                    # u_zero_I branch (active-set masked solve used by the adjoints)
                    I = torch.tensor(rng.uniform(size=(T, B, m)) < 0.3)
                    lb = riccati_closure(R.lqr_step_backup, n, m, T, u_zero_I=I)
                    Ks, ks, _ = lb(ctx, Ct, ct, Ft, None)
                    out[f"{name}_zI"] = np_(I)
                    out[f"{name}_zI_K"], out[f"{name}_zI_k"] = np_(Ks[::-1]), np_(ks[::-1])
            save(f"riccati_{tname(dt)}", **out)


# --------------------------------------------------------------------------
# C. pnqp box QP
# --------------------------------------------------------------------------
def case_pnqp():
    print("C. pnqp")
    for dt in (torch.float64, torch.float32):
        with default_dtype(dt):
            out = {}
            for m in (1, 3):
                rng = np.random.RandomState(3 + m)
                B = 64
                L = rng.normal(size=(B, m, m))
                H = L @ np.swapaxes(L, 1, 2) + 0.2 * np.eye(m)
                q = rng.normal(size=(B, m)) * 3
                lo = -rng.uniform(0.1, 1.5, (B, m))
                hi = rng.uniform(0.1, 1.5, (B, m))
                x0 = rng.uniform(-2, 2, (B, m))
                Ht, qt, lot, hit, x0t = (torch.tensor(a, dtype=dt) for a in (H, q, lo, hi, x0))
                out.update({f"m{m}_H": H, f"m{m}_q": q, f"m{m}_lo": lo, f"m{m}_hi": hi, f"m{m}_x0": x0})
                with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
                    x, _, If, it = R.pnqp.pnqp(Ht, qt, lot, hit)
                    out[f"m{m}_x"], out[f"m{m}_If"], out[f"m{m}_it"] = np_(x), np_(If), np.array(it)
                    x, _, If, it = R.pnqp.pnqp(Ht, qt, -0.7, 0.7, x_init=x0t)
                    out[f"m{m}_xf"], out[f"m{m}_Iff"], out[f"m{m}_itf"] = np_(x), np_(If), np.array(it)
                    # per-problem calls (batch size 1): the reference semantics without batch coupling
                    xs, its = [], []
                    for b in range(B):
                        x, _, If, it = R.pnqp.pnqp(Ht[b:b+1], qt[b:b+1], lot[b:b+1], hit[b:b+1])
                        xs.append(np_(x)[0]); its.append(it)
                    out[f"m{m}_x_pp"], out[f"m{m}_it_pp"] = np.stack(xs), np.array(its)
            save(f"pnqp_{tname(dt)}", **out)


# --------------------------------------------------------------------------
# helpers for the solver-level cases
# --------------------------------------------------------------------------
def xinit_for(name, B, rng):
    if name == "pendulum":       # il_env.py:63-66
        th = rng.uniform(-np.pi / 2, np.pi / 2, B)
        return np.stack([np.cos(th), np.sin(th), rng.uniform(-1, 1, B)], 1)
    if name == "cartpole":       # il_env.py:71-75 without the *0
        th = rng.uniform(-np.pi, np.pi, B)
        return np.stack([rng.uniform(-.5, .5, B), rng.uniform(-.5, .5, B), np.cos(th), np.sin(th),
                         rng.uniform(-1, 1, B)], 1)
    if name == "rocket":         # near hover
        r = rng.uniform([0, -4, -2.5], [10, 4, 2.5], (B, 3))
        v = rng.normal(0, 0.1, (B, 3))
        q = np.array([1., 0, 0, 0]) + 0.05 * rng.normal(size=(B, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        w = rng.normal(0, 0.02, (B, 3))
        return np.concatenate([r, v, q, w], 1)


def true_cost(dx, T, B, dt):
    q, p = dx.get_true_obj()       # il_env.py:159-162 materialisation
    Q = torch.diag(q).to(dt).unsqueeze(0).unsqueeze(0).repeat(T, B, 1, 1)
    P = p.to(dt).unsqueeze(0).repeat(T, B, 1)
    return Q, P


# --------------------------------------------------------------------------
# D. one LQRStep (explicit) forward: Riccati + rollout/line search
# --------------------------------------------------------------------------
def case_lqrstep():
    print("D. lqr step")
    for dt in (torch.float64, torch.float32):
        with default_dtype(dt):
            out = {}
            for tag, bounds in (("unc", None), ("box", (-5.0, 5.0))):
                dx = model("cartpole")
                T, B = 25, 16
                rng = np.random.RandomState(11)
                x0 = xinit_for("cartpole", B, rng)
                u = rng.uniform(-2, 2, (T, B, 1))
                X0, U = torch.tensor(x0, dtype=dt), torch.tensor(u, dtype=dt)
                Q, P = true_cost(dx, T, B, dt)
                mpc_ = R.mpc_explicit.MPC(5, 1, T, lqr_iter=1)
                with torch.no_grad():
                    X = R.util.get_traj(T, U, x_init=X0, dynamics=dx)
                    F, f = mpc_.linearize_dynamics(X, U, dx, diff=False)
                    kw = {} if bounds is None else dict(u_lower=bounds[0], u_upper=bounds[1])
                    step = R.lqr_step_explicit.LQRStep(
                        5, 1, T, true_cost=R.mpc_explicit.QuadCost(Q, P), true_dynamics=dx,
                        current_x=X, current_u=U, linesearch_decay=0.5, max_linesearch_iter=2, **kw)
                    nx, nu, nqp, costs, du, malpha = step(X0, Q, P, F, f, None)
                out.update({f"{tag}_x0": x0, f"{tag}_u": u, f"{tag}_x": np_(X), f"{tag}_F": np_(F),
                            f"{tag}_f": np_(f), f"{tag}_nx": np_(nx), f"{tag}_nu": np_(nu),
                            f"{tag}_costs": np_(costs), f"{tag}_du": np_(du), f"{tag}_malpha": np_(malpha),
                            f"{tag}_nqp": np_(nqp)})
            save(f"lqrstep_{tname(dt)}", **out)


# --------------------------------------------------------------------------
# E. full MPC (mpc_explicit) solves
# --------------------------------------------------------------------------
MPC_CASES = {
    # name: (model, T, B, lqr_iter, bounds, eps, not_improved_lim, decay, max_ls)
    "cart_unc": ("cartpole", 25, 64, 10, None, 0.0, 10 ** 9, 0.5, 2),
    "cart_box10": ("cartpole", 25, 64, 10, (-10.0, 10.0), 0.0, 10 ** 9, 0.5, 2),
    "cart_il": ("cartpole", 25, 64, 40, (-100.0, 100.0), 1e-4, 5, 0.5, 2),
    "pend_unc": ("pendulum", 10, 64, 10, None, 0.0, 10 ** 9, 0.2, 5),
    "pend_box": ("pendulum", 10, 64, 10, (-2.0, 2.0), 0.0, 10 ** 9, 0.2, 5),
    "rocket_unc": ("rocket", 30, 64, 5, None, 0.0, 10 ** 9, 0.2, 5),
}


def run_mpc(name, dt, lqr_iter_override=None):
    mname, T, B, it, bounds, eps, nil, decay, mls = MPC_CASES[name]
    dx = model(mname)
    rng = np.random.RandomState(0)
    x0 = xinit_for(mname, B, rng)
    X0 = torch.tensor(x0, dtype=dt)
    Q, P = true_cost(dx, T, B, dt)
    kw = {} if bounds is None else dict(u_lower=bounds[0], u_upper=bounds[1])
    m = R.mpc_explicit.MPC(dx.n_state, dx.n_ctrl, T, lqr_iter=lqr_iter_override or it, eps=eps,
                           not_improved_lim=nil, linesearch_decay=decay, max_linesearch_iter=mls,
                           exit_unconverged=False, detach_unconverged=False, verbose=-1,
                           grad_method=R.mpc_explicit.GradMethods.ANALYTIC, **kw)
    with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
        x, u, costs = m(X0, R.mpc_explicit.QuadCost(Q, P), dx)
    return x0, np_(x), np_(u), np_(costs)


MPC_ITERATE_CASES = ("cart_unc", "cart_box10", "pend_box")   # per-iteration goldens (lqr_iter 1, 2, 3)


def case_mpc_iterates():
    """Only the per-iteration entries of MPC_ITERATE_CASES, merged into the
    existing mpc_{f64,f32}.npz (the rest of those files is left as it is)."""
    print("E'. mpc per-iteration entries")
    for dt in (torch.float64, torch.float32):
        with default_dtype(dt):
            path = os.path.join(OUT, f"mpc_{tname(dt)}.npz")
            with np.load(path) as old:
                out = {k: old[k] for k in old.files}
            for name in MPC_ITERATE_CASES:
                for k in (1, 2, 3):
                    _, x, u, costs = run_mpc(name, dt, lqr_iter_override=k)
                    out.update({f"{name}_it{k}_x": x, f"{name}_it{k}_u": u, f"{name}_it{k}_costs": costs})
            save(f"mpc_{tname(dt)}", **out)


def case_mpc():
    print("E. mpc")
    for dt in (torch.float64, torch.float32):
        with default_dtype(dt):
            out = {}
            for name in MPC_CASES:
                x0, x, u, costs = run_mpc(name, dt)
                out.update({f"{name}_x0": x0, f"{name}_x": x, f"{name}_u": u, f"{name}_costs": costs})
                if name in MPC_ITERATE_CASES:
                    for k in (1, 2, 3):
                        _, x, u, costs = run_mpc(name, dt, lqr_iter_override=k)
                        out.update({f"{name}_it{k}_x": x, f"{name}_it{k}_u": u, f"{name}_it{k}_costs": costs})
            save(f"mpc_{tname(dt)}", **out)


# --------------------------------------------------------------------------
# F. classic differentiable LQR (mpc.py + lqr_step.py backward)
# --------------------------------------------------------------------------
def case_classic_adjoint():
    print("F. classic adjoint")
    dt = torch.float64
    with default_dtype(dt):
        out = {}
        for tag, (n, m, T, B, bounds) in {"m1": (5, 1, 10, 3, None), "m3": (4, 3, 8, 3, None),
                                            "m1box": (5, 1, 10, 3, (-0.5, 0.5)),
                                            "m3box": (4, 3, 8, 3, (-0.5, 0.5))}.items():
            rng = np.random.RandomState(21)
            C, c, F, f = random_lqr(n, m, T, B, rng)
            x0 = rng.normal(size=(B, n))
            wx, wu = rng.normal(size=(T, B, n)), rng.normal(size=(T, B, m))
            Ct, ct, Ft, ft, x0t = (torch.tensor(a, dtype=dt, requires_grad=True) for a in (C, c, F, f, x0))
            kw = {} if bounds is None else dict(u_lower=bounds[0], u_upper=bounds[1])
            mpc_ = R.mpc.MPC(n, m, T, lqr_iter=1, n_batch=B, detach_unconverged=False,
                             exit_unconverged=False, verbose=-1, **kw)
            with contextlib.redirect_stdout(io.StringIO()):
                x, u, _ = mpc_(x0t, R.mpc.QuadCost(Ct, ct), R.mpc.LinDx(Ft, ft))
                loss = (x * torch.tensor(wx)).sum() + (u * torch.tensor(wu)).sum()
                loss.backward()
            out.update({f"{tag}_C": C, f"{tag}_c": c, f"{tag}_F": F, f"{tag}_f": f, f"{tag}_x0": x0,
                        f"{tag}_wx": wx, f"{tag}_wu": wu, f"{tag}_x": np_(x), f"{tag}_u": np_(u),
                        f"{tag}_dx0": np_(x0t.grad), f"{tag}_dC": np_(Ct.grad), f"{tag}_dc": np_(ct.grad),
                        f"{tag}_dF": np_(Ft.grad), f"{tag}_df": np_(ft.grad)})
        save("adjoint_f64", **out)


# --------------------------------------------------------------------------
# G. DiLQR implicit backward (lqr_step_explicit.py:653-712)
# --------------------------------------------------------------------------
def implicit_once(mname, T, B, bounds, x, u, x0, Q, P, wx, wu, dt):
    dx = model(mname)
    theta = dx.params.detach().clone().to(dt).requires_grad_(True)
    Qg, Pg = Q.clone().requires_grad_(True), P.clone().requires_grad_(True)
    m = R.mpc_explicit.MPC(dx.n_state, dx.n_ctrl, T, grad_method=R.mpc_explicit.GradMethods.ANALYTIC)
    X, U = torch.tensor(x, dtype=dt), torch.tensor(u, dtype=dt)
    F, f = m.linearize_dynamics(X, U, dx, diff=True)
    F, f = F.detach(), f.detach()
    kw = {} if bounds is None else dict(u_lower=bounds[0], u_upper=bounds[1])
    step = R.lqr_step_explicit.LQRStep(
        dx.n_state, dx.n_ctrl, T, true_cost=R.mpc_explicit.QuadCost(Qg, Pg), true_dynamics=dx,
        current_x=X, current_u=U, back_eps=m.back_eps, no_op_forward=True, **kw)
    with contextlib.redirect_stdout(io.StringIO()):
        x2, u2 = step(torch.tensor(x0, dtype=dt), Qg, Pg, F, f, theta)
        loss = (x2 * torch.tensor(wx, dtype=dt)).sum() + (u2 * torch.tensor(wu, dtype=dt)).sum()
        loss.backward()
    return np_(Qg.grad), np_(Pg.grad), np_(theta.grad), np_(F), np_(f)


IMPLICIT_CASES = {
    # tag: (model, T, B, bounds, MPC_CASES entry for decay / max_ls)
    "cart_unc": ("cartpole", 10, 4, None, "cart_unc"),
    "cart_box": ("cartpole", 10, 4, (-5.0, 5.0), "cart_box10"),
    "pend_box": ("pendulum", 10, 4, (-2.0, 2.0), "pend_box"),
    # rocket: the reference's D_x/D_u/D_params/x_xtm1 builders (rocket.py:541-820)
    "rock_unc": ("rocket", 10, 4, None, "rocket_unc"),
    "rock_box": ("rocket", 10, 4, (-10.0, 10.0), "rocket_unc"),
}
# config 4's own horizon (SURVEY.md §8(c) case G): cartpole T=25, B=8; T*B=200
# stays under the reference's CPU-path threshold (lqr_step_explicit.py:699-700)
IMPLICIT25_CASES = {
    "cart25_unc": ("cartpole", 25, 8, None, "cart_unc"),
    "cart25_box10": ("cartpole", 25, 8, (-10.0, 10.0), "cart_box10"),
    "cart25_box100": ("cartpole", 25, 8, (-100.0, 100.0), "cart_box10"),
}


def case_implicit25():
    case_implicit(IMPLICIT25_CASES, "implicit25")


def case_implicit(cases=IMPLICIT_CASES, fname="implicit"):
    print(f"G. implicit backward ({fname})")
    for dt in (torch.float64, torch.float32):
        with default_dtype(dt):
            out = {}
            for tag, (mname, T, B, bounds, mpc_case) in cases.items():
                dx = model(mname)
                rng = np.random.RandomState(5)
                x0 = xinit_for(mname, B, rng)
                Q, P = true_cost(dx, T, B, dt)
                kw = {} if bounds is None else dict(u_lower=bounds[0], u_upper=bounds[1])
                _, _, _, _, _, _, _, decay, mls = MPC_CASES[mpc_case]
                m = R.mpc_explicit.MPC(dx.n_state, dx.n_ctrl, T, lqr_iter=30, eps=1e-6,
                                       linesearch_decay=decay, max_linesearch_iter=mls,
                                       exit_unconverged=False, detach_unconverged=False, verbose=-1,
                                       grad_method=R.mpc_explicit.GradMethods.ANALYTIC, **kw)
                with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
                    x, u, _ = m(torch.tensor(x0, dtype=dt), R.mpc_explicit.QuadCost(Q, P), dx)
                x, u = np_(x), np_(u)
                wx = rng.normal(size=x.shape)
                wu = rng.normal(size=u.shape)
                # MKL's batched getrf hangs on the rocket's 160x160 KKT systems with
                # 8 threads in this image (lqr_step_explicit.py:570); one thread is fine
                torch.set_num_threads(1 if mname == "rocket" or T * (dx.n_state + dx.n_ctrl) > 100 else 8)
                dQ, dP, dth, F, f = implicit_once(mname, T, B, bounds, x, u, x0, Q, P, wx, wu, dt)
                # per-problem d theta: weight only problem j
                dth_b = []
                for j in range(B):
                    mx, mu = np.zeros_like(wx), np.zeros_like(wu)
                    mx[:, j], mu[:, j] = wx[:, j], wu[:, j]
                    dth_b.append(implicit_once(mname, T, B, bounds, x, u, x0, Q, P, mx, mu, dt)[2])
                out.update({f"{tag}_x0": x0, f"{tag}_x": x, f"{tag}_u": u, f"{tag}_Q": np_(Q),
                            f"{tag}_P": np_(P), f"{tag}_wx": wx, f"{tag}_wu": wu, f"{tag}_F": F,
                            f"{tag}_f": f, f"{tag}_dQ": dQ, f"{tag}_dP": dP, f"{tag}_dtheta": dth,
                            f"{tag}_dtheta_b": np.stack(dth_b)})
            save(f"{fname}_{tname(dt)}", **out)


# --------------------------------------------------------------------------
# H. the reference's own known-answer datasets (data/*.pkl), parsed statically
# --------------------------------------------------------------------------
def parse_dataset(path):
    data = open(path, "rb").read()
    ops = list(pickletools.genops(data))
    scalars, tensors = {}, {}
    last_key = None
    for i, (op, arg, _pos) in enumerate(ops):
        if op.name in ("SHORT_BINUNICODE", "BINUNICODE") and isinstance(arg, str):
            last_key = arg
        elif op.name in ("BININT1", "BININT2", "BININT", "BINFLOAT") and last_key is not None:
            scalars.setdefault(last_key, arg)
            last_key = None
        elif op.name == "BINBYTES":
            storage = torch.load(io.BytesIO(arg), weights_only=True)
            flat = torch.tensor(storage.tolist(), dtype=storage.dtype)
            # following ops: offset, size tuple, stride tuple (torch._utils._rebuild_tensor_v2)
            ints = []
            for op2, arg2, _ in ops[i + 1:i + 40]:
                if op2.name in ("BININT1", "BININT2", "BININT"):
                    ints.append(arg2)
                if op2.name in ("NEWTRUE", "NEWFALSE"):
                    break
            off, rest = ints[0], ints[1:]
            nd = len(rest) // 2
            size, stride = rest[:nd], rest[nd:]
            owner = [k for k in ("params", "goal_state", "goal_weights", "train_data", "val_data",
                                 "test_data") if k not in tensors][0]
            tensors[owner] = torch.as_strided(flat, size, stride, off).clone().numpy()
    return scalars, tensors


def case_datasets():
    print("H. datasets")
    out = {}
    for env in ("cartpole", "pendulum"):
        scalars, tensors = parse_dataset(os.path.join(REF, "data", env + ".pkl"))
        for k in ("train_data", "val_data", "test_data", "params"):
            out[f"{env}_{k}"] = tensors[k]
        for k in ("lqr_iter", "mpc_T", "linesearch_decay", "max_linesearch_iter", "mpc_eps", "lower", "upper"):
            out[f"{env}_{k}"] = np.array(scalars[k])
    save("datasets", **out)


# --------------------------------------------------------------------------
# I. the IL training loop (il_exp.py:183-429) on a reference dataset
# --------------------------------------------------------------------------
IL_CASES = {
    # name: (dataset, mode, learn_cost, learn_dx, n_train, n_batch, n_epoch, lqr_iter)
    "pend_sysid": ("pendulum", "sysid", False, True, 10, 5, 3, None),
    "pend_empc_dx": ("pendulum", "empc", False, True, 10, 5, 2, 30),
    "pend_empc_cost": ("pendulum", "empc", True, False, 10, 5, 2, 30),
    # the north-star model's dataset (data/cartpole.pkl: 2 train / 1 val / 1 test
    # trajectories, T=35, lqr_iter 100 from the dataset): n_batch 2 (the reference
    # prints matrix_rank(A[1]), lqr_step_explicit.py:561, so a batch needs 2), 4 epochs
    "cart_empc_dx": ("cartpole", "empc", False, True, 2, 2, 4, None),
}


def case_il():
    """IL_Exp(...).run() with its dataset handed over WITHOUT unpickling: the
    IL_Env is rebuilt from the statically parsed dataset and il_exp's `pkl.load`
    is pointed at it (pkl.dump of the best model is a no-op).  setproctitle and
    IPython (absent here) are stand-in modules used only by il_exp's process
    title and excepthook.  The losses/parameter histories come from the CSV
    files run() writes."""
    print("I. il loop")
    import csv
    import shutil
    import tempfile
    st = types.ModuleType("setproctitle")
    st.setproctitle = lambda *a, **k: None
    sys.modules.setdefault("setproctitle", st)
    ip, ipc, ub = types.ModuleType("IPython"), types.ModuleType("IPython.core"), types.ModuleType("IPython.core.ultratb")
    ub.FormattedTB = lambda *a, **k: sys.excepthook
    ip.core, ipc.ultratb = ipc, ub
    for k, v in (("IPython", ip), ("IPython.core", ipc), ("IPython.core.ultratb", ub)):
        sys.modules.setdefault(k, v)
    import il_env
    import il_exp
    out = {}
    for name, (ds, mode, lc, ldx, n_train, n_batch, n_epoch, lqr_iter) in IL_CASES.items():
        scalars, tensors = parse_dataset(os.path.join(REF, "data", ds + ".pkl"))
        env = il_env.IL_Env(ds, lqr_iter=lqr_iter or int(scalars["lqr_iter"]), mpc_T=int(scalars["mpc_T"]))
        for k in ("train_data", "val_data", "test_data"):
            setattr(env, k, torch.tensor(tensors[k], dtype=torch.float32))
        il_exp.pkl = types.SimpleNamespace(load=lambda f, _e=env: _e, dump=lambda *a, **k: None)
        # MKL's multi-threaded getrf/laswp fails on the >100-wide KKT systems
        # (T=35, d=6 -> 210) in this image (see case_implicit); one thread is fine
        torch.set_num_threads(1 if ds == "cartpole" else 8)
        work = tempfile.mkdtemp()
        lin = R.mpc_explicit.MPC.linearize_dynamics
        if mode == "empc":
            # SURVEY.md §8(c) implicit-backward recipe inside the reference's own
            # MPC: the closing linearisation (mpc_explicit.py:302-310) gets the
            # best iterate detached.  The reference makes x, u fresh leaves
            # (.detach().requires_grad_(True)) whose views get_linear_dyn then
            # writes through, which torch 2.10 refuses at backward ("leaf
            # variable has been moved into the graph interior"); those leaves'
            # gradients are consumed by nothing, so detaching them changes no
            # gradient that reaches the parameters (F is built from
            # params.detach(), f = dynamics(x, u) - F tau keeps the params graph,
            # and the no-op LQRStep gets theta = dx.params, 325).
            def lin_detached(self, x, u, dynamics, diff, _lin=lin):
                return _lin(self, x.detach() if diff else x, u.detach() if diff else u, dynamics, diff)
            R.mpc_explicit.MPC.linearize_dynamics = lin_detached
        try:
            exp = il_exp.IL_Exp(data=os.path.join(REF, "data", ds + ".pkl"), work=work, save=os.path.join(work, "s"),
                                n_batch=n_batch, mode=mode, learn_cost=lc, learn_dx=ldx, no_cuda=True, seed=5,
                                n_epoch=n_epoch, n_train=n_train, device="cpu")
            with contextlib.redirect_stdout(io.StringIO()):
                exp.run()
            rd = lambda f: np.array([[float(v) for v in row] for row in list(csv.reader(open(os.path.join(exp.save, f))))[1:]])
            out[f"{name}_train"] = rd("train_losses.csv")
            out[f"{name}_val_test"] = rd("val_test_losses.csv")
            if ldx:
                out[f"{name}_dx_hist"] = np.array([[float(v) for v in row] for row in csv.reader(open(os.path.join(exp.save, "dx_hist.csv")))])
            if lc:
                out[f"{name}_cost_hist"] = np.array([[float(v) for v in row] for row in csv.reader(open(os.path.join(exp.save, "cost_hist.csv")))])
            print(f"  {name}: ok")
        except Exception as e:          # the reference's own failure is recorded, not hidden
            print(f"  {name}: reference raised {type(e).__name__}: {e}")
            out[f"{name}_error"] = np.array(f"{type(e).__name__}: {e}")
        finally:
            R.mpc_explicit.MPC.linearize_dynamics = lin
            shutil.rmtree(work, ignore_errors=True)
    save("il", **out)


# --------------------------------------------------------------------------
# J. generic dynamics / costs: NNDynamics with
#    AUTO_DIFF / FINITE_DIFF / ANALYTIC (grad_input) linearisation through the
#    classic mpc.MPC (+ its backward into the network), an env_dx model with
#    AUTO_DIFF through mpc_explicit, a non-quadratic cost (approximate_cost),
#    and the slew-rate augmentation.  fp64 and fp32.
# --------------------------------------------------------------------------
class NQCost(torch.nn.Module):
    """A smooth non-quadratic stage cost: 1/2|tau|^2 + 0.1 sum tau^4 + w . tau."""

    def __init__(self, w):
        super().__init__()
        self.w = w

    def forward(self, tau):
        return 0.5 * (tau ** 2).sum(-1) + 0.1 * (tau ** 4).sum(-1) + (tau * self.w).sum(-1)


def case_generic():
    print("J. generic dynamics / costs")
    for dt in (torch.float64, torch.float32):
        generic_one(dt)


def generic_one(dt):
    import dynamics as ref_dyn
    out = {}
    with default_dtype(dt), contextlib.redirect_stdout(io.StringIO()):
        T, B = 10, 8
        rng = np.random.RandomState(21)
        # ---- NNDynamics (n=5, m=1, one hidden layer of 32 sigmoids), classic MPC
        torch.manual_seed(3)
        nn_dx = ref_dyn.NNDynamics(5, 1, hidden_sizes=[32], activation="sigmoid")
        for i, fc in enumerate(nn_dx.fcs):
            out[f"nn_W{i}"], out[f"nn_b{i}"] = np_(fc.weight), np_(fc.bias)
        x0 = 0.3 * rng.normal(size=(B, 5))
        L = rng.normal(size=(T, B, 6, 6)) * 0.3
        C = L @ np.swapaxes(L, -1, -2) + np.eye(6)
        c = 0.1 * rng.normal(size=(T, B, 6))
        wx, wu = rng.normal(size=(T, B, 5)), rng.normal(size=(T, B, 1))
        out.update(nn_x0=x0, nn_C=C, nn_c=c, nn_wx=wx, nn_wu=wu)
        for tag, gm in (("auto", R.mpc.GradMethods.AUTO_DIFF), ("fd", R.mpc.GradMethods.FINITE_DIFF),
                        ("analytic", R.mpc.GradMethods.ANALYTIC)):
            for p_ in nn_dx.parameters():
                p_.grad = None
            X0 = torch.tensor(x0, dtype=dt, requires_grad=True)
            Ct, ct = torch.tensor(C, dtype=dt, requires_grad=True), torch.tensor(c, dtype=dt, requires_grad=True)
            m = R.mpc.MPC(5, 1, T, lqr_iter=4, grad_method=gm, u_lower=-1.0, u_upper=1.0, n_batch=B,
                          exit_unconverged=False, detach_unconverged=False, linesearch_decay=0.2,
                          max_linesearch_iter=10)
            x, u, costs = m(X0, R.mpc.QuadCost(Ct, ct), nn_dx)
            ((x * torch.tensor(wx, dtype=dt)).sum() + (u * torch.tensor(wu, dtype=dt)).sum()).backward()
            out.update({f"nn_{tag}_x": np_(x), f"nn_{tag}_u": np_(u), f"nn_{tag}_costs": np_(costs),
                        f"nn_{tag}_dx0": np_(X0.grad), f"nn_{tag}_dC": np_(Ct.grad), f"nn_{tag}_dc": np_(ct.grad)})
            for i, fc in enumerate(nn_dx.fcs):
                out[f"nn_{tag}_dW{i}"] = np_(fc.weight.grad)
                out[f"nn_{tag}_db{i}"] = np_(fc.bias.grad)
        # ---- cartpole through mpc_explicit with AUTO_DIFF (forward)
        dx = model("cartpole")
        x0c = xinit_for("cartpole", B, rng)
        Q, P = true_cost(dx, T, B, dt)
        m = R.mpc_explicit.MPC(5, 1, T, lqr_iter=5, grad_method=R.mpc_explicit.GradMethods.AUTO_DIFF,
                               exit_unconverged=False, detach_unconverged=False, linesearch_decay=0.5,
                               max_linesearch_iter=2, eps=0.0, not_improved_lim=10 ** 9)
        x, u, costs = m(torch.tensor(x0c, dtype=dt), R.mpc_explicit.QuadCost(Q, P), dx)
        out.update(cart_auto_x0=x0c, cart_auto_x=np_(x), cart_auto_u=np_(u), cart_auto_costs=np_(costs))
        # ---- cartpole with a slew-rate penalty: mpc_explicit ANALYTIC and mpc AUTO_DIFF (forward)
        for tag, mod, gm in (("slew_explicit", R.mpc_explicit, R.mpc_explicit.GradMethods.ANALYTIC),
                             ("slew_classic", R.mpc, R.mpc.GradMethods.AUTO_DIFF)):
            m = mod.MPC(5, 1, T, lqr_iter=5, grad_method=gm, slew_rate_penalty=0.1, exit_unconverged=False,
                        detach_unconverged=False, linesearch_decay=0.5, max_linesearch_iter=2, eps=0.0,
                        not_improved_lim=10 ** 9)
            x, u, costs = m(torch.tensor(x0c, dtype=dt), mod.QuadCost(Q, P), dx)
            out.update({f"{tag}_x": np_(x), f"{tag}_u": np_(u), f"{tag}_costs": np_(costs)})
        # ---- cartpole with the delta_u trust region (lqr_step_explicit.py:205-213)
        m = R.mpc_explicit.MPC(5, 1, T, lqr_iter=5, grad_method=R.mpc_explicit.GradMethods.ANALYTIC,
                               u_lower=-10.0, u_upper=10.0, delta_u=1.0, exit_unconverged=False,
                               detach_unconverged=False, linesearch_decay=0.5, max_linesearch_iter=2, eps=0.0,
                               not_improved_lim=10 ** 9)
        x, u, costs = m(torch.tensor(x0c, dtype=dt), R.mpc_explicit.QuadCost(Q, P), dx)
        out.update(delta_u_x=np_(x), delta_u_u=np_(u), delta_u_costs=np_(costs))
        # ---- pendulum with a non-quadratic cost: mpc AUTO_DIFF and mpc_explicit ANALYTIC (forward)
        dxp = model("pendulum")
        x0p = xinit_for("pendulum", B, rng)
        wq = 0.3 * rng.normal(size=4)
        out.update(nq_x0=x0p, nq_w=wq)
        for tag, mod, gm in (("nq_classic", R.mpc, R.mpc.GradMethods.AUTO_DIFF),
                             ("nq_explicit", R.mpc_explicit, R.mpc_explicit.GradMethods.ANALYTIC)):
            m = mod.MPC(3, 1, T, lqr_iter=5, grad_method=gm, n_batch=B, exit_unconverged=False,
                        detach_unconverged=False, linesearch_decay=0.2, max_linesearch_iter=5, eps=0.0,
                        not_improved_lim=10 ** 9, u_lower=-2.0, u_upper=2.0)
            x, u, costs = m(torch.tensor(x0p, dtype=dt), NQCost(torch.tensor(wq, dtype=dt)), dxp)
            out.update({f"{tag}_x": np_(x), f"{tag}_u": np_(u), f"{tag}_costs": np_(costs)})
    save(f"generic_{tname(dt)}", **out)


# --------------------------------------------------------------------------
# K. API options: delta_u on LQRStep, u_zero_I on both MPCs and the implicit step
# --------------------------------------------------------------------------
def case_api():
    print("K. api options")
    for dt in (torch.float64, torch.float32):
        out = {}
        with default_dtype(dt), contextlib.redirect_stdout(io.StringIO()):
            # ---- LQRStep(delta_u) (lqr_step_explicit.py:132-135, 205-213), the lqrstep 'box' setup
            dx = model("cartpole")
            T, B = 25, 16
            rng = np.random.RandomState(11)
            x0 = xinit_for("cartpole", B, rng)
            u = rng.uniform(-2, 2, (T, B, 1))
            X0, U = torch.tensor(x0, dtype=dt), torch.tensor(u, dtype=dt)
            Q, P = true_cost(dx, T, B, dt)
            mpc_ = R.mpc_explicit.MPC(5, 1, T, lqr_iter=1)
            with torch.no_grad():
                X = R.util.get_traj(T, U, x_init=X0, dynamics=dx)
                F, f = mpc_.linearize_dynamics(X, U, dx, diff=False)
                step = R.lqr_step_explicit.LQRStep(
                    5, 1, T, u_lower=-5.0, u_upper=5.0, delta_u=0.5, true_cost=R.mpc_explicit.QuadCost(Q, P),
                    true_dynamics=dx, current_x=X, current_u=U, linesearch_decay=0.5, max_linesearch_iter=2)
                nx, nu, nqp, costs, du, malpha = step(X0, Q, P, F, f, None)
            out.update(dlt_x0=x0, dlt_u=u, dlt_x=np_(X), dlt_F=np_(F), dlt_f=np_(f), dlt_nx=np_(nx),
                       dlt_nu=np_(nu), dlt_costs=np_(costs), dlt_malpha=np_(malpha))
            # ---- MPC(u_zero_I): cartpole unconstrained / +-10, rocket (m = 3) unconstrained
            for tag, mname, T, B, it, bounds in (("zi_cart", "cartpole", 10, 8, 5, None),
                                                 ("zi_cartbox", "cartpole", 10, 8, 5, (-10.0, 10.0)),
                                                 ("zi_rock", "rocket", 10, 4, 3, None)):
                dxm = model(mname)
                rng = np.random.RandomState(7)
                x0 = xinit_for(mname, B, rng)
                zI = rng.uniform(size=(T, B, dxm.n_ctrl)) < 0.25
                Q, P = true_cost(dxm, T, B, dt)
                kw = {} if bounds is None else dict(u_lower=bounds[0], u_upper=bounds[1])
                decay, mls = (0.5, 2) if mname == "cartpole" else (0.2, 5)
                m = R.mpc_explicit.MPC(dxm.n_state, dxm.n_ctrl, T, lqr_iter=it, eps=0.0, not_improved_lim=10 ** 9,
                                       linesearch_decay=decay, max_linesearch_iter=mls, exit_unconverged=False,
                                       detach_unconverged=False, verbose=-1, u_zero_I=torch.tensor(zI),
                                       grad_method=R.mpc_explicit.GradMethods.ANALYTIC, **kw)
                with torch.no_grad():
                    x, uu, costs = m(torch.tensor(x0, dtype=dt), R.mpc_explicit.QuadCost(Q, P), dxm)
                out.update({f"{tag}_x0": x0, f"{tag}_zI": zI, f"{tag}_x": np_(x), f"{tag}_u": np_(uu),
                            f"{tag}_costs": np_(costs)})
            # ---- the DiLQR no-op step with u_zero_I (its Riccati gains feed the implicit backward)
            mname, T, B = "cartpole", 10, 4
            dxm = model(mname)
            rng = np.random.RandomState(9)
            x0 = xinit_for(mname, B, rng)
            u = rng.uniform(-1, 1, (T, B, 1))
            zI = rng.uniform(size=(T, B, 1)) < 0.25
            Q, P = true_cost(dxm, T, B, dt)
            wx, wu = rng.normal(size=(T, B, 5)), rng.normal(size=(T, B, 1))
            X = R.util.get_traj(T, torch.tensor(u, dtype=dt), x_init=torch.tensor(x0, dtype=dt), dynamics=dxm)
            theta = dxm.params.detach().clone().to(dt).requires_grad_(True)
            Qg, Pg = Q.clone().requires_grad_(True), P.clone().requires_grad_(True)
            mm = R.mpc_explicit.MPC(5, 1, T, grad_method=R.mpc_explicit.GradMethods.ANALYTIC)
            F, f = mm.linearize_dynamics(X, torch.tensor(u, dtype=dt), dxm, diff=True)
            step = R.lqr_step_explicit.LQRStep(5, 1, T, u_zero_I=torch.tensor(zI), true_cost=R.mpc_explicit.QuadCost(
                Qg, Pg), true_dynamics=dxm, current_x=X.detach(), current_u=torch.tensor(u, dtype=dt),
                back_eps=mm.back_eps, no_op_forward=True)
            x2, u2 = step(torch.tensor(x0, dtype=dt), Qg, Pg, F.detach(), f.detach(), theta)
            ((x2 * torch.tensor(wx, dtype=dt)).sum() + (u2 * torch.tensor(wu, dtype=dt)).sum()).backward()
            out.update(zim_x0=x0, zim_u=u, zim_x=np_(X), zim_zI=zI, zim_wx=wx, zim_wu=wu, zim_dQ=np_(Qg.grad),
                       zim_dP=np_(Pg.grad), zim_dtheta=np_(theta.grad))
        save(f"api_{tname(dt)}", **out)


# --------------------------------------------------------------------------
# M. LQRStep (both variants) with a generic true_cost / true_dynamics: the line
#    search evaluates true_cost(new_xut) and true_dynamics(x, u)
#    (lqr_step_explicit.py:226-236, lqr_step.py:224-234)
# --------------------------------------------------------------------------
def case_stepgen():
    import dynamics as ref_dyn
    print("M. LQRStep with generic true_cost / true_dynamics")
    dt = torch.float64
    out = {}
    with default_dtype(dt), contextlib.redirect_stdout(io.StringIO()):
        # ---- pendulum, non-quadratic true_cost, the sweep on the true objective's C, c
        T, B = 10, 8
        rng = np.random.RandomState(31)
        dxp = model("pendulum")
        x0 = xinit_for("pendulum", B, rng)
        u = rng.uniform(-1, 1, (T, B, 1))
        wq = 0.3 * rng.normal(size=4)
        X0, U = torch.tensor(x0), torch.tensor(u)
        Q, P = true_cost(dxp, T, B, dt)
        cost = NQCost(torch.tensor(wq))
        with torch.no_grad():
            X = R.util.get_traj(T, U, x_init=X0, dynamics=dxp)
            F, f = R.mpc_explicit.MPC(3, 1, T, lqr_iter=1).linearize_dynamics(X, U, dxp, diff=False)
        out.update(nq_x0=x0, nq_u=u, nq_w=wq, nq_X=np_(X), nq_F=np_(F), nq_f=np_(f))
        for tag, mod in (("explicit", R.lqr_step_explicit), ("classic", R.lqr_step)):
            step = mod.LQRStep(3, 1, T, u_lower=-2.0, u_upper=2.0, true_cost=cost, true_dynamics=dxp,
                               current_x=X, current_u=U, linesearch_decay=0.2, max_linesearch_iter=5)
            args = (X0, Q, P, F, f) + ((None,) if tag == "explicit" else ())
            with torch.no_grad():
                nx, nu, nqp, costs, du, malpha = step(*args)
            out.update({f"nq_{tag}_nx": np_(nx), f"nq_{tag}_nu": np_(nu), f"nq_{tag}_costs": np_(costs),
                        f"nq_{tag}_du": np_(du), f"nq_{tag}_malpha": np_(malpha), f"nq_{tag}_nqp": np_(nqp)})
        # ---- NNDynamics true_dynamics (n=5, m=1), quadratic true_cost, AUTO_DIFF linearisation
        torch.manual_seed(5)
        nn_dx = ref_dyn.NNDynamics(5, 1, hidden_sizes=[32], activation="sigmoid")
        for i, fc in enumerate(nn_dx.fcs):
            out[f"nn_W{i}"], out[f"nn_b{i}"] = np_(fc.weight), np_(fc.bias)
        x0 = 0.3 * rng.normal(size=(B, 5))
        u = 0.3 * rng.normal(size=(T, B, 1))
        L = rng.normal(size=(T, B, 6, 6)) * 0.3
        C = L @ np.swapaxes(L, -1, -2) + np.eye(6)
        c = 0.1 * rng.normal(size=(T, B, 6))
        X0, U, Ct, ct = (torch.tensor(a) for a in (x0, u, C, c))
        X = R.util.get_traj(T, U, x_init=X0, dynamics=nn_dx).detach()
        F, f = R.mpc_explicit.MPC(5, 1, T, lqr_iter=1, grad_method=R.mpc_explicit.GradMethods.AUTO_DIFF
                                  ).linearize_dynamics(X, U, nn_dx, diff=False)
        F, f = F.detach(), f.detach()
        out.update(nn_x0=x0, nn_u=u, nn_C=C, nn_c=c, nn_X=np_(X), nn_F=np_(F), nn_f=np_(f))
        for tag, mod in (("explicit", R.lqr_step_explicit), ("classic", R.lqr_step)):
            step = mod.LQRStep(5, 1, T, u_lower=-1.0, u_upper=1.0, true_cost=R.mpc_explicit.QuadCost(Ct, ct),
                               true_dynamics=nn_dx, current_x=X, current_u=U, linesearch_decay=0.2,
                               max_linesearch_iter=10)
            args = (X0, Ct, ct, F, f) + ((None,) if tag == "explicit" else ())
            with torch.no_grad():
                nx, nu, nqp, costs, du, malpha = step(*args)
            out.update({f"nn_{tag}_nx": np_(nx), f"nn_{tag}_nu": np_(nu), f"nn_{tag}_costs": np_(costs),
                        f"nn_{tag}_du": np_(du), f"nn_{tag}_malpha": np_(malpha), f"nn_{tag}_nqp": np_(nqp)})
    save("stepgen_f64", **out)


# --------------------------------------------------------------------------
# L. the 5-parameter pendulum (pendulum.py simple=False, il_env.py:40-42
#    'pendulum-complex'): forward, its autograd Jacobian (the reference's own
#    closed forms unpack three parameters and fail for it), and MPC solves
#    through mpc_explicit.MPC with GradMethods.AUTO_DIFF, the runnable path
# --------------------------------------------------------------------------
COMPLEX_PARAMS = (10., 1., 1., 1.0, 0.1)        # il_env.py:41
COMPLEX_MPC = {
    # name: (T, B, lqr_iter, eps, not_improved_lim)  bounds +-2, decay 0.2, max_ls 5 (pendulum.py:52-58)
    "fixed": (20, 16, 10, 0.0, 10 ** 9),
    "il": (20, 16, 40, 1e-3, 5),
}


def case_complex():
    print("L. pendulum-complex")
    for dt in (torch.float64, torch.float32):
        with default_dtype(dt):
            out = {}
            dxm = R.pendulum.PendulumDx(torch.tensor(COMPLEX_PARAMS, dtype=dt), simple=False)
            rng = np.random.RandomState(21)
            x, u = sample_states("pendulum", 256, rng)
            X = torch.tensor(x, dtype=dt, requires_grad=True)
            U = torch.tensor(u, dtype=dt, requires_grad=True)
            nx = dxm(X, U)
            rows = [torch.autograd.grad(nx[:, j].sum(), [X, U], retain_graph=True) for j in range(3)]
            D = torch.stack([torch.cat(r, 1) for r in rows], 1)          # [N, n, d], as AUTO_DIFF forms it
            out.update(x=x, u=u, fwd=np_(nx), jac=np_(D))
            for name, (T, B, it, eps, nil) in COMPLEX_MPC.items():
                rng = np.random.RandomState(3)
                x0 = xinit_for("pendulum", B, rng)
                Q, P = true_cost(dxm, T, B, dt)
                m = R.mpc_explicit.MPC(3, 1, T, u_lower=-2.0, u_upper=2.0, lqr_iter=it, eps=eps,
                                       not_improved_lim=nil, linesearch_decay=0.2, max_linesearch_iter=5,
                                       exit_unconverged=False, detach_unconverged=False, verbose=-1,
                                       grad_method=R.mpc_explicit.GradMethods.AUTO_DIFF)
                # AUTO_DIFF differentiates the dynamics with torch.autograd.grad
                # (mpc_explicit.py:562-566): grad mode stays on
                with contextlib.redirect_stdout(io.StringIO()):
                    xs, us, costs = m(torch.tensor(x0, dtype=dt), R.mpc_explicit.QuadCost(Q, P), dxm)
                out.update({f"{name}_x0": x0, f"{name}_x": np_(xs), f"{name}_u": np_(us),
                            f"{name}_costs": np_(costs)})
            save(f"complex_{tname(dt)}", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["models", "riccati", "pnqp", "lqrstep", "mpc", "adjoint", "implicit",
                             "implicit25", "datasets", "il", "generic", "api", "complex", "stepgen"]
    table = {"models": case_models, "riccati": case_riccati, "pnqp": case_pnqp,
             "lqrstep": case_lqrstep, "mpc": case_mpc, "mpc_iterates": case_mpc_iterates,
             "adjoint": case_classic_adjoint,
             "implicit": case_implicit, "implicit25": case_implicit25, "datasets": case_datasets, "il": case_il,
             "generic": case_generic, "api": case_api, "complex": case_complex, "stepgen": case_stepgen}
    for w in which:
        table[w]()
