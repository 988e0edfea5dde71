"""Pin the numpy oracle against golden vectors produced by the reference itself.

CPU-only.  The goldens (tests/golden/*.npz) were written by
tests/golden/gen_golden.py, which ran the reference in the build container.
fp64 goldens are compared tightly (the oracle restates the same algorithm, so
only summation-order rounding differs); fp32 goldens loosely.
"""
import numpy as np
import pytest

from oracle import adjoint, lqr, models, mpc

MODELS = models.MODELS


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))


# ---------------------------------------------------------------- models
@pytest.mark.parametrize("name", ["pendulum", "cartpole", "rocket"])
@pytest.mark.parametrize("prec,tol", [("f64", 1e-12), ("f32", 2e-5)])
def test_model_forward_and_jacobian(golden, name, prec, tol):
    g = golden(f"models_{prec}")
    dt = np.float64 if prec == "f64" else np.float32
    M = MODELS[name]
    x, u = g[f"{name}_x"].astype(dt), g[f"{name}_u"].astype(dt)
    assert rel(M.forward(x, u), g[f"{name}_fwd"]) < tol
    assert rel(M.get_linear_dyn(x, u), g[f"{name}_D"]) < tol * 10




@pytest.mark.parametrize("name", ["pendulum", "cartpole", "rocket"])
def test_model_get_matrices(golden, name):
    g = golden("models_f64")
    M = MODELS[name]
    x, u = g[f"{name}_x"][:16], g[f"{name}_u"][:16]
    mats = M.get_matrices(x, u)
    for key, val in zip(("D", "D_params", "D_x", "D_u", "x_theta", "x_xtm1", "x_utm1"), mats):
        ref = g[f"{name}_gm_{key}"]
        assert ref.shape == val.shape, (key, ref.shape, val.shape)
        assert rel(val, ref) < 1e-10, key


@pytest.mark.parametrize("name", ["pendulum", "cartpole", "rocket"])
def test_model_grad_input(golden, name):
    g = golden("models_f64")
    M = MODELS[name]
    out = M.grad_input(g[f"{name}_gi_X"], g[f"{name}_gi_U"], g[f"{name}_gi_K"])
    for key, val in zip(("grad_D", "grad_d", "D_x", "D_u", "D", "d_x", "d_u"), out):
        ref = g[f"{name}_gi_{key}"]
        assert ref.shape == val.shape, (key, ref.shape, val.shape)
        assert rel(val, ref) < 1e-10, key


# ---------------------------------------------------------------- Riccati
SHAPES = {"pendulum": (3, 1, 10, 16), "cartpole": (5, 1, 25, 16), "rocket": (13, 3, 30, 8)}


@pytest.mark.parametrize("name", list(SHAPES))
@pytest.mark.parametrize("variant", ["", "chol_", "zI_", "box_"])
def test_riccati(golden, name, variant):
    g = golden("riccati_f64")
    n, m, T, B = SHAPES[name]
    C, c, F, u = g[f"{name}_C"], g[f"{name}_c"], g[f"{name}_F"], g[f"{name}_u"]
    kw = {}
    if variant == "chol_":
        kw = dict(m_solver="chol")
    elif variant == "zI_":
        kw = dict(m_solver="chol", u_zero_I=g[f"{name}_zI"])
    elif variant == "box_":
        kw = dict(u=u, u_lower=-1.0, u_upper=1.0)
    K, k, _ = lqr.lqr_backward(C, c, F, n, m, **kw)
    assert rel(K, g[f"{name}_{variant}K"]) < 1e-9
    assert rel(k, g[f"{name}_{variant}k"]) < 1e-9


# ---------------------------------------------------------------- pnqp
@pytest.mark.parametrize("m", [1, 3])
def test_pnqp(golden, m):
    g = golden("pnqp_f64")
    H, q, lo, hi, x0 = (g[f"m{m}_{k}"] for k in ("H", "q", "lo", "hi", "x0"))
    x, _, If, it = lqr.pnqp(H, q, lo, hi)
    assert rel(x, g[f"m{m}_x"]) < 1e-10 and it == g[f"m{m}_it"]
    np.testing.assert_array_equal(If, g[f"m{m}_If"])
    x, _, If, it = lqr.pnqp(H, q, -0.7, 0.7, x_init=x0)
    assert rel(x, g[f"m{m}_xf"]) < 1e-10 and it == g[f"m{m}_itf"]
    x, _, _, its = lqr.pnqp(H, q, lo, hi, per_problem=True)
    assert rel(x, g[f"m{m}_x_pp"]) < 1e-10
    np.testing.assert_array_equal(its, g[f"m{m}_it_pp"])


# ---------------------------------------------------------------- one LQR step
@pytest.mark.parametrize("tag,bounds", [("unc", None), ("box", (-5.0, 5.0))])
def test_lqr_step(golden, tag, bounds):
    g = golden("lqrstep_f64")
    M = MODELS["cartpole"]
    x0, u, x = g[f"{tag}_x0"], g[f"{tag}_u"], g[f"{tag}_x"]
    T, B, _ = u.shape
    assert rel(lqr.get_traj(T, u, x0, M.forward), x) < 1e-12
    F, f = mpc.linearize(M, x, u)
    assert rel(F, g[f"{tag}_F"]) < 1e-12 and rel(f, g[f"{tag}_f"]) < 1e-12
    q, p = M.true_obj()
    C, c = mpc.expand_cost(np.diag(q), p, T, B)
    lo, hi = bounds if bounds else (None, None)
    K, k, _ = lqr.lqr_backward(C, lqr.c_back(C, c, x, u), F, 5, 1, u=u, u_lower=lo, u_upper=hi)
    nx, nu, costs, du, _, malpha, _ = lqr.lqr_forward(x0, C, c, x, u, K, k, M.forward, lo, hi, None, 0.5, 2)
    assert rel(nx, g[f"{tag}_nx"]) < 1e-10
    assert rel(nu, g[f"{tag}_nu"]) < 1e-10
    assert rel(costs, g[f"{tag}_costs"]) < 1e-10
    assert rel(du, g[f"{tag}_du"]) < 1e-10
    assert abs(malpha - g[f"{tag}_malpha"]) < 1e-12


# ---------------------------------------------------------------- MPC solves
MPC_CASES = {
    "cart_unc": ("cartpole", 25, 10, None, 0.0, 10 ** 9, 0.5, 2),
    "cart_box10": ("cartpole", 25, 10, (-10.0, 10.0), 0.0, 10 ** 9, 0.5, 2),
    "cart_il": ("cartpole", 25, 40, (-100.0, 100.0), 1e-4, 5, 0.5, 2),
    "pend_unc": ("pendulum", 10, 10, None, 0.0, 10 ** 9, 0.2, 5),
    "pend_box": ("pendulum", 10, 10, (-2.0, 2.0), 0.0, 10 ** 9, 0.2, 5),
    "rocket_unc": ("rocket", 30, 5, None, 0.0, 10 ** 9, 0.2, 5),
}


def run_oracle_mpc(g, name, dt, **over):
    mname, T, it, bounds, eps, nil, decay, mls = MPC_CASES[name]
    M = MODELS[mname]
    x0 = g[f"{name}_x0"].astype(dt)
    B = x0.shape[0]
    q, p = M.true_obj()
    C, c = mpc.expand_cost(np.diag(q).astype(dt), p.astype(dt), T, B)
    lo, hi = bounds if bounds else (None, None)
    kw = dict(u_lower=lo, u_upper=hi, lqr_iter=it, eps=eps, not_improved_lim=nil,
              linesearch_decay=decay, max_linesearch_iter=mls)
    kw.update(over)
    return mpc.mpc_forward(M, x0, C, c, T, **kw)


@pytest.mark.parametrize("name", list(MPC_CASES))
def test_mpc_f64(golden, name):
    g = golden("mpc_f64")
    x, u, costs, _ = run_oracle_mpc(g, name, np.float64)
    assert rel(x, g[f"{name}_x"]) < 1e-8
    assert rel(u, g[f"{name}_u"]) < 1e-8
    assert rel(costs, g[f"{name}_costs"]) < 1e-8


@pytest.mark.parametrize("name", ["cart_unc", "cart_box10", "pend_box"])
def test_mpc_iterates_f64(golden, name):
    g = golden("mpc_f64")
    if f"{name}_it1_u" not in g:
        pytest.skip("no per-iteration goldens for this case")
    for k in (1, 2, 3):
        x, u, costs, _ = run_oracle_mpc(g, name, np.float64, lqr_iter=k)
        assert rel(u, g[f"{name}_it{k}_u"]) < 1e-9, k


@pytest.mark.parametrize("name", ["cart_unc", "cart_box10", "pend_unc", "pend_box"])
def test_mpc_f32(golden, name):
    """fp32 oracle vs fp32 reference: same algorithm, different summation
    order; line-search/active-set decisions can flip on 1-ulp differences, so
    the bar is the trajectory cost."""
    g = golden("mpc_f32")
    x, u, costs, _ = run_oracle_mpc(g, name, np.float32)
    ref = g[f"{name}_costs"]
    assert np.max(np.abs(costs - ref) / np.maximum(1.0, np.abs(ref))) < 1e-3


# ---------------------------------------------------------------- 5-parameter pendulum
@pytest.mark.parametrize("prec,tol", [("f64", 1e-12), ("f32", 2e-5)])
def test_pendulum_complex_forward_and_jacobian(golden, prec, tol):
    """pendulum.py simple=False: forward and its autograd Jacobian (the
    reference's AUTO_DIFF linearisation, mpc_explicit.py:562-566)."""
    g = golden(f"complex_{prec}")
    dt = np.float64 if prec == "f64" else np.float32
    x, u = g["x"].astype(dt), g["u"].astype(dt)
    PC = models.PendulumComplex
    assert rel(PC.forward(x, u), g["fwd"]) < tol
    assert rel(PC.get_linear_dyn(x, u), g["jac"]) < 10 * tol


@pytest.mark.parametrize("name", ["fixed", "il"])
def test_pendulum_complex_mpc_f64(golden, name):
    """mpc_explicit.MPC(GradMethods.AUTO_DIFF) on the 5-parameter pendulum,
    bounds +-2, decay 0.2, max_ls 5 (the reference's fp64 run)."""
    g = golden("complex_f64")
    T, B = g[f"{name}_u"].shape[:2]
    it, eps, nil = {"fixed": (10, 0.0, 10 ** 9), "il": (40, 1e-3, 5)}[name]
    q, p = models.PendulumComplex.true_obj()
    C, c = mpc.expand_cost(np.diag(q), p, T, B)
    x, u, costs, _ = mpc.mpc_forward(models.PendulumComplex, g[f"{name}_x0"], C, c, T, u_lower=-2.0, u_upper=2.0,
                                     lqr_iter=it, eps=eps, not_improved_lim=nil, linesearch_decay=0.2,
                                     max_linesearch_iter=5)
    assert rel(u, g[f"{name}_u"]) < 1e-8 and rel(x, g[f"{name}_x"]) < 1e-8
    assert rel(costs, g[f"{name}_costs"]) < 1e-8


# ---------------------------------------------------------------- classic adjoint
@pytest.mark.parametrize("tag,bounds", [("m1", None), ("m3", None), ("m1box", (-0.5, 0.5)),
                                        ("m3box", (-0.5, 0.5))])
def test_classic_adjoint(golden, tag, bounds):
    g = golden("adjoint_f64")
    C, c, F, f, x0 = (g[f"{tag}_{k}"] for k in ("C", "c", "F", "f", "x0"))
    T, B, d = c.shape
    n = x0.shape[1]
    m = d - n
    lo, hi = bounds if bounds else (None, None)
    x, u, costs, _ = mpc.mpc_forward(("lin", F, f), x0, C, c, T, u_lower=lo, u_upper=hi, lqr_iter=1)
    assert rel(x, g[f"{tag}_x"]) < 1e-10 and rel(u, g[f"{tag}_u"]) < 1e-10
    dx0, dC, dc, dF, df = adjoint.classic_backward(g[f"{tag}_wx"], g[f"{tag}_wu"], x0, C, c, F, f,
                                                   x, u, lo, hi)
    for key, val in (("dx0", dx0), ("dC", dC), ("dc", dc), ("dF", dF), ("df", df)):
        assert rel(val, g[f"{tag}_{key}"]) < 1e-9, key


# ---------------------------------------------------------------- DiLQR implicit backward
IMPLICIT = {"cart_unc": ("cartpole", None), "cart_box": ("cartpole", (-5.0, 5.0)),
            "pend_box": ("pendulum", (-2.0, 2.0)), "rock_unc": ("rocket", None),
            "rock_box": ("rocket", (-10.0, 10.0)),
            # config 4's horizon: cartpole T=25, B=8 (gen_golden.py IMPLICIT25_CASES)
            "cart25_unc": ("cartpole", None), "cart25_box10": ("cartpole", (-10.0, 10.0)),
            "cart25_box100": ("cartpole", (-100.0, 100.0))}


def implicit_file(tag, prec="f64"):
    return f"implicit25_{prec}" if tag.startswith("cart25") else f"implicit_{prec}"


@pytest.mark.parametrize("tag", list(IMPLICIT))
def test_implicit_backward_f64(golden, tag):
    g = golden(implicit_file(tag))
    mname, bounds = IMPLICIT[tag]
    M = MODELS[mname]
    x, u, Q, P, F = (g[f"{tag}_{k}"] for k in ("x", "u", "Q", "P", "F"))
    T, B, n = x.shape
    m = u.shape[2]
    Fo, fo = mpc.linearize(M, x, u)
    assert rel(Fo, F) < 1e-12
    lo, hi = bounds if bounds else (None, None)
    K, _, _ = lqr.lqr_backward(Q, lqr.c_back(Q, P, x, u), Fo, n, m, u=u, u_lower=lo, u_upper=hi)
    dC, dc, dth = adjoint.implicit_backward(M, g[f"{tag}_wx"], g[f"{tag}_wu"], Q, P, Fo, fo, x, u,
                                            K[::-1], lo, hi)
    assert rel(dth, g[f"{tag}_dtheta_b"]) < 1e-6
    assert rel(dth.sum(0), g[f"{tag}_dtheta"]) < 1e-6
    assert rel(dC, g[f"{tag}_dQ"]) < 1e-6
    assert rel(dc, g[f"{tag}_dP"]) < 1e-6


# ---------------------------------------------------------------- the reference's own datasets
def test_dataset_cartpole_known_answer(golden):
    """data/cartpole.pkl: expert trajectories made by the reference solver
    (il_env.py:81-94) at fp32, T=35, lqr_iter=100, bounds +-100, eps 1e-4,
    decay 0.5, max_ls 2, start th = pi/1.05.  Re-solve from their x_init."""
    g = golden("datasets")
    tau = np.concatenate([g["cartpole_train_data"], g["cartpole_val_data"], g["cartpole_test_data"]])
    tau = tau.astype(np.float32)
    M = MODELS["cartpole"]
    T = int(g["cartpole_mpc_T"])
    x0 = tau[:, 0, :5]
    B = x0.shape[0]
    q, p = M.true_obj()
    C, c = mpc.expand_cost(np.diag(q).astype(np.float32), p.astype(np.float32), T, B)
    x, u, costs, _ = mpc.mpc_forward(M, x0, C, c, T, u_lower=float(g["cartpole_lower"]),
                                     u_upper=float(g["cartpole_upper"]), lqr_iter=int(g["cartpole_lqr_iter"]),
                                     eps=float(g["cartpole_mpc_eps"]), linesearch_decay=float(g["cartpole_linesearch_decay"]),
                                     max_linesearch_iter=int(g["cartpole_max_linesearch_iter"]))
    got = np.concatenate([x, u], 2).transpose(1, 0, 2)
    assert np.max(np.abs(got - tau)) < 5e-3


@pytest.mark.parametrize("tag", list(IMPLICIT))
def test_implicit_backward_fast_f64(golden, tag):
    """The O(T d^3) algebra (the one the HIP kernels use, and the checker the
    full-size GPU tests call) against the reference's (T d)^3 KKT solve."""
    g = golden(implicit_file(tag))
    mname, bounds = IMPLICIT[tag]
    M = MODELS[mname]
    x, u, Q, P = (g[f"{tag}_{k}"] for k in ("x", "u", "Q", "P"))
    T, B, n = x.shape
    m = u.shape[2]
    Fo, fo = mpc.linearize(M, x, u)
    lo, hi = bounds if bounds else (None, None)
    K, _, _ = lqr.lqr_backward(Q, lqr.c_back(Q, P, x, u), Fo, n, m, u=u, u_lower=lo, u_upper=hi)
    dC, dc, dth = adjoint.implicit_backward_fast(M, g[f"{tag}_wx"], g[f"{tag}_wu"], Q, P, Fo, fo, x, u,
                                                 K[::-1], lo, hi)
    # rocket: the reference's dense 160x160 KKT solve (lqr_step_explicit.py:570)
    # is ill-conditioned enough to move its fp64 dtheta by ~6.5e-6 relative to
    # the recursion's; every other case agrees to < 1e-6
    tol = 2e-5 if mname == "rocket" else 1e-6
    assert rel(dth, g[f"{tag}_dtheta_b"]) < tol
    assert rel(dC, g[f"{tag}_dQ"]) < tol
    assert rel(dc, g[f"{tag}_dP"]) < tol
