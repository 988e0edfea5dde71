"""API-fidelity tests of the MPC classes on the GPU (round 5):

  * `verbose > 0` prints the reference's per-iteration table
    (mpc_explicit.py:236-241, 285-295; util.table_log, util.py:80-101) from
    figures the device recorded, one row per iteration the solve ran;
  * the classic mpc.MPC sends a gradient into an env_dx model's params the
    way the reference's AUTO_DIFF linearisation does (mpc.py:538-551: F as
    data, f = dynamics(x, u) - F tau with the params graph), and refuses it for
    the 5-parameter pendulum instead of dropping it.
"""
import re

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def cartpole_case(B, T, seed=0):
    from dilqr.env_dx.cartpole import CartpoleDx
    rng = np.random.RandomState(seed)
    th = rng.uniform(-np.pi, np.pi, B)
    x0 = np.stack([rng.uniform(-.5, .5, B), rng.uniform(-.5, .5, B), np.cos(th), np.sin(th),
                   rng.uniform(-1, 1, B)], 1)
    dx = CartpoleDx()
    q, p = dx.get_true_obj()
    C = torch.diag(q).repeat(T, B, 1, 1).to(DEV)
    c = p.repeat(T, B, 1).to(DEV)
    return dx, torch.tensor(x0, dtype=torch.float32, device=DEV), C, c


ROW = re.compile(r"^\| (\d+) \| (\S+) \| (\S+) \| (\S+) \| (\S+) \|$")


@pytest.mark.parametrize("mode", ["stop_rule", "fixed", "box", "u_zero_I"])
def test_verbose_table(capsys, mode):
    """The verbose report: 'Initial mean(cost)', the table header once, then one
    row per iteration that ran; the last row's mean(cost) is the returned costs'
    mean and every row's figures are finite.  A verbose solve returns the same
    bits as a quiet one (the same launches, one iteration per call)."""
    import dilqr
    from dilqr import util
    util._seen_tables.discard("lqr")
    T, B = 12, 256
    dx, x0, C, c = cartpole_case(B, T)
    kw = dict(lqr_iter=8, exit_unconverged=False, detach_unconverged=False, linesearch_decay=0.5,
              max_linesearch_iter=2)
    if mode == "stop_rule":
        kw.update(eps=1e-2, not_improved_lim=3)
    elif mode == "fixed":
        kw.update(eps=0.0, not_improved_lim=10 ** 9)
    elif mode == "box":
        kw.update(eps=1e-3, u_lower=-2.0, u_upper=2.0)
    else:
        zI = torch.zeros(T, B, 1, dtype=torch.bool, device=DEV)
        zI[-3:] = True
        kw.update(eps=1e-3, u_zero_I=zI)
    quiet = dilqr.MPC(5, 1, T, verbose=0, **kw)
    loud = dilqr.MPC(5, 1, T, verbose=1, **kw)
    with torch.no_grad():
        xq, uq, cq = quiet(x0, dilqr.QuadCost(C, c), dx)
        capsys.readouterr()
        xv, uv, cv = loud(x0, dilqr.QuadCost(C, c), dx)
    out = capsys.readouterr().out.strip().splitlines()
    assert torch.equal(xq, xv) and torch.equal(uq, uv) and torch.equal(cq, cv)
    assert out[0].startswith("Initial mean(cost): ")
    assert np.isfinite(float(out[0].split(":")[1]))
    assert out[1] == "| iter | mean(cost) | ||full_du||_max | mean(alphas) | total_qp_iters |"
    rows = [ROW.match(l) for l in out[2:]]
    assert rows and all(rows), out
    its = [int(r.group(1)) for r in rows]
    assert its == list(range(len(its)))
    sv = loud.last_solve
    assert len(its) == sv.log["iterations"]
    if mode == "fixed":
        assert len(its) == 8
    last = rows[-1]
    assert float(last.group(2)) == pytest.approx(float(cv.mean()), rel=1e-4)
    for r in rows:
        assert np.isfinite(float(r.group(3))) and np.isfinite(float(r.group(4)))
        assert r.group(5) == ("-" if mode == "box" else "0")
    print(f"verbose {mode}: {len(its)} rows")


def test_verbose_log_fused_equals_unfused():
    """The fused loop (stop rule on device, decision applied by the next
    iteration's prologue) and the unfused host-stepped loop (k_mpc_control
    after every iteration) record the same rows: the same iteration count and
    the same per-iteration figures (their iterates agree bit for bit,
    test_fused_iteration_equals_unfused)."""
    from dilqr import _native as N
    from dilqr import ops
    T, B = 10, 128
    dx, x0, C, c = cartpole_case(B, T, seed=3)
    th = ops.theta_of(dx, x0)
    for eps, lim in ((5e-2, 5), (1e-6, 1)):
        kw = dict(lqr_iter=12, eps=eps, linesearch_decay=0.5, max_linesearch_iter=2, not_improved_lim=lim,
                  verbose=1)
        sv = ops.mpc_solve(N.MODEL_CARTPOLE, th, x0, C.contiguous(), c.contiguous(), T, **kw)[4]
        ws = ops.mpc_solve_unfused(N.MODEL_CARTPOLE, th, x0, C.contiguous(), c.contiguous(), T, **kw)
        a, b = sv.log, ws.log
        print(f"eps {eps} lim {lim}: fused {a['iterations']} rows, unfused {b['iterations']}")
        assert a["iterations"] == b["iterations"]
        k = a["iterations"]
        assert torch.allclose(a["stats"][:k], b["stats"][:k], rtol=1e-6, atol=0)
        assert float(a["initial_mean_cost"]) == pytest.approx(float(b["initial_mean_cost"]), rel=1e-6)


def test_classic_mpc_params_gradient_matches_autodiff():
    """Classic mpc.MPC, cartpole with params requiring grad: the fused
    (ANALYTIC) path's gradient into params equals the generic AUTO_DIFF path's
    (the reference's wiring, mpc.py:538-551) at the same solution.  Before
    round 5 the fused path left params.grad None."""
    from dilqr import mpc as cmpc
    from dilqr.env_dx.cartpole import CartpoleDx
    T, B = 10, 16
    _, x0, C, c = cartpole_case(B, T, seed=1)
    grads = {}
    sols = {}
    for gm in (cmpc.GradMethods.ANALYTIC, cmpc.GradMethods.AUTO_DIFF):
        params = torch.tensor((9.8, 1.0, 0.1, 0.5), device=DEV, requires_grad=True)
        dx = CartpoleDx(params)
        m = cmpc.MPC(5, 1, T, lqr_iter=20, eps=1e-5, grad_method=gm, exit_unconverged=False,
                     detach_unconverged=False, linesearch_decay=0.5, max_linesearch_iter=2, n_batch=B)
        x, u, _ = m(x0, cmpc.QuadCost(C, c), dx)
        w = torch.linspace(-1, 1, T * B, device=DEV).view(T, B, 1)
        (u * w).sum().backward()
        assert params.grad is not None, gm
        grads[gm] = params.grad.detach().cpu().numpy().astype(np.float64)
        sols[gm] = u.detach().cpu().numpy()
    a, b = grads[cmpc.GradMethods.ANALYTIC], grads[cmpc.GradMethods.AUTO_DIFF]
    du = np.max(np.abs(sols[cmpc.GradMethods.ANALYTIC] - sols[cmpc.GradMethods.AUTO_DIFF]))
    err = np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))
    print(f"classic params grad: fused {a}, generic {b}, rel err {err:.2e} (solutions differ by {du:.2e})")
    assert np.all(np.isfinite(a)) and np.any(a != 0)
    assert err < 1e-3


def test_classic_mpc_pendulum_complex_params_gradient_refused():
    """The 5-parameter pendulum through the classic MPC: the solve runs, a
    backward into params raises (no device derivative in theta) instead of
    leaving params.grad silently None."""
    from dilqr import mpc as cmpc
    from dilqr.env_dx.pendulum import PendulumDx
    from oracle import models as omodels
    dx = PendulumDx(torch.tensor(omodels.PendulumComplex.default_params), simple=False)
    dx.params = dx.params.clone().to(DEV).requires_grad_(True)
    T, B = 5, 4
    q, p = dx.get_true_obj()
    m = cmpc.MPC(3, 1, T, u_lower=-2.0, u_upper=2.0, lqr_iter=3, exit_unconverged=False, detach_unconverged=False)
    x0 = torch.tensor(np.tile([1.0, 0.0, 0.0], (B, 1)), dtype=torch.float32, device=DEV)
    x, u, _ = m(x0, cmpc.QuadCost(torch.diag(q).repeat(T, B, 1, 1).to(DEV), p.repeat(T, B, 1).to(DEV)), dx)
    with pytest.raises(NotImplementedError, match="5-parameter"):
        u.sum().backward()


@pytest.mark.parametrize("name,n,m", [("pendulum", 3, 1), ("cartpole", 5, 1), ("rocket", 13, 3)])
def test_qp_total_vs_golden_and_per_step_maxima(golden, name, n, m):
    """LQRStep's n_total_qp_iter (ops.lqr_backward qp_total: the per-step batch
    maximum of the pnqp iterations from the sweep's atomic max, plus 1 per step,
    lqr_step_explicit.py:137-150) on the reference's bounded Riccati case
    (riccati golden, box +-1): equal to the per-problem oracle's
    sum_t (1 + max_b it[t, b]) exactly, and to the reference's own batch-coupled
    count (its Armijo loop exits on the batch max, pnqp.py:75; parity of the
    count is then by this case: the golden's value).  rocket (m = 3) takes the
    16-lane group sweep, the others the one-lane sweep."""
    from dilqr import ops
    from oracle import lqr as olqr
    g = golden("riccati_f64")
    C, c, F, u = g[f"{name}_C"], g[f"{name}_c"], g[f"{name}_F"], g[f"{name}_u"]
    dev = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device=DEV)  # noqa: E731
    _, _, total = ops.lqr_backward(dev(C), dev(c), dev(F), n, m, u=dev(u), u_lower=-1.0, u_upper=1.0,
                                   qp_total=True)
    _, _, o_total = olqr.lqr_backward(C, c, F, n, m, u=u, u_lower=-1.0, u_upper=1.0, per_problem=True)
    ref = int(g[f"{name}_box_nqp"])
    print(f"{name}: qp_total {total}, per-problem oracle {o_total}, reference {ref}")
    assert total == o_total
    assert total == ref


@pytest.mark.parametrize("model,B,bounds,eps,lim", [
    ("cartpole", 32, (-100.0, 100.0), 1e-4, 5),       # the IL loop's settings (il_env.py:153-188), n_batch 32
    ("cartpole", 100, None, 5e-2, 5),                 # stops on max full_du_norm < eps
    ("cartpole", 256, (-10.0, 10.0), 1e-3, 1),        # one full workgroup; n_not_improved > 1 can stop it
    ("pendulum", 77, (-2.0, 2.0), 1e-3, 5),
    ("cartpole", 64, None, 0.0, 3),                   # eps 0: only the not-improved rule
])
def test_small_batch_solve_equals_per_iteration_launches(model, B, bounds, eps, lim):
    """dilqr_mpc_solve_small_f32 (the whole stop-rule loop in ONE workgroup,
    the rule applied in-kernel) leaves exactly the state of begin + the
    per-iteration launches (fused iteration + k_mpc_norm_rows + the next
    prologue's mpc_decide): best trajectories, costs, best_du, full_du_norm,
    step sizes, slots and the iteration the rule stopped at."""
    from dilqr import _native as N
    from dilqr import ops
    from dilqr.env_dx.cartpole import CartpoleDx
    from dilqr.env_dx.pendulum import PendulumDx
    T, iters = (35, 60) if model == "cartpole" else (20, 60)
    dx = CartpoleDx() if model == "cartpole" else PendulumDx()
    rng = np.random.RandomState(B)
    if model == "cartpole":
        th = rng.uniform(-np.pi, np.pi, B)
        x0 = np.stack([rng.uniform(-.5, .5, B), rng.uniform(-.5, .5, B), np.cos(th), np.sin(th),
                       rng.uniform(-1, 1, B)], 1)
        decay, mls = 0.5, 2
    else:
        th = rng.uniform(-np.pi / 2, np.pi / 2, B)
        x0 = np.stack([np.cos(th), np.sin(th), rng.uniform(-1, 1, B)], 1)
        decay, mls = 0.2, 5
    x0 = torch.tensor(x0, dtype=torch.float32, device=DEV)
    q, p = dx.get_true_obj()
    C = torch.diag(q).repeat(T, B, 1, 1).to(DEV).contiguous()
    c = p.repeat(T, B, 1).to(DEV).contiguous()
    th_ = ops.theta_of(dx, x0)
    n, m = dx.n_state, dx.n_ctrl
    nb, keep = N.make_bounds(*(bounds if bounds else (None, None)))
    a = ops.MPCSolve(T, B, n, m, DEV)
    a.solve_small(dx.model_id, th_, x0, C, c, nb, decay, mls, iters, 1e-4, eps, lim)
    b = ops.MPCSolve(T, B, n, m, DEV)
    b.begin(dx.model_id, th_, x0)
    for i in range(iters):
        b.iterate(dx.model_id, th_, x0, C, c, nb, decay, mls, i, 1e-4, eps, lim)
    print(f"{model} B={B}: small solve ran {a.iterations} (stopped {a.stopped}), per-iteration {b.iterations} "
          f"(stopped {b.stopped})")
    assert a.iterations == b.iterations and a.stopped == b.stopped
    assert b.stopped or b.iterations == iters
    # the control word itself (iter, stopped, n_not_improved, max) is the same,
    # stopped or not
    assert torch.equal(a._ctrl_now(), b._ctrl_now())
    xa, ua = a.gather_best()
    xb, ub = b.gather_best()
    assert torch.equal(xa, xb) and torch.equal(ua, ub)
    for f in ("best_cost", "best_du", "full_du_norm", "cost", "alpha", "slot", "improved"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    del keep


@pytest.mark.parametrize("mls,decay,bounds", [(1, 0.2, None), (2, 0.5, None), (3, 0.2, None), (4, 0.2, None),
                                              (6, 0.3, None), (9, 0.2, None), (6, 0.2, (-5.0, 5.0))])
def test_rocket_quad_search_any_max_ls_equals_unfused(golden, mls, decay, bounds):
    """The rocket MPC's quad-lane line search (k_mpc_search_quad: four passes per
    round, cost only, pass 0 written speculatively, the winner re-rolled) over
    max_ls from 1 (the only pass is the last: accepted unrolled-for-comparison)
    to 9 (three rounds, the last pass alone in round 2): iterates, costs and
    best iterates equal the unfused kernels' sequential search bit for bit."""
    import dilqr
    from dilqr import ops
    from dilqr.env_dx.rocket import RocketDx
    g = golden("mpc_f64")
    x0 = g["rocket_unc_x0"]
    T, it = 30, 8
    dx = RocketDx()
    B = x0.shape[0]
    q, p = dx.get_true_obj()
    C = torch.diag(q).repeat(T, B, 1, 1).to(DEV)
    c = p.repeat(T, B, 1).to(DEV)
    lo, hi = bounds if bounds else (None, None)
    xi = torch.tensor(x0, dtype=torch.float32, device=DEV)
    m = dilqr.MPC(13, 3, T, u_lower=lo, u_upper=hi, lqr_iter=it, eps=0.0, not_improved_lim=10 ** 9,
                  linesearch_decay=decay, max_linesearch_iter=mls, exit_unconverged=False, detach_unconverged=False)
    with torch.no_grad():
        xa, ua, ca = m(xi, dilqr.QuadCost(C, c), dx)
    ws = ops.mpc_solve_unfused(dx.model_id, ops.theta_of(dx, C), xi, C, c, T, u_lower=lo, u_upper=hi, lqr_iter=it,
                               eps=0.0, linesearch_decay=decay, max_linesearch_iter=mls, not_improved_lim=10 ** 9)
    alphas = m.last_solve.alpha.cpu().numpy()
    print(f"max_ls {mls} decay {decay}: final step sizes {np.unique(alphas)}")
    for a, b in ((xa, ws.best_x), (ua, ws.best_u), (ca, ws.best_cost)):
        assert torch.equal(a, b), float((a - b).abs().max())


@pytest.mark.parametrize("B,T,iters,mls", [(1, 1, 1, 1), (3, 2, 3, 1), (5, 7, 1, 2), (129, 4, 6, 2)])
def test_small_batch_solve_edges(B, T, iters, mls):
    """The one-workgroup solve at its edges — one problem, a one-step horizon,
    one iteration (the rule never applied), one line-search pass, a batch that
    is not a multiple of 64 — equals begin + the per-iteration launches."""
    from dilqr import _native as N
    from dilqr import ops
    from dilqr.env_dx.cartpole import CartpoleDx
    dx = CartpoleDx()
    rng = np.random.RandomState(T * 100 + B)
    th = rng.uniform(-np.pi, np.pi, B)
    x0 = torch.tensor(np.stack([rng.uniform(-.5, .5, B), rng.uniform(-.5, .5, B), np.cos(th), np.sin(th),
                                rng.uniform(-1, 1, B)], 1), dtype=torch.float32, device=DEV)
    q, p = dx.get_true_obj()
    C = torch.diag(q).repeat(T, B, 1, 1).to(DEV).contiguous()
    c = p.repeat(T, B, 1).to(DEV).contiguous()
    th_ = ops.theta_of(dx, x0)
    nb, keep = N.make_bounds(None, None)
    a = ops.MPCSolve(T, B, 5, 1, DEV)
    a.solve_small(dx.model_id, th_, x0, C, c, nb, 0.5, mls, iters, 1e-4, 1e-3, 2)
    b = ops.MPCSolve(T, B, 5, 1, DEV)
    b.begin(dx.model_id, th_, x0)
    for i in range(iters):
        b.iterate(dx.model_id, th_, x0, C, c, nb, 0.5, mls, i, 1e-4, 1e-3, 2)
    assert a.iterations == b.iterations and a.stopped == b.stopped
    assert b.stopped or b.iterations == iters
    assert torch.equal(a._ctrl_now(), b._ctrl_now())
    xa, ua = a.gather_best()
    xb, ub = b.gather_best()
    assert torch.equal(xa, xb) and torch.equal(ua, ub)
    for f in ("best_cost", "best_du", "full_du_norm", "cost", "alpha"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    del keep


@pytest.mark.parametrize("model,bounds,eps,lim,iters", [("pendulum", (-2.0, 2.0), 1e-3, 5, 60),
                                                      ("cartpole", None, 5e-2, 5, 60),
                                                      ("cartpole", (-10.0, 10.0), 1e-4, 5, 40),
                                                      ("cartpole", (-10.0, 10.0), 0.0, 2, 40)])
def test_pipelined_stop_polls_equal_blocking_polls(model, bounds, eps, lim, iters):
    """Above SMALL_BATCH_MAX the stop-rule loop runs per-iteration launches and
    polls the stop flag through pinned-memory copies behind events, waiting
    only POLL_AHEAD runs behind the device (round 6).  The result — best
    trajectories, costs, best_du, the iterations that ran, the stop flag — is
    the blocking poll's (POLL_AHEAD = 0) and the plain per-iteration loop's
    (iterations after a stop are device no-ops), stopped early or not."""
    from dilqr import _native as N
    from dilqr import ops
    from dilqr.env_dx.cartpole import CartpoleDx
    from dilqr.env_dx.pendulum import PendulumDx
    B = 512
    rng = np.random.RandomState(12)
    if model == "cartpole":
        T, dx, decay, mls = 25, CartpoleDx(), 0.5, 2
        th = rng.uniform(-np.pi, np.pi, B)
        x0 = np.stack([rng.uniform(-.5, .5, B), rng.uniform(-.5, .5, B), np.cos(th), np.sin(th),
                       rng.uniform(-1, 1, B)], 1)
    else:
        T, dx, decay, mls = 20, PendulumDx(), 0.2, 5
        th = rng.uniform(-np.pi / 2, np.pi / 2, B)
        x0 = np.stack([np.cos(th), np.sin(th), rng.uniform(-1, 1, B)], 1)
    x0 = torch.tensor(x0, dtype=torch.float32, device=DEV)
    n, m = dx.n_state, dx.n_ctrl
    lo, hi = bounds if bounds else (None, None)
    q, p = dx.get_true_obj()
    C = torch.diag(q).repeat(T, B, 1, 1).to(DEV).contiguous()
    c = p.repeat(T, B, 1).to(DEV).contiguous()
    th_ = ops.theta_of(dx, x0)
    assert B > ops.SMALL_BATCH_MAX
    out = {}
    keep = ops.POLL_AHEAD
    try:
        for pa in (2, 0):
            ops.POLL_AHEAD = pa
            x, u, cost, du, sv = ops.mpc_solve(dx.model_id, th_, x0, C, c, T, u_lower=lo, u_upper=hi,
                                               lqr_iter=iters, eps=eps, linesearch_decay=decay,
                                               max_linesearch_iter=mls, not_improved_lim=lim)
            out[pa] = (x, u, cost, du, sv.iterations, sv.stopped)
    finally:
        ops.POLL_AHEAD = keep
    nb, kb = N.make_bounds(lo, hi)
    ref = ops.MPCSolve(T, B, n, m, DEV)
    ref.begin(dx.model_id, th_, x0)
    for i in range(iters):
        ref.iterate(dx.model_id, th_, x0, C, c, nb, decay, mls, i, 1e-4, eps, lim)
    xr, ur = ref.gather_best()
    print(f"\n{model} {bounds} eps {eps} lim {lim}: ran {out[2][4]} of {iters} (stopped {out[2][5]}), "
          f"reference loop {ref.iterations}")
    if model == "pendulum":
        assert out[2][5], "this case is meant to stop early"
    for pa in (2, 0):
        x, u, cost, du, its, stopped = out[pa]
        assert torch.equal(x, xr) and torch.equal(u, ur), pa
        assert torch.equal(cost, ref.best_cost) and torch.equal(du, ref.best_du), pa
        assert its == ref.iterations and stopped == ref.stopped, (pa, its, ref.iterations)
    del kb
