"""GPU parity of the generic-dynamics / generic-cost MPC loop (dilqr.generic,
SURVEY.md §8(f) #4) against the reference run in fp32 (tests/golden/gen_golden.py
case J):
  * NNDynamics with AUTO_DIFF, FINITE_DIFF and ANALYTIC (grad_input)
    linearisation through the classic mpc.MPC, plus its backward (classic adjoint
    kernel -> autograd through the linearisation into the network, C, c, x_init);
  * an env_dx model (cartpole) with AUTO_DIFF through mpc_explicit.MPC;
  * the slew-rate penalty (CtrlPassthroughDynamics augmentation) through both MPCs;
  * a non-quadratic cost (autograd Hessian expansion, approximate_cost).
Tolerances (fp32 solver vs the fp32 reference): 1e-3 relative on trajectories and
costs for the model cases.  The NNDynamics problem has flat cost directions:
the reference itself, run in fp64 instead of fp32 on the same weights, moves u
by 2.0e-3 (AUTO_DIFF) / 2.3e-2 (FINITE_DIFF, central differences at eps = 1e-4)
while its costs agree to 2e-7 / 3e-6 — so there the costs are held to 1e-4 /
1e-3 and the trajectories and gradients to that measured spread (5e-3 / 5e-2).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b))))


def gpu(a, grad=False):
    return torch.tensor(np.asarray(a), dtype=torch.float32, device=DEV, requires_grad=grad)


def cpu(t):
    return t.detach().cpu().numpy().astype(np.float64)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def nn_model(g):
    from dilqr.dynamics import NNDynamics
    nn_dx = NNDynamics(5, 1, hidden_sizes=[32], activation="sigmoid").to(DEV)
    with torch.no_grad():
        for i, fc in enumerate(nn_dx.fcs):
            fc.weight.copy_(gpu(g[f"nn_W{i}"]))
            fc.bias.copy_(gpu(g[f"nn_b{i}"]))
    return nn_dx


@pytest.mark.parametrize("tag", ["auto", "fd", "analytic"])
def test_nn_dynamics_classic_mpc(golden, tag):
    import dilqr.mpc as cmpc
    from dilqr import QuadCost
    g = golden("generic_f32")
    nn_dx = nn_model(g)
    T, B = g["nn_C"].shape[:2]
    gm = {"auto": cmpc.GradMethods.AUTO_DIFF, "fd": cmpc.GradMethods.FINITE_DIFF,
          "analytic": cmpc.GradMethods.ANALYTIC}[tag]
    X0, C, c = gpu(g["nn_x0"], True), gpu(g["nn_C"], True), gpu(g["nn_c"], True)
    m = cmpc.MPC(5, 1, T, lqr_iter=4, grad_method=gm, u_lower=-1.0, u_upper=1.0, n_batch=B,
                 exit_unconverged=False, detach_unconverged=False, linesearch_decay=0.2, max_linesearch_iter=10)
    x, u, costs = m(X0, QuadCost(C, c), nn_dx)
    tol, ctol = (5e-2, 1e-3) if tag == "fd" else (5e-3, 1e-4)
    assert relerr(cpu(costs), g[f"nn_{tag}_costs"]) < ctol
    assert relerr(cpu(u), g[f"nn_{tag}_u"]) < tol
    assert relerr(cpu(x), g[f"nn_{tag}_x"]) < tol
    ((x * gpu(g["nn_wx"])).sum() + (u * gpu(g["nn_wu"])).sum()).backward()
    gtol = tol
    assert relerr(cpu(X0.grad), g[f"nn_{tag}_dx0"]) < gtol
    assert relerr(cpu(C.grad), g[f"nn_{tag}_dC"]) < gtol
    assert relerr(cpu(c.grad), g[f"nn_{tag}_dc"]) < gtol
    for i, fc in enumerate(nn_dx.fcs):
        assert relerr(cpu(fc.weight.grad), g[f"nn_{tag}_dW{i}"]) < gtol
        assert relerr(cpu(fc.bias.grad), g[f"nn_{tag}_db{i}"]) < gtol


def cart_cost(T, B):
    from dilqr.env_dx.cartpole import CartpoleDx
    dx = CartpoleDx()
    q, p = dx.get_true_obj()
    return dx, torch.diag(q).repeat(T, B, 1, 1).to(DEV), p.repeat(T, B, 1).to(DEV)


def test_cartpole_autodiff_explicit(golden):
    import dilqr
    g = golden("generic_f32")
    T, B = g["cart_auto_x"].shape[:2]
    dx, C, c = cart_cost(T, B)
    m = dilqr.MPC(5, 1, T, lqr_iter=5, grad_method=dilqr.GradMethods.AUTO_DIFF, exit_unconverged=False,
                  detach_unconverged=False, linesearch_decay=0.5, max_linesearch_iter=2, eps=0.0,
                  not_improved_lim=10 ** 9)
    with torch.no_grad():
        x, u, costs = m(gpu(g["cart_auto_x0"]), dilqr.QuadCost(C, c), dx)
    assert relerr(cpu(costs), g["cart_auto_costs"]) < 1e-3
    assert relerr(cpu(u), g["cart_auto_u"]) < 1e-3


@pytest.mark.parametrize("tag", ["slew_explicit", "slew_classic"])
def test_slew_rate_penalty(golden, tag):
    import dilqr
    import dilqr.mpc as cmpc
    g = golden("generic_f32")
    T, B = g[f"{tag}_x"].shape[:2]
    dx, C, c = cart_cost(T, B)
    mod, gm = (dilqr, dilqr.GradMethods.ANALYTIC) if tag == "slew_explicit" else (cmpc, cmpc.GradMethods.AUTO_DIFF)
    m = mod.MPC(5, 1, T, lqr_iter=5, grad_method=gm, slew_rate_penalty=0.1, exit_unconverged=False,
                detach_unconverged=False, linesearch_decay=0.5, max_linesearch_iter=2, eps=0.0,
                not_improved_lim=10 ** 9)
    with torch.no_grad():
        x, u, costs = m(gpu(g["cart_auto_x0"]), dilqr.QuadCost(C, c), dx)
    assert relerr(cpu(costs), g[f"{tag}_costs"]) < 1e-3
    assert relerr(cpu(u), g[f"{tag}_u"]) < 1e-3
    assert relerr(cpu(x), g[f"{tag}_x"]) < 1e-3


class NQCost(torch.nn.Module):
    """The fixture's non-quadratic stage cost: 1/2|tau|^2 + 0.1 sum tau^4 + w . tau."""

    def __init__(self, w):
        super().__init__()
        self.w = w

    def forward(self, tau):
        return 0.5 * (tau ** 2).sum(-1) + 0.1 * (tau ** 4).sum(-1) + (tau * self.w).sum(-1)


@pytest.mark.parametrize("tag", ["nq_classic", "nq_explicit"])
def test_non_quadratic_cost(golden, tag):
    import dilqr
    import dilqr.mpc as cmpc
    from dilqr.env_dx.pendulum import PendulumDx
    g = golden("generic_f32")
    T, B = g[f"{tag}_x"].shape[:2]
    mod, gm = (cmpc, cmpc.GradMethods.AUTO_DIFF) if tag == "nq_classic" else (dilqr, dilqr.GradMethods.ANALYTIC)
    m = mod.MPC(3, 1, T, lqr_iter=5, grad_method=gm, n_batch=B, exit_unconverged=False, detach_unconverged=False,
                linesearch_decay=0.2, max_linesearch_iter=5, eps=0.0, not_improved_lim=10 ** 9, u_lower=-2.0,
                u_upper=2.0)
    with torch.no_grad():
        x, u, costs = m(gpu(g["nq_x0"]), NQCost(gpu(g["nq_w"])), PendulumDx())
    assert relerr(cpu(costs), g[f"{tag}_costs"]) < 1e-3
    assert relerr(cpu(u), g[f"{tag}_u"]) < 1e-3


def test_delta_u_trust_region(golden):
    """delta_u: each step's control stays within +-delta_u of the current one,
    inside the box (lqr_step_explicit.py:205-213)."""
    import dilqr
    g = golden("generic_f32")
    T, B = g["delta_u_x"].shape[:2]
    dx, C, c = cart_cost(T, B)
    m = dilqr.MPC(5, 1, T, lqr_iter=5, u_lower=-10.0, u_upper=10.0, delta_u=1.0, exit_unconverged=False,
                  detach_unconverged=False, linesearch_decay=0.5, max_linesearch_iter=2, eps=0.0,
                  not_improved_lim=10 ** 9)
    with torch.no_grad():
        x, u, costs = m(gpu(g["cart_auto_x0"]), dilqr.QuadCost(C, c), dx)
    assert relerr(cpu(costs), g["delta_u_costs"]) < 1e-3
    assert relerr(cpu(u), g["delta_u_u"]) < 1e-3


@pytest.mark.parametrize("variant", ["explicit", "classic"])
@pytest.mark.parametrize("case", ["nq", "nn"])
def test_lqrstep_generic_true_cost_and_dynamics(golden, variant, case):
    """One LQRStep forward (both variants) whose line search evaluates a
    non-quadratic true_cost (pendulum, "nq") or a Module true_dynamics
    (NNDynamics, "nn"), lqr_step_explicit.py:226-236 / lqr_step.py:224-234:
    the HIP Riccati sweep, the rollout in torch.  Against the reference's fp64
    step on the same inputs (case M of gen_golden.py): new x, u, costs,
    full_du_norm, mean step size and the pnqp iteration count."""
    import dilqr
    import dilqr.lqr_step as classic
    g = golden("stepgen_f64")
    mod = dilqr if variant == "explicit" else classic
    if case == "nq":
        from dilqr.env_dx.pendulum import PendulumDx
        T, B = g["nq_u"].shape[:2]
        dx = PendulumDx()
        q, p = dx.get_true_obj()
        C, c = torch.diag(q).repeat(T, B, 1, 1).to(DEV), p.repeat(T, B, 1).to(DEV)
        cost, lo, hi, mls = NQCost(gpu(g["nq_w"])), -2.0, 2.0, 5
    else:
        from dilqr.dynamics import NNDynamics
        T, B = g["nn_u"].shape[:2]
        dx = NNDynamics(5, 1, hidden_sizes=[32], activation="sigmoid").to(DEV)
        with torch.no_grad():
            for i, fc in enumerate(dx.fcs):
                fc.weight.copy_(gpu(g[f"nn_W{i}"]))
                fc.bias.copy_(gpu(g[f"nn_b{i}"]))
        C, c = gpu(g["nn_C"]), gpu(g["nn_c"])
        cost, lo, hi, mls = dilqr.QuadCost(C, c), -1.0, 1.0, 10
    X, U = gpu(g[f"{case}_X"]), gpu(g[f"{case}_u"])
    step = mod.LQRStep(X.shape[2], 1, T, u_lower=lo, u_upper=hi, true_cost=cost, true_dynamics=dx, current_x=X,
                       current_u=U, linesearch_decay=0.2, max_linesearch_iter=mls)
    args = (gpu(g[f"{case}_x0"]), C, c, gpu(g[f"{case}_F"]), gpu(g[f"{case}_f"]))
    with torch.no_grad():
        nx, nu, nqp, costs, du, malpha = step(*args, None) if variant == "explicit" else step(*args)
    k = f"{case}_{variant}"
    errs = {name: relerr(cpu(a), g[f"{k}_{name}"]) for name, a in
            (("nx", nx), ("nu", nu), ("costs", costs), ("du", du), ("malpha", malpha))}
    print(f"\n[LQRStep {variant} {case}] " + ", ".join(f"{a} {b:.2e}" for a, b in errs.items()))
    assert max(errs.values()) < 1e-4, errs
    assert float(nqp[0]) == float(g[f"{k}_nqp"][0])
