"""Host-side pieces of the generic loop (dilqr.generic, dilqr.dynamics) on CPU:
the NNDynamics mirror's analytic grad_input against autograd, the batched
linearisations against each other, the autograd cost expansion of a quadratic
cost (exact), and the slew-rate augmentation's structure (mpc_explicit.py:383-466)."""
import types

import torch

from dilqr import generic
from dilqr.definitions import QuadCost
from dilqr.dynamics import CtrlPassthroughDynamics, NNDynamics
from dilqr.mpc_explicit import GradMethods


def jac_autograd(f, x, u):
    J = torch.autograd.functional.jacobian(lambda a, b: f(a, b).sum(0), (x, u))
    return J[0].permute(1, 0, 2), J[1].permute(1, 0, 2)


def test_nn_grad_input_matches_autograd():
    torch.manual_seed(0)
    for act in ("sigmoid", "relu"):
        nn_dx = NNDynamics(4, 2, hidden_sizes=[16, 8], activation=act).double()
        x, u = torch.randn(7, 4, dtype=torch.float64), torch.randn(7, 2, dtype=torch.float64)
        nn_dx(x, u)
        R, S = nn_dx.grad_input(x, u)
        Ra, Sa = jac_autograd(nn_dx, x, u)
        assert torch.allclose(R, Ra, atol=1e-12) and torch.allclose(S, Sa, atol=1e-12)


def test_linearisations_agree():
    torch.manual_seed(1)
    nn_dx = NNDynamics(3, 1, hidden_sizes=[12]).double()
    T, B = 5, 4
    x = torch.randn(T, B, 3, dtype=torch.float64)
    u = torch.randn(T, B, 1, dtype=torch.float64)
    out = {}
    for gm in (GradMethods.AUTO_DIFF, GradMethods.FINITE_DIFF, GradMethods.ANALYTIC):
        out[gm] = generic.linearize(types.SimpleNamespace(grad_method=gm), x, u, nn_dx, diff=False)
    Fa, fa = out[GradMethods.AUTO_DIFF]
    for gm in (GradMethods.FINITE_DIFF, GradMethods.ANALYTIC):
        F, f = out[gm]
        assert F.shape == (T - 1, B, 3, 4) and f.shape == (T - 1, B, 3)
        tol = 1e-7 if gm == GradMethods.FINITE_DIFF else 1e-12
        assert torch.allclose(F, Fa, atol=tol) and torch.allclose(f, fa, atol=tol)


def test_approximate_cost_of_a_quadratic_is_exact():
    torch.manual_seed(2)
    T, B, d = 4, 3, 5
    L = torch.randn(d, d, dtype=torch.float64)
    Q = L @ L.T
    p = torch.randn(d, dtype=torch.float64)
    x, u = torch.randn(T, B, 3, dtype=torch.float64), torch.randn(T, B, 2, dtype=torch.float64)
    H, c, val = generic.approximate_cost(x, u, lambda tau: 0.5 * generic.bquad(tau, Q) + tau @ p, diff=False)
    assert torch.allclose(H, Q.expand(T, B, d, d), atol=1e-12)
    assert torch.allclose(c, p.expand(T, B, d), atol=1e-12)


def test_slew_augmentation_structure():
    T, B, n, m = 4, 2, 3, 1
    mpc = types.SimpleNamespace(T=T, n_state=n, n_ctrl=m, slew_rate_penalty=0.5, prev_ctrl=None)
    C = torch.eye(n + m).expand(T, B, n + m, n + m).clone()
    c = torch.ones(T, B, n + m)
    F = torch.randn(T - 1, B, n, n + m)
    x, u = torch.randn(T, B, n), torch.randn(T, B, m)
    dyn = lambda xx, uu: xx + uu.sum(1, keepdim=True)
    x0 = torch.randn(B, n)
    _x0, _C, _c, _F, _f, _dyn, _cost, _x = generic.slew_augment(mpc, x0, C, c, F, None, QuadCost(C, c), dyn, x, u)
    assert _C.shape == (T, B, n + 2 * m, n + 2 * m) and _F.shape == (T - 1, B, n + m, n + 2 * m)
    # the slew block gamma/2 [[I, -I], [-I, I]] on (u_{t-1}, u_t) plus the original C
    assert torch.allclose(_C[0, 0, :m, :m], torch.tensor([[0.5]])) and torch.allclose(_C[0, 0, :m, -m:], torch.tensor([[-0.5]]))
    assert torch.allclose(_C[0, 0, -m:, -m:], torch.tensor([[1.5]]))
    # the passthrough row copies u_t into the new state's first block
    assert torch.allclose(_F[0, 0, :m, -m:], torch.eye(m)) and torch.allclose(_x[1:, :, :m], u[:-1])
    assert isinstance(_dyn, CtrlPassthroughDynamics)
    xt = torch.randn(B, n + m)
    assert torch.allclose(_dyn(xt, u[0])[:, :m], u[0])
