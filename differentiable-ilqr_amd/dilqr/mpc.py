"""Classic mpc.pytorch MPC (mpc.py:57-601) on the HIP path.

Takes model dynamics or a LinDx (and, through dilqr.generic, any dynamics
Module, AUTO_DIFF / FINITE_DIFF linearisation, non-quadratic costs and the
slew-rate penalty).  The forward loop runs on device; gradients
flow through a no-op classic LQR step (lqr_step.py:277-282) whose backward is
the classic adjoint kernel, exactly like mpc.py:302-335.  With model dynamics
the reference differentiates the autograd linearisation (mpc.py:538-551): F is
data, f = dynamics(x, u) - F tau keeps the graph to the model's parameters; here
F comes from the kernel and, when dx.params requires grad, f is formed the same
way through the model's device vjp, so gradients reach (x_init, C, c), the
parameters and, for LinDx, (F, f).
"""
import warnings

import torch
from torch.nn import Module

from . import _native as N
from . import ops
from .definitions import LinDx, QuadCost
from .lqr_step import LQRStep
from .mpc_explicit import MPC as ExplicitMPC
from .mpc_explicit import GradMethods, expand_cost


class _RefuseThetaGrad(torch.autograd.Function):
    """f with a graph to the 5-parameter pendulum's params whose backward
    raises: the solve runs, a gradient into params is refused rather than
    silently dropped (the explicit MPC refuses it in its implicit backward)."""

    @staticmethod
    def forward(ctx, f, params):
        return f.clone()

    @staticmethod
    def backward(ctx, gf):
        raise NotImplementedError("dilqr: gradients into the 5-parameter pendulum's params are not implemented "
                                  "(no device derivative in theta; the reference's grad_input has no 5-parameter "
                                  "form either, pendulum.py:157)")


class MPC(Module):
    def __init__(self, n_state, n_ctrl, T, u_lower=None, u_upper=None, u_zero_I=None, u_init=None,
                 lqr_iter=10, grad_method=GradMethods.ANALYTIC, delta_u=None, verbose=0, eps=1e-7,
                 back_eps=1e-7, n_batch=None, linesearch_decay=0.2, max_linesearch_iter=10,
                 exit_unconverged=True, detach_unconverged=True, backprop=True, slew_rate_penalty=None,
                 prev_ctrl=None, not_improved_lim=5, best_cost_eps=1e-4):
        super().__init__()
        assert (u_lower is None) == (u_upper is None)
        assert max_linesearch_iter > 0
        self.u_zero_I = None if u_zero_I is None else u_zero_I.detach()
        self.delta_u, self.slew_rate_penalty, self.prev_ctrl = delta_u, slew_rate_penalty, prev_ctrl
        self.n_state, self.n_ctrl, self.T = n_state, n_ctrl, T
        self.u_lower = u_lower if (u_lower is None or isinstance(u_lower, float)) else u_lower.detach()
        self.u_upper = u_upper if (u_upper is None or isinstance(u_upper, float)) else u_upper.detach()
        self.u_init = None if u_init is None else u_init.detach()
        self.lqr_iter, self.grad_method, self.verbose = lqr_iter, grad_method, verbose
        self.eps, self.back_eps, self.n_batch = eps, back_eps, n_batch
        self.linesearch_decay, self.max_linesearch_iter = linesearch_decay, max_linesearch_iter
        self.exit_unconverged, self.detach_unconverged, self.backprop = exit_unconverged, detach_unconverged, backprop
        self.not_improved_lim, self.best_cost_eps = not_improved_lim, best_cost_eps

    # generic dynamics / costs share the explicit MPC's driver
    forward_generic = ExplicitMPC.forward_generic
    _detach_unconverged = ExplicitMPC._detach_unconverged

    def fused(self, cost, dx):
        """The device-resident loop: env_dx model (ANALYTIC) or LinDx, quadratic
        cost, no slew-rate penalty / delta_u; anything else -> dilqr.generic."""
        model_ok = isinstance(dx, LinDx) or (getattr(dx, "model_id", None) is not None and (
            self.grad_method == GradMethods.ANALYTIC
            or (self.grad_method == GradMethods.AUTO_DIFF and getattr(dx, "jacobian_is_autograd", False))))
        return isinstance(cost, QuadCost) and model_ok and self.slew_rate_penalty is None and self.delta_u is None

    def _f_with_params_graph(self, dx, model_id, F, x, u):
        """f = dynamics(x_t, u_t) - F_t tau_t with the dynamics' graph to its
        parameters, F a constant — what the reference's AUTO_DIFF linearisation
        hands the LQR step (mpc.py:538-551: torch.autograd.grad without
        create_graph gives F as data, new_x keeps the params graph), so a
        gradient reaches dx.params through f.  The 5-parameter pendulum has no
        device derivative in theta (its dynamics_vjp is refused), so a
        gradient there raises instead of being silently dropped."""
        if model_id == N.MODEL_PENDULUM_COMPLEX:
            return _RefuseThetaGrad.apply(ops.linearize(model_id, ops.theta_of(dx, x), x, u)[1], dx.params)
        T, B, n = x.shape
        m = u.shape[2]
        xs, us = x[:-1].reshape(-1, n).detach(), u[:-1].reshape(-1, m).detach()
        new_x = dx(xs, us).view(T - 1, B, n)
        tau = torch.cat((x[:-1], u[:-1]), 2).detach()
        return new_x - (F @ tau.unsqueeze(-1)).squeeze(-1)

    def forward(self, x_init, cost, dx):
        if not x_init.is_cuda:
            raise RuntimeError("dilqr: x_init must be on the GPU (no CPU path)")
        if not self.fused(cost, dx):
            return self.forward_generic(x_init, cost, dx, classic=True)
        n_batch = self.n_batch if self.n_batch is not None else (
            cost.C.size(1) if cost.C.ndimension() == 4 else None)
        if n_batch is None:
            raise ValueError("MPC Error: Could not infer batch size, pass in as n_batch")
        T, n, m = self.T, self.n_state, self.n_ctrl
        C, c = expand_cost(cost.C, cost.c, T, n_batch, n + m)
        model_id = ops.model_id_of(dx)
        lin = model_id == N.MODEL_LINDX
        theta = None if lin else ops.theta_of(dx, x_init)
        Fd = fd = None
        if lin:
            Fd = dx.F.detach().contiguous()
            fd = None if (dx.f is None or dx.f.nelement() == 0) else dx.f.detach().contiguous()
        with torch.no_grad():
            if not lin and self.u_zero_I is None:
                # an env_dx model: the device-resident fused loop (its iterates equal
                # the unfused pipeline's bit for bit, test_fused_iteration_equals_unfused)
                x, u, costs, full_du_norm, _sv = ops.mpc_solve(
                    model_id, theta, x_init.detach(), C.detach().contiguous(), c.detach().contiguous(), T,
                    u_init=self.u_init, u_lower=self.u_lower, u_upper=self.u_upper, lqr_iter=self.lqr_iter,
                    eps=self.eps, linesearch_decay=self.linesearch_decay,
                    max_linesearch_iter=self.max_linesearch_iter, not_improved_lim=self.not_improved_lim,
                    best_cost_eps=self.best_cost_eps, verbose=self.verbose)
            else:
                ws = ops.mpc_solve_unfused(model_id, theta, x_init.detach(), C.detach().contiguous(),
                                           c.detach().contiguous(), T, F=Fd, f=fd, u_init=self.u_init,
                                           u_lower=self.u_lower, u_upper=self.u_upper, lqr_iter=self.lqr_iter,
                                           eps=self.eps, linesearch_decay=self.linesearch_decay,
                                           max_linesearch_iter=self.max_linesearch_iter,
                                           not_improved_lim=self.not_improved_lim,
                                           best_cost_eps=self.best_cost_eps, u_zero_I=self.u_zero_I,
                    verbose=self.verbose)
                x, u, costs, full_du_norm, _sv = ws.best_x, ws.best_u, ws.best_cost, ws.best_du, ws
        if self.verbose > 0:                                    # mpc.py:270-275, 368-379
            from .util import print_solve_log
            print_solve_log(_sv.log)
        if torch.is_grad_enabled() and self.backprop:
            if lin:
                F, f = dx.F, (dx.f if dx.f is not None else torch.empty(0, device=x.device))
            else:
                F, f = ops.linearize(model_id, theta, x, u)
                params = getattr(dx, "params", None)
                if isinstance(params, torch.Tensor) and params.requires_grad:
                    f = self._f_with_params_graph(dx, model_id, F, x, u)
            step = LQRStep(n, m, T, u_lower=self.u_lower, u_upper=self.u_upper, u_zero_I=self.u_zero_I,
                           true_cost=QuadCost(C, c), true_dynamics=dx, current_x=x, current_u=u,
                           back_eps=self.back_eps, no_op_forward=True)
            x, u = step(x_init, C, c, F, f)
        if self.detach_unconverged and float(full_du_norm.max()) > self.eps:    # mpc.py:321-334
            if self.exit_unconverged:
                raise AssertionError("LQR did not converge (exit_unconverged=True)")
            if self.verbose >= 0:
                warnings.warn("LQR Warning: All examples did not converge to a fixed point. "
                              "Detaching and *not* backpropping through the bad examples.")
            I = (full_du_norm < self.eps)
            Ix = I.view(1, -1, 1).expand_as(x).to(x.dtype)
            Iu = I.view(1, -1, 1).expand_as(u).to(u.dtype)
            x = x * Ix + x.clone().detach() * (1. - Ix)
            u = u * Iu + u.clone().detach() * (1. - Iu)
        return x, u, costs
