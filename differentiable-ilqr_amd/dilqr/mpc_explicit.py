"""MPC of DiLQR (mpc_explicit.py:57-627) on the HIP path.

Same constructor and `forward(x_init, QuadCost(C, c), dx) -> (x, u, costs)` as
the reference.  The whole iLQR loop — rollout, on-the-fly linearisation, Riccati
sweep (+pnqp), line search, best-iterate tracking and the stop rule — runs on
the GPU (ops.mpc_solve); the host only polls the stop flag every few
iterations.  Differentiation goes through LQRStep(no_op_forward=True) at the
best iterate, exactly as the reference wires it (mpc_explicit.py:302-325).
"""
import warnings
from enum import Enum

import torch
from torch.nn import Module

from . import _native as N
from . import ops
from .definitions import LinDx, QuadCost
from .lqr_step_explicit import LQRStep


class GradMethods(Enum):
    AUTO_DIFF = 1
    FINITE_DIFF = 2
    ANALYTIC = 3
    ANALYTIC_CHECK = 4


def expand_cost(C, c, T, n_batch, d):
    """mpc_explicit.py:203-224."""
    if C.ndimension() == 2:
        C = C.unsqueeze(0).unsqueeze(0).expand(T, n_batch, d, -1)
    elif C.ndimension() == 3:
        C = C.unsqueeze(1).expand(T, n_batch, d, -1)
    if c.ndimension() == 1:
        c = c.unsqueeze(0).unsqueeze(0).expand(T, n_batch, -1)
    elif c.ndimension() == 2:
        c = c.unsqueeze(1).expand(T, n_batch, -1)
    if C.ndimension() != 4 or c.ndimension() != 3:
        raise ValueError("MPC Error: Unexpected QuadCost shape.")
    return C, c


class MPC(Module):
    def __init__(self, n_state, n_ctrl, T, u_lower=None, u_upper=None, u_zero_I=None, u_init=None,
                 lqr_iter=10, grad_method=GradMethods.ANALYTIC, delta_u=None, verbose=0, eps=1e-7,
                 back_eps=1e-7, n_batch=None, linesearch_decay=0.2, max_linesearch_iter=10,
                 exit_unconverged=True, detach_unconverged=True, backprop=True, slew_rate_penalty=None,
                 prev_ctrl=None, not_improved_lim=5, best_cost_eps=1e-4):
        super().__init__()
        assert (u_lower is None) == (u_upper is None)
        assert max_linesearch_iter > 0
        self.n_state, self.n_ctrl, self.T = n_state, n_ctrl, T
        self.u_lower = u_lower if (u_lower is None or isinstance(u_lower, float)) else u_lower.detach()
        self.u_upper = u_upper if (u_upper is None or isinstance(u_upper, float)) else u_upper.detach()
        self.u_zero_I = None if u_zero_I is None else u_zero_I.detach()
        self.u_init = None if u_init is None else u_init.detach()
        self.lqr_iter = lqr_iter
        self.grad_method = grad_method
        self.delta_u = delta_u
        self.verbose = verbose
        self.eps = eps
        self.back_eps = back_eps
        self.n_batch = n_batch
        self.linesearch_decay = linesearch_decay
        self.max_linesearch_iter = max_linesearch_iter
        self.exit_unconverged = exit_unconverged
        self.detach_unconverged = detach_unconverged
        self.backprop = backprop
        self.not_improved_lim = not_improved_lim
        self.best_cost_eps = best_cost_eps
        self.slew_rate_penalty = slew_rate_penalty
        self.prev_ctrl = prev_ctrl
        if grad_method == GradMethods.ANALYTIC_CHECK:
            raise NotImplementedError("dilqr: ANALYTIC_CHECK is disabled in the reference too (mpc_explicit.py:578)")

    def fused(self, cost, dx):
        """The whole loop on device in HIP kernels: an env_dx model with its
        analytic Jacobian, a quadratic cost, no slew-rate penalty / delta_u
        (the fused iteration; with a u_zero_I mask the unfused kernels).
        AUTO_DIFF takes the same path for a model whose Jacobian is the autograd
        one (the 5-parameter pendulum).  Anything else runs the generic loop
        (dilqr.generic)."""
        jac_ok = self.grad_method == GradMethods.ANALYTIC or (
            self.grad_method == GradMethods.AUTO_DIFF and getattr(dx, "jacobian_is_autograd", False))
        return (isinstance(cost, QuadCost) and getattr(dx, "model_id", None) is not None and jac_ok
                and self.slew_rate_penalty is None and self.delta_u is None)

    def forward(self, x_init, cost, dx):
        if not x_init.is_cuda:
            raise RuntimeError("dilqr: x_init must be on the GPU (no CPU path)")
        if not self.fused(cost, dx):
            return self.forward_generic(x_init, cost, dx, classic=False)
        n_batch = self.n_batch if self.n_batch is not None else (
            cost.C.size(1) if cost.C.ndimension() == 4 else None)
        if n_batch is None:
            raise ValueError("MPC Error: Could not infer batch size, pass in as n_batch")
        T, n, m = self.T, self.n_state, self.n_ctrl
        C, c = expand_cost(cost.C, cost.c, T, n_batch, n + m)
        assert x_init.ndimension() == 2 and x_init.size(0) == n_batch
        model_id = ops.model_id_of(dx)
        theta = ops.theta_of(dx, x_init)
        Cd, cd = C.detach().contiguous(), c.detach().contiguous()
        with torch.no_grad():
            if self.u_zero_I is None:
                x, u, costs, full_du_norm, sv = ops.mpc_solve(
                    model_id, theta, x_init.detach(), Cd, cd, T, u_init=self.u_init, u_lower=self.u_lower,
                    u_upper=self.u_upper, lqr_iter=self.lqr_iter, eps=self.eps,
                    linesearch_decay=self.linesearch_decay, max_linesearch_iter=self.max_linesearch_iter,
                    not_improved_lim=self.not_improved_lim, best_cost_eps=self.best_cost_eps,
                    verbose=self.verbose)
            else:
                # controls held at zero (mpc_explicit.py:369, 452 -> LQRStep u_zero_I):
                # the unfused kernels take the mask (masked gain solve, zeroed rollout)
                sv = ops.mpc_solve_unfused(
                    model_id, theta, x_init.detach(), Cd, cd, T, u_init=self.u_init, u_lower=self.u_lower,
                    u_upper=self.u_upper, lqr_iter=self.lqr_iter, eps=self.eps,
                    linesearch_decay=self.linesearch_decay, max_linesearch_iter=self.max_linesearch_iter,
                    not_improved_lim=self.not_improved_lim, best_cost_eps=self.best_cost_eps, u_zero_I=self.u_zero_I,
                    verbose=self.verbose)
                x, u, costs, full_du_norm = sv.best_x, sv.best_u, sv.best_cost, sv.best_du
        self.last_solve = sv
        if self.verbose > 0:
            from .util import print_solve_log
            print_solve_log(sv.log)

        need_grad = torch.is_grad_enabled() and self.backprop and (
            C.requires_grad or c.requires_grad or
            (isinstance(getattr(dx, "params", None), torch.Tensor) and dx.params.requires_grad))
        if need_grad:
            # mpc_explicit.py:302-325: linearise at the best iterate and hand theta
            # to the implicit backward through a no-op LQR step.
            F, f = ops.linearize(model_id, theta, x, u)
            th = dx.params if isinstance(dx.params, torch.Tensor) else torch.tensor(dx.params)
            step = LQRStep(n, m, T, u_lower=self.u_lower, u_upper=self.u_upper, u_zero_I=self.u_zero_I,
                           true_cost=QuadCost(C, c), true_dynamics=dx, current_x=x, current_u=u,
                           back_eps=self.back_eps, no_op_forward=True)
            x, u = step(x_init, C, c, F, f, th)
        return self._detach_unconverged(x, u, costs, full_du_norm)

    def forward_generic(self, x_init, cost, dx, classic):
        """Generic dynamics / costs: dilqr.generic's loop,
        the HIP Riccati sweep inside, then the closing no-op LQR step."""
        from . import generic
        if self.n_batch is not None:
            n_batch = self.n_batch
        elif isinstance(cost, QuadCost) and cost.C.ndimension() == 4:
            n_batch = cost.C.size(1)
        else:
            raise ValueError("MPC Error: Could not infer batch size, pass in as n_batch")
        T, n, m = self.T, self.n_state, self.n_ctrl
        if isinstance(cost, QuadCost):
            C, c = expand_cost(cost.C, cost.c, T, n_batch, n + m)
            cost = QuadCost(C, c)
        assert x_init.ndimension() == 2 and x_init.size(0) == n_batch
        x, u, costs, full_du_norm = generic.solve(self, x_init, cost, dx, n_batch)
        need_grad = torch.is_grad_enabled() and self.backprop
        if need_grad:
            x, u = generic.final_step(self, x_init, cost, dx, x, u, classic)
        return self._detach_unconverged(x, u, costs, full_du_norm)

    def _detach_unconverged(self, x, u, costs, full_du_norm):
        if self.detach_unconverged:
            # mpc_explicit.py:343-356
            if float(full_du_norm.max()) > self.eps:
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
