"""LQRStep of DiLQR (lqr_step_explicit.py:24-718) on the HIP path.

`LQRStep(...)` returns a callable with the reference's signature
`apply(x_init, C, c, F, f=None, theta=None)`:

  * regular forward  -> (new_x, new_u, Tensor([n_total_qp_iter]), costs,
                         full_du_norm, mean_alphas)      (lqr_step_explicit.py:625-650)
  * no_op_forward    -> (current_x, current_u) with the Riccati gains of the
                         current trajectory saved for the implicit backward
                         (lqr_step_explicit.py:604-623)

The backward of the no-op step is the DiLQR implicit differentiation
(lqr_step_explicit.py:653-712) and returns (None, dC, dc, None, None,
dtheta [B,p], None); autograd sums dtheta over the batch like the reference.
"""
import torch
from torch.autograd import Function

from . import _native as N
from . import generic, ops
from .definitions import LinDx, QuadCost


def _bounds_arg(v):
    if v is None or isinstance(v, (int, float)):
        return v
    return v.detach()


def LQRStep(n_state, n_ctrl, T, u_lower=None, u_upper=None, u_zero_I=None, delta_u=None,
            linesearch_decay=0.2, max_linesearch_iter=10, true_cost=None, true_dynamics=None,
            delta_space=True, current_x=None, current_u=None, verbose=0, back_eps=1e-3,
            no_op_forward=False, theta=None):
    if not delta_space:
        raise NotImplementedError("dilqr: delta_space=False is unimplemented in the reference too (639)")
    if delta_u is not None and u_lower is None:
        raise NotImplementedError("dilqr: delta_u without u_lower is unimplemented in the reference too (197)")
    lo, hi = _bounds_arg(u_lower), _bounds_arg(u_upper)
    zI = None if u_zero_I is None else u_zero_I.detach()

    def sweep(C, c, F, x, u, qp_total=False):
        """lqr_backward (54-162): c_back fused into the kernel; with delta_u the
        box is relative and clipped to +-delta_u (132-135), c_back formed here;
        the u_zero_I mask applies only without bounds (the pnqp branch ignores it)."""
        if delta_u is not None:
            rlo, rhi = ops.delta_u_sweep_bounds(lo, hi, u, delta_u)
            return ops.lqr_backward(C, ops.c_back(C.detach(), c.detach(), x, u), F, n_state, n_ctrl,
                                    u_lower=rlo, u_upper=rhi, qp_total=qp_total)
        return ops.lqr_backward(C, c, F, n_state, n_ctrl, x=x, u=u, u_lower=lo, u_upper=hi,
                                u_zero_I=zI if lo is None else None, qp_total=qp_total)

    class LQRStepFn(Function):
        @staticmethod
        def forward(ctx, x_init, C, c, F, f=None, theta=None, if_converge=False):
            assert current_x is not None and current_u is not None
            x, u = current_x.detach(), current_u.detach()
            m_id = ops.generic_model_id(true_dynamics)
            if no_op_forward:
                K, _, _ = sweep(C, c, F, x, u)
                ctx.save_for_backward(x_init, C, c, F, f, x, u, theta, K)
                ctx.model = true_dynamics
                return x.clone(), u.clone()
            if not isinstance(true_cost, QuadCost) or m_id is None:
                # a generic true_cost / true_dynamics (lqr_step_explicit.py:226-236):
                # the HIP sweep, the rollout with the user's Modules in torch
                nx, nu, costs, full_du_norm, alphas, n_qp = generic.lqr_step_forward(
                    T, n_state, n_ctrl, x_init, C, c, F, x, u, true_cost, true_dynamics, lo, hi, delta_u,
                    linesearch_decay, max_linesearch_iter, u_zero_I=zI, extras=True)
                ctx.save_for_backward(x_init, C, c, F, f, nx, nu)
                return nx, nu, torch.tensor([float(n_qp)]), costs, full_du_norm, alphas.mean()
            K, k, nqp = sweep(C, c, F, x, u, qp_total=lo is not None)
            if m_id == N.MODEL_LINDX:
                th, Fd, fd = None, true_dynamics.F, true_dynamics.f
                if fd is not None and fd.nelement() == 0:
                    fd = None
            else:
                th, Fd, fd = ops.theta_of(true_dynamics, x_init), None, None
            Ct, ct = true_cost
            flo, fhi = (lo, hi) if delta_u is None else ops.delta_u_rollout_bounds(lo, hi, u, delta_u)
            nx, nu, costs, du_sq, alphas = ops.lqr_forward(
                m_id, th, x_init, Ct, ct, x, u, K, k, F=Fd, f=fd, u_lower=flo, u_upper=fhi, u_zero_I=zI,
                linesearch_decay=linesearch_decay, max_linesearch_iter=max_linesearch_iter)
            full_du_norm = ops.quirk_norm(du_sq)
            n_qp = nqp if isinstance(nqp, int) else 0
            ctx.save_for_backward(x_init, C, c, F, f, nx, nu)
            return nx, nu, torch.tensor([float(n_qp)]), costs, full_du_norm, alphas.mean()

        @staticmethod
        def backward(ctx, dl_dx, dl_du, *unused):
            if len(ctx.saved_tensors) != 9:
                # the reference's backward unpacks 9 saved tensors and fails the
                # same way after a regular (non no-op) forward (656)
                raise RuntimeError("LQRStep backward needs a no_op_forward step (lqr_step_explicit.py:656)")
            from .implicit import implicit_backward
            x_init, C, c, F, f, x, u, th, K = ctx.saved_tensors
            dC, dc, dtheta = implicit_backward(ctx.model, dl_dx, dl_du, C, c, F, f, x, u, K, lo, hi, th)
            return None, dC, dc, None, None, dtheta, None

    return LQRStepFn.apply
