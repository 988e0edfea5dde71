"""Classic differentiable LQR step of mpc.pytorch (lqr_step.py:23-409) on the HIP path.

`LQRStep(...)` returns `apply(x_init, C, c, F, f=None)`; forward is the same
Riccati sweep + line-search rollout as the DiLQR step, backward is the classic
adjoint (lqr_step.py:312-407) returning (dx_init, dC, dc, dF, df), computed by
one fused kernel (dilqr_lqr_adjoint_f32).
"""
import torch
from torch.autograd import Function

from . import _native as N
from . import generic, ops
from .definitions import QuadCost


def LQRStep(n_state, n_ctrl, T, u_lower=None, u_upper=None, u_zero_I=None, delta_u=None,
            linesearch_decay=0.2, max_linesearch_iter=10, true_cost=None, true_dynamics=None,
            delta_space=True, current_x=None, current_u=None, verbose=0, back_eps=1e-3,
            no_op_forward=False):
    if not delta_space:
        raise NotImplementedError("dilqr: delta_space=False is unimplemented in the reference too")
    if delta_u is not None and u_lower is None:
        raise NotImplementedError("dilqr: delta_u without u_lower is unimplemented in the reference too (195)")
    lo = u_lower if (u_lower is None or isinstance(u_lower, (int, float))) else u_lower.detach()
    hi = u_upper if (u_upper is None or isinstance(u_upper, (int, float))) else u_upper.detach()
    zI = None if u_zero_I is None else u_zero_I.detach()

    class LQRStepFn(Function):
        @staticmethod
        def forward(ctx, x_init, C, c, F, f=None):
            x, u = current_x.detach(), current_u.detach()
            if no_op_forward:                                   # lqr_step.py:277-282
                ctx.save_for_backward(x_init, C, c, F, f, x, u)
                return x.clone(), u.clone()
            m_id = ops.generic_model_id(true_dynamics)
            if not isinstance(true_cost, QuadCost) or m_id is None:
                # a generic true_cost / true_dynamics (lqr_step.py:224-234): the HIP
                # sweep, the rollout with the user's Modules in torch
                nx, nu, costs, full_du_norm, alphas, n_qp = generic.lqr_step_forward(
                    T, n_state, n_ctrl, x_init, C, c, F, x, u, true_cost, true_dynamics, lo, hi, delta_u,
                    linesearch_decay, max_linesearch_iter, u_zero_I=zI, extras=True)
                ctx.save_for_backward(x_init, C, c, F, f, nx, nu)
                return nx, nu, torch.tensor([float(n_qp)]), costs, full_du_norm, alphas.mean()
            if delta_u is not None:                             # lqr_step.py:130-135
                rlo, rhi = ops.delta_u_sweep_bounds(lo, hi, u, delta_u)
                K, k, nqp = ops.lqr_backward(C, ops.c_back(C.detach(), c.detach(), x, u), F, n_state, n_ctrl,
                                             u_lower=rlo, u_upper=rhi, qp_total=True)
            else:
                K, k, nqp = ops.lqr_backward(C, c, F, n_state, n_ctrl, x=x, u=u, u_lower=lo, u_upper=hi,
                                             u_zero_I=zI if lo is None else None, qp_total=lo is not None)
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
            x_init, C, c, F, f, nx, nu = ctx.saved_tensors
            has_f = f is not None and f.nelement() > 0
            dx0, dC, dc, dF, df = ops.lqr_adjoint(C, c, F, nx, nu, dl_dx.contiguous(), dl_du.contiguous(),
                                                  u_lower=lo, u_upper=hi, m_solver=N.SOLVE_INV, want_df=has_f)
            return dx0, dC, dc, dF, (df if has_f else None)

    return LQRStepFn.apply
