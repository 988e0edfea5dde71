"""Shared model plumbing: every model's forward / get_linear_dyn runs on the GPU
through libdilqr.so; the module holds the reference's constants."""
import torch
from torch import nn

from .. import _native as N


class _DynamicsFn(torch.autograd.Function):
    """forward() with the gradient autograd gives the reference (its forward is
    eager torch): dilqr_dynamics_f32 forward, dilqr_dynamics_vjp_f32 backward."""

    @staticmethod
    def forward(ctx, x, u, theta, model_id):
        x, u, th = x.detach().contiguous(), u.detach().contiguous(), theta.detach().contiguous()
        out = torch.empty_like(x)
        N.call("dilqr_dynamics_f32", model_id, x.shape[0], N.ptr(th), N.ptr(x), N.ptr(u), N.ptr(out),
               N.stream(x.device))
        ctx.save_for_backward(x, u, th)
        ctx.model_id = model_id
        return out

    @staticmethod
    def backward(ctx, gout):
        x, u, th = ctx.saved_tensors
        gout = gout.detach().float().contiguous()
        gth = torch.empty(x.shape[0], th.shape[0], device=x.device)
        gx, gu = torch.empty_like(x), torch.empty_like(u)
        N.call("dilqr_dynamics_vjp_f32", ctx.model_id, x.shape[0], N.ptr(th), N.ptr(x), N.ptr(u), N.ptr(gout),
               N.ptr(gth), N.ptr(gx), N.ptr(gu), N.stream(x.device))
        return gx, gu, gth.sum(0), None


class HipDynamics(nn.Module):
    model_id = None
    n_state = n_ctrl = None

    def _theta(self, like):
        p = self.params
        if not isinstance(p, torch.Tensor):
            p = torch.tensor(p)
        return p.detach().to(device=like.device, dtype=torch.float32).contiguous()

    def forward(self, x, u):
        squeeze = x.ndimension() == 1
        if squeeze:
            x, u = x.unsqueeze(0), u.unsqueeze(0)
        p = self.params if isinstance(self.params, torch.Tensor) else torch.tensor(self.params)
        needs_grad = torch.is_grad_enabled() and (x.requires_grad or u.requires_grad or p.requires_grad)
        if needs_grad:
            th = p.to(device=x.device, dtype=torch.float32)
            out = _DynamicsFn.apply(x.float(), u.float(), th, self.model_id)
        else:
            x = x.detach().contiguous()
            u = u.detach().contiguous()
            out = torch.empty_like(x)
            N.call("dilqr_dynamics_f32", self.model_id, x.shape[0], N.ptr(self._theta(x)), N.ptr(x), N.ptr(u),
                   N.ptr(out), N.stream(x.device))
        return out.squeeze(0) if squeeze else out

    def get_linear_dyn(self, x, u):
        x = x.detach().contiguous()
        u = u.detach().contiguous()
        D = torch.empty(x.shape[0], self.n_state, self.n_state + self.n_ctrl, device=x.device)
        N.call("dilqr_linear_dyn_f32", self.model_id, x.shape[0], N.ptr(self._theta(x)), N.ptr(x), N.ptr(u),
               N.ptr(D), N.stream(x.device))
        return D

    def get_matrices(self, x, u):
        """(D, D_grad_params, D_grad_x, D_grad_u, x_grad_theta, x_grad_xtm1,
        x_grad_utm1) per row (cartpole.py:105-716, pendulum.py:152-382,
        rocket.py:258-261): one HIP kernel, dilqr_get_matrices_f32."""
        x = x.detach().float().contiguous()
        u = u.detach().float().contiguous()
        Nr, n, m = x.shape[0], self.n_state, self.n_ctrl
        d, p = n + m, N.lib().dilqr_model_num_params(self.model_id)
        dev = x.device
        outs = [torch.empty(Nr, *sh, device=dev) for sh in ((n, d), (n, d, p), (n, d, n), (n, d, m), (n, p),
                                                              (n, n), (n, m))]
        N.call("dilqr_get_matrices_f32", self.model_id, Nr, N.ptr(self._theta(x)), N.ptr(x), N.ptr(u),
               *[N.ptr(o) for o in outs], N.stream(dev))
        return tuple(outs)

    def grad_input(self, X, U, K=None):
        """The closed-loop total derivatives of the reference's grad_input
        (cartpole.py:717-788, pendulum.py:383-443, rocket.py:263-323):
        (grad_D [T-1,B,n,d,p], grad_d [T-1,B,n,p], D_x [T-1,B,n,d,n],
        D_u [T-1,B,n,d,m], D [T-1,B,n,d], d_x [T-1,B,n,n], d_u [T-1,B,n,m]).
        K [T,B,m,n] is consumed as K[t] (the order the caller stacks it; the
        implicit backward passes the reversed Riccati stack); None = zeros."""
        T, B, n = X.shape
        m = U.shape[2]
        d, p = n + m, N.lib().dilqr_model_num_params(self.model_id)
        dev = X.device
        Xc, Uc = X.detach().float().contiguous(), U.detach().float().contiguous()
        Kc = None
        if K is not None:
            if isinstance(K, (list, tuple)):        # the reference's per-step list (lqr_backward's Ks)
                K = torch.stack([torch.as_tensor(k) for k in K])
            Kc = torch.as_tensor(K).detach().to(device=dev, dtype=torch.float32).contiguous()
            if tuple(Kc.shape) != (T, B, m, n):   # k_grad_input reads K[t] for every t < T
                raise ValueError(f"grad_input: K must be [T, B, m, n] = {(T, B, m, n)}, got {tuple(Kc.shape)}")
        D, Dp, Dx, Du, xth, xx, xu = self.get_matrices(Xc.view(T * B, n), Uc.view(T * B, m))
        Tm = max(T - 1, 0)
        gD = torch.empty(Tm, B, n, d, p, device=dev)
        gd = torch.empty(Tm, B, n, p, device=dev)
        dX = torch.empty(Tm, B, n, n, device=dev)
        dU = torch.empty(Tm, B, n, m, device=dev)
        N.call("dilqr_grad_input_f32", self.model_id, T, B, N.ptr(Xc), N.ptr(Uc), N.ptr(Kc),
               *[N.ptr(a) for a in (D, Dp, Dx, Du, xth, xx, xu, gD, gd, dX, dU)], N.stream(dev))
        sh = lambda a: a.view(T, B, *a.shape[1:])[:Tm]  # noqa: E731
        return gD, gd, sh(Dx), sh(Du), sh(D), dX, dU

    def get_true_obj(self):
        q = torch.cat((self.goal_weights, self.ctrl_penalty * torch.ones(self.n_ctrl)))
        px = -torch.sqrt(self.goal_weights) * self.goal_state
        p = torch.cat((px, torch.zeros(self.n_ctrl)))
        return q, p
