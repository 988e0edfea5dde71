"""DiLQR implicit backward (lqr_step_explicit.py:653-712) on the HIP path: one
fused kernel per call (dilqr_implicit_backward_f32): one lane per problem for
pendulum and cartpole, a 16-lane group per problem for rocket."""
import torch

from . import _native as N
from . import ops


def implicit_backward(model, dl_dx, dl_du, C, c, F, f, x, u, K, u_lower, u_upper, theta):
    """Returns (dC [T,B,d,d], dc [T,B,d], dtheta [B,p]).  K: the no-op step's
    gains in natural time order (the kernel applies the reference's reversed
    stacking).  F, f are not needed: the kernel re-linearises at (x, u)."""
    mid = ops.model_id_of(model)
    if mid == N.MODEL_PENDULUM_COMPLEX:
        raise NotImplementedError(
            "dilqr: no implicit backward for the 5-parameter pendulum: the reference's grad_input / get_matrices "
            "exist for the 3-parameter model only (pendulum.py:157 unpacks g, m, l)")
    if mid not in (N.MODEL_CARTPOLE, N.MODEL_PENDULUM, N.MODEL_ROCKET):
        raise NotImplementedError("dilqr: the implicit backward needs a pendulum, cartpole or rocket model")
    T, B, n = x.shape
    m = u.shape[2]
    d = n + m
    dev = x.device
    th = ops.theta_of(model, x)
    bounds, keep = N.make_bounds(u_lower, u_upper)
    rec = N.lib().dilqr_implicit_ws_floats(mid)
    ws = torch.empty(T * B * rec, device=dev)
    dC = torch.empty(T, B, d, d, device=dev)
    dc = torch.empty(T, B, d, device=dev)
    dth = torch.empty(B, th.shape[0], device=dev)
    args = [ops._f32(a) for a in (C, c, x, u, K, dl_dx, dl_du)]
    N.call("dilqr_implicit_backward_f32", mid, T, B, N.ptr(th), *[N.ptr(a) for a in args], bounds, N.ptr(ws),
           N.ptr(dC), N.ptr(dc), N.ptr(dth), N.stream(dev))
    del keep
    if isinstance(theta, torch.Tensor):
        dth = dth.to(device=theta.device, dtype=theta.dtype)
    return dC.to(C.dtype), dc.to(c.dtype), dth
