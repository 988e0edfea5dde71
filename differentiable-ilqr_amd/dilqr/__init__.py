"""dilqr — MI355X-native batched differentiable iLQR (drop-in for the hot path of
josef-w/Differentiable-iLQR).

Modules mirror the reference's: definitions (QuadCost, LinDx), mpc_explicit
(DiLQR MPC + GradMethods), lqr_step_explicit (DiLQR LQRStep), mpc / lqr_step
(classic differentiable LQR), env_dx (cartpole, pendulum models).  All compute
runs in libdilqr.so (HIP, gfx950) — see include/dilqr.h.
"""
from .definitions import LinDx, QuadCost  # noqa: F401
from .mpc_explicit import MPC, GradMethods  # noqa: F401
from .lqr_step_explicit import LQRStep  # noqa: F401
from . import env_dx, ops  # noqa: F401

__version__ = "0.1.0"
