"""Pendulum (env_dx/pendulum.py): n=3 [cos th, sin th, dth], m=1, dt = 0.05,
|u| <= 2.  simple=True: theta = (g, m, l) = (10, 1, 1) (pendulum.py:40-42);
simple=False: theta = (g, m, l, d, b) = (10, 1, 1, 0, 0), a damping d*th and a
gravity bias b (pendulum.py:43-45, 84-89; il_env.py:40-42 'pendulum-complex'
uses (10, 1, 1, 1, 0.1)).

The 5-parameter variant has no closed-form Jacobian in the reference (its
get_linear_dyn and get_matrices unpack three parameters, pendulum.py:157, 448,
so mpc_explicit.MPC with GradMethods.ANALYTIC raises there); its runnable path
is GradMethods.AUTO_DIFF, autograd through forward().  Here its Jacobian
(dilqr_models.h PendulumComplex) IS that autograd derivative, so ANALYTIC and
AUTO_DIFF both run the fused HIP iteration with it.  The second-order terms the
implicit backward needs do not exist in the reference for this variant
(grad_input -> get_matrices fails the same way), so gradients through an MPC
solve of it raise NotImplementedError."""
import torch

from .. import _native as N
from ._base import HipDynamics


class PendulumDx(HipDynamics):

    def __init__(self, params=None, simple=True):
        super().__init__()
        self.simple = simple
        self.max_torque = 2.0
        self.dt = 0.05
        self.n_state, self.n_ctrl = 3, 1
        if params is None:                                                               # pendulum.py:40-45
            params = torch.tensor((10., 1., 1.)) if simple else torch.tensor((10., 1., 1., 0., 0.))
        self.params = params
        assert len(self.params) == (3 if simple else 5)
        self.goal_state = torch.tensor([1., 0., 0.])
        self.goal_weights = torch.tensor([1., 1., 0.1])
        self.ctrl_penalty = 0.001
        self.lower, self.upper = -2., 2.
        self.mpc_eps = 1e-3                                                              # pendulum.py:56-58
        self.linesearch_decay = 0.2
        self.max_linesearch_iter = 5

    @property
    def model_id(self):
        return N.MODEL_PENDULUM if self.simple else N.MODEL_PENDULUM_COMPLEX

    @property
    def jacobian_is_autograd(self):
        """get_linear_dyn equals autograd through forward() (the clamp's gate on
        u included): true for the 5-parameter variant only — the reference's
        closed forms for the 3-parameter one are taken at the unclamped u."""
        return not self.simple
