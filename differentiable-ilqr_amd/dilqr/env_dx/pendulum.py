"""Pendulum (env_dx/pendulum.py, simple variant): n=3 [cos th, sin th, dth], m=1,
theta = (g, m, l) = (10, 1, 1), dt = 0.05, |u| <= 2."""
import torch

from .. import _native as N
from ._base import HipDynamics


class PendulumDx(HipDynamics):
    model_id = N.MODEL_PENDULUM

    def __init__(self, params=None, simple=True):
        super().__init__()
        if not simple:
            raise NotImplementedError("dilqr: the 5-parameter pendulum (simple=False) is not on the HIP path")
        self.simple = True
        self.max_torque = 2.0
        self.dt = 0.05
        self.n_state, self.n_ctrl = 3, 1
        self.params = torch.tensor((10., 1., 1.)) if params is None else params          # pendulum.py:42
        assert len(self.params) == 3
        self.goal_state = torch.tensor([1., 0., 0.])
        self.goal_weights = torch.tensor([1., 1., 0.1])
        self.ctrl_penalty = 0.001
        self.lower, self.upper = -2., 2.
        self.mpc_eps = 1e-3                                                              # pendulum.py:56-58
        self.linesearch_decay = 0.2
        self.max_linesearch_iter = 5
