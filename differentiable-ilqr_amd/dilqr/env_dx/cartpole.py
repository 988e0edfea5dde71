"""Cartpole (env_dx/cartpole.py): n=5 [x, dx, cos th, sin th, dth], m=1,
theta = (g, m_cart, m_pole, l) = (9.8, 1, 0.1, 0.5), dt = 0.05, |u| <= 100."""
import torch

from .. import _native as N
from ._base import HipDynamics


class CartpoleDx(HipDynamics):
    model_id = N.MODEL_CARTPOLE

    def __init__(self, params=None):
        super().__init__()
        self.n_state, self.n_ctrl = 5, 1
        self.params = torch.tensor((9.8, 1.0, 0.1, 0.5)) if params is None else params   # cartpole.py:39
        assert len(self.params) == 4
        self.force_mag = 100.
        self.theta_threshold_radians = 3.141592653589793
        self.x_threshold = 2.4
        self.max_velocity = 10
        self.dt = 0.05
        self.lower, self.upper = -self.force_mag, self.force_mag
        self.goal_state = torch.tensor([0., 0., 1., 0., 0.])
        self.goal_weights = torch.tensor([0.1, 0.1, 1., 1., 0.1])
        self.ctrl_penalty = 0.001
        self.mpc_eps = 1e-4                                                            # cartpole.py:60-62
        self.linesearch_decay = 0.5
        self.max_linesearch_iter = 2
