"""Rocket (env_dx/rocket.py): n=13 [r(3), v(3), q(4), w(3)], m=3 thrust
[f, f_side1, f_side2], theta = (Jx, Jy, Jz, mass, l) = (0.5, 1, 1, 1, 1), dt = 0.1,
thrust clamped to +-400 inside the dynamics, |u| <= 20 for the MPC.

Like the reference, forward() returns the UNNORMALISED quaternion
(rocket.py:156-164 normalises a copy it does not return)."""
import torch

from .. import _native as N
from ._base import HipDynamics


class RocketDx(HipDynamics):
    model_id = N.MODEL_ROCKET

    def __init__(self, params=None):
        super().__init__()
        self.dt = 0.1
        self.n_state, self.n_ctrl = 13, 3
        self.params = torch.tensor((0.5, 1.0, 1.0, 1.0, 1.0)) if params is None else params   # rocket.py:27-30
        assert len(self.params) == 5
        self.goal_state = torch.zeros(13)
        self.goal_state[6] = 1.0                                                # rocket.py:33-42
        self.goal_weights = torch.ones(13)
        self.goal_weights[0:3] = 10.0
        self.goal_weights[6:10] = 0.1                                           # rocket.py:44-53
        self.side_penalty, self.thrust_penalty = 1, 0.4
        self.ctrl_penalty = torch.tensor([self.side_penalty, self.side_penalty, self.thrust_penalty])
        self.tilt_penalty = 50.0
        self.max_thrust = 20 ** 2
        self.max_tilt_angle = 0.3
        self.mpc_eps = 1e-3                                                     # rocket.py:68-70
        self.linesearch_decay = 0.2
        self.max_linesearch_iter = 5
        self.tilt_Q = self.tilt_penalty * torch.tensor([0., 0., 4., 4.])        # rocket.py:75-79
        self.tilt_p = self.tilt_penalty * torch.tensor([0., 0., 0., 0.])
        self.lower, self.upper = torch.tensor([-20., -20., -20.]), torch.tensor([20., 20., 20.])

    def get_true_obj(self):
        """rocket.py:212-232 (tilt_penalty applied a second time, as there)."""
        q = torch.cat((self.goal_weights, self.ctrl_penalty))
        q[6:10] = self.tilt_Q * self.tilt_penalty
        px = -torch.sqrt(self.goal_weights) * self.goal_state
        px[6:10] = -self.tilt_p * self.tilt_penalty
        p = torch.cat((px, torch.zeros(self.n_ctrl)))
        return q, p

    def get_cost_matrices(self, n_batch, mpc_T):
        """rocket.py:234-256, literally: adding the 4-vector tilt_Q to the 13x13
        state block does not broadcast, so this raises as the reference does;
        callers build diag(get_true_obj()) instead (il_env.py:159-162)."""
        q, p = self.get_true_obj()
        Q = torch.diag(q).clone()
        Q[:self.n_state, :self.n_state] += self.tilt_Q
        Q = Q.unsqueeze(0).unsqueeze(0).repeat(mpc_T, n_batch, 1, 1)
        p = p.unsqueeze(0).unsqueeze(0).repeat(mpc_T, n_batch, 1)
        return Q, p
