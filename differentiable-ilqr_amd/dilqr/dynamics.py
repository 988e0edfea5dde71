"""Generic dynamics modules of the reference (dynamics.py), for the MPC's
generic loop (dilqr.generic).

They are plain torch Modules — evaluated by torch on the GPU — with the
reference's constructor arguments, parameter layout (so its state dicts load)
and `grad_input` Jacobians.  The fused HIP kernels never see them: the MPC
routes any dynamics other than the env_dx models through dilqr.generic, whose
Riccati sweeps are the HIP kernel.
"""
import torch
import torch.nn.functional as Fn
from torch import nn

from .generic import CtrlPassthroughDynamics  # noqa: F401  (dynamics.py:133-156)

ACTS = {"sigmoid": torch.sigmoid, "relu": Fn.relu, "elu": Fn.elu}


class NNDynamics(nn.Module):
    """dynamics.py:15-130: x' = MLP([x; u]) (+ x with passthrough)."""

    def __init__(self, n_state, n_ctrl, hidden_sizes=(100,), activation="sigmoid", passthrough=True):
        super().__init__()
        self.passthrough = passthrough
        sizes = list(hidden_sizes) + [n_state]
        fcs, in_sz = [], n_state + n_ctrl
        for out_sz in sizes:
            fcs.append(nn.Linear(in_sz, out_sz))
            in_sz = out_sz
        self.fcs = nn.ModuleList(fcs)
        if activation not in ACTS:
            raise ValueError(f"activation must be one of {sorted(ACTS)}")
        self.activation = activation
        self.acts = [ACTS[activation]] * (len(self.fcs) - 1) + [lambda z: z]
        self.zs = []

    @property
    def Ws(self):
        return [fc.weight for fc in self.fcs]

    def forward(self, x, u):
        x_dim, u_dim = x.ndimension(), u.ndimension()
        if x_dim == 1:
            x = x.unsqueeze(0)
        if u_dim == 1:
            u = u.unsqueeze(0)
        self.zs = []
        z = torch.cat((x, u), 1)
        for act, fc in zip(self.acts, self.fcs):
            z = act(fc(z))
            self.zs.append(z)
        self.zs = self.zs[:-1]            # the hidden activations (dynamics.py:82-83)
        if self.passthrough:
            z = z + x
        return z.squeeze(0) if x_dim == 1 else z

    def grad_input(self, x, u):
        """dynamics.py:92-130: R = d x'/d x, S = d x'/d u from the weights and the
        last forward's activations."""
        n_batch, n_state = x.size()
        diff = x.requires_grad or u.requires_grad
        Ws = self.Ws if diff else [W.detach() for W in self.Ws]
        zs = self.zs if diff else [z.detach() for z in self.zs]
        grad = Ws[-1].unsqueeze(0).repeat(n_batch, 1, 1)
        for i in range(len(zs) - 1, -1, -1):
            n_out, n_in = Ws[i].size()
            if self.activation == "relu":
                Wi = Ws[i].unsqueeze(0).repeat(n_batch, 1, 1)
                Wi = Wi * (zs[i] > 0.).to(Wi.dtype).unsqueeze(2)
            elif self.activation == "sigmoid":
                d = (zs[i] * (1. - zs[i])).unsqueeze(2).expand(n_batch, n_out, n_in)
                Wi = Ws[i].unsqueeze(0).repeat(n_batch, 1, 1) * d
            else:
                raise NotImplementedError("grad_input: relu and sigmoid only (as the reference)")
            grad = grad.bmm(Wi)
        R, S = grad[:, :, :n_state], grad[:, :, n_state:]
        if self.passthrough:
            R = R + torch.eye(n_state, dtype=R.dtype, device=R.device).unsqueeze(0)
        return R, S


class AffineDynamics(nn.Module):
    """dynamics.py:159-202: x' = A x + B u + c."""

    def __init__(self, A, B, c=None):
        super().__init__()
        assert A.ndimension() == 2 and B.ndimension() == 2
        self.A, self.B, self.c = A, B, c

    def forward(self, x, u):
        x_dim = x.ndimension()
        if x_dim == 1:
            x = x.unsqueeze(0)
        if u.ndimension() == 1:
            u = u.unsqueeze(0)
        z = x.mm(self.A.t()) + u.mm(self.B.t()) + (self.c if self.c is not None else 0.)
        return z.squeeze(0) if x_dim == 1 else z

    def grad_input(self, x, u):
        n_batch = x.size(0)
        return self.A.unsqueeze(0).repeat(n_batch, 1, 1), self.B.unsqueeze(0).repeat(n_batch, 1, 1)
