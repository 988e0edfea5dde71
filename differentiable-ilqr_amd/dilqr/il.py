"""The imitation-learning loop around the solver (SURVEY.md §8 f #1-2) on the
HIP path: the reference's IL_Env (il_env.py:31-188), the empc / sysid training
epochs of IL_Exp.run (il_exp.py:183-429) and dataset_loss (440-495), and its
datasets (data/*.pkl) read without unpickling.

Everything numeric runs through dilqr.mpc_explicit.MPC (device-resident iLQR
loop forward, fused implicit backward); the host keeps the reference's control
flow: warm-start buffers, RMSprop over (learn_q_logit, learn_p, env_params),
the q/p round robin every 10 epochs.  Out of scope: the
argparse CLI, CSV logging, pickled checkpoints, the 'nn' LSTM baseline, and the
'pendulum-complex' NNDynamics variant.
"""
import io
import pickletools
import warnings

import numpy as np
import torch
from torch import optim
from torch.utils.data import DataLoader, TensorDataset

from .definitions import QuadCost
from .env_dx.cartpole import CartpoleDx
from .env_dx.pendulum import PendulumDx
from .mpc_explicit import MPC, GradMethods

_ENVS = {"pendulum": PendulumDx, "cartpole": CartpoleDx}


# ---------------------------------------------------------------- datasets
def load_il_dataset(path):
    """Read a reference dataset (a pickled IL_Env, il_exp.py:75-77) WITHOUT
    unpickling: the pickle opcode stream is walked with pickletools, scalar
    attributes are taken from their (key, value) opcode pairs, and each
    embedded tensor storage is loaded with torch.load(weights_only=True) and
    viewed with the offset/size/stride that follow it in the stream.  Returns
    {"env": name, scalars..., "params", "goal_state", "goal_weights",
    "train_data", "val_data", "test_data"} with float tensors on the CPU."""
    data = open(path, "rb").read()
    ops = list(pickletools.genops(data))
    out, tensors, last_key = {}, [], None
    for i, (op, arg, _pos) in enumerate(ops):
        if op.name in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE") and isinstance(arg, str):
            if last_key == "env" and "env" not in out:
                out["env"] = arg
                last_key = None
                continue
            last_key = arg
        elif op.name in ("BININT1", "BININT2", "BININT", "BINFLOAT") and last_key is not None:
            out.setdefault(last_key, arg)
            last_key = None
        elif op.name == "BINBYTES":
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")          # TypedStorage deprecation
                storage = torch.load(io.BytesIO(arg), weights_only=True)
                flat = torch.tensor(storage.tolist(), dtype=storage.dtype)
            # torch._utils._rebuild_tensor_v2(storage, offset, size, stride, ...)
            ints = []
            for op2, arg2, _ in ops[i + 1:i + 40]:
                if op2.name in ("BININT1", "BININT2", "BININT"):
                    ints.append(arg2)
                if op2.name in ("NEWTRUE", "NEWFALSE"):
                    break
            off, rest = ints[0], ints[1:]
            nd = len(rest) // 2
            tensors.append(torch.as_strided(flat, rest[:nd], rest[nd:], off).clone())
    # the IL_Env's tensors in pickling order: true_dx.params, goal_state,
    # goal_weights, then train/val/test data (il_env.py:31-54, 81-94)
    names = ("params", "goal_state", "goal_weights", "train_data", "val_data", "test_data")
    for name, t in zip(names, tensors):
        out[name] = t.float()
    return out


# ---------------------------------------------------------------- IL_Env
class IL_Env:
    """il_env.py:31-188 for 'pendulum' and 'cartpole', tensors on `device`."""

    def __init__(self, env, lqr_iter=100, mpc_T=35, device="cuda"):
        if env not in _ENVS:
            raise NotImplementedError(f"dilqr: IL env {env!r} is not on the HIP path")
        self.env = env
        self.device = torch.device(device)
        self.true_dx = _ENVS[env]()
        self.lqr_iter = lqr_iter
        self.mpc_T = mpc_T
        self.grad_method = GradMethods.ANALYTIC
        self.train_data = self.val_data = self.test_data = None

    @classmethod
    def from_dataset(cls, path, device="cuda"):
        """An IL_Env carrying a reference dataset (load_il_dataset)."""
        d = load_il_dataset(path)
        env = cls(d["env"], lqr_iter=int(d["lqr_iter"]), mpc_T=int(d["mpc_T"]), device=device)
        env.train_data, env.val_data, env.test_data = d["train_data"], d["val_data"], d["test_data"]
        return env

    def sample_xinit(self, n_batch=1):
        """il_env.py:59-79 (CPU generator, as the reference draws it)."""
        def uniform(shape, low, high):
            return torch.rand(shape) * (high - low) + low
        if self.env == "pendulum":
            th = uniform(n_batch, -(1 / 2) * np.pi, (1 / 2) * np.pi)
            thdot = uniform(n_batch, -1., 1.)
            return torch.stack((torch.cos(th), torch.sin(th), thdot), dim=1)
        x = uniform(n_batch, -0.5, 0.5) * 0
        dx = uniform(n_batch, -0.5, 0.5) * 0
        th = uniform(n_batch, -np.pi, np.pi) * 0 + torch.ones(n_batch) * 3.1415926 / 1.05
        dth = uniform(n_batch, -1., 1.) * 0
        return torch.stack((x, dx, torch.cos(th), torch.sin(th), dth), dim=1)

    def populate_data(self, n_train, n_val, n_test, seed=0):
        """il_env.py:81-94: expert trajectories from the true model, one batched
        MPC solve on the GPU."""
        torch.manual_seed(seed)
        xinit = self.sample_xinit(n_batch=n_train + n_val + n_test).to(self.device)
        q, p = self.true_dx.get_true_obj()
        with torch.no_grad():
            x, u = self.mpc(self.true_dx, xinit, q.to(self.device), p.to(self.device))
        tau = torch.cat((x, u), dim=2).transpose(0, 1)
        self.train_data = tau[:n_train]
        self.val_data = tau[n_train:n_train + n_val]
        self.test_data = tau[-n_test:]

    def mpc(self, dx, xinit, q, p, u_init=None, eps_override=None, lqr_iter_override=None):
        """il_env.py:153-188."""
        n_batch = xinit.shape[0]
        Q = torch.diag(q).unsqueeze(0).unsqueeze(0).repeat(self.mpc_T, n_batch, 1, 1)
        p = p.unsqueeze(0).repeat(self.mpc_T, n_batch, 1)
        eps = eps_override if eps_override else self.true_dx.mpc_eps
        lqr_iter = lqr_iter_override if lqr_iter_override else self.lqr_iter
        x_mpc, u_mpc, _ = MPC(
            self.true_dx.n_state, self.true_dx.n_ctrl, self.mpc_T,
            u_lower=float(self.true_dx.lower), u_upper=float(self.true_dx.upper), u_init=u_init,
            lqr_iter=lqr_iter, verbose=0, exit_unconverged=False, detach_unconverged=True,
            linesearch_decay=self.true_dx.linesearch_decay,
            max_linesearch_iter=self.true_dx.max_linesearch_iter,
            grad_method=self.grad_method, eps=eps)(xinit, QuadCost(Q, p), dx)
        return x_mpc, u_mpc


# ---------------------------------------------------------------- IL_Exp (training)
class ILTrainer:
    """The empc / sysid training loop of IL_Exp.run (il_exp.py:183-429) and
    dataset_loss (440-495), without the CLI/logging/checkpoint plumbing.
    `history` collects the rows the reference writes to train_losses.csv
    (epoch fraction, im_loss[, sysid_loss]) and val_test_losses.csv."""

    RESTART_WARMSTART_EVERY = 50          # il_exp.py:82
    ROUND_ROBIN = 10                      # il_exp.py:282

    def __init__(self, env, mode="empc", learn_cost=False, learn_dx=False, n_batch=32, n_train=100, seed=5,
                 env_params=None):
        if mode not in ("empc", "imempc", "sysid"):
            raise NotImplementedError(f"dilqr: IL mode {mode!r} is not on the HIP path")
        if mode in ("empc", "imempc"):
            assert learn_cost or learn_dx
        if mode == "sysid":
            learn_dx = True
        self.env, self.mode = env, mode
        self.learn_cost, self.learn_dx = learn_cost, learn_dx
        self.n_batch, self.n_train, self.seed = n_batch, n_train, seed
        dev = env.device
        self.device = dev
        self.n_state, self.n_ctrl = env.true_dx.n_state, env.true_dx.n_ctrl
        torch.manual_seed(seed)
        true_q, true_p = env.true_dx.get_true_obj()
        self.true_q, self.true_p = true_q.to(dev), true_p.to(dev)
        self.learn_q_logit = torch.zeros_like(self.true_q).requires_grad_()      # il_exp.py:128-132
        self.learn_p = torch.zeros_like(self.true_p).requires_grad_()
        if learn_dx:
            init = {"pendulum": (15., 3., 0.5), "cartpole": (9.8, 3.0, 0.1, 1.0)}[env.env]   # 136-141
            p0 = torch.tensor(init if env_params is None else env_params, dtype=torch.float32)
        else:
            p0 = env.true_dx.params.detach().clone().float()
        self.env_params = p0.to(dev).requires_grad_()
        if mode == "sysid":
            self.opt = optim.RMSprop([{"params": [self.env_params], "lr": 1e-2, "alpha": 0.5}])
        else:
            params1 = ([self.learn_q_logit, self.learn_p] if learn_cost else []) + \
                      ([self.env_params] if learn_dx else [])
            self.opt = optim.RMSprop([{"params": params1, "lr": 1e-2, "alpha": 0.5}])
        self.history = {"train": [], "val_test": [], "params": []}
        self.cost_update_q = False
        self.epoch = 0

    # -- il_exp.py:432-439 (the same DataLoader, so shuffling draws the global
    # generator exactly as the reference's loop does)
    def _loader(self, data, shuffle=False):
        data = data.to(self.device)
        xs, us = data[:, :, :self.n_state], data[:, :, -self.n_ctrl:]
        xinits = xs[:, 0]
        ds = TensorDataset(xinits, xs, us, torch.arange(0, xinits.shape[0], device=self.device))
        return DataLoader(ds, batch_size=self.n_batch, shuffle=shuffle)

    def _dx(self):
        return self.env.true_dx.__class__(self.env_params)

    def _qp(self):
        if self.learn_cost:
            q = torch.sigmoid(self.learn_q_logit)
            return q, q.sqrt() * self.learn_p
        return self.true_q, self.true_p

    def fit(self, n_epoch):
        env, T = self.env, self.env.mpc_T
        if self.epoch == 0:
            torch.manual_seed(self.seed)                      # il_exp.py:184
            self.train = self._loader(env.train_data[:self.n_train], shuffle=True)
            self.val = self._loader(env.val_data)
            self.test = self._loader(env.test_data)
            self.train_warmstart = torch.zeros(len(self.train.dataset), T, self.n_ctrl, device=self.device)
            self.val_warmstart = torch.zeros(len(self.val.dataset), T, self.n_ctrl, device=self.device)
            self.test_warmstart = torch.zeros(len(self.test.dataset), T, self.n_ctrl, device=self.device)
        n_batches = len(self.train)
        for _ in range(n_epoch):
            i = self.epoch
            if i > 0 and i % self.ROUND_ROBIN == 0:
                self.cost_update_q = not self.cost_update_q
            if i % self.RESTART_WARMSTART_EVERY == 0:
                self.train_warmstart.zero_(); self.val_warmstart.zero_(); self.test_warmstart.zero_()
            for j, (xinits, xs, us, idxs) in enumerate(self.train):
                dx = self._dx()
                q, p = self._qp()
                nom_x, nom_u = env.mpc(dx, xinits, q, p, u_init=self.train_warmstart[idxs].transpose(0, 1))
                nom_u = nom_u.transpose(0, 1)
                self.train_warmstart[idxs] = nom_u.detach()
                im_loss = (us.detach() - nom_u).pow(2).mean()
                row = [i + j / n_batches, float(im_loss.detach())]
                sysid_loss = None
                if self.learn_dx:
                    xs_flat = xs[:, :-1].reshape(-1, self.n_state)
                    us_flat = us[:, :-1].reshape(-1, self.n_ctrl)
                    pred_next_x = dx(xs_flat, us_flat).view(xs.shape[0], T - 1, self.n_state)
                    sysid_loss = (xs[:, 1:].detach() - pred_next_x).pow(2).mean()
                    row.append(float(sysid_loss.detach()))
                self.history["train"].append(row)
                self.opt.zero_grad()
                (sysid_loss if self.mode == "sysid" else im_loss).backward()
                if self.learn_cost:
                    if self.cost_update_q:
                        self.learn_p.grad.zero_()
                    else:
                        self.learn_q_logit.grad.zero_()
                # dx_hist.csv / cost_hist.csv rows: the parameters this step used
                self.history["params"].append(self.env_params.detach().cpu().numpy().copy())
                if self.learn_cost:
                    q, p = self._qp()
                    self.history.setdefault("cost", []).append(torch.cat((q, p)).detach().cpu().numpy().copy())
                self.opt.step()
            val = self.dataset_loss(self.val, self.val_warmstart)
            test = self.dataset_loss(self.test, self.test_warmstart)
            self.history["val_test"].append([i, val, test])
            self.epoch += 1
        return self.history

    @torch.no_grad()
    def dataset_loss(self, loader, warmstart):
        """il_exp.py:440-495."""
        losses = []
        for xinits, xs, us, idxs in loader:
            q, p = self._qp()
            _, pred_u = self.env.mpc(self._dx(), xinits, q, p, u_init=warmstart[idxs].transpose(0, 1))
            pred_u = pred_u.transpose(0, 1)
            warmstart[idxs] = pred_u
            losses.append((us - pred_u).pow(2).mean(dim=1))
        return float(torch.cat(losses).mean())
