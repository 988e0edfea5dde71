"""The iLQR loop for generic dynamics and costs.

What the fused HIP iteration cannot take — dynamics that are an arbitrary
torch Module (e.g. the reference's NNDynamics, dynamics.py:15-130), the
GradMethods.AUTO_DIFF / FINITE_DIFF linearisations (mpc_explicit.py:547-627),
non-quadratic costs expanded by autograd (approximate_cost, 468-508), the
slew-rate augmentation with CtrlPassthroughDynamics (383-466, dynamics.py:
133-156) and the delta_u trust region (lqr_step_explicit.py:202-215) — runs
here: the user's Module is evaluated by torch on the GPU, batched over the
whole horizon wherever the reference loops over t, and every Riccati sweep
(+pnqp) is the HIP kernel (ops.lqr_backward, c_back fused).  The line search
follows lqr_step_explicit.py:166-263 with per-problem step sizes (the
reference's `torch.diag(alphas).mm(kt)` is O(B^2); here it is a broadcast),
the best-iterate bookkeeping and stop rule follow mpc_explicit.py:262-299.

Nothing here is on the HIP hot path of the headline: those solves go through
ops.mpc_solve.  This module exists so that a user of the reference with any
dynamics or cost finds the same MPC API working on the GPU.
"""
import torch

from . import _native as N
from . import ops
from .definitions import LinDx, QuadCost


# ---------------------------------------------------------------- batched helpers (util.py:42-56)
def bmv(X, y):
    return torch.matmul(X, y.unsqueeze(-1)).squeeze(-1)


def bquad(x, Q):
    return (x.unsqueeze(-2) @ Q @ x.unsqueeze(-1)).squeeze(-1).squeeze(-1)


def bdot(x, y):
    return (x * y).sum(-1)


def eclamp(x, lo, hi):
    """util.eclamp (util.py:58-72): the bound values are written exactly."""
    lo_t = lo if isinstance(lo, torch.Tensor) else torch.full_like(x, float(lo))
    hi_t = hi if isinstance(hi, torch.Tensor) else torch.full_like(x, float(hi))
    x = torch.where(x < lo_t, lo_t, x)
    return torch.where(x > hi_t, hi_t, x)


def quad_stage_cost(tau, C, c):
    return 0.5 * bquad(tau, C) + bdot(tau, c)


# ---------------------------------------------------------------- dynamics / cost wrappers
class CtrlPassthroughDynamics(torch.nn.Module):
    """dynamics.py:133-156: state [u_{t-1}; x_t] -> [u_t; f(x_t, u_t)]."""

    def __init__(self, dynamics):
        super().__init__()
        self.dynamics = dynamics

    def forward(self, tilde_x, u):
        squeeze = tilde_x.ndimension() == 1
        if squeeze:
            tilde_x = tilde_x.unsqueeze(0)
        if u.ndimension() == 1:
            u = u.unsqueeze(0)
        n_ctrl = u.size(1)
        out = torch.cat((u, self.dynamics(tilde_x[:, n_ctrl:], u)), dim=1)
        return out.squeeze(0) if squeeze else out


class SlewRateCost(torch.nn.Module):
    """mpc_explicit.py:35-55: cost(true tau) + 1/2 tau^T slew_C tau."""

    def __init__(self, cost, slew_C, n_state, n_ctrl):
        super().__init__()
        self.cost, self.slew_C, self.n_state, self.n_ctrl = cost, slew_C, n_state, n_ctrl

    def forward(self, tau):
        return self.cost(tau[:, self.n_ctrl:]) + 0.5 * bquad(tau, self.slew_C[0])


def rollout(T, u, x_init, dynamics):
    """util.get_traj (util.py:104-127)."""
    x = [x_init.detach()]
    with torch.no_grad():
        for t in range(T - 1):
            if isinstance(dynamics, LinDx):
                nx = bmv(dynamics.F[t], torch.cat((x[t], u[t]), 1))
                if dynamics.f is not None and dynamics.f.nelement() > 0:
                    nx = nx + dynamics.f[t]
            else:
                nx = dynamics(x[t], u[t].detach())
            x.append(nx.detach())
    return torch.stack(x, 0)


def traj_cost(T, x, u, cost):
    """util.get_cost (util.py:130-153) on a given trajectory; returns [B]."""
    with torch.no_grad():
        tau = torch.cat((x, u), 2)
        if isinstance(cost, QuadCost):
            return quad_stage_cost(tau, cost.C, cost.c).sum(0)
        return torch.stack([cost(tau[t]) for t in range(T)], 0).sum(0)


# ---------------------------------------------------------------- linearisation
def linearize(mpc, x, u, dynamics, diff):
    """MPC.linearize_dynamics (mpc_explicit.py:511-627, mpc.py:490-601) for
    every grad method, batched over the horizon: the (T-1)*B rows go through
    the dynamics as one batch (the reference loops over t; per-row dynamics give
    the same rows).  Returns F [T-1,B,n,n+m], f [T-1,B,n]."""
    from .mpc_explicit import GradMethods
    T, B, n = x.shape
    m = u.shape[2]
    dev = x.device
    if T < 2:
        return torch.zeros(0, B, n, n + m, device=dev), torch.zeros(0, B, n, device=dev)
    mid = getattr(dynamics, "model_id", None)
    gm = mpc.grad_method
    if gm == GradMethods.ANALYTIC and mid is not None and not diff:
        # the env_dx models: the HIP linearisation (get_linear_dyn, unclamped u)
        return ops.linearize(mid, ops.theta_of(dynamics, x), x.detach(), u.detach())
    xs = x[:-1].detach().reshape(-1, n)
    us = u[:-1].detach().reshape(-1, m)
    if gm == GradMethods.ANALYTIC:
        if mid is not None:
            # env_dx model, differentiable linearisation: get_linear_dyn
            # (mpc_explicit.py:516-546) on the autograd path of the model
            with torch.enable_grad():
                new_x = dynamics(xs, us)
                D = dynamics.get_linear_dyn(xs, us)
            f = new_x - bmv(D, torch.cat((xs, us), 1))
            return D.view(T - 1, B, n, n + m), f.view(T - 1, B, n)
        if not hasattr(dynamics, "grad_input"):
            raise ValueError("GradMethods.ANALYTIC needs dynamics.grad_input(x, u) -> (R, S)")
        # mpc.py:494-519: R, S from the model's grad_input (NNDynamics: the
        # chain of its weights, differentiable when diff)
        xs = xs.clone().requires_grad_(True)
        us = us.clone().requires_grad_(True)
        with torch.enable_grad():
            new_x = dynamics(xs, us)
            if not diff:
                new_x, xs, us = new_x.detach(), xs.detach(), us.detach()
            R, S = dynamics.grad_input(xs, us)
            f = new_x - bmv(R, xs) - bmv(S, us)
        F = torch.cat((R, S), 2)
        if not diff:
            F, f = F.detach(), f.detach()
        return F.view(T - 1, B, n, n + m), f.view(T - 1, B, n)
    if gm == GradMethods.AUTO_DIFF:
        # mpc_explicit.py:566-576: one backward per state component, without
        # create_graph (so F carries no graph; f does, through new_x)
        xs = xs.clone().requires_grad_(True)
        us = us.clone().requires_grad_(True)
        with torch.enable_grad():
            new_x = dynamics(xs, us)
            Rs, Ss = [], []
            for j in range(n):
                Rj, Sj = torch.autograd.grad(new_x[:, j].sum(), [xs, us], retain_graph=True)
                Rs.append(Rj)
                Ss.append(Sj)
            R, S = torch.stack(Rs, 1), torch.stack(Ss, 1)
            if not diff:
                new_x, xs, us = new_x.detach(), xs.detach(), us.detach()
            f = new_x - bmv(R, xs) - bmv(S, us)
        F = torch.cat((R, S), 2)
        if not diff:
            f = f.detach()
        return F.view(T - 1, B, n, n + m), f.view(T - 1, B, n)
    if gm == GradMethods.FINITE_DIFF:
        # mpc_explicit.py:598-611 with util.jacobian (util.py:10-20): central
        # differences, eps = 1e-4, every row at once.  With diff the quotients
        # keep their graph (the reference differentiates F through them too)
        eps = 1e-4
        with torch.set_grad_enabled(diff):
            new_x = dynamics(xs, us)
            Rc, Sc = [], []
            for i in range(n):
                e = torch.zeros_like(xs)
                e[:, i] = eps
                Rc.append((dynamics(xs + e, us) - dynamics(xs - e, us)) / (2. * eps))
            for i in range(m):
                e = torch.zeros_like(us)
                e[:, i] = eps
                Sc.append((dynamics(xs, us + e) - dynamics(xs, us - e)) / (2. * eps))
            R, S = torch.stack(Rc, 2), torch.stack(Sc, 2)
            f = new_x - bmv(R, xs) - bmv(S, us)
        F = torch.cat((R, S), 2)
        if not diff:
            f = f.detach()
        return F.view(T - 1, B, n, n + m), f.view(T - 1, B, n)
    raise NotImplementedError(f"dilqr: grad_method {gm} is not implemented")


def approximate_cost(x, u, cost, diff):
    """MPC.approximate_cost (mpc_explicit.py:468-508): the cost's Hessian and
    gradient at tau by autograd, all T*B rows at once.  Returns C [T,B,d,d],
    c [T,B,d] (= grad - H tau), stage costs [T,B]."""
    T, B, n = x.shape
    d = n + u.shape[2]
    with torch.enable_grad():
        tau = torch.cat((x, u), 2).detach().reshape(T * B, d).requires_grad_(True)
        val = cost(tau)
        grad = torch.autograd.grad(val.sum(), tau, create_graph=True)[0]
        H = torch.stack([torch.autograd.grad(grad[:, i].sum(), tau, create_graph=True)[0] for i in range(d)], -1)
        c = grad - bmv(H, tau)
    H, c, val = H.view(T, B, d, d), c.view(T, B, d), val.view(T, B)
    if not diff:
        return H.detach(), c.detach(), val.detach()
    return H, c, val


# ---------------------------------------------------------------- one LQR step (forward)
def lqr_step_forward(T, n, m, x_init, C, c, F, x, u, true_cost, true_dynamics, u_lower, u_upper, delta_u,
                     decay, max_ls, u_zero_I=None, extras=False):
    """LQRStepFn.forward of the DiLQR step (lqr_step_explicit.py:625-650): the
    HIP Riccati sweep in delta space (c_back = C tau + c fused), then the line
    search of lqr_forward (166-263) with the true dynamics/cost.  Returns
    (new_x, new_u, costs [B], full_du_norm [B]); with extras also the final
    step sizes [B] (one decay undone where the last pass still failed,
    254-255) and the sweep's pnqp iteration count."""
    B = x.shape[1]
    lo = u_lower if (u_lower is None or isinstance(u_lower, float)) else u_lower.detach().contiguous()
    hi = u_upper if (u_upper is None or isinstance(u_upper, float)) else u_upper.detach().contiguous()
    if delta_u is not None and lo is None:
        raise NotImplementedError("dilqr: delta_u without u_lower is unimplemented in the reference too "
                                  "(lqr_step_explicit.py:197)")
    zI = None if u_zero_I is None else u_zero_I.detach().bool()
    xd, ud = x.detach().contiguous(), u.detach().contiguous()
    Cd, cd, Fd = C.detach().contiguous(), c.detach().contiguous(), F.detach().contiguous()
    if delta_u is not None:
        # lqr_step_explicit.py:132-135: the sweep's relative box clipped to
        # +-delta_u (exact values), c_back formed here
        rlo, rhi = ops.delta_u_sweep_bounds(lo, hi, ud, delta_u)
        K, k, nqp = ops.lqr_backward(Cd, ops.c_back(Cd, cd, xd, ud), Fd, n, m, u_lower=rlo, u_upper=rhi,
                                     qp_total=extras)
    else:
        K, k, nqp = ops.lqr_backward(Cd, cd, Fd, n, m, x=xd, u=ud, u_lower=lo, u_upper=hi,
                                     u_zero_I=zI if lo is None else None, qp_total=extras and lo is not None)
    old_cost = traj_cost(T, x, u, true_cost)
    alphas = torch.ones(B, device=x.device)
    cur_cost, full_du_norm = None, None
    i = 0
    with torch.no_grad():
        while (cur_cost is None or bool((cur_cost > old_cost).any())) and i < max_ls:
            new_u, new_x, dxs, objs = [], [x_init.detach()], torch.zeros_like(x_init), []
            for t in range(T):
                nu = bmv(K[t], dxs) + u[t] + alphas.unsqueeze(1) * k[t]
                if zI is not None:                              # lqr_step_explicit.py:199-200
                    nu = torch.where(zI[t], torch.zeros_like(nu), nu)
                if lo is not None:
                    lb = lo if isinstance(lo, float) else lo[t]
                    ub = hi if isinstance(hi, float) else hi[t]
                    if delta_u is not None:                 # lqr_step_explicit.py:205-213
                        lb_lim, ub_lim = lb, ub
                        lb = u[t] - delta_u
                        ub = u[t] + delta_u
                        lb = torch.where(lb < lb_lim, torch.as_tensor(lb_lim, device=lb.device).expand_as(lb), lb)
                        ub = torch.where(ub > ub_lim, torch.as_tensor(ub_lim, device=ub.device).expand_as(ub), ub)
                    nu = eclamp(nu, lb, ub)
                new_u.append(nu)
                tau = torch.cat((new_x[t], nu), 1)
                if t < T - 1:
                    if isinstance(true_dynamics, LinDx):
                        nx = bmv(true_dynamics.F[t], tau)
                        if true_dynamics.f is not None and true_dynamics.f.nelement() > 0:
                            nx = nx + true_dynamics.f[t]
                    else:
                        nx = true_dynamics(new_x[t], nu)
                    new_x.append(nx)
                    dxs = nx - x[t + 1]
                if isinstance(true_cost, QuadCost):
                    objs.append(quad_stage_cost(tau, true_cost.C[t], true_cost.c[t]))
                else:
                    objs.append(true_cost(tau))
            cur_cost = torch.stack(objs).sum(0)
            new_u = torch.stack(new_u)
            new_x = torch.stack(new_x)
            if full_du_norm is None:                        # 245-247: the batch-mixing view
                full_du_norm = (u - new_u).transpose(1, 2).contiguous().view(B, -1).norm(2, 1)
            alphas = torch.where(cur_cost > old_cost, alphas * decay, alphas)
            i += 1
        if extras:
            alphas = torch.where(cur_cost > old_cost, alphas / decay, alphas)
    if extras:
        n_qp = nqp if isinstance(nqp, int) else 0
        return new_x, new_u, cur_cost, full_du_norm, alphas, n_qp
    return new_x, new_u, cur_cost, full_du_norm


# ---------------------------------------------------------------- the slew-rate augmentation
def slew_augment(mpc, x_init, C, c, F, f, cost, dynamics, x, u):
    """solve_lqr_subproblem's slew-rate branch (mpc_explicit.py:383-466): the
    state becomes [u_{t-1}; x_t] with cost gamma/2 |u_t - u_{t-1}|^2 added."""
    T, n, m = mpc.T, mpc.n_state, mpc.n_ctrl
    B = C.size(1)
    nsc = n + m
    _nsc = nsc + m
    dev, dt = C.device, C.dtype
    _C = torch.zeros(T, B, _nsc, _nsc, device=dev, dtype=dt)
    half_gamI = mpc.slew_rate_penalty * torch.eye(m, device=dev, dtype=dt).expand(T, B, m, m)
    _C[:, :, :m, :m] = half_gamI
    _C[:, :, -m:, :m] = -half_gamI
    _C[:, :, :m, -m:] = -half_gamI
    _C[:, :, -m:, -m:] = half_gamI
    slew_C = _C.clone()
    _C = _C + torch.nn.functional.pad(C, (m, 0, m, 0))
    _c = torch.cat((torch.zeros(T, B, m, device=dev, dtype=dt), c), 2)
    _F0 = torch.cat((torch.zeros(m, n + m, device=dev, dtype=dt), torch.eye(m, device=dev, dtype=dt)), 1)
    _F0 = _F0.expand(T - 1, B, m, nsc + m)
    _F1 = torch.cat((torch.zeros(T - 1, B, n, m, device=dev, dtype=dt), F), 3)
    _F = torch.cat((_F0, _F1), 2)
    _f = None if f is None else torch.cat((torch.zeros(T - 1, B, m, device=dev, dtype=dt), f), 2)
    if mpc.prev_ctrl is not None:
        prev_u = mpc.prev_ctrl.detach()
        if prev_u.ndimension() == 1:
            prev_u = prev_u.unsqueeze(0)
        if prev_u.ndimension() == 2:
            prev_u = prev_u.unsqueeze(0)
    else:
        prev_u = torch.zeros(1, B, m, device=dev, dtype=dt)
    utm1s = torch.cat((prev_u.expand(1, B, m), u.detach()[:-1]))
    _x = torch.cat((utm1s, x), 2)
    _x_init = torch.cat((prev_u[0].expand(B, m), x_init), 1)
    _dyn = None if isinstance(dynamics, LinDx) else CtrlPassthroughDynamics(dynamics)
    _cost = QuadCost(_C, _c) if isinstance(cost, QuadCost) else SlewRateCost(cost, slew_C, n, m)
    return _x_init, _C, _c, _F, _f, _dyn, _cost, _x


def solve_subproblem(mpc, x_init, C, c, F, f, cost, dynamics, x, u, extras=False):
    """One LQR step of the outer loop (solve_lqr_subproblem, mpc_explicit.py:360-466).
    extras: also the step sizes and the pnqp count (the verbose table)."""
    T, n, m = mpc.T, mpc.n_state, mpc.n_ctrl
    if mpc.slew_rate_penalty is None or isinstance(cost, torch.nn.Module):
        return lqr_step_forward(T, n, m, x_init, C, c, F, x, u, cost, dynamics, mpc.u_lower, mpc.u_upper,
                                mpc.delta_u, mpc.linesearch_decay, mpc.max_linesearch_iter,
                                getattr(mpc, "u_zero_I", None), extras=extras)
    _x_init, _C, _c, _F, _f, _dyn, _cost, _x = slew_augment(mpc, x_init, C, c, F, f, cost, dynamics, x, u)
    true_dyn = _dyn if _dyn is not None else LinDx(_F, _f)
    out = lqr_step_forward(T, n + m, m, _x_init, _C, _c, _F, _x, u, _cost, true_dyn, mpc.u_lower,
                           mpc.u_upper, mpc.delta_u, mpc.linesearch_decay, mpc.max_linesearch_iter,
                           getattr(mpc, "u_zero_I", None), extras=extras)
    return (out[0][:, :, m:],) + tuple(out[1:])


# ---------------------------------------------------------------- the outer loop
def solve(mpc, x_init, cost, dx, n_batch):
    """mpc_explicit.MPC.forward / mpc.MPC.forward loop (mpc_explicit.py:226-299)
    for generic dynamics/costs.  Returns (best x, best u, best costs, best
    full_du_norm), all detached."""
    T, n, m = mpc.T, mpc.n_state, mpc.n_ctrl
    dev = x_init.device
    if mpc.u_init is None:
        u = torch.zeros(T, n_batch, m, device=dev, dtype=x_init.dtype)
    else:
        u = mpc.u_init.to(device=dev, dtype=x_init.dtype)
        if u.ndimension() == 2:
            u = u.unsqueeze(1).expand(T, n_batch, -1).clone()
    x_init = x_init.detach()
    best = None
    n_not_improved = 0
    verbose = getattr(mpc, "verbose", 0) > 0
    if verbose:                                                          # mpc_explicit.py:236-241
        x0 = rollout(T, u, x_init, dx)
        print("Initial mean(cost): {:.4e}".format(float(traj_cost(T, x0, u, cost).mean())))
    for it in range(mpc.lqr_iter):
        u = u.detach()
        x = rollout(T, u, x_init, dx)
        if isinstance(dx, LinDx):
            F, f = dx.F.detach(), (None if dx.f is None or dx.f.nelement() == 0 else dx.f.detach())
        else:
            F, f = linearize(mpc, x, u, dx, diff=False)
        if isinstance(cost, QuadCost):
            C, c = cost.C.detach(), cost.c.detach()
        else:
            C, c, _ = approximate_cost(x, u, cost, diff=False)
        out = solve_subproblem(mpc, x_init, C, c, F, f, cost, dx, x, u, extras=verbose)
        x, u, costs, full_du_norm = out[:4]
        n_not_improved += 1
        if best is None:
            best = {"x": x.clone(), "u": u.clone(), "costs": costs.clone(), "fdn": full_du_norm.clone()}
        else:
            take = costs <= best["costs"] + mpc.best_cost_eps           # mpc_explicit.py:277-283
            if bool(take.any()):
                n_not_improved = 0
            best["x"][:, take] = x[:, take]
            best["u"][:, take] = u[:, take]
            best["costs"][take] = costs[take]
            best["fdn"][take] = full_du_norm[take]
        if verbose:                                                      # mpc_explicit.py:285-295
            from .util import table_log
            table_log("lqr", (("iter", it), ("mean(cost)", float(best["costs"].mean()), "{:.4e}"),
                              ("||full_du||_max", float(full_du_norm.max()), "{:.2e}"),
                              ("mean(alphas)", float(out[4].mean()), "{:.2e}"), ("total_qp_iters", out[5])))
        if float(full_du_norm.max()) < mpc.eps or n_not_improved > mpc.not_improved_lim:   # 297-299
            break
    return best["x"], best["u"], best["costs"], best["fdn"]


def final_step(mpc, x_init, cost, dx, x, u, classic):
    """The reference's closing no-op LQR step (mpc_explicit.py:302-325,
    mpc.py:299-318): linearise at the best iterate WITH gradients (the
    autograd linearisation / cost expansion graphs carry them to the dynamics'
    and cost's parameters), then the no-op step whose backward is the classic
    adjoint kernel (classic=True) or the DiLQR implicit backward."""
    from .lqr_step import LQRStep as ClassicStep
    from .lqr_step_explicit import LQRStep as ExplicitStep
    T, n, m = mpc.T, mpc.n_state, mpc.n_ctrl
    if isinstance(dx, LinDx):
        F, f = dx.F, dx.f
    else:
        F, f = linearize(mpc, x, u, dx, diff=True)
    if isinstance(cost, QuadCost):
        C, c = cost.C, cost.c
    else:
        C, c, _ = approximate_cost(x, u, cost, diff=True)
    if f is None:
        f = torch.empty(0, device=x.device)
    if mpc.slew_rate_penalty is not None and not isinstance(cost, torch.nn.Module):
        _x_init, _C, _c, _F, _f, _dyn, _cost, _x = slew_augment(mpc, x_init, C, c, F, f if f.nelement() else None,
                                                                cost, dx, x, u)
        if not classic:
            raise NotImplementedError("dilqr: the DiLQR implicit backward with a slew-rate penalty")
        step = ClassicStep(n + m, m, T, u_lower=mpc.u_lower, u_upper=mpc.u_upper, true_cost=_cost,
                           true_dynamics=_dyn if _dyn is not None else LinDx(_F, _f), current_x=_x.detach(),
                           current_u=u.detach(), back_eps=mpc.back_eps, no_op_forward=True)
        xa, ua = step(_x_init, _C, _c, _F, _f if _f is not None else torch.empty(0, device=x.device))
        return xa[:, :, m:], ua
    if classic:
        step = ClassicStep(n, m, T, u_lower=mpc.u_lower, u_upper=mpc.u_upper, true_cost=QuadCost(C, c),
                           true_dynamics=dx, current_x=x.detach(), current_u=u.detach(), back_eps=mpc.back_eps,
                           no_op_forward=True)
        return step(x_init, C, c, F, f)
    if getattr(dx, "model_id", None) not in (N.MODEL_CARTPOLE, N.MODEL_PENDULUM, N.MODEL_ROCKET):
        # the DiLQR implicit backward needs an env_dx model's second derivatives
        # (the reference reads dx.params and dx.grad_input and raises without
        # them, mpc_explicit.py:325, lqr_step_explicit.py:703): a caller whose
        # inputs carry gradients gets the same refusal, never a silently
        # detached solution; without gradients there is nothing to attach
        wants = [t for t in (x_init, C, c, F, f) if isinstance(t, torch.Tensor) and t.requires_grad]
        if wants:
            raise NotImplementedError(
                "dilqr: mpc_explicit.MPC differentiates through the DiLQR implicit backward, which needs an "
                "env_dx model (cartpole, pendulum, rocket); use mpc.MPC (classic adjoint) for LinDx or "
                "generic dynamics, or solve under torch.no_grad()")
        return x.detach(), u.detach()
    th = dx.params if isinstance(dx.params, torch.Tensor) else torch.tensor(dx.params)
    # the no-op step's sweep (its gains feed the implicit backward) sees the
    # same mask / trust region as the loop's (mpc_explicit.py:369, 452)
    step = ExplicitStep(n, m, T, u_lower=mpc.u_lower, u_upper=mpc.u_upper, u_zero_I=getattr(mpc, "u_zero_I", None),
                        delta_u=mpc.delta_u, true_cost=QuadCost(C, c), true_dynamics=dx, current_x=x.detach(),
                        current_u=u.detach(), back_eps=mpc.back_eps, no_op_forward=True)
    return step(x_init, C, c, F, f, th)
