"""CPU baseline: the reference's iLQR forward path restated in fp32 torch on the
host cores, with the reference's OP STRUCTURE (one batched torch op per
timestep per quantity, a Python loop over the horizon, the per-problem Python
best-iterate loop), so its timing stands in for the reference's CPU PyTorch
path on a machine the reference itself never reaches (the GPU box).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): bench.py's cpu_baseline leg
times it; tests/test_torch_cpu.py pins it to the reference's fp32 goldens and to
the numpy oracle.  Written from the reference's math, not copied:

  * get_traj                 util.py:104-127 (Python loop over t, dx.forward per t)
  * linearize (ANALYTIC)     mpc_explicit.py:516-546 (one batched forward and
                             get_linear_dyn over the (T-1)*B rows)
  * c_back                   lqr_step_explicit.py:630-636 (loop over t of bmv)
  * lqr_backward (m = 1)     lqr_step_explicit.py:54-162 (Q = C + F^T V F by bmm,
                             K = -Q_ux/Q_uu, V/v update by bmm/bmv)
  * lqr_forward              lqr_step_explicit.py:166-263, including the
                             reference's diag(alphas).mm(k_t) step (O(B^2) per
                             step and pass: why the reference is run in chunks)
  * MPC loop                 mpc_explicit.py:246-299 with the per-problem Python
                             loop of the best-iterate update (277-283)

Cartpole only (config 2 of BASELINE.json: unconstrained, m = 1), the model
equations of cartpole.py:64-97 and the closed-form Jacobian of cartpole.py:
790-839 (derivative of the same equations).
"""
import os
import time

import torch

DT = 0.05
THETA = (9.8, 1.0, 0.1, 0.5)      # g, m_cart, m_pole, l (cartpole.py:39)
FORCE_MAG = 100.0


def bmv(X, y):
    return torch.bmm(X, y.unsqueeze(2)).squeeze(2)


def cartpole_forward(state, u, th=THETA):
    """cartpole.py:64-97: clamp, atan2 angle, accelerations, explicit Euler."""
    g, mc, mp, l = th
    total = mc + mp
    pml = mp * l
    uu = torch.clamp(u[:, 0], -FORCE_MAG, FORCE_MAG)
    x, dx, c, s, dth = state.unbind(1)
    ang = torch.atan2(s, c)
    cart_in = (uu + pml * dth ** 2 * s) / total
    th_acc = (g * s - c * cart_in) / (l * (4. / 3. - mp * c ** 2 / total))
    xacc = cart_in - pml * th_acc * c / total
    ang = ang + DT * dth
    return torch.stack((x + DT * dx, dx + DT * xacc, torch.cos(ang), torch.sin(ang), dth + DT * th_acc), 1)


def cartpole_jacobian(state, u, th=THETA):
    """d forward / d [x; u] at the unclamped u (cartpole.py:790-839), [N,5,6]."""
    g, mc, mp, l = th
    total = mc + mp
    pml = mp * l
    c, s, w = state[:, 2], state[:, 3], state[:, 4]
    uu = u[:, 0]
    A = uu + pml * w ** 2 * s
    den = l * (4. / 3. - mp * c ** 2 / total)
    num = g * s - c * A / total
    tha = num / den
    A_s, A_w = pml * w ** 2, 2 * pml * w * s
    den_c = -2 * l * mp * c / total
    tha_c = (-A / total - tha * den_c) / den
    tha_s = (g - c * A_s / total) / den
    tha_w = (-c * A_w / total) / den
    tha_u = (-c / total) / den
    k = pml / total
    xa_c = -k * (tha_c * c + tha)
    xa_s = A_s / total - k * tha_s * c
    xa_w = A_w / total - k * tha_w * c
    xa_u = 1. / total - k * tha_u * c
    ang = torch.atan2(s, c) + DT * w
    cs, sn = torch.cos(ang), torch.sin(ang)
    r2 = c ** 2 + s ** 2
    N = state.shape[0]
    D = torch.zeros(N, 5, 6, dtype=state.dtype)
    D[:, 0, 0] = 1.
    D[:, 0, 1] = DT
    D[:, 1, 1] = 1.
    D[:, 1, 2], D[:, 1, 3], D[:, 1, 4], D[:, 1, 5] = DT * xa_c, DT * xa_s, DT * xa_w, DT * xa_u
    D[:, 2, 2], D[:, 2, 3], D[:, 2, 4] = s * sn / r2, -c * sn / r2, -DT * sn
    D[:, 3, 2], D[:, 3, 3], D[:, 3, 4] = -s * cs / r2, c * cs / r2, DT * cs
    D[:, 4, 2], D[:, 4, 3], D[:, 4, 4], D[:, 4, 5] = DT * tha_c, DT * tha_s, 1. + DT * tha_w, DT * tha_u
    return D


def get_traj(T, u, x_init):
    xs = [x_init]
    for t in range(T - 1):
        xs.append(cartpole_forward(xs[t], u[t]))
    return torch.stack(xs)


def bquad(x, Q):
    return x.unsqueeze(1).bmm(Q).bmm(x.unsqueeze(2)).squeeze(1).squeeze(1)


def get_cost(T, C, c, x, u):
    """util.get_cost on a given trajectory: a loop over t of 1/2 bquad + bdot."""
    objs = []
    for t in range(T):
        xut = torch.cat((x[t], u[t]), 1)
        objs.append(0.5 * bquad(xut, C[t]) + (xut * c[t]).sum(1))
    return torch.stack(objs).sum(0)


def linearize(x, u):
    T, B, n = x.shape
    m = u.shape[2]
    xs, us = x[:-1].reshape(-1, n), u[:-1].reshape(-1, m)
    nx = cartpole_forward(xs, us)
    D = cartpole_jacobian(xs, us)
    f = nx - bmv(D, torch.cat((xs, us), 1))
    return D.view(T - 1, B, n, n + m), f.view(T - 1, B, n)


def lqr_backward(C, c_back, F, n):
    """m = 1, unconstrained, delta space (f_back = None)."""
    T = C.shape[0]
    Ks, ks = [None] * T, [None] * T
    V = v = None
    for t in range(T - 1, -1, -1):
        if t == T - 1:
            Q, q = C[t], c_back[t]
        else:
            Ft = F[t]
            FtT = Ft.transpose(1, 2)
            Q = C[t] + FtT.bmm(V).bmm(Ft)
            q = c_back[t] + bmv(FtT, v)
        Qxx, Qxu, Qux, Quu = Q[:, :n, :n], Q[:, :n, n:], Q[:, n:, :n], Q[:, n:, n:]
        qx, qu = q[:, :n], q[:, n:]
        K = -(1. / Quu) * Qux
        k = -(1. / Quu.squeeze(2)) * qu
        KT = K.transpose(1, 2)
        V = Qxx + Qxu.bmm(K) + KT.bmm(Qux) + KT.bmm(Quu).bmm(K)
        v = qx + bmv(Qxu, k) + bmv(KT, qu) + bmv(KT.bmm(Quu), k)
        Ks[t], ks[t] = K, k
    return Ks, ks


def lqr_forward(x_init, C, c, x, u, Ks, ks, decay, max_ls):
    T, B, n = x.shape
    old_cost = get_cost(T, C, c, x, u)
    alphas = torch.ones(B, dtype=x.dtype)
    cost = full_du_norm = None
    i = 0
    while (cost is None or bool((cost > old_cost).any())) and i < max_ls:
        new_x, new_u = [x_init], []
        dx = torch.zeros_like(x_init)
        objs = []
        for t in range(T):
            nu = bmv(Ks[t], dx) + u[t] + torch.diag(alphas).mm(ks[t])
            new_u.append(nu)
            tau = torch.cat((new_x[t], nu), 1)
            if t < T - 1:
                nx = cartpole_forward(new_x[t], nu)
                new_x.append(nx)
                dx = nx - x[t + 1]
            objs.append(0.5 * bquad(tau, C[t]) + (tau * c[t]).sum(1))
        cost = torch.stack(objs).sum(0)
        new_u = torch.stack(new_u)
        new_x = torch.stack(new_x)
        if full_du_norm is None:                 # the batch-mixing view (lqr_step_explicit.py:245-247)
            full_du_norm = (u - new_u).transpose(1, 2).contiguous().view(B, -1).norm(2, 1)
        alphas[cost > old_cost] *= decay
        i += 1
    alphas[cost > old_cost] /= decay
    alpha_du_norm = (u - new_u).transpose(1, 2).contiguous().view(B, -1).norm(2, 1)   # 255-256
    return new_x, new_u, cost, full_du_norm, alpha_du_norm, torch.mean(alphas)


def mpc_forward(x_init, C, c, T, lqr_iter, decay=0.5, max_ls=2, best_cost_eps=1e-4, eps=0.0,
                not_improved_lim=10 ** 9):
    """The unconstrained loop (stop rule evaluated as the reference does, with
    the builtin max over the batch): returns best x, u, costs."""
    B, n = x_init.shape
    u = torch.zeros(T, B, 1, dtype=x_init.dtype)
    best = None
    n_not_improved = 0
    for _ in range(lqr_iter):
        x = get_traj(T, u, x_init)
        F, _f = linearize(x, u)
        cb = torch.stack([bmv(C[t], torch.cat((x[t], u[t]), 1)) + c[t] for t in range(T)])   # 630-636
        Ks, ks = lqr_backward(C, cb, F, n)
        x, u, costs, full_du_norm, _adn, _ma = lqr_forward(x_init, C, c, x, u, Ks, ks, decay, max_ls)
        n_not_improved += 1
        if best is None:
            best = {"x": list(torch.split(x, 1, dim=1)), "u": list(torch.split(u, 1, dim=1)), "costs": costs,
                    "full_du_norm": full_du_norm}
        else:
            for j in range(B):                               # mpc_explicit.py:277-283
                if costs[j] <= best["costs"][j] + best_cost_eps:
                    n_not_improved = 0
                    best["x"][j] = x[:, j].unsqueeze(1)
                    best["u"][j] = u[:, j].unsqueeze(1)
                    best["costs"][j] = costs[j]
                    best["full_du_norm"][j] = full_du_norm[j]
        if max(full_du_norm) < eps or n_not_improved > not_improved_lim:   # 297-299
            break
    return torch.cat(best["x"], 1), torch.cat(best["u"], 1), best["costs"]


def host_threads():
    """The host cores this process may use: OMP_NUM_THREADS when set (the GPU
    box sets it to the box's CPU share), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def time_config2(make_problems, T=25, chunks=(512, 1024, 2048, 4096), iters=6, reps=3, budget_s=30.0,
                 threads=None):
    """Problem-iterations/s of the reference-structured CPU path on config 2
    (cartpole T=25, unconstrained, decay 0.5, max_ls 2), chunked: per chunk size,
    per-iteration time = (t(iters) - t(1)) / (iters - 1), best of `reps`
    (SURVEY.md §8(d) protocol); the best chunk is the baseline.  Stops adding
    chunk sizes once `budget_s` is spent."""
    threads = threads or host_threads()
    torch.set_num_threads(threads)
    q = torch.tensor([0.1, 0.1, 1., 1., 0.1, 0.001])
    p = torch.tensor([0., 0., -1., 0., 0., 0.])
    out = {}
    t_start = time.perf_counter()
    with torch.no_grad():
        for B in chunks:
            if time.perf_counter() - t_start > budget_s and out:
                break
            x0 = torch.tensor(make_problems(B, seed=1)[0])
            C = torch.diag(q).expand(T, B, 6, 6).contiguous()
            c = p.expand(T, B, 6).contiguous()
            mpc_forward(x0, C, c, T, 1)                     # warm-up
            best = {}
            for k in (1, iters):
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    mpc_forward(x0, C, c, T, k)
                    ts.append(time.perf_counter() - t0)
                best[k] = min(ts)
            per_iter = (best[iters] - best[1]) / (iters - 1)
            out[B] = B / per_iter
    bestB = max(out, key=out.get)
    return {"value": out[bestB], "chunk": bestB, "by_chunk": {str(k): v for k, v in out.items()},
            "threads": threads, "elapsed_s": time.perf_counter() - t_start}
