"""Oracle LQR kernels (numpy): Riccati sweep, pnqp, rollout + line search, cost.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

All tensors are time-major like the reference: C [T,B,d,d], c [T,B,d],
F [T-1,B,n,d], x [T,B,n], u [T,B,m].  Gains are returned in NATURAL time order
K [T,B,m,n], k [T,B,m] (the reference appends them T-1 -> 0,
lqr_step_explicit.py:63,154).

Batch semantics.  The reference's pnqp is batch-coupled (its Armijo loop exits on
the batch max, pnqp.py:65-76, and it returns early only when every problem has
converged, pnqp.py:56-59).  `per_problem=True` evaluates pnqp one problem at a
time, which is the reference's own behaviour at batch size 1 and the semantics
the HIP kernels implement (one problem per lane).  Everything else here is
per-problem already.
"""
import numpy as np

GAMMA = 0.1


def bmv(X, y):
    return (X @ y[..., None])[..., 0]


def eclamp(x, lower, upper):
    """util.py:58-72 (in place in the reference; here on a copy)."""
    x = x.copy()
    lo = lower if np.ndim(lower) == 0 else lower
    hi = upper if np.ndim(upper) == 0 else upper
    I = x < lo
    x[I] = lo if np.ndim(lo) == 0 else lo[I]
    I = x > hi
    x[I] = hi if np.ndim(hi) == 0 else hi[I]
    return x


def _slice(v, sl):
    return v if np.ndim(v) == 0 else v[sl]


def _note(margins, key, vals):
    """margins[key] = elementwise min(margins[key], vals) (per problem)."""
    if margins is None:
        return
    vals = np.asarray(vals, np.float64)
    margins[key] = vals if key not in margins else np.minimum(margins[key], vals)


def pnqp(H, q, lower, upper, x_init=None, n_iter=20, per_problem=False, margins=None):
    """Projected-Newton box QP, pnqp.py:5-82.

    Returns (x [B,m], H_free [B,m,m] (the masked matrix whose LU/inverse the
    reference returns), If [B,m] free mask, n_iter_done).
    With per_problem=True, n_iter_done is an int array [B].

    margins (dict, per_problem only): per problem, the smallest distance of any
    of its discrete decisions from its threshold — the clamp of a candidate
    (|x - bound|, relative), the clamped-set sign test (|g_i| at a bound), the
    stop test (| ||dx|| - 1e-4 |) and the Armijo test (|armijo - GAMMA|) —
    so a test can tell a near-tie decision (which fp32 may take the other way)
    from real error.  Key 'pnqp'.
    """
    if per_problem:
        B = H.shape[0]
        mb = [dict() if margins is not None else None for _ in range(B)]
        outs = [pnqp(H[b:b + 1], q[b:b + 1], _slice(lower, slice(b, b + 1)),
                     _slice(upper, slice(b, b + 1)),
                     None if x_init is None else x_init[b:b + 1], n_iter, margins=mb[b]) for b in range(B)]
        if margins is not None:
            _note(margins, "pnqp", [m_.get("pnqp", [np.inf])[0] for m_ in mb])
        return (np.concatenate([o[0] for o in outs]), np.concatenate([o[1] for o in outs]),
                np.concatenate([o[2] for o in outs]), np.array([o[3] for o in outs]))
    dt = H.dtype
    B, n, _ = H.shape
    eye = np.eye(n, dtype=dt)

    def obj(x):
        return 0.5 * np.einsum("bi,bij,bj->b", x, H, x) + np.einsum("bi,bi->b", q, x)

    if x_init is None:                                   # pnqp.py:14-19
        if n == 1:
            x_init = -(1. / H[:, :, 0]) * q
        else:
            x_init = -np.linalg.solve(H, q[..., None])[..., 0]
    def bound_gap(z):                                    # distance of z from the nearer bound
        sc = np.maximum(1.0, np.abs(z))
        return np.min(np.minimum(np.abs(z - lower), np.abs(z - upper)) / sc, axis=1)

    if margins is not None:
        _note(margins, "pnqp", bound_gap(x_init))
    x = eclamp(x_init, lower, upper)

    H_ = If = None
    for i in range(n_iter):                              # pnqp.py:28-78
        g = bmv(H, x) + q
        if margins is not None:
            at = (x == lower) | (x == upper)
            _note(margins, "pnqp", np.min(np.where(at, np.abs(g), np.inf), axis=1))
        Ic = (((x == lower) & (g > 0)) | ((x == upper) & (g < 0))).astype(dt)
        If = 1 - Ic
        Hff = If[:, :, None] * If[:, None, :]
        g_ = g.copy()
        g_[Ic.astype(bool)] = 0.
        H_ = H.copy()
        H_[(1 - Hff).astype(bool)] = 0.
        H_ = H_ + dt.type(1e-11) * eye
        if n == 1:
            dx = -(1. / H_[:, :, 0]) * g_
        else:
            dx = -np.linalg.solve(H_, g_[..., None])[..., 0]
        J = np.linalg.norm(dx, axis=1) >= 1e-4
        if margins is not None:
            _note(margins, "pnqp", np.abs(np.linalg.norm(dx, axis=1) - 1e-4) / 1e-4)
        if J.sum() == 0:
            return x, H_, If, i
        alpha = np.ones(B, dt)
        max_armijo = GAMMA
        count = 0
        while max_armijo <= GAMMA and count < 10:
            if margins is not None:
                _note(margins, "pnqp", bound_gap(x + alpha[:, None] * dx))
            maybe_x = eclamp(x + alpha[:, None] * dx, lower, upper)
            armijos = np.full(B, GAMMA + 1e-6, dt)
            with np.errstate(divide="ignore", invalid="ignore"):
                num = obj(x) - obj(maybe_x)
                den = np.einsum("bi,bi->b", g, x - maybe_x)
                armijos[J] = (num / den)[J]
            I = armijos <= GAMMA
            if margins is not None:
                _note(margins, "pnqp", np.where(J, np.abs(armijos - GAMMA), np.inf))
            alpha[I] *= dt.type(0.1)
            max_armijo = np.max(armijos)
            count += 1
        x = maybe_x
    return x, H_, If, i


def lqr_backward(C, c_back, F, n, m, u=None, u_lower=None, u_upper=None, u_zero_I=None,
                 m_solver="pinv", per_problem=False, margins=None):
    """Backward Riccati sweep in delta space (f_back=None), lqr_step_explicit.py:54-162.

    m_solver: 'pinv'  -> per-sample pinverse for m>1 (lqr_step_explicit.py:90-96)
              'chol'  -> cholesky(Q_uu + 1e-6 I) (lqr_step_backup.py:199-208)
    u_zero_I [T,B,m] bool: the masked solve of lqr_step_backup.py:210-232.
    Returns K [T,B,m,n], k [T,B,m], n_total_qp_iter.
    """
    T, B = C.shape[:2]
    dt = C.dtype
    K = np.zeros((T, B, m, n), dt)
    k = np.zeros((T, B, m), dt)
    V = v = None
    prev_kt = None
    n_qp = 0
    for t in range(T - 1, -1, -1):
        if t == T - 1:
            Q, q = C[t], c_back[t]
        else:
            Ft = F[t]
            FtT = np.swapaxes(Ft, 1, 2)
            Q = C[t] + FtT @ V @ Ft
            q = c_back[t] + bmv(FtT, v)
        Qxx, Qxu, Qux, Quu = Q[:, :n, :n], Q[:, :n, n:], Q[:, n:, :n], Q[:, n:, n:]
        qx, qu = q[:, :n], q[:, n:]
        if u_lower is None:
            if m == 1 and u_zero_I is None:
                Kt = -(1. / Quu) * Qux
                kt = -(1. / Quu[:, :, 0]) * qu
            elif u_zero_I is None:
                if m_solver == "pinv":
                    Qi = np.stack([np.linalg.pinv(Quu[b]) for b in range(B)])
                elif m_solver == "lu":
                    Qi = np.linalg.inv(Quu)
                else:
                    L = np.linalg.cholesky(Quu + dt.type(1e-6) * np.eye(m, dtype=dt))
                    Qi = np.linalg.inv(np.swapaxes(L, 1, 2)) @ np.linalg.inv(L)
                Kt = -Qi @ Qux
                kt = bmv(-Qi, qu)
            else:
                I = u_zero_I[t].astype(dt)
                notI = 1 - I
                qu_ = qu.copy()
                qu_[I.astype(bool)] = 0
                Quu_ = Quu.copy()
                Quu_[(1 - notI[:, :, None] * notI[:, None, :]).astype(bool)] = 0.
                diag = np.zeros_like(Quu_, dtype=bool)
                for j in range(m):
                    diag[:, j, j] = I[:, j].astype(bool)
                Quu_[diag] += dt.type(1e-8)
                Qux_ = Qux.copy()
                Qux_[np.repeat(I[:, :, None], n, 2).astype(bool)] = 0.
                if m == 1:
                    Kt = -(1. / Quu_) * Qux_
                    kt = -(1. / Quu[:, :, 0]) * qu_
                else:
                    Kt = -np.linalg.solve(Quu_, Qux_)
                    kt = -np.linalg.solve(Quu_, qu_[..., None])[..., 0]
        else:
            lo = u_lower if np.ndim(u_lower) == 0 else u_lower[t]
            hi = u_upper if np.ndim(u_upper) == 0 else u_upper[t]
            lb = lo - u[t]
            ub = hi - u[t]
            kt, Hf, If, it = pnqp(Quu, qu, lb, ub, x_init=prev_kt, n_iter=20, per_problem=per_problem,
                                  margins=margins)
            n_qp += 1 + (int(np.max(it)) if per_problem else it)
            prev_kt = kt
            Qux_ = Qux.copy()
            Qux_[np.repeat((1 - If)[:, :, None], n, 2).astype(bool)] = 0
            if m == 1:
                Kt = -((1. / Hf) * Qux_)
            else:
                Kt = -np.linalg.solve(Hf, Qux_)
        K[t], k[t] = Kt, kt
        KtT = np.swapaxes(Kt, 1, 2)
        V = Qxx + Qxu @ Kt + KtT @ Qux + KtT @ Quu @ Kt
        v = qx + bmv(Qxu, kt) + bmv(KtT, qu) + bmv(KtT @ Quu, kt)
    return K, k, n_qp


def c_back(C, c, x, u):
    """Delta-space linear term C_t tau_t + c_t (lqr_step_explicit.py:630-636)."""
    tau = np.concatenate([x, u], -1)
    return bmv(C, tau) + c


def quad_cost_terms(C, c, tau):
    """0.5 tau^T C tau + c^T tau per (t,b), util.py:130-153."""
    return 0.5 * np.einsum("tbi,tbij,tbj->tb", tau, C, tau) + np.einsum("tbi,tbi->tb", tau, c)


def get_traj(T, u, x_init, dyn):
    """util.py:104-127.  dyn is a callable (x,u)->x' or ('lin', F, f)."""
    x = [x_init]
    for t in range(T - 1):
        if isinstance(dyn, tuple):
            _, F, f = dyn
            nx = bmv(F[t], np.concatenate([x[t], u[t]], 1))
            if f is not None:
                nx = nx + f[t]
        else:
            nx = dyn(x[t], u[t])
        x.append(nx)
    return np.stack(x)


def quirk_du_norm(u, new_u):
    """The reference's `(u-new_u).transpose(1,2).contiguous().view(n_batch,-1).norm(2,1)`
    (lqr_step_explicit.py:245-247, 255-256): the [T,m,B] buffer is re-viewed as
    [B, T*m], so row r mixes several problems unless m*T divides B's layout.
    Restated exactly."""
    T, B, m = u.shape
    flat = np.ascontiguousarray(np.transpose(u - new_u, (0, 2, 1))).reshape(B, T * m)
    return np.linalg.norm(flat, axis=1)


def lqr_forward(x_init, C, c, x, u, K, k, dyn, u_lower=None, u_upper=None, u_zero_I=None,
                linesearch_decay=0.2, max_linesearch_iter=10, margins=None, force_alpha=None):
    """Rollout with batched backtracking line search, lqr_step_explicit.py:166-263.

    dyn: callable true dynamics, or ('lin', F, f) for a LinDx.
    Returns new_x, new_u, costs, full_du_norm, alpha_du_norm, mean_alphas, alphas.
    margins (dict): per problem, the smallest relative distance of an accept
    test it took (|cost_p - old| / max(1, |old|), key 'linesearch') and of a
    control it clamped or kept from a bound (key 'clamp').
    force_alpha [B] (test use): after the line search has made (and recorded)
    its own decisions, return instead the rollout at these step sizes — the
    trajectory the search returns when it settles on them — so a test can
    replay another implementation's decisions and compare arithmetic alone.
    The returned alphas stay this search's own choices.
    """
    T, B, n = x.shape
    dt = x.dtype
    old_cost = quad_cost_terms(C, c, np.concatenate([x, u], -1)).sum(0)
    alphas = np.ones(B, dt)
    current_cost = None
    full_du_norm = None
    live = np.ones(B, bool)                              # problems still deciding (the rest repeat their pass)
    i = 0
    while (current_cost is None or np.any(current_cost > old_cost)) and i < max_linesearch_iter:
        new_x = [x_init]
        new_u = []
        dx = np.zeros_like(x_init)
        for t in range(T):
            nut = bmv(K[t], dx) + u[t] + alphas[:, None] * k[t]
            if u_zero_I is not None:
                nut[u_zero_I[t]] = 0.
            if u_lower is not None:
                lo = u_lower if np.ndim(u_lower) == 0 else u_lower[t]
                hi = u_upper if np.ndim(u_upper) == 0 else u_upper[t]
                if margins is not None:
                    gap = np.minimum(np.abs(nut - lo), np.abs(nut - hi)) / np.maximum(1.0, np.abs(nut))
                    _note(margins, "clamp", np.where(live, np.min(gap, axis=1), np.inf))
                nut = eclamp(nut, lo, hi)
            new_u.append(nut)
            if t < T - 1:
                if isinstance(dyn, tuple):
                    _, F, f = dyn
                    nxt = bmv(F[t], np.concatenate([new_x[t], nut], 1))
                    if f is not None:
                        nxt = nxt + f[t]
                else:
                    nxt = dyn(new_x[t], nut)
                new_x.append(nxt)
                dx = nxt - x[t + 1]
        new_x, new_u = np.stack(new_x), np.stack(new_u)
        current_cost = quad_cost_terms(C, c, np.concatenate([new_x, new_u], -1)).sum(0)
        if margins is not None:
            rel = np.abs(current_cost - old_cost) / np.maximum(1.0, np.abs(old_cost))
            last = i == max_linesearch_iter - 1                  # the last pass is accepted regardless
            _note(margins, "linesearch", np.where(live & (not last), rel, np.inf))
            live = live & (current_cost > old_cost)
        if full_du_norm is None:
            full_du_norm = quirk_du_norm(u, new_u)
        alphas[current_cost > old_cost] *= dt.type(linesearch_decay)
        i += 1
    alphas[current_cost > old_cost] /= dt.type(linesearch_decay)
    if force_alpha is not None:
        new_x, new_u = rollout_at(x_init, x, u, K, k, dyn, np.asarray(force_alpha, dt), u_lower, u_upper, u_zero_I)
        current_cost = quad_cost_terms(C, c, np.concatenate([new_x, new_u], -1)).sum(0)
    alpha_du_norm = quirk_du_norm(u, new_u)
    return new_x, new_u, current_cost, full_du_norm, alpha_du_norm, np.mean(alphas), alphas


def rollout_at(x_init, x, u, K, k, dyn, alphas, u_lower=None, u_upper=None, u_zero_I=None):
    """One pass of lqr_forward's rollout at per-problem step sizes alphas [B]."""
    T = x.shape[0]
    new_x, new_u = [x_init], []
    dx = np.zeros_like(x_init)
    for t in range(T):
        nut = bmv(K[t], dx) + u[t] + alphas[:, None] * k[t]
        if u_zero_I is not None:
            nut[u_zero_I[t]] = 0.
        if u_lower is not None:
            lo = u_lower if np.ndim(u_lower) == 0 else u_lower[t]
            hi = u_upper if np.ndim(u_upper) == 0 else u_upper[t]
            nut = eclamp(nut, lo, hi)
        new_u.append(nut)
        if t < T - 1:
            if isinstance(dyn, tuple):
                _, F, f = dyn
                nxt = bmv(F[t], np.concatenate([new_x[t], nut], 1))
                if f is not None:
                    nxt = nxt + f[t]
            else:
                nxt = dyn(new_x[t], nut)
            new_x.append(nxt)
            dx = nxt - x[t + 1]
    return np.stack(new_x), np.stack(new_u)
