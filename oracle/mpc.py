"""Oracle iLQR outer loop (numpy), restating mpc_explicit.MPC.forward
(mpc_explicit.py:182-358) with GradMethods.ANALYTIC linearisation
(mpc_explicit.py:511-546).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
import numpy as np

from . import lqr


def linearize(model, x, u, params=None):
    """mpc_explicit.py:516-546: F = get_linear_dyn(x,u), f = f(x,u) - F [x;u],
    over the first T-1 steps."""
    T, B, n = x.shape
    m = u.shape[2]
    _x = x[:-1].reshape(-1, n)
    _u = u[:-1].reshape(-1, m)
    nx = model.forward(_x, _u, params)
    D = model.get_linear_dyn(_x, _u, params)
    d = nx - np.einsum("bnm,bm->bn", D, np.concatenate([_x, _u], -1))
    return D.reshape(T - 1, B, n, n + m), d.reshape(T - 1, B, n)


def mpc_forward(model, x_init, C, c, T, u_init=None, u_lower=None, u_upper=None, lqr_iter=10,
                eps=1e-7, linesearch_decay=0.2, max_linesearch_iter=10, not_improved_lim=5,
                best_cost_eps=1e-4, params=None, per_problem=False, m_solver="pinv", trace=None, margins=None,
                force=None):
    """Returns (x [T,B,n], u [T,B,m], costs [B], info).

    `model` is one of oracle.models.MODELS, or ('lin', F, f) for a LinDx.
    C/c must already be materialised [T,B,d,d] / [T,B,d].
    margins (dict): per problem, the smallest relative distance of each kind of
    discrete decision of the solve from its threshold (keys 'linesearch',
    'clamp', 'pnqp' from lqr.lqr_forward / lqr.pnqp, 'best' for the best-iterate
    test cost <= best + best_cost_eps, 'stop' for the batch-wide eps test);
    margins['min'] is their minimum.  A problem with a clear margin everywhere
    follows the same decision path in fp32 as in this fp64 restatement.
    force (test use): force(i) -> (alphas [B], take [B] bool) of iteration i as
    another implementation decided them; the loop then follows those decisions
    (the trajectory at those step sizes, those best-iterate updates) while the
    trace still records its own (trace entries 'alpha_free', 'take_free' and the
    iteration's decision margins 'ls_margin', 'best_margin').
    """
    B, n = x_init.shape
    d = C.shape[-1]
    m = d - n
    dt = x_init.dtype
    if isinstance(model, tuple):
        dyn = model
    else:
        def dyn(xx, uu):
            return model.forward(xx, uu, params)
    u = np.zeros((T, B, m), dt) if u_init is None else np.array(u_init, dtype=dt)
    if u.ndim == 2:
        u = np.repeat(u[:, None], B, 1)
    best = None
    n_not_improved = 0
    n_iters = 0
    for i in range(lqr_iter):                                     # mpc_explicit.py:246
        fa, ft = force(i) if force is not None else (None, None)
        it_m = {} if (margins is not None or trace is not None) else None
        x = lqr.get_traj(T, u, x_init, dyn)
        if isinstance(model, tuple):
            F, f = model[1], model[2]
        else:
            F, f = linearize(model, x, u, params)
        cb = lqr.c_back(C, c, x, u)
        K, k, nqp = lqr.lqr_backward(C, cb, F, n, m, u=u, u_lower=u_lower, u_upper=u_upper,
                                     m_solver=m_solver, per_problem=per_problem, margins=it_m)
        x, u, costs, full_du_norm, _, mean_alpha, alphas = lqr.lqr_forward(
            x_init, C, c, x, u, K, k, dyn, u_lower=u_lower, u_upper=u_upper,
            linesearch_decay=linesearch_decay, max_linesearch_iter=max_linesearch_iter, margins=it_m,
            force_alpha=fa)
        n_iters += 1
        n_not_improved += 1
        take_free = np.ones(B, bool)
        if best is None:                                          # mpc_explicit.py:269-283
            best = dict(x=x.copy(), u=u.copy(), costs=costs.copy(), du=full_du_norm.copy())
        else:
            take_free = costs <= best["costs"] + best_cost_eps
            if it_m is not None:
                lqr._note(it_m, "best", np.abs(costs - (best["costs"] + best_cost_eps))
                          / np.maximum(1.0, np.abs(best["costs"])))
            take = take_free if ft is None else np.asarray(ft, bool)
            for j in range(B):
                if take[j]:
                    n_not_improved = 0
                    best["x"][:, j] = x[:, j]
                    best["u"][:, j] = u[:, j]
                    best["costs"][j] = costs[j]
                    best["du"][j] = full_du_norm[j]
        if it_m is not None and margins is not None:
            for k_, v in it_m.items():
                lqr._note(margins, k_, v)
        if trace is not None:
            inf = np.full(B, np.inf)
            trace.append(dict(x=x.copy(), u=u.copy(), costs=costs.copy(), du=full_du_norm.copy(),
                              mean_alpha=mean_alpha, nqp=nqp, alpha_free=alphas.copy(), take_free=take_free,
                              ls_margin=it_m.get("linesearch", inf), best_margin=it_m.get("best", inf),
                              pnqp_margin=it_m.get("pnqp", inf), clamp_margin=it_m.get("clamp", inf)))
        if margins is not None and eps > 0:                       # batch-wide: every problem
            lqr._note(margins, "stop", np.full(B, abs(max(full_du_norm) - eps) / eps))
        if max(full_du_norm) < eps or n_not_improved > not_improved_lim:   # mpc_explicit.py:297-299
            break
    if margins is not None:
        margins["min"] = np.min(np.stack([v for k_, v in margins.items() if k_ != "min"] or [np.full(B, np.inf)]), 0)
    info = dict(n_iters=n_iters, full_du_norm=best["du"],
                converged=bool(max(best["du"]) <= eps))
    return best["x"], best["u"], best["costs"], info


def expand_cost(C, c, T, B):
    """mpc_explicit.py:203-224 broadcasting of QuadCost([d,d]|[T,d,d]|[T,B,d,d], ...)."""
    C = np.asarray(C)
    c = np.asarray(c)
    if C.ndim == 2:
        C = np.broadcast_to(C, (T, B) + C.shape)
    elif C.ndim == 3:
        C = np.broadcast_to(C[:, None], (T, B) + C.shape[1:])
    if c.ndim == 1:
        c = np.broadcast_to(c, (T, B) + c.shape)
    elif c.ndim == 2:
        c = np.broadcast_to(c[:, None], (T, B) + c.shape[1:])
    return np.ascontiguousarray(C), np.ascontiguousarray(c)
