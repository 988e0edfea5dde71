"""Oracle backward passes (numpy).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

  classic_backward   lqr_step.py:312-407 (LQRStepFn.backward of mpc.pytorch):
                     one adjoint LQR solve + costate recursions.
  kkt_gradient       lqr_step_explicit.py:276-355 on an arbitrary RHS batch,
                     with the adjoint engine of lqr_step_backup.py/mpc_backup.py.
  implicit_backward  lqr_step_explicit.py:653-712 + fix_point_equ 458-598:
                     the DiLQR implicit differentiation through the iLQR fixed
                     point, restated literally (unit-RHS expansion, dense A).
"""
import numpy as np

from . import lqr


def adjoint_lqr_solve(C, r, F, n, m, I=None, engine="backup", back_eps=1e-7):
    """The nested MPC(lqr_iter=1, u_zero_I=I)(0, QuadCost(C,-r), LinDx(F,None))
    solve (lqr_step.py:328-340, lqr_step_explicit.py:277-289).

    x_init = 0, u = 0, so x = 0, c_back = -r; one Riccati sweep and one rollout
    with the default line search (decay 0.2, 10 passes) of that MPC.
    engine='classic' -> lqr_step.py (pinverse for m>1); 'backup' ->
    lqr_step_backup.py (cholesky + 1e-6 I for m>1).
    """
    T, B, d = r.shape
    dt = C.dtype
    x0 = np.zeros((B, n), dt)
    x = np.zeros((T, B, n), dt)
    u = np.zeros((T, B, m), dt)
    cb = -r
    K, k, _ = lqr.lqr_backward(C, cb, F, n, m, u=u, u_zero_I=I,
                               m_solver="pinv" if engine == "classic" else "chol")
    dxs, dus, *_ = lqr.lqr_forward(x0, C, -r, x, u, K, k, ("lin", F, None), u_zero_I=I,
                                   linesearch_decay=0.2, max_linesearch_iter=10)
    return dxs, dus


def _active_set(new_u, u_lower, u_upper):
    if u_lower is None:
        return None
    return (np.abs(new_u - u_lower) <= 1e-8) | (np.abs(new_u - u_upper) <= 1e-8)


def kkt_gradient(r, C, c, F, f, new_x, new_u, I, n, m, engine="backup"):
    """lqr_step_explicit.py:276-355 (also lqr_step.py:328-405).
    Returns dx_init, dC, dc, dF, df."""
    T = C.shape[0]
    dx, du = adjoint_lqr_solve(C, r, F, n, m, I=I, engine=engine)
    dxu = np.concatenate([dx, du], 2)
    xu = np.concatenate([new_x, new_u], 2)
    dC = -0.5 * (dxu[..., :, None] * xu[..., None, :] + xu[..., :, None] * dxu[..., None, :])
    dc = -dxu
    lams = [None] * T
    prev = None
    for t in range(T - 1, -1, -1):
        lam = lqr.bmv(C[t, :, :n, :n], new_x[t]) + lqr.bmv(C[t, :, :n, n:], new_u[t]) + c[t, :, :n]
        if prev is not None:
            lam = lam + lqr.bmv(np.swapaxes(F[t, :, :, :n], 1, 2), prev)
        lams[t] = prev = lam
    dlams = [None] * T
    prev = None
    for t in range(T - 1, -1, -1):
        dlam = lqr.bmv(C[t, :, :n, :n], dx[t]) + lqr.bmv(C[t, :, :n, n:], du[t]) - r[t, :, :n]
        if prev is not None:
            dlam = dlam + lqr.bmv(np.swapaxes(F[t, :, :, :n], 1, 2), prev)
        dlams[t] = prev = dlam
    dlams = np.stack(dlams)
    dF = np.zeros_like(F)
    for t in range(T - 1):
        dF[t] = -(dlams[t + 1][:, :, None] * xu[t][:, None, :] + lams[t + 1][:, :, None] * dxu[t][:, None, :])
    df = -dlams[1:] if (f is not None and f.size > 0) else None
    return -dlams[0], dC, dc, dF, df


def classic_backward(dl_dx, dl_du, x_init, C, c, F, f, new_x, new_u, u_lower=None, u_upper=None):
    """lqr_step.py:312-407.  Returns (dx_init, dC, dc, dF, df)."""
    n, m = new_x.shape[2], new_u.shape[2]
    r = np.concatenate([dl_dx, dl_du], 2)
    I = _active_set(new_u, u_lower, u_upper)
    return kkt_gradient(r, C, c, F, f, new_x, new_u, I, n, m, engine="classic")


def implicit_backward(model, dl_dx, dl_du, C, c, F, f, new_x, new_u, K_rev, u_lower=None,
                      u_upper=None, params=None):
    """lqr_step_explicit.py:653-712 (+ fix_point_equ 458-598).

    K_rev: the gains of the no-op forward's Riccati sweep STACKED IN THE ORDER
    THE REFERENCE STACKS THEM (reverse time, lqr_step_explicit.py:617-618), and
    consumed by grad_input as K[t] (cartpole.py:761) - a reference quirk kept.
    Returns (dC [T,B,d,d], dc [T,B,d], dtheta [B,p]).
    """
    T, B, n = dl_dx.shape
    m = dl_du.shape[2]
    d = n + m
    dt = C.dtype
    p = model.n_params
    TD = T * d
    NB = B * TD
    # unit right-hand sides (lqr_step_explicit.py:665-671)
    r_new = np.zeros((T, NB, d), dt)
    for b in range(B):
        for t in range(T):
            for k in range(d):
                r_new[t, b * TD + t * d + k, k] = 1
    rep = lambda a: np.repeat(a, TD, axis=1)                     # noqa: E731 (repeat_interleave)
    C_n, c_n, F_n, f_n = rep(C), rep(c), rep(F), rep(f)
    x_n, u_n = rep(new_x), rep(new_u)
    I_n = _active_set(u_n, u_lower, u_upper)
    _, dtau_dC, dtau_dc, dtau_dF, dtau_df = kkt_gradient(r_new, C_n, c_n, F_n, f_n, x_n, u_n, I_n,
                                                         n, m, engine="backup")
    gD, gd, Dx, Du, D, d_x, d_u = model.grad_input(new_x, new_u, K_rev, params)
    return fix_point_equ(dl_dx, dl_du, (dtau_dC, dtau_dc, dtau_dF, dtau_df, gD, gd, Dx, Du, D, d_x, d_u), p)


def fix_point_equ(dl_dx, dl_du, mats, p):
    """lqr_step_explicit.py:458-598."""
    T, B, n = dl_dx.shape
    m = dl_du.shape[2]
    d = n + m
    dt = dl_dx.dtype
    dtau_dC, dtau_dc, dtau_dF, dtau_df, gD, gd, Dx, Du, D, d_x, d_u = mats
    tD = dtau_dF.reshape(T - 1, B, T, d, n, d).transpose(1, 2, 3, 0, 4, 5)
    X_D = tD[:, :, :n].reshape(B, T * n, T - 1, n, d)
    U_D = tD[:, :, n:].reshape(B, T * m, T - 1, n, d)
    td = dtau_df.reshape(T - 1, B, T, d, n).transpose(1, 2, 3, 0, 4)
    X_d = td[:, :, :n].reshape(B, T * n, T - 1, n)
    U_d = td[:, :, n:].reshape(B, T * m, T - 1, n)
    tC = dtau_dC.reshape(T, B, T, d, d, d).transpose(1, 2, 3, 0, 4, 5)
    X_C = tC[:, :, :n].reshape(B, T * n, T * d * d)
    U_C = tC[:, :, n:].reshape(B, T * m, T * d * d)
    tc = dtau_dc.reshape(T, B, T, d, d).transpose(1, 2, 3, 0, 4)
    X_c = tc[:, :, :n].reshape(B, T * n, T * d)
    U_c = tc[:, :, n:].reshape(B, T * m, T * d)
    Dx, Du = Dx.transpose(1, 0, 2, 3, 4), Du.transpose(1, 0, 2, 3, 4)
    d_x, d_u = d_x.transpose(1, 0, 2, 3), d_u.transpose(1, 0, 2, 3)
    gD, gd = gD.transpose(1, 0, 2, 3, 4), gd.transpose(1, 0, 2, 3)

    def pad(a, k):                                   # the zero block for t = T-1 (515-523)
        return np.concatenate([a, np.zeros(a.shape[:2] + (1, k), dt)], 2)

    e5 = lambda a, b: np.einsum("bptnm,btnmk->bptk", a, b)      # noqa: E731
    e4 = lambda a, b: np.einsum("bptn,btnk->bptk", a, b)        # noqa: E731
    X_X = (pad(e5(X_D, Dx), n) + pad(e4(X_d, d_x), n)).reshape(B, T * n, T * n)
    U_U = (pad(e5(U_D, Du), m) + pad(e4(U_d, d_u), m)).reshape(B, T * m, T * m)
    X_U = (pad(e5(X_D, Du), m) + pad(e4(X_d, d_u), m)).reshape(B, T * n, T * m)
    U_X = (pad(e5(U_D, Dx), n) + pad(e4(U_d, d_x), n)).reshape(B, T * m, T * n)
    F_th = np.einsum("bptnm,btnmk->bpk", X_D, gD) + np.einsum("bptn,btnk->bpk", X_d, gd)
    G_th = np.einsum("bptnm,btnmk->bpk", U_D, gD) + np.einsum("bptn,btnk->bpk", U_d, gd)
    A = np.zeros((B, T * d, T * d), dt)
    A[:, :T * n, :T * n] = np.eye(T * n, dtype=dt) - X_X
    A[:, :T * n, T * n:] = -X_U
    A[:, T * n:, :T * n] = -U_X
    A[:, T * n:, T * n:] = np.eye(T * m, dtype=dt) - U_U
    sol_th = np.linalg.solve(A, np.concatenate([F_th, G_th], 1))
    rhs_C = np.concatenate([X_C, U_C], 1)
    rhs_c = np.concatenate([X_c, U_c], 1)
    sol_C = np.stack([np.linalg.lstsq(A[b], rhs_C[b], rcond=None)[0] for b in range(B)])
    sol_c = np.stack([np.linalg.lstsq(A[b], rhs_c[b], rcond=None)[0] for b in range(B)])
    g = np.concatenate([dl_dx.transpose(1, 0, 2).reshape(B, T * n), dl_du.transpose(1, 0, 2).reshape(B, T * m)], 1)
    dtheta = np.einsum("bi,bij->bj", g, sol_th)
    dC = np.einsum("bi,bij->bj", g, sol_C).reshape(B, T, d, d).transpose(1, 0, 2, 3)
    dc = np.einsum("bi,bij->bj", g, sol_c).reshape(B, T, d).transpose(1, 0, 2)
    return dC, dc, dtheta


def implicit_backward_fast(model, dl_dx, dl_du, C, c, F, f, new_x, new_u, K_rev, u_lower=None,
                           u_upper=None, params=None):
    """The same result as implicit_backward, by the algebra the HIP kernel uses.

    The reference solves A^T w = g (A = I - J, (T d)^2) after forming J from T*d
    unit-RHS adjoint solves.  Two identities collapse that:
      (1) J[p,(t,k)] = -sum_j dtau_t(e_p)[j] M_t[j,k] with
          M_t[j,k] = sum_i lam_{t+1}[i] dD_t[i,j]/dtau_k — the dlam terms of
          X_D_X and X_d_X cancel (d_grad_X = -D_grad_x . tau), so J = -P M with
          P the adjoint-LQR solution operator (dtau(r) = P r) and M = blkdiag(M_t);
      (2) w = g - M^T y with y = P w  <=>  y solves the LQR with cost matrices
          C_t + M_t^T and linear term -g (same dynamics F, same active set).
    Then dC, dc, dtheta are the KKT gradients of the adjoint solve with r = w, whose
    trajectory is y itself.  Cost: O(T d^3) per problem instead of O((T d)^3).
    """
    T, B, n = dl_dx.shape
    m = dl_du.shape[2]
    d = n + m
    dt = C.dtype
    p = model.n_params
    g = np.concatenate([dl_dx, dl_du], 2)
    I = _active_set(new_u, u_lower, u_upper)
    gD, gd, Dx, Du, D, d_x, d_u = model.grad_input(new_x, new_u, K_rev, params)
    # primal costates (lqr_step_explicit.py:305-319)
    lams = [None] * T
    prev = None
    for t in range(T - 1, -1, -1):
        lam = lqr.bmv(C[t, :, :n, :n], new_x[t]) + lqr.bmv(C[t, :, :n, n:], new_u[t]) + c[t, :, :n]
        if prev is not None:
            lam = lam + lqr.bmv(np.swapaxes(F[t, :, :, :n], 1, 2), prev)
        lams[t] = prev = lam
    # M_t = sum_i lam_{t+1}[i] dD_t[i,:,:]/dtau
    M = np.zeros((T, B, d, d), dt)
    Dtau = np.concatenate([Dx, Du], -1)                       # [T-1,B,n,d,d]
    for t in range(T - 1):
        M[t] = np.einsum("bi,bijk->bjk", lams[t + 1], Dtau[t])
    Cp = C + np.swapaxes(M, 2, 3)
    y = adjoint_lqr_linear(Cp, g, F, n, m, I)
    w = g - np.einsum("tbjk,tbj->tbk", M, y)
    # KKT gradient of the adjoint solve with r = w (trajectory y)
    xu = np.concatenate([new_x, new_u], 2)
    dC = -0.5 * (y[..., :, None] * xu[..., None, :] + xu[..., :, None] * y[..., None, :])
    dc = -y
    dlam = [None] * T
    prev = None
    for t in range(T - 1, -1, -1):
        dl = lqr.bmv(C[t, :, :n, :n], y[t, :, :n]) + lqr.bmv(C[t, :, :n, n:], y[t, :, n:]) - w[t, :, :n]
        if prev is not None:
            dl = dl + lqr.bmv(np.swapaxes(F[t, :, :, :n], 1, 2), prev)
        dlam[t] = prev = dl
    dtheta = np.zeros((B, p), dt)
    for t in range(T - 1):
        dF = -(dlam[t + 1][:, :, None] * xu[t][:, None, :] + lams[t + 1][:, :, None] * y[t][:, None, :])
        df = -dlam[t + 1]
        dtheta += np.einsum("bnm,bnmk->bk", dF, gD[t]) + np.einsum("bn,bnk->bk", df, gd[t])
    return dC, dc, dtheta


def adjoint_lqr_linear(C, g, F, n, m, I=None):
    """tau = argmin of 1/2 tau^T C tau - g^T tau s.t. x_0 = 0, x_{t+1} = F_t tau_t
    (controls in the active set I fixed to 0), by the Riccati elimination — valid
    for a non-symmetric C (it eliminates the linear KKT system).  No line search."""
    T, B, d = g.shape
    dt = C.dtype
    K, k, _ = lqr.lqr_backward(C, -g, F, n, m, u_zero_I=I, m_solver="lu")
    x = np.zeros((B, n), dt)
    out = np.zeros((T, B, d), dt)
    for t in range(T):
        u = lqr.bmv(K[t], x) + k[t]
        if I is not None:
            u[I[t]] = 0.
        out[t, :, :n], out[t, :, n:] = x, u
        if t < T - 1:
            x = lqr.bmv(F[t], np.concatenate([x, u], 1))
    return out
