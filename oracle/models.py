"""Oracle dynamics models (numpy), restating env_dx/{pendulum,cartpole,rocket}.py.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

`forward` restates each model's forward() op by op.  The derivative tensors
(get_linear_dyn, get_matrices) are derived symbolically with sympy from the
same equations WITHOUT the control clamp, which is what the reference's
closed-form expressions are (the analytic Jacobians ignore
the clamp).  The derivations are pinned against the reference's own outputs in
tests/test_oracle_golden.py.
"""
import functools

import numpy as np
import sympy as sp


class _Model:
    name = None
    n_state = n_ctrl = n_params = None
    default_params = None
    lower = upper = None
    linesearch_decay = max_linesearch_iter = mpc_eps = None

    # ---- symbolic core --------------------------------------------------
    @classmethod
    def _sym_next_state(cls, xs, us, ps):
        raise NotImplementedError

    @classmethod
    @functools.lru_cache(maxsize=None)
    def _lambdas(cls):
        n, m, p = cls.n_state, cls.n_ctrl, cls.n_params
        xs = sp.symbols(f"x0:{n}", real=True)
        us = sp.symbols(f"u0:{m}", real=True)
        ps = sp.symbols(f"p0:{p}", real=True)
        f = sp.Matrix(cls._sym_next_state(xs, us, ps))
        tau = list(xs) + list(us)
        D = f.jacobian(tau)                                   # [n, d]
        args = list(xs) + list(us) + list(ps)

        def lam(expr_list):
            return sp.lambdify(args, expr_list, modules="numpy", cse=True)

        d = n + m
        D_flat = [D[i, j] for i in range(n) for j in range(d)]
        Dx = [sp.diff(D[i, j], xs[k]) for i in range(n) for j in range(d) for k in range(n)]
        Du = [sp.diff(D[i, j], us[k]) for i in range(n) for j in range(d) for k in range(m)]
        Dp = [sp.diff(D[i, j], ps[k]) for i in range(n) for j in range(d) for k in range(p)]
        fp = [sp.diff(f[i], ps[k]) for i in range(n) for k in range(p)]
        return dict(D=lam(D_flat), Dx=lam(Dx), Du=lam(Du), Dp=lam(Dp), fp=lam(fp))

    @classmethod
    def _eval(cls, key, x, u, params, shape):
        params = cls.default_params if params is None else params
        fn = cls._lambdas()[key]
        N = x.shape[0]
        dt = x.dtype
        args = [x[:, i] for i in range(cls.n_state)] + [u[:, i] for i in range(cls.n_ctrl)] + \
               [dt.type(params[i]) for i in range(cls.n_params)]
        vals = fn(*args)
        out = np.empty((N, len(vals)), dtype=dt)
        for j, v in enumerate(vals):
            out[:, j] = np.broadcast_to(np.asarray(v, dtype=dt), (N,))
        return out.reshape((N,) + shape)

    # ---- public API (mirrors the reference model protocol) ---------------
    @classmethod
    def get_linear_dyn(cls, x, u, params=None):
        """Analytic Jacobian d x_{t+1} / d [x_t, u_t] at the UNCLAMPED u."""
        return cls._eval("D", x, u, params, (cls.n_state, cls.n_state + cls.n_ctrl))

    @classmethod
    def get_matrices(cls, x, u, params=None):
        """(D, D_params, D_x, D_u, x_theta, x_xtm1, x_utm1), the tuple of e.g.
        cartpole.py:105-716 get_matrices."""
        n, m, p = cls.n_state, cls.n_ctrl, cls.n_params
        d = n + m
        D = cls._eval("D", x, u, params, (n, d))
        Dp = cls._eval("Dp", x, u, params, (n, d, p))
        Dx = cls._eval("Dx", x, u, params, (n, d, n))
        Du = cls._eval("Du", x, u, params, (n, d, m))
        fp = cls._eval("fp", x, u, params, (n, p))
        return D, Dp, Dx, Du, fp, D[:, :, :n].copy(), D[:, :, n:].copy()

    @classmethod
    def grad_input(cls, X, U, K, params=None):
        """Closed-loop total derivatives, restating cartpole.py:717-788 (the same
        code sits in pendulum.py:383-443 and rocket.py:263-323).

        X [T,B,n], U [T,B,m], K [T,B,m,n] consumed as K[t] (the caller passes
        the Riccati gains in the order the reference stacks them).
        Returns (grad_D [T-1,B,n,d,p], grad_d [T-1,B,n,p], D_x [T-1,B,n,d,n],
                 D_u [T-1,B,n,d,m], D [T-1,B,n,d], d_x [T-1,B,n,n], d_u [T-1,B,n,m]).
        """
        T, B, n = X.shape
        m = U.shape[2]
        p = cls.n_params
        d = n + m
        dt = X.dtype
        D, Dp, Dx, Du, x_th, x_x, x_u = cls.get_matrices(X.reshape(T * B, n), U.reshape(T * B, m), params)
        D, Dp, Dx, Du = (a.reshape((T, B) + a.shape[1:]) for a in (D, Dp, Dx, Du))
        x_th, x_x, x_u = (a.reshape((T, B) + a.shape[1:]) for a in (x_th, x_x, x_u))
        XU = np.concatenate([X, U], -1)
        d_X = np.einsum("tbnmk,tbm->tbnk", -Dx, XU)           # cartpole.py:752
        d_U = np.einsum("tbnmk,tbm->tbnk", -Du, XU)           # cartpole.py:753
        gradx = np.zeros((B, n, p), dt)
        grad_D, grad_d = [], []
        Ktm1 = None
        for t in range(T):                                    # cartpole.py:755-782
            Kt = K[t]
            if t > 0:
                gradxtm1 = gradx
                gradx = x_th[t] + (x_x[t] + x_u[t] @ Ktm1) @ gradx
            if t < T - 1:
                # D_grad_params[t] + (D_x[t] + D_u[t] @ K_t) @ gradx, per row n
                DxK = Dx[t] + Du[t] @ Kt[:, None]             # [B,n,d,n]
                gD = Dp[t] + DxK @ gradx[:, None]             # [B,n,d,p]
                grad_D.append(gD)
            if t > 0:
                xu_par = np.concatenate([gradxtm1, Ktm1 @ gradxtm1], 1)   # [B,d,p]
                xu_tm1 = XU[t - 1]
                gd = gradx - np.einsum("bnmk,bm->bnk", grad_D[t - 1], xu_tm1) - D[t - 1] @ xu_par
                grad_d.append(gd)
            Ktm1 = Kt
        return (np.stack(grad_D), np.stack(grad_d), Dx[:T - 1], Du[:T - 1], D[:T - 1],
                d_X[:T - 1], d_U[:T - 1])

    @classmethod
    def true_obj(cls):
        raise NotImplementedError


class Pendulum(_Model):
    """env_dx/pendulum.py (simple variant), n=3 [cos th, sin th, dth], m=1."""
    name = "pendulum"
    n_state, n_ctrl, n_params = 3, 1, 3
    default_params = (10.0, 1.0, 1.0)           # g, m, l  (pendulum.py:42)
    dt = 0.05
    max_torque = 2.0
    lower, upper = -2.0, 2.0
    mpc_eps, linesearch_decay, max_linesearch_iter = 1e-3, 0.2, 5      # pendulum.py:56-58

    @classmethod
    def forward(cls, x, u, params=None):
        """pendulum.py:60-95."""
        g, m, l = (x.dtype.type(v) for v in (params if params is not None else cls.default_params))
        dt = x.dtype.type(cls.dt)
        uu = np.clip(u, -cls.max_torque, cls.max_torque)[:, 0]
        c, s, dth = x[:, 0], x[:, 1], x[:, 2]
        th = np.arctan2(s, c)
        newdth = dth + dt * (-3. * g / (2. * l) * (-s) + 3. * uu / (m * l ** 2))
        newth = th + newdth * dt
        return np.stack([np.cos(newth), np.sin(newth), newdth], 1)

    @classmethod
    def _sym_next_state(cls, xs, us, ps):
        c, s, dth = xs
        (u,) = us
        g, m, l = ps
        th = sp.atan2(s, c)
        newdth = dth + sp.Float(cls.dt) * (-3 * g / (2 * l) * (-s) + 3 * u / (m * l ** 2))
        newth = th + newdth * sp.Float(cls.dt)
        return [sp.cos(newth), sp.sin(newth), newdth]

    @classmethod
    def true_obj(cls):
        """pendulum.py:117-125."""
        goal_state = np.array([1., 0., 0.])
        goal_weights = np.array([1., 1., 0.1])
        q = np.concatenate([goal_weights, [0.001]])
        p = np.concatenate([-np.sqrt(goal_weights) * goal_state, [0.]])
        return q, p


class PendulumComplex(_Model):
    """env_dx/pendulum.py with simple=False (pendulum.py:30-49, 76-95): theta =
    (g, m, l, d, b), damping d*th and a gravity bias inside sin(th + b).  The
    reference has no closed-form Jacobian for it (get_linear_dyn unpacks three
    parameters, pendulum.py:448); its runnable linearisation is AUTO_DIFF
    (mpc_explicit.py:562-566), i.e. autograd through forward(): the clamp's gate
    on u included.  get_linear_dyn here is that derivative."""
    name = "pendulum_complex"
    n_state, n_ctrl, n_params = 3, 1, 5
    default_params = (10.0, 1.0, 1.0, 1.0, 0.1)     # il_env.py:41
    dt = 0.05
    max_torque = 2.0
    lower, upper = -2.0, 2.0
    mpc_eps, linesearch_decay, max_linesearch_iter = 1e-3, 0.2, 5

    @classmethod
    def forward(cls, x, u, params=None):
        """pendulum.py:76-95 (simple=False branch)."""
        g, m, l, d, b = (x.dtype.type(v) for v in (params if params is not None else cls.default_params))
        dt = x.dtype.type(cls.dt)
        uu = np.clip(u, -cls.max_torque, cls.max_torque)[:, 0]
        c, s, dth = x[:, 0], x[:, 1], x[:, 2]
        th = np.arctan2(s, c)
        newdth = dth + dt * (-3. * g / (2. * l) * (-np.sin(th + b)) + 3. * uu / (m * l ** 2) - d * th)
        newth = th + newdth * dt
        return np.stack([np.cos(newth), np.sin(newth), newdth], 1)

    @classmethod
    def _sym_next_state(cls, xs, us, ps):
        c, s, dth = xs
        (u,) = us
        g, m, l, d, b = ps
        th = sp.atan2(s, c)
        newdth = dth + sp.Float(cls.dt) * (3 * g / (2 * l) * sp.sin(th + b) + 3 * u / (m * l ** 2) - d * th)
        newth = th + newdth * sp.Float(cls.dt)
        return [sp.cos(newth), sp.sin(newth), newdth]

    @classmethod
    def get_linear_dyn(cls, x, u, params=None):
        """Autograd's Jacobian of forward(): the symbolic one at the clamped u,
        its u column gated by lo <= u <= hi (torch.clamp's backward)."""
        uc = np.clip(u, cls.lower, cls.upper)
        D = cls._eval("D", x, uc, params, (cls.n_state, cls.n_state + cls.n_ctrl))
        gate = ((u >= cls.lower) & (u <= cls.upper)).astype(x.dtype)          # [N, m]
        D[:, :, cls.n_state:] *= gate[:, None, :]
        return D

    @classmethod
    def get_matrices(cls, x, u, params=None):
        raise NotImplementedError("the reference's get_matrices has no 5-parameter form (pendulum.py:157)")

    @classmethod
    def true_obj(cls):
        return Pendulum.true_obj()


class Cartpole(_Model):
    """env_dx/cartpole.py, n=5 [x, dx, cos th, sin th, dth], m=1."""
    name = "cartpole"
    n_state, n_ctrl, n_params = 5, 1, 4
    default_params = (9.8, 1.0, 0.1, 0.5)      # g, m_cart, m_pole, l  (cartpole.py:39)
    dt = 0.05
    force_mag = 100.0
    lower, upper = -100.0, 100.0
    mpc_eps, linesearch_decay, max_linesearch_iter = 1e-4, 0.5, 2      # cartpole.py:60-62

    @classmethod
    def forward(cls, state, u, params=None):
        """cartpole.py:64-97."""
        g, mc, mp, l = (state.dtype.type(v) for v in (params if params is not None else cls.default_params))
        dt = state.dtype.type(cls.dt)
        total_mass = mp + mc
        pml = mp * l
        uu = np.clip(u[:, 0], -cls.force_mag, cls.force_mag)
        x, dx, c, s, dth = (state[:, i] for i in range(5))
        th = np.arctan2(s, c)
        cart_in = (uu + pml * dth ** 2 * s) / total_mass
        th_acc = (g * s - c * cart_in) / (l * (4. / 3. - mp * c ** 2 / total_mass))
        xacc = cart_in - pml * th_acc * c / total_mass
        x = x + dt * dx
        dx = dx + dt * xacc
        th = th + dt * dth
        dth = dth + dt * th_acc
        return np.stack([x, dx, np.cos(th), np.sin(th), dth], 1)

    @classmethod
    def _sym_next_state(cls, xs, us, ps):
        x, dx, c, s, dth = xs
        (u,) = us
        g, mc, mp, l = ps
        dt = sp.Float(cls.dt)
        total = mp + mc
        pml = mp * l
        th = sp.atan2(s, c)
        cart_in = (u + pml * dth ** 2 * s) / total
        th_acc = (g * s - c * cart_in) / (l * (sp.Rational(4, 3) - mp * c ** 2 / total))
        xacc = cart_in - pml * th_acc * c / total
        th2 = th + dt * dth
        return [x + dt * dx, dx + dt * xacc, sp.cos(th2), sp.sin(th2), dth + dt * th_acc]

    @classmethod
    def get_matrices(cls, x, u, params=None):
        """cartpole.py:105-716.  The sympy derivatives agree with the reference's
        hand-derived closed forms everywhere except five entries, which are
        restated here exactly as the reference writes them:
          * x_grad_xtm1[0,0] = 0 (cartpole.py:666: first row starts with a zero,
            where d x_{t+1} / d x_t is 1);
          * D_grad_params[4,3,1] (matrix_2_part_2, row 4, col 3: d/d m_c) and
            D_grad_params[4,3..5,2] (matrix_2_part_3, row 4, cols 3-5: d/d m_p),
            whose closed forms differ from the derivative of D[4,:].
        """
        D, Dp, Dx, Du, fp, x_x, x_u = super().get_matrices(x, u, params)
        g, m_c, m_p, l = (x.dtype.type(v) for v in (params if params is not None else cls.default_params))
        dt = x.dtype.type(cls.dt)
        c, s, dth = x[:, 2], x[:, 3], x[:, 4]
        M = m_c + m_p
        den = -c ** 2 * m_p / M + 4 / 3
        Dp[:, 4, 3, 1] = dt * (-c ** 2 * m_p * (-c * dth ** 2 * l * m_p / M + g) / (l * M ** 2 * den ** 2)
                               + c * dt * dth ** 2 * m_p / (M ** 2 * den))
        Dp[:, 4, 3, 2] = dt * (-c ** 2 * m_p * (-c * dth ** 2 * l * m_p / M + g) / (l * den ** 2)
                               + c * dt * dth ** 2 * l * m_p / M ** 2)
        Dp[:, 4, 4, 2] = (-2 * c * dt * dth * m_p * s * (-c ** 2 * m_p / M ** 2 + c ** 2 / M) / (M * den ** 2)
                          + 2 * c * dt * dth * m_p * s / (M ** 2 * den))
        Dp[:, 4, 5, 2] = c * dt / (l * M ** 2 * den)
        x_x[:, 0, 0] = 0
        return D, Dp, Dx, Du, fp, x_x, x_u

    @classmethod
    def true_obj(cls):
        """cartpole.py:859-867."""
        goal_state = np.array([0., 0., 1., 0., 0.])
        goal_weights = np.array([0.1, 0.1, 1., 1., 0.1])
        q = np.concatenate([goal_weights, [0.001]])
        p = np.concatenate([-np.sqrt(goal_weights) * goal_state, [0.]])
        return q, p


class Rocket(_Model):
    """env_dx/rocket.py, n=13 [r(3), v(3), q(4), w(3)], m=3, theta=(Jx,Jy,Jz,mass,l)."""
    name = "rocket"
    n_state, n_ctrl, n_params = 13, 3, 5
    default_params = (0.5, 1.0, 1.0, 1.0, 1.0)     # rocket.py:29
    dt = 0.1
    max_thrust = 400.0
    lower, upper = -20.0, 20.0
    mpc_eps, linesearch_decay, max_linesearch_iter = 1e-3, 0.2, 5      # rocket.py:68-70

    @classmethod
    def forward(cls, x, u, params=None):
        """rocket.py:82-164.  Returns the UNNORMALISED quaternion (the reference
        computes new_x_out with a normalised q but returns new_x, 159-164)."""
        Jx, Jy, Jz, mass, l = (x.dtype.type(v) for v in (params if params is not None else cls.default_params))
        dt = x.dtype.type(cls.dt)
        v, q, w = x[:, 3:6], x[:, 6:10], x[:, 10:13]
        T_B = np.clip(u, -cls.max_thrust, cls.max_thrust)
        q0, q1, q2, q3 = (q[:, i] for i in range(4))
        C_B_I = np.stack([
            np.stack([1 - 2 * (q2 ** 2 + q3 ** 2), 2 * (q1 * q2 + q0 * q3), 2 * (q1 * q3 - q0 * q2)], -1),
            np.stack([2 * (q1 * q2 - q0 * q3), 1 - 2 * (q1 ** 2 + q3 ** 2), 2 * (q2 * q3 + q0 * q1)], -1),
            np.stack([2 * (q1 * q3 + q0 * q2), 2 * (q2 * q3 - q0 * q1), 1 - 2 * (q1 ** 2 + q2 ** 2)], -1)],
            1)
        C_I_B = np.swapaxes(C_B_I, 1, 2)
        g = np.array([-10., 0., 0.], dtype=x.dtype)
        thrust = (C_I_B @ T_B[:, :, None])[:, :, 0]
        dv = thrust / mass + g
        wx, wy, wz = w[:, 0], w[:, 1], w[:, 2]
        dq = 0.5 * np.stack([-wx * q1 - wy * q2 - wz * q3,
                             wx * q0 + wz * q2 - wy * q3,
                             wy * q0 - wz * q1 + wx * q3,
                             wz * q0 + wy * q1 - wx * q2], 1)
        torque = np.stack([np.zeros_like(wx), (l / 2) * T_B[:, 2], -(l / 2) * T_B[:, 1]], 1)
        J = np.array([Jx, Jy, Jz], dtype=x.dtype)
        Jw = w * J
        wxJw = np.cross(w, Jw)
        dw = (torque - wxJw) / J
        deriv = np.concatenate([v, dv, dq, dw], 1)
        return x + deriv * dt

    @classmethod
    def _sym_next_state(cls, xs, us, ps):
        r0, r1, r2, v0, v1, v2, q0, q1, q2, q3, wx, wy, wz = xs
        ux, uy, uz = us
        Jx, Jy, Jz, mass, l = ps
        dt = sp.Float(cls.dt)
        CBI = sp.Matrix([[1 - 2 * (q2 ** 2 + q3 ** 2), 2 * (q1 * q2 + q0 * q3), 2 * (q1 * q3 - q0 * q2)],
                         [2 * (q1 * q2 - q0 * q3), 1 - 2 * (q1 ** 2 + q3 ** 2), 2 * (q2 * q3 + q0 * q1)],
                         [2 * (q1 * q3 + q0 * q2), 2 * (q2 * q3 - q0 * q1), 1 - 2 * (q1 ** 2 + q2 ** 2)]])
        Tb = sp.Matrix([ux, uy, uz])
        dv = CBI.T * Tb / mass + sp.Matrix([-10, 0, 0])
        w = sp.Matrix([wx, wy, wz])
        q = sp.Matrix([q0, q1, q2, q3])
        Om = sp.Matrix([[0, -wx, -wy, -wz], [wx, 0, wz, -wy], [wy, -wz, 0, wx], [wz, wy, -wx, 0]])
        dq = Om * q / 2
        torque = sp.Matrix([0, l / 2 * uz, -l / 2 * uy])
        J = sp.diag(Jx, Jy, Jz)
        dw = J.inv() * (torque - w.cross(J * w))
        deriv = [v0, v1, v2] + list(dv) + list(dq) + list(dw)
        return [xi + di * dt for xi, di in zip(xs, deriv)]

    @classmethod
    def get_matrices(cls, x, u, params=None):
        """rocket.py:258-261 with the reference's build_batched_* tensors.  D,
        x_grad_theta and x_grad_utm1 equal the derivatives (sympy); the builders
        of D_grad_params (738-820), D_grad_x (677-735), D_grad_u (633-675) and
        x_grad_xtm1 (541-631) are sparse closed forms that do NOT follow the
        derivative of D (most entries sit at shifted indices), and are restated
        here entry by entry as the reference writes them."""
        D, _Dp, _Dx, _Du, fp, _xx, x_u = super().get_matrices(x, u, params)
        Jx, Jy, Jz, mass, l = (x.dtype.type(v) for v in (params if params is not None else cls.default_params))
        dt = x.dtype.type(cls.dt)
        N = x.shape[0]
        z = lambda *shape: np.zeros((N,) + shape, x.dtype)
        ux, uy, uz = u[:, 0], u[:, 1], u[:, 2]
        q0, q1, q2, q3 = x[:, 6], x[:, 7], x[:, 8], x[:, 9]
        wx, wy, wz = x[:, 10], x[:, 11], x[:, 12]
        # ---- x_grad_xtm1 (rocket.py:541-631)
        xx = z(13, 13)
        for i in range(13):
            xx[:, i, i] = 1.0
        xx[:, 3, 0] = dt; xx[:, 4, 1] = dt; xx[:, 5, 2] = dt
        xx[:, 6, 3] = dt * ((uz * 2 * q2 - uy * 2 * q3)) / mass
        xx[:, 6, 4] = dt * ((ux * 2 * q3 - uz * 2 * q1)) / mass
        xx[:, 6, 5] = dt * ((uy * 2 * q1 - ux * 2 * q2)) / mass
        xx[:, 6, 10] = dt * 0.5 * wx; xx[:, 6, 11] = dt * 0.5 * wy; xx[:, 6, 12] = dt * 0.5 * wz
        xx[:, 7, 3] = dt * ((uy * 2 * q2 + uz * 2 * q3)) / mass
        xx[:, 7, 4] = dt * ((ux * 2 * q2 - uy * 4 * q1 - uz * 2 * q0)) / mass
        xx[:, 7, 5] = dt * ((ux * 2 * q3 + uy * 2 * q0 - uz * 4 * q1)) / mass
        xx[:, 7, 10] = -dt * 0.5 * wx; xx[:, 7, 11] = -dt * 0.5 * wz; xx[:, 7, 12] = dt * 0.5 * wy
        xx[:, 8, 3] = dt * ((uy * 2 * q1 - ux * 4 * q2 + uz * 2 * q0)) / mass
        xx[:, 8, 4] = dt * ((ux * 2 * q1 + uz * 2 * q3)) / mass
        xx[:, 8, 5] = dt * ((uy * 2 * q3 - ux * 2 * q0 - uz * 4 * q2)) / mass
        xx[:, 8, 10] = -dt * 0.5 * wy; xx[:, 8, 11] = dt * 0.5 * wz; xx[:, 8, 12] = -dt * 0.5 * wx
        xx[:, 9, 3] = dt * ((uz * 2 * q1 - ux * 4 * q3 - uy * 2 * q0)) / mass
        xx[:, 9, 4] = dt * ((ux * 2 * q0 - uy * 4 * q3 + uz * 2 * q2)) / mass
        xx[:, 9, 5] = dt * ((ux * 2 * q1 + uy * 2 * q2)) / mass
        xx[:, 9, 10] = -dt * 0.5 * wz; xx[:, 9, 11] = -dt * 0.5 * wy; xx[:, 9, 12] = dt * 0.5 * wx
        xx[:, 10, 6] = -dt * 0.5 * q1; xx[:, 10, 7] = dt * 0.5 * q0
        xx[:, 10, 8] = dt * 0.5 * q3; xx[:, 10, 9] = -dt * 0.5 * q2
        xx[:, 10, 11] = -dt * ((wz * Jx - wz * Jz)) / Jy
        xx[:, 10, 12] = -dt * ((wy * Jy - wy * Jx)) / Jz
        xx[:, 11, 6] = -dt * 0.5 * q2; xx[:, 11, 7] = -dt * 0.5 * q3
        xx[:, 11, 8] = dt * 0.5 * q0; xx[:, 11, 9] = dt * 0.5 * q1
        xx[:, 11, 10] = -dt * ((wz * Jz - wz * Jy)) / Jx
        xx[:, 11, 12] = -dt * ((wx * Jy - wx * Jx)) / Jz
        xx[:, 12, 6] = -dt * 0.5 * q3; xx[:, 12, 7] = dt * 0.5 * q2
        xx[:, 12, 8] = -dt * 0.5 * q1; xx[:, 12, 9] = dt * 0.5 * q0
        xx[:, 12, 10] = -dt * ((wy * Jz - wy * Jy)) / Jx
        xx[:, 12, 11] = -dt * ((wx * Jx - wx * Jz)) / Jy
        # ---- D_grad_u (rocket.py:633-675)
        Du = z(13, 16, 3)
        Du[:, 5, 5, 0] = dt * (2 * q3 / mass); Du[:, 5, 6, 0] = -dt * (2 * q2 / mass)
        Du[:, 6, 5, 1] = -dt * (2 * q3 / mass); Du[:, 6, 7, 1] = dt * (2 * q1 / mass)
        Du[:, 7, 5, 2] = dt * (2 * q2 / mass); Du[:, 7, 6, 2] = -dt * (2 * q1 / mass)
        # ---- D_grad_x (rocket.py:677-735)
        Dx = z(13, 16, 13)
        Dx[:, 5, 5, 6] = -dt * (2 * uz / mass) * q3
        Dx[:, 5, 6, 6] = dt * 0.5; Dx[:, 5, 7, 6] = dt * 0.5; Dx[:, 5, 8, 6] = dt * 0.5
        Dx[:, 5, 5, 7] = dt * (2 * uy / mass) * q3
        Dx[:, 6, 5, 7] = dt * (2 * ux / mass) * q2 + dt * (2 * uy / mass) * q1
        Dx[:, 5, 5, 8] = dt * (2 * uz / mass) * q0 - dt * (2 * ux / mass) * q3
        Dx[:, 6, 5, 8] = dt * (2 * ux / mass) * q1 - dt * (4 * uy / mass) * q0 - dt * (2 * uz / mass) * q3
        Dx[:, 5, 5, 9] = -dt * (2 * uy / mass) * q0 + dt * (2 * ux / mass) * q1
        Dx[:, 6, 5, 9] = dt * (2 * ux / mass) * q0 - dt * (2 * uz / mass) * q2
        Dx[:, 9, 9, 10] = -dt * 0.5
        Dx[:, 10, 10, 10] = -dt * (Jy - Jx) / Jz * wy
        Dx[:, 10, 11, 10] = dt * (Jx - Jz) / Jy * wz
        Dx[:, 9, 10, 11] = dt * 0.5
        Dx[:, 11, 10, 11] = -dt * (Jy - Jx) / Jz * wx
        Dx[:, 11, 12, 11] = dt * (Jz - Jy) / Jx * wz
        Dx[:, 9, 11, 12] = dt * 0.5
        Dx[:, 9, 12, 12] = -dt * 0.5
        Dx[:, 12, 11, 12] = -dt * (Jx - Jz) / Jy * wy
        Dx[:, 12, 10, 12] = dt * (Jz - Jy) / Jx * wx
        # ---- D_grad_params (rocket.py:738-820)
        Dp = z(13, 16, 5)
        Dp[:, 11, 10, 0] = -dt * (wz / Jy); Dp[:, 12, 10, 0] = dt * (wy / Jz)
        Dp[:, 11, 12, 0] = dt * ((wy * Jz - wy * Jy) / Jx ** 2); Dp[:, 12, 11, 0] = dt * (wx / Jz)
        Dp[:, 11, 10, 1] = dt * ((wz * Jx - wz * Jz) / Jy ** 2); Dp[:, 12, 10, 1] = -dt * (wy / Jz)
        Dp[:, 11, 13, 1] = dt * (wz / Jx); Dp[:, 12, 11, 1] = -dt * (wx / Jz)
        Dp[:, 11, 14, 1] = dt * (wy / Jx)
        Dp[:, 12, 12, 1] = dt * ((wx * Jx - wx * Jz) / Jy ** 2)
        Dp[:, 11, 15, 1] = -dt * ((l / 2) / Jy ** 2)
        Dp[:, 11, 10, 2] = dt * (wz / Jy)
        Dp[:, 12, 10, 2] = dt * ((wy * Jy - wy * Jx) / Jz ** 2)
        Dp[:, 11, 13, 2] = -dt * (wz / Jx)
        Dp[:, 12, 11, 2] = dt * ((wx * Jy - wx * Jx) / Jz ** 2)
        Dp[:, 11, 14, 2] = -dt * (wy / Jx)
        Dp[:, 12, 12, 2] = dt * (wx / Jy)
        Dp[:, 12, 14, 2] = dt * ((l / 2) / Jz ** 2)
        m2 = mass ** 2
        Dp[:, 3, 13, 3] = -dt * (1 - 2 * (q2 ** 2 + q3 ** 2)) / m2
        Dp[:, 4, 13, 3] = -dt * (2 * (q1 * q2 + q0 * q3)) / m2
        Dp[:, 5, 13, 3] = -dt * (2 * (q1 * q3 - q0 * q2)) / m2
        Dp[:, 3, 14, 3] = -dt * (2 * (q1 * q2 - q0 * q3)) / m2
        Dp[:, 4, 14, 3] = -dt * (1 - 2 * (q1 ** 2 + q3 ** 2)) / m2
        Dp[:, 5, 14, 3] = -dt * (2 * (q2 * q3 + q0 * q1)) / m2
        Dp[:, 3, 15, 3] = -dt * (2 * (q1 * q3 + q0 * q2)) / m2
        Dp[:, 4, 15, 3] = -dt * (2 * (q2 * q3 - q0 * q1)) / m2
        Dp[:, 5, 15, 3] = -dt * (1 - 2 * (q1 ** 2 + q2 ** 2)) / m2
        Dp[:, 3, 13, 3] += -dt * ((uz * 2 * q2 - uy * 2 * q3)) / m2
        Dp[:, 4, 13, 3] += -dt * ((ux * 2 * q3 - uz * 2 * q1)) / m2
        Dp[:, 5, 13, 3] += -dt * ((uy * 2 * q1 - ux * 2 * q2)) / m2
        Dp[:, 3, 14, 3] += -dt * ((uy * 2 * q2 + uz * 2 * q3)) / m2
        Dp[:, 4, 14, 3] += -dt * ((ux * 2 * q2 - uy * 4 * q1 - uz * 2 * q0)) / m2
        Dp[:, 5, 14, 3] += -dt * ((ux * 2 * q3 + uy * 2 * q0 - uz * 4 * q1)) / m2
        Dp[:, 3, 15, 3] += -dt * ((uy * 2 * q1 - ux * 4 * q2 + uz * 2 * q0)) / m2
        Dp[:, 4, 15, 3] += -dt * ((ux * 2 * q1 + uz * 2 * q3)) / m2
        Dp[:, 5, 15, 3] += -dt * ((uy * 2 * q3 - ux * 2 * q0 - uz * 4 * q2)) / m2
        Dp[:, 3, 15, 3] += -dt * (uz * 2 * q1 - ux * 4 * q3 - uy * 2 * q0) / m2
        Dp[:, 4, 15, 3] += -dt * (ux * 2 * q0 - uy * 4 * q3 + uz * 2 * q2) / m2
        Dp[:, 5, 15, 3] += -dt * (ux * 2 * q1 + uy * 2 * q2) / m2
        Dp[:, 11, 15, 4] = dt * 0.5 / Jy ** 2
        Dp[:, 12, 14, 4] = -dt * 0.5 / Jz ** 2
        return D, Dp, Dx, Du, fp, xx, x_u

    @classmethod
    def true_obj(cls):
        """rocket.py:212-232, including its double application of tilt_penalty
        (tilt_Q is pre-multiplied at rocket.py:77 and again at 225)."""
        goal_state = np.zeros(13)
        goal_state[6] = 1.0
        goal_weights = np.ones(13)
        goal_weights[0:3] = 10.0
        goal_weights[6:10] = 0.1
        tilt_Q = 50.0 * np.array([0., 0., 4., 4.])
        tilt_p = 50.0 * np.zeros(4)
        q = np.concatenate([goal_weights, [1., 1., 0.4]])
        q[6:10] = tilt_Q * 50.0
        px = -np.sqrt(goal_weights) * goal_state
        px[6:10] = -tilt_p * 50.0
        p = np.concatenate([px, np.zeros(3)])
        return q, p


MODELS = {"pendulum": Pendulum, "cartpole": Cartpole, "rocket": Rocket, "pendulum_complex": PendulumComplex}
