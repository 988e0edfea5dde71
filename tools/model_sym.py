"""Symbolic model equations for tools/gen_model_derivs.py (code generation only).

The generator derives the implicit backward's second-order terms from these.
They restate the reference's env_dx models independently of oracle/ (which is
test infrastructure the generator must not run); tests/test_models_gen.py checks
the generated code against the oracle, which is itself pinned to the reference's
get_matrices outputs.

  pendulum   env_dx/pendulum.py:63-80     (forward, control clamp dropped)
  cartpole   env_dx/cartpole.py:64-97     (+ four D_grad_params closed forms, 400-560)
  rocket     env_dx/rocket.py:82-164      (+ the build_batched_* builders, 541-820)

The analytic Jacobians of the reference ignore the control clamp, so none is
applied here either.
"""
import sympy as sp


def symbols(n, m, p):
    return (sp.symbols(f"x0:{n}", real=True), sp.symbols(f"u0:{m}", real=True),
            sp.symbols(f"th0:{p}", real=True))


# ------------------------------------------------------------------ pendulum
class Pendulum:
    n, m, p = 3, 1, 3
    xx00_zero = False         # x_grad_xtm1 is D[:, :n] as computed (pendulum.py:152-382)
    dt = 0.05

    @classmethod
    def next_state(cls, xs, us, ps):
        c, s, dth = xs
        (u,) = us
        g, m, l = ps
        th = sp.atan2(s, c)
        newdth = dth + sp.Float(cls.dt) * (-3 * g / (2 * l) * (-s) + 3 * u / (m * l ** 2))
        newth = th + newdth * sp.Float(cls.dt)
        return [sp.cos(newth), sp.sin(newth), newdth]

    @classmethod
    def dp_overrides(cls):
        return {}


# ------------------------------------------------------------------ cartpole
class Cartpole:
    n, m, p = 5, 1, 4
    xx00_zero = True          # the reference writes x_grad_xtm1[0,0] = 0 (cartpole.py:666)
    dt = 0.05

    @classmethod
    def next_state(cls, xs, us, ps):
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
    def dp_overrides(cls):
        """The reference's closed forms for D_grad_params[4,3,1], [4,3,2], [4,4,2],
        [4,5,2] (cartpole.py matrix_2_part_2 / matrix_2_part_3, row 4), which are
        not the derivative of D[4,:]."""
        dt = sp.Float(cls.dt)

        def common(xs, ps):
            c, s, w = xs[2], xs[3], xs[4]
            g, mc, mp, l = ps
            Mt = mc + mp
            den = -c ** 2 * mp / Mt + sp.Rational(4, 3)
            return c, s, w, g, mc, mp, l, Mt, den

        def e431(xs, us, ps):
            c, s, w, g, mc, mp, l, Mt, den = common(xs, ps)
            return dt * (-c ** 2 * mp * (-c * w ** 2 * l * mp / Mt + g) / (l * Mt ** 2 * den ** 2)
                         + c * dt * w ** 2 * mp / (Mt ** 2 * den))

        def e432(xs, us, ps):
            c, s, w, g, mc, mp, l, Mt, den = common(xs, ps)
            return dt * (-c ** 2 * mp * (-c * w ** 2 * l * mp / Mt + g) / (l * den ** 2)
                         + c * dt * w ** 2 * l * mp / Mt ** 2)

        def e442(xs, us, ps):
            c, s, w, g, mc, mp, l, Mt, den = common(xs, ps)
            return (-2 * c * dt * w * mp * s * (-c ** 2 * mp / Mt ** 2 + c ** 2 / Mt) / (Mt * den ** 2)
                    + 2 * c * dt * w * mp * s / (Mt ** 2 * den))

        def e452(xs, us, ps):
            c, s, w, g, mc, mp, l, Mt, den = common(xs, ps)
            return c * dt / (l * Mt ** 2 * den)

        return {(4, 3, 1): e431, (4, 3, 2): e432, (4, 4, 2): e442, (4, 5, 2): e452}


# ------------------------------------------------------------------ rocket
class Rocket:
    n, m, p = 13, 3, 5
    dt = 0.1

    @classmethod
    def next_state(cls, xs, us, ps):
        r0, r1, r2, v0, v1, v2, q0, q1, q2, q3, wx, wy, wz = xs
        ux, uy, uz = us
        Jx, Jy, Jz, mass, l = ps
        dt = sp.Float(cls.dt)
        CBI = sp.Matrix([[1 - 2 * (q2 ** 2 + q3 ** 2), 2 * (q1 * q2 + q0 * q3), 2 * (q1 * q3 - q0 * q2)],
                         [2 * (q1 * q2 - q0 * q3), 1 - 2 * (q1 ** 2 + q3 ** 2), 2 * (q2 * q3 + q0 * q1)],
                         [2 * (q1 * q3 + q0 * q2), 2 * (q2 * q3 - q0 * q1), 1 - 2 * (q1 ** 2 + q2 ** 2)]])
        dv = CBI.T * sp.Matrix([ux, uy, uz]) / mass + sp.Matrix([-10, 0, 0])
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
    def builders(cls, xs, us, ps):
        """The reference's build_batched_x_xtm1 (rocket.py:541-631), _D_u (633-675),
        _D_x (677-735) and _D_params (738-820): sparse closed forms that are NOT
        the derivatives of D (most entries sit at shifted indices).  Returned as
        dicts {(i, j[, k]): expr}; `+=` entries of the reference are summed."""
        dt = sp.Float(cls.dt)
        half = sp.Float(0.5)
        Jx, Jy, Jz, mass, l = ps
        ux, uy, uz = us
        q0, q1, q2, q3 = xs[6:10]
        wx, wy, wz = xs[10:13]
        xx = {(i, i): sp.Integer(1) for i in range(13)}
        xx.update({
            (3, 0): dt, (4, 1): dt, (5, 2): dt,
            (6, 3): dt * (uz * 2 * q2 - uy * 2 * q3) / mass,
            (6, 4): dt * (ux * 2 * q3 - uz * 2 * q1) / mass,
            (6, 5): dt * (uy * 2 * q1 - ux * 2 * q2) / mass,
            (6, 10): dt * half * wx, (6, 11): dt * half * wy, (6, 12): dt * half * wz,
            (7, 3): dt * (uy * 2 * q2 + uz * 2 * q3) / mass,
            (7, 4): dt * (ux * 2 * q2 - uy * 4 * q1 - uz * 2 * q0) / mass,
            (7, 5): dt * (ux * 2 * q3 + uy * 2 * q0 - uz * 4 * q1) / mass,
            (7, 10): -dt * half * wx, (7, 11): -dt * half * wz, (7, 12): dt * half * wy,
            (8, 3): dt * (uy * 2 * q1 - ux * 4 * q2 + uz * 2 * q0) / mass,
            (8, 4): dt * (ux * 2 * q1 + uz * 2 * q3) / mass,
            (8, 5): dt * (uy * 2 * q3 - ux * 2 * q0 - uz * 4 * q2) / mass,
            (8, 10): -dt * half * wy, (8, 11): dt * half * wz, (8, 12): -dt * half * wx,
            (9, 3): dt * (uz * 2 * q1 - ux * 4 * q3 - uy * 2 * q0) / mass,
            (9, 4): dt * (ux * 2 * q0 - uy * 4 * q3 + uz * 2 * q2) / mass,
            (9, 5): dt * (ux * 2 * q1 + uy * 2 * q2) / mass,
            (9, 10): -dt * half * wz, (9, 11): -dt * half * wy, (9, 12): dt * half * wx,
            (10, 6): -dt * half * q1, (10, 7): dt * half * q0, (10, 8): dt * half * q3, (10, 9): -dt * half * q2,
            (10, 11): -dt * (wz * Jx - wz * Jz) / Jy, (10, 12): -dt * (wy * Jy - wy * Jx) / Jz,
            (11, 6): -dt * half * q2, (11, 7): -dt * half * q3, (11, 8): dt * half * q0, (11, 9): dt * half * q1,
            (11, 10): -dt * (wz * Jz - wz * Jy) / Jx, (11, 12): -dt * (wx * Jy - wx * Jx) / Jz,
            (12, 6): -dt * half * q3, (12, 7): dt * half * q2, (12, 8): -dt * half * q1, (12, 9): dt * half * q0,
            (12, 10): -dt * (wy * Jz - wy * Jy) / Jx, (12, 11): -dt * (wx * Jx - wx * Jz) / Jy,
        })
        Du = {
            (5, 5, 0): dt * (2 * q3 / mass), (5, 6, 0): -dt * (2 * q2 / mass),
            (6, 5, 1): -dt * (2 * q3 / mass), (6, 7, 1): dt * (2 * q1 / mass),
            (7, 5, 2): dt * (2 * q2 / mass), (7, 6, 2): -dt * (2 * q1 / mass),
        }
        Dx = {
            (5, 5, 6): -dt * (2 * uz / mass) * q3,
            (5, 6, 6): dt * half, (5, 7, 6): dt * half, (5, 8, 6): dt * half,
            (5, 5, 7): dt * (2 * uy / mass) * q3,
            (6, 5, 7): dt * (2 * ux / mass) * q2 + dt * (2 * uy / mass) * q1,
            (5, 5, 8): dt * (2 * uz / mass) * q0 - dt * (2 * ux / mass) * q3,
            (6, 5, 8): dt * (2 * ux / mass) * q1 - dt * (4 * uy / mass) * q0 - dt * (2 * uz / mass) * q3,
            (5, 5, 9): -dt * (2 * uy / mass) * q0 + dt * (2 * ux / mass) * q1,
            (6, 5, 9): dt * (2 * ux / mass) * q0 - dt * (2 * uz / mass) * q2,
            (9, 9, 10): -dt * half,
            (10, 10, 10): -dt * (Jy - Jx) / Jz * wy,
            (10, 11, 10): dt * (Jx - Jz) / Jy * wz,
            (9, 10, 11): dt * half,
            (11, 10, 11): -dt * (Jy - Jx) / Jz * wx,
            (11, 12, 11): dt * (Jz - Jy) / Jx * wz,
            (9, 11, 12): dt * half,
            (9, 12, 12): -dt * half,
            (12, 11, 12): -dt * (Jx - Jz) / Jy * wy,
            (12, 10, 12): dt * (Jz - Jy) / Jx * wx,
        }
        m2 = mass ** 2
        Dp = {
            (11, 10, 0): -dt * (wz / Jy), (12, 10, 0): dt * (wy / Jz),
            (11, 12, 0): dt * ((wy * Jz - wy * Jy) / Jx ** 2), (12, 11, 0): dt * (wx / Jz),
            (11, 10, 1): dt * ((wz * Jx - wz * Jz) / Jy ** 2), (12, 10, 1): -dt * (wy / Jz),
            (11, 13, 1): dt * (wz / Jx), (12, 11, 1): -dt * (wx / Jz),
            (11, 14, 1): dt * (wy / Jx),
            (12, 12, 1): dt * ((wx * Jx - wx * Jz) / Jy ** 2),
            (11, 15, 1): -dt * ((l / 2) / Jy ** 2),
            (11, 10, 2): dt * (wz / Jy),
            (12, 10, 2): dt * ((wy * Jy - wy * Jx) / Jz ** 2),
            (11, 13, 2): -dt * (wz / Jx),
            (12, 11, 2): dt * ((wx * Jy - wx * Jx) / Jz ** 2),
            (11, 14, 2): -dt * (wy / Jx),
            (12, 12, 2): dt * (wx / Jy),
            (12, 14, 2): dt * ((l / 2) / Jz ** 2),
            (11, 15, 4): dt * half / Jy ** 2,
            (12, 14, 4): -dt * half / Jz ** 2,
        }
        acc = [
            ((3, 13, 3), -dt * (1 - 2 * (q2 ** 2 + q3 ** 2)) / m2),
            ((4, 13, 3), -dt * (2 * (q1 * q2 + q0 * q3)) / m2),
            ((5, 13, 3), -dt * (2 * (q1 * q3 - q0 * q2)) / m2),
            ((3, 14, 3), -dt * (2 * (q1 * q2 - q0 * q3)) / m2),
            ((4, 14, 3), -dt * (1 - 2 * (q1 ** 2 + q3 ** 2)) / m2),
            ((5, 14, 3), -dt * (2 * (q2 * q3 + q0 * q1)) / m2),
            ((3, 15, 3), -dt * (2 * (q1 * q3 + q0 * q2)) / m2),
            ((4, 15, 3), -dt * (2 * (q2 * q3 - q0 * q1)) / m2),
            ((5, 15, 3), -dt * (1 - 2 * (q1 ** 2 + q2 ** 2)) / m2),
            ((3, 13, 3), -dt * (uz * 2 * q2 - uy * 2 * q3) / m2),
            ((4, 13, 3), -dt * (ux * 2 * q3 - uz * 2 * q1) / m2),
            ((5, 13, 3), -dt * (uy * 2 * q1 - ux * 2 * q2) / m2),
            ((3, 14, 3), -dt * (uy * 2 * q2 + uz * 2 * q3) / m2),
            ((4, 14, 3), -dt * (ux * 2 * q2 - uy * 4 * q1 - uz * 2 * q0) / m2),
            ((5, 14, 3), -dt * (ux * 2 * q3 + uy * 2 * q0 - uz * 4 * q1) / m2),
            ((3, 15, 3), -dt * (uy * 2 * q1 - ux * 4 * q2 + uz * 2 * q0) / m2),
            ((4, 15, 3), -dt * (ux * 2 * q1 + uz * 2 * q3) / m2),
            ((5, 15, 3), -dt * (uy * 2 * q3 - ux * 2 * q0 - uz * 4 * q2) / m2),
            ((3, 15, 3), -dt * (uz * 2 * q1 - ux * 4 * q3 - uy * 2 * q0) / m2),
            ((4, 15, 3), -dt * (ux * 2 * q0 - uy * 4 * q3 + uz * 2 * q2) / m2),
            ((5, 15, 3), -dt * (ux * 2 * q1 + uy * 2 * q2) / m2),
        ]
        for key, e in acc:
            Dp[key] = Dp.get(key, sp.Integer(0)) + e
        return xx, Du, Dx, Dp
