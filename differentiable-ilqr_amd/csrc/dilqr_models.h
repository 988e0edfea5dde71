// dilqr_models.h — device dynamics of the reference's env_dx models.
//
// forward(): the reference forward's arithmetic, restated for the GPU: rocket
// op for op (contraction off); pendulum and cartpole with the angle update
// through angle_step (dilqr_device.h: the angle-sum identity instead of
// atan2 -> add -> sin/cos) and the divisions as reciprocal products — the same
// function to a few ulp (tests: dynamics vs the reference at 2e-5).
// jacobian(): d x_{t+1} / d [x_t;u_t] at the UNCLAMPED u, as get_linear_dyn
// writes it, derived by hand with common subexpressions.
#pragma once
#include "dilqr_device.h"

namespace dilqr {

// ---------------------------------------------------------------- pendulum
// env_dx/pendulum.py: x = [cos th, sin th, dth], u = [torque], theta = (g, m, l)
struct Pendulum {
  static constexpr int N = 3, M = 1, P = 3;
  static constexpr float DT = 0.05f;
  static constexpr float ULIM = 2.0f;      // forward() clamps u to [-ULIM, ULIM]
  float g, m, l;
  float kg, ku;                            // 3g/(2l), 3/(m l^2)
  DEV void load(const float* __restrict__ th) {
    g = th[0]; m = th[1]; l = th[2];
    kg = 3.0f * g / (2.0f * l);
    ku = 3.0f / (m * (l * l));
  }

  static constexpr bool kJacFromNext = false;   // its Jacobian angle uses the unclamped u
  DEV void jacobian_next(const float (&x)[N], const float (&u)[M], const float (&)[N], float (&D)[N][N + M]) const {
    jacobian(x, u, D);
  }

  struct FSparsity {      // pendulum.py:448-474: row 2 has a structural zero at cos
    static constexpr bool nz(int i, int j) { return !(i == 2 && j == 0); }
  };

  // pendulum.py:60-95; S = float, or f2 for two trajectories at once.  The
  // angle update th' = atan2(sin, cos) + dt * dth' goes through angle_step (no
  // atan2; sin and cos of the increment only)
  template <class S>
  DEV void forward(const S (&x)[N], const S (&u)[M], S (&o)[N]) const {
    S uu = vclamp(u[0], -2.0f, 2.0f);
    S c = x[0], s = x[1], dth = x[2];
    S newdth = dth + DT * (kg * s + ku * uu);
    angle_step(c, s, newdth * DT, o[0], o[1]);
    o[2] = newdth;
  }

  // cos and sin of the integrated angle at the UNCLAMPED u, as the Jacobian
  // uses them (and the implicit backward's second-order terms, which take them
  // as inputs: gen::PendulumD2 next_cs is the same pair by atan2f/cosf/sinf)
  DEV void next_cs(const float (&x)[N], const float (&u)[M], float& cs, float& sn) const {
    angle_step(x[0], x[1], DT * (DT * (kg * x[1] + ku * u[0]) + x[2]), cs, sn);
  }

  // pendulum.py:444-475
  DEV void jacobian(const float (&x)[N], const float (&u)[M], float (&D)[N][N + M]) const {
    float sn, cs;
    next_cs(x, u, cs, sn);
    jacobian_sc(x, u, cs, sn, D);
  }
  DEV void jacobian_sc(const float (&x)[N], const float (&u)[M], float cs, float sn, float (&D)[N][N + M]) const {
    float c = x[0], s = x[1];
    float ir2 = vrcp(c * c + s * s);
    float dc = -s * ir2;                // d newth / d cos
    float ds = c * ir2 + DT * DT * kg;  // d newth / d sin
    float dw = DT;                      // d newth / d dth
    float du = DT * DT * ku;            // d newth / d u
    D[0][0] = -sn * dc; D[0][1] = -sn * ds; D[0][2] = -sn * dw; D[0][3] = -sn * du;
    D[1][0] = cs * dc;  D[1][1] = cs * ds;  D[1][2] = cs * dw;  D[1][3] = cs * du;
    D[2][0] = 0.f;      D[2][1] = DT * kg;  D[2][2] = 1.f;      D[2][3] = DT * ku;
  }
};

// ---------------------------------------------------------------- pendulum, 5 parameters
// env_dx/pendulum.py with simple=False (pendulum.py:30-49, 76-95; il_env.py:40-42
// 'pendulum-complex'): theta = (g, m, l, d, b), a damping d*th and a gravity bias
// b inside sin(th + b).  The damping needs th itself, so forward() follows the
// reference's ops: th = atan2(sin, cos), th' = th + dt*dth', cos/sin of th'.
// The reference has no closed-form Jacobian for this variant (get_linear_dyn
// and get_matrices unpack three parameters, pendulum.py:157, 448, so its
// ANALYTIC path fails); its runnable path linearises by autograd
// (GradMethods.AUTO_DIFF, mpc_explicit.py:547-627), so jacobian() is that
// derivative: atan2's partials, and the clamp's gate on u (torch.clamp passes
// the gradient where lo <= u <= hi).
struct PendulumComplex {
  static constexpr int N = 3, M = 1, P = 5;
  static constexpr float DT = 0.05f;
  static constexpr float ULIM = 2.0f;
  float kg, ku, dmp, bias;                 // 3g/(2l), 3/(m l^2), d, b
  DEV void load(const float* __restrict__ th) {
    const float g = th[0], m = th[1], l = th[2];
    kg = 3.0f * g / (2.0f * l);
    ku = 3.0f / (m * (l * l));
    dmp = th[3];
    bias = th[4];
  }

  static constexpr bool kJacFromNext = false;
  DEV void jacobian_next(const float (&x)[N], const float (&u)[M], const float (&)[N], float (&D)[N][N + M]) const {
    jacobian(x, u, D);
  }
  struct FSparsity {      // every entry of the 3 x 4 Jacobian is a function of the state
    static constexpr bool nz(int, int) { return true; }
  };

  template <class S>
  DEV void forward(const S (&x)[N], const S (&u)[M], S (&o)[N]) const {
    S uu = vclamp(u[0], -2.0f, 2.0f);
    S th = vatan2(x[1], x[0]);
    S newdth = x[2] + DT * ((kg * vsin(th + bias) + ku * uu) - dmp * th);
    S newth = th + newdth * DT;
    S sn, cs;
    vsincos(newth, sn, cs);
    o[0] = cs; o[1] = sn; o[2] = newdth;
  }

  DEV void jacobian(const float (&x)[N], const float (&u)[M], float (&D)[N][N + M]) const {
    const float c = x[0], s = x[1], w = x[2];
    const float gate = (u[0] >= -2.0f && u[0] <= 2.0f) ? 1.0f : 0.0f;
    const float uu = fminf(fmaxf(u[0], -2.0f), 2.0f);
    const float th = atan2f(s, c);
    float sb, cb;
    sincosf(th + bias, &sb, &cb);
    const float newdth = w + DT * ((kg * sb + ku * uu) - dmp * th);
    float sn, cs;
    sincosf(th + newdth * DT, &sn, &cs);
    const float ir2 = 1.0f / (c * c + s * s);
    const float th_c = -s * ir2, th_s = c * ir2;      // d atan2(s, c)
    const float a = DT * (kg * cb - dmp);             // d newdth / d th
    const float nd[4] = {a * th_c, a * th_s, 1.0f, DT * ku * gate};
    const float nt[4] = {th_c + DT * nd[0], th_s + DT * nd[1], DT, DT * nd[3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      D[0][j] = -sn * nt[j];
      D[1][j] = cs * nt[j];
      D[2][j] = nd[j];
    }
  }
};

// ---------------------------------------------------------------- cartpole
// env_dx/cartpole.py: x = [x, dx, cos th, sin th, dth], u = [force],
// theta = (g, m_cart, m_pole, l)
struct Cartpole {
  static constexpr int N = 5, M = 1, P = 4;
  static constexpr float DT = 0.05f;
  static constexpr float ULIM = 100.0f;
  float g, mc, mp, l;
  float iM, pml, mpM, pmlM;                // 1/(mc+mp), mp l, mp/(mc+mp), mp l/(mc+mp)
  DEV void load(const float* __restrict__ th) {
    g = th[0]; mc = th[1]; mp = th[2]; l = th[3];
    iM = 1.0f / (mp + mc);
    pml = mp * l;
    mpM = mp * iM;
    pmlM = pml * iM;
  }

  // structural nonzeros of jacobian() (cartpole.py:802-838): rows x, dx, cos, sin, dth
  struct FSparsity {
    static constexpr bool nz(int i, int j) {
      return i == 0 ? (j <= 1) : i == 1 ? (j >= 1) : i == 4 ? (j >= 2) : (j >= 2 && j <= 4);
    }
  };

  // cartpole.py:64-97; S = float, or f2 for two trajectories at once.  The
  // divisions by the mass are products with 1/(mc+mp), the one by the
  // pole-inertia term a hardware reciprocal, and th' = atan2(sin, cos) + dt*dth
  // goes through angle_step (no atan2; sin and cos of dt*dth only).
  template <class S>
  DEV void forward(const S (&s_)[N], const S (&u)[M], S (&o)[N]) const {
    S uu = vclamp(u[0], -100.0f, 100.0f);
    S x = s_[0], dx = s_[1], c = s_[2], s = s_[3], dth = s_[4];
    S cart_in = (uu + (pml * (dth * dth)) * s) * iM;
    S th_acc = (g * s - c * cart_in) * vrcp(l * (4.0f / 3.0f - mpM * (c * c)));
    S xacc = cart_in - (pmlM * th_acc) * c;
    o[0] = x + DT * dx;
    o[1] = dx + DT * xacc;
    angle_step(c, s, DT * dth, o[2], o[3]);
    o[4] = dth + DT * th_acc;
  }

  // cos and sin of the integrated angle (independent of u), as forward() and the
  // Jacobian form them (gen::CartpoleD2 next_cs: the same pair by atan2f/cosf/sinf)
  DEV void next_cs(const float (&s_)[N], const float (&)[M], float& cs, float& sn) const {
    angle_step(s_[2], s_[3], DT * s_[4], cs, sn);
  }

  // cartpole.py:790-839 (closed form of the same derivative)
  DEV void jacobian(const float (&s_)[N], const float (&u)[M], float (&D)[N][N + M]) const {
    float sn, cs;
    next_cs(s_, u, cs, sn);
    jacobian_sc(s_, u, cs, sn, D);
  }

  // The Jacobian's cos/sin of the integrated angle are exactly components 2 and
  // 3 of forward(x, u) (the same angle_step call, independent of u), so along a
  // rollout the fused sweep takes them from x_{t+1} instead of recomputing them.
  static constexpr bool kJacFromNext = true;
  DEV void jacobian_next(const float (&s_)[N], const float (&u)[M], const float (&xn)[N],
                         float (&D)[N][N + M]) const {
    jacobian_sc(s_, u, xn[2], xn[3], D);
  }

  DEV void jacobian_sc(const float (&s_)[N], const float (&u)[M], float cs, float sn, float (&D)[N][N + M]) const {
    float c = s_[2], s = s_[3], w = s_[4], uu = u[0];
    float A = uu + pml * w * w * s;                 // cart_in * M
    float den = l * (4.0f / 3.0f - mp * c * c * iM);
    float iden = vrcp(den);
    float num = g * s - c * A * iM;
    float tha = num * iden;                         // th_acc
    // partials of A, den, num wrt (c, s, w, u)
    float A_s = pml * w * w, A_w = 2.0f * pml * w * s;
    float den_c = -2.0f * l * mp * c * iM;
    float num_c = -A * iM, num_s = g - c * A_s * iM, num_w = -c * A_w * iM, num_u = -c * iM;
    float tha_c = (num_c - tha * den_c) * iden;
    float tha_s = num_s * iden, tha_w = num_w * iden, tha_u = num_u * iden;
    float k = pmlM;
    float xa_c = -k * (tha_c * c + tha);
    float xa_s = A_s * iM - k * tha_s * c;
    float xa_w = A_w * iM - k * tha_w * c;
    float xa_u = iM - k * tha_u * c;
    float ir2 = vrcp(c * c + s * s);
    D[0][0] = 1.f; D[0][1] = DT;  D[0][2] = 0.f;            D[0][3] = 0.f;            D[0][4] = 0.f;            D[0][5] = 0.f;
    D[1][0] = 0.f; D[1][1] = 1.f; D[1][2] = DT * xa_c;      D[1][3] = DT * xa_s;      D[1][4] = DT * xa_w;      D[1][5] = DT * xa_u;
    D[2][0] = 0.f; D[2][1] = 0.f; D[2][2] = s * sn * ir2;   D[2][3] = -c * sn * ir2;  D[2][4] = -DT * sn;       D[2][5] = 0.f;
    D[3][0] = 0.f; D[3][1] = 0.f; D[3][2] = -s * cs * ir2;  D[3][3] = c * cs * ir2;   D[3][4] = DT * cs;        D[3][5] = 0.f;
    D[4][0] = 0.f; D[4][1] = 0.f; D[4][2] = DT * tha_c;     D[4][3] = DT * tha_s;     D[4][4] = 1.f + DT * tha_w; D[4][5] = DT * tha_u;
  }
};

// ---------------------------------------------------------------- LinDx
// definitions.py LinDx: x_{t+1} = F_t [x_t; u_t] + f_t (util.py:199-204,
// lqr_step_explicit.py:220-224).  Step-dependent, so it is applied inline by the
// kernels rather than through this model interface.

}  // namespace dilqr

#include "dilqr_models_gen.h"
#include "dilqr_d2_sparsity.h"

namespace dilqr {
// Second-order terms of each model for the implicit backward.  XX00_ZERO: the
// reference's x_grad_xtm1 has a 0 where d x_{t+1}/d x_t is 1 (cartpole.py:666).
// hess_nz / dparam_nz / ftheta_nz (dilqr_d2_sparsity.h): the generated
// pieces' structural zeros, skipped by the implicit backward at compile time.
template <class Model> struct D2Of;
template <> struct D2Of<Pendulum> : gen::PendulumD2Z {
  using type = gen::PendulumD2;
  static constexpr bool XX00_ZERO = false;
};
template <> struct D2Of<Cartpole> : gen::CartpoleD2Z {
  using type = gen::CartpoleD2;
  static constexpr bool XX00_ZERO = true;
};
}  // namespace dilqr

namespace dilqr {
// ---------------------------------------------------------------- rocket
// env_dx/rocket.py: x = [r(3), v(3), q(4), w(3)], u = thrust (3), theta =
// (Jx, Jy, Jz, mass, l), dt = 0.1.  The reference returns the UNNORMALISED
// quaternion (rocket.py:159-164: new_x_out is built but new_x is returned).
struct Rocket {
  static constexpr int N = 13, M = 3, P = 5;
  static constexpr float DT = 0.1f;
  float Jx, Jy, Jz, mass, l;
  // 1/mass, 1/Jx, 1/Jy, 1/Jz: the same IEEE quotients deriv() and jac_row
  // formed per call, formed once per launch (theta is the same for every
  // problem: readfirstlane keeps them in scalar registers, no VGPRs)
  float im, iJx, iJy, iJz;
  // jac_row's coefficients, per launch (scalar registers): dt/m, 2 dt/m, and
  // the angular rows' -dt (J_j - J_k)/J_i and +-dt (l/2)/J_i
  float s1, s2, w10, w11, w12, l11, l12;
  DEV void load(const float* __restrict__ th) {
    Jx = th[0]; Jy = th[1]; Jz = th[2]; mass = th[3]; l = th[4];
    im = uniform(1.f / mass); iJx = uniform(1.f / Jx); iJy = uniform(1.f / Jy); iJz = uniform(1.f / Jz);
    s1 = uniform(DT * im);
    s2 = uniform(2.f * s1);
    w10 = uniform((-DT * (Jz - Jy)) * iJx);
    w11 = uniform((-DT * (Jx - Jz)) * iJy);
    w12 = uniform((-DT * (Jy - Jx)) * iJz);
    l11 = uniform((DT * (l / 2.f)) * iJy);
    l12 = uniform((-DT * (l / 2.f)) * iJz);
  }
  static DEV float uniform(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

  struct FSparsity {    // rocket.py:324-426 (69 nonzeros)
    static constexpr bool nz(int i, int j) {
      return i == j || (i < 3 && j == i + 3) || (i >= 3 && i < 6 && j >= 6 && j <= 9) ||
             (i >= 3 && i < 6 && j >= 13) || (i >= 6 && i < 10 && j >= 6 && j <= 12) ||
             (i >= 10 && j >= 10 && j <= 12) || (i == 11 && j == 15) || (i == 12 && j == 14);
    }
  };

  // derivative of state component r (rocket.py:94-156), contraction off so the
  // rounding follows the reference's eager ops — except that the three
  // divisions by the mass are products with one reciprocal, formed per call
  // (in the 16-lane kernels every lane's row is a different case of the
  // switch, so a wave executes all of them; the reciprocal is not kept live
  // across the kernel: four more live VGPRs cost those kernels an occupancy
  // step)
  DEV float deriv(int r, const float (&x)[N], const float (&u)[M]) const {
#pragma clang fp contract(off)
    const float q0 = x[6], q1 = x[7], q2 = x[8], q3 = x[9], wx = x[10], wy = x[11], wz = x[12];
    const float Tx = fminf(fmaxf(u[0], -400.f), 400.f);
    const float Ty = fminf(fmaxf(u[1], -400.f), 400.f);
    const float Tz = fminf(fmaxf(u[2], -400.f), 400.f);
    switch (r) {
      case 0: case 1: case 2: return x[3 + r];
      case 3: return (((1.f - 2.f * (q2 * q2 + q3 * q3)) * Tx + 2.f * (q1 * q2 - q0 * q3) * Ty) +
                      2.f * (q1 * q3 + q0 * q2) * Tz) * im + -10.f;
      case 4: return ((2.f * (q1 * q2 + q0 * q3) * Tx + (1.f - 2.f * (q1 * q1 + q3 * q3)) * Ty) +
                      2.f * (q2 * q3 - q0 * q1) * Tz) * im + 0.f;
      case 5: return ((2.f * (q1 * q3 - q0 * q2) * Tx + 2.f * (q2 * q3 + q0 * q1) * Ty) +
                      (1.f - 2.f * (q1 * q1 + q2 * q2)) * Tz) * im + 0.f;
      case 6: return 0.5f * (((-wx * q1) + (-wy * q2)) + (-wz * q3));
      case 7: return 0.5f * (((wx * q0) + (wz * q2)) + (-wy * q3));
      case 8: return 0.5f * (((wy * q0) + (-wz * q1)) + (wx * q3));
      case 9: return 0.5f * (((wz * q0) + (wy * q1)) + (-wx * q2));
      case 10: return iJx * (0.f - (wy * (Jz * wz) - wz * (Jy * wy)));
      case 11: return iJy * ((l / 2.f) * Tz - (wz * (Jx * wx) - wx * (Jz * wz)));
      default: return iJz * (-(l / 2.f) * Ty - (wx * (Jy * wy) - wy * (Jx * wx)));
    }
  }

  DEV void forward(const float (&x)[N], const float (&u)[M], float (&o)[N]) const {
#pragma clang fp contract(off)
#pragma unroll
    for (int r = 0; r < N; ++r) o[r] = x[r] + deriv(r, x, u) * DT;
  }
  // component r of forward() (the 16-lanes-per-problem kernels, dilqr_group.h)
  DEV float forward_row(int r, const float (&x)[N], const float (&u)[M]) const {
#pragma clang fp contract(off)
    return x[r] + deriv(r, x, u) * DT;
  }
  // row r of get_linear_dyn (rocket.py:324-426), unclamped u, factored over
  // the per-launch coefficients of load(): rows 3-5 are 2 dt/m times the
  // derivative of R(q) T (d/dq: bilinear in q and T; d/dT: R(q)), rows 6-9
  // +-dt/2 times w or q, rows 10-12 a coefficient times one rate (27 divisions
  // and ~50 products per Jacobian in the reference's order become ~15
  // products: the 16- and 8-lane kernels evaluate the whole Jacobian in every
  // lane).  The same real numbers as the reference's expressions, rounded in
  // another order (parity at 1e-4 against the float64 oracle).
  DEV void jac_row(int r, const float (&x)[N], const float (&u)[M], float (&D)[N + M]) const {
    const float dt = DT;
    const float q0 = x[6], q1 = x[7], q2 = x[8], q3 = x[9], wx = x[10], wy = x[11], wz = x[12];
    const float ux = u[0], uy = u[1], uz = u[2];
    const float a = s2;
#pragma unroll
    for (int j = 0; j < N + M; ++j) D[j] = (j == r) ? 1.f : 0.f;
    switch (r) {
      case 0: case 1: case 2: D[r + 3] = dt; break;
      case 3:
        D[6] = a * (uz * q2 - uy * q3);
        D[7] = a * (uy * q2 + uz * q3);
        D[8] = a * ((uy * q1 - 2.f * ux * q2) + uz * q0);
        D[9] = a * ((uz * q1 - 2.f * ux * q3) - uy * q0);
        D[13] = s1 - a * (q2 * q2 + q3 * q3);
        D[14] = a * (q1 * q2 - q0 * q3);
        D[15] = a * (q1 * q3 + q0 * q2);
        break;
      case 4:
        D[6] = a * (ux * q3 - uz * q1);
        D[7] = a * ((ux * q2 - 2.f * uy * q1) - uz * q0);
        D[8] = a * (ux * q1 + uz * q3);
        D[9] = a * ((ux * q0 - 2.f * uy * q3) + uz * q2);
        D[13] = a * (q1 * q2 + q0 * q3);
        D[14] = s1 - a * (q1 * q1 + q3 * q3);
        D[15] = a * (q2 * q3 - q0 * q1);
        break;
      case 5:
        D[6] = a * (uy * q1 - ux * q2);
        D[7] = a * ((ux * q3 + uy * q0) - 2.f * uz * q1);
        D[8] = a * ((uy * q3 - ux * q0) - 2.f * uz * q2);
        D[9] = a * (ux * q1 + uy * q2);
        D[13] = a * (q1 * q3 - q0 * q2);
        D[14] = a * (q2 * q3 + q0 * q1);
        D[15] = s1 - a * (q1 * q1 + q2 * q2);
        break;
      case 6:
        D[7] = -dt * 0.5f * wx; D[8] = -dt * 0.5f * wy; D[9] = -dt * 0.5f * wz;
        D[10] = -dt * 0.5f * q1; D[11] = -dt * 0.5f * q2; D[12] = -dt * 0.5f * q3;
        break;
      case 7:
        D[6] = dt * 0.5f * wx; D[8] = dt * 0.5f * wz; D[9] = -dt * 0.5f * wy;
        D[10] = dt * 0.5f * q0; D[11] = -dt * 0.5f * q3; D[12] = dt * 0.5f * q2;
        break;
      case 8:
        D[6] = dt * 0.5f * wy; D[7] = -dt * 0.5f * wz; D[9] = dt * 0.5f * wx;
        D[10] = dt * 0.5f * q3; D[11] = dt * 0.5f * q0; D[12] = -dt * 0.5f * q1;
        break;
      case 9:
        D[6] = dt * 0.5f * wz; D[7] = dt * 0.5f * wy; D[8] = -dt * 0.5f * wx;
        D[10] = -dt * 0.5f * q2; D[11] = dt * 0.5f * q1; D[12] = dt * 0.5f * q0;
        break;
      case 10: D[11] = w10 * wz; D[12] = w10 * wy; break;
      case 11: D[10] = w11 * wz; D[12] = w11 * wx; D[15] = l11; break;
      default: D[10] = w12 * wy; D[11] = w12 * wx; D[14] = l12; break;   // 12
    }
  }
  // Every row evaluated in every lane (compile-time rows: no divergence) and
  // lane r keeping row r by selects — a switch on the lane's row makes the
  // wave run all 13 cases behind exec-mask branches and merge the whole row
  // after each (~24 register moves per case)
  DEV void jac_row_sel(int r, const float (&x)[N], const float (&u)[M], float (&D)[N + M]) const {
#pragma unroll
    for (int j = 0; j < N + M; ++j) D[j] = 0.f;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float Di[N + M];
      jac_row(i, x, u, Di);
#pragma unroll
      for (int j = 0; j < N + M; ++j)
        if (j == i || FSparsity::nz(i, j)) D[j] = r == i ? Di[j] : D[j];
    }
  }

  DEV void jacobian(const float (&x)[N], const float (&u)[M], float (&D)[N][N + M]) const {
#pragma unroll
    for (int r = 0; r < N; ++r) jac_row(r, x, u, D[r]);
  }
};
}  // namespace dilqr
