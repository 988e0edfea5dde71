// dilqr_models.h — device dynamics of the reference's env_dx models.
//
// forward(): op-for-op restatement of the reference forward (contraction off,
// so every product/sum rounds like the reference's eager fp32 ops).
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
  float g, m, l;
  DEV void load(const float* __restrict__ th) { g = th[0]; m = th[1]; l = th[2]; }

  struct FSparsity {      // pendulum.py:448-474: row 2 has a structural zero at cos
    static constexpr bool nz(int i, int j) { return !(i == 2 && j == 0); }
  };

  // pendulum.py:60-95
  DEV void forward(const float (&x)[N], const float (&u)[M], float (&o)[N]) const {
#pragma clang fp contract(off)
    float uu = fminf(fmaxf(u[0], -2.0f), 2.0f);
    float c = x[0], s = x[1], dth = x[2];
    float th = atan2f(s, c);
    float a = (-3.0f * g) / (2.0f * l) * (-s);
    float b = (3.0f * uu) / (m * (l * l));
    float newdth = dth + DT * (a + b);
    float newth = th + newdth * DT;
    o[0] = cosf(newth);
    o[1] = sinf(newth);
    o[2] = newdth;
  }

  // pendulum.py:444-475
  DEV void jacobian(const float (&x)[N], const float (&u)[M], float (&D)[N][N + M]) const {
    float c = x[0], s = x[1], dth = x[2], uu = u[0];
    float r2 = c * c + s * s;
    float kg = 3.0f * g / (2.0f * l);
    float ku = 3.0f / (l * l * m);
    float newth = DT * (DT * (kg * s + ku * uu) + dth) + atan2f(s, c);
    float sn = sinf(newth), cs = cosf(newth);
    float dc = -s / r2;                 // d newth / d cos
    float ds = c / r2 + DT * DT * kg;   // d newth / d sin
    float dw = DT;                      // d newth / d dth
    float du = DT * DT * ku;            // d newth / d u
    D[0][0] = -sn * dc; D[0][1] = -sn * ds; D[0][2] = -sn * dw; D[0][3] = -sn * du;
    D[1][0] = cs * dc;  D[1][1] = cs * ds;  D[1][2] = cs * dw;  D[1][3] = cs * du;
    D[2][0] = 0.f;      D[2][1] = DT * kg;  D[2][2] = 1.f;      D[2][3] = DT * ku;
  }
};

// ---------------------------------------------------------------- cartpole
// env_dx/cartpole.py: x = [x, dx, cos th, sin th, dth], u = [force],
// theta = (g, m_cart, m_pole, l)
struct Cartpole {
  static constexpr int N = 5, M = 1, P = 4;
  static constexpr float DT = 0.05f;
  float g, mc, mp, l;
  DEV void load(const float* __restrict__ th) { g = th[0]; mc = th[1]; mp = th[2]; l = th[3]; }

  // structural nonzeros of jacobian() (cartpole.py:802-838): rows x, dx, cos, sin, dth
  struct FSparsity {
    static constexpr bool nz(int i, int j) {
      return i == 0 ? (j <= 1) : i == 1 ? (j >= 1) : i == 4 ? (j >= 2) : (j >= 2 && j <= 4);
    }
  };

  // cartpole.py:64-97
  DEV void forward(const float (&s_)[N], const float (&u)[M], float (&o)[N]) const {
#pragma clang fp contract(off)
    float total_mass = mp + mc;
    float pml = mp * l;
    float uu = fminf(fmaxf(u[0], -100.0f), 100.0f);
    float x = s_[0], dx = s_[1], c = s_[2], s = s_[3], dth = s_[4];
    float th = atan2f(s, c);
    float cart_in = (uu + (pml * (dth * dth)) * s) / total_mass;
    float th_acc = (g * s - c * cart_in) / (l * (4.0f / 3.0f - (mp * (c * c)) / total_mass));
    float xacc = cart_in - ((pml * th_acc) * c) / total_mass;
    o[0] = x + DT * dx;
    o[1] = dx + DT * xacc;
    float th2 = th + DT * dth;
    o[2] = cosf(th2);
    o[3] = sinf(th2);
    o[4] = dth + DT * th_acc;
  }

  // cartpole.py:790-839 (closed form of the same derivative)
  DEV void jacobian(const float (&s_)[N], const float (&u)[M], float (&D)[N][N + M]) const {
    float c = s_[2], s = s_[3], w = s_[4], uu = u[0];
    float Mt = mc + mp, iM = 1.0f / Mt;
    float pml = mp * l;
    float A = uu + pml * w * w * s;                 // cart_in * M
    float den = l * (4.0f / 3.0f - mp * c * c * iM);
    float iden = 1.0f / den;
    float num = g * s - c * A * iM;
    float tha = num * iden;                         // th_acc
    // partials of A, den, num wrt (c, s, w, u)
    float A_s = pml * w * w, A_w = 2.0f * pml * w * s;
    float den_c = -2.0f * l * mp * c * iM;
    float num_c = -A * iM, num_s = g - c * A_s * iM, num_w = -c * A_w * iM, num_u = -c * iM;
    float tha_c = (num_c - tha * den_c) * iden;
    float tha_s = num_s * iden, tha_w = num_w * iden, tha_u = num_u * iden;
    float k = pml * iM;
    float xa_c = -k * (tha_c * c + tha);
    float xa_s = A_s * iM - k * tha_s * c;
    float xa_w = A_w * iM - k * tha_w * c;
    float xa_u = iM - k * tha_u * c;
    float ir2 = 1.0f / (c * c + s * s);
    float th2 = DT * w + atan2f(s, c);
    float sn = sinf(th2), cs = cosf(th2);
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

namespace dilqr {
// Second-order terms of each model for the implicit backward.  XX00_ZERO: the
// reference's x_grad_xtm1 has a 0 where d x_{t+1}/d x_t is 1 (cartpole.py:666).
template <class Model> struct D2Of;
template <> struct D2Of<Pendulum> { using type = gen::PendulumD2; static constexpr bool XX00_ZERO = false; };
template <> struct D2Of<Cartpole> { using type = gen::CartpoleD2; static constexpr bool XX00_ZERO = true; };
}  // namespace dilqr
