// tu_models.hip — dynamics, Jacobians, rollouts, linearisation, standalone pnqp,
// the quirk du-norm; the library version and build id.
#include "dilqr_common.h"

namespace dilqr {

// ============================================================ model kernels
template <class Model>
__global__ void __launch_bounds__(kBlock) k_dynamics(int N, const float* __restrict__ theta,
                                                     const float* __restrict__ x, const float* __restrict__ u,
                                                     float* __restrict__ out) {
  constexpr int n = Model::N, m = Model::M;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  Model md; md.load(theta);
  float xi[n], ui[m], o[n];
  ld(xi, x + (size_t)i * n); ld(ui, u + (size_t)i * m);
  md.forward(xi, ui, o);
  st(out + (size_t)i * n, o);
}

// Vector-Jacobian product of forward() (the sysid loss's backward,
// il_exp.py:338-347, which the reference gets from autograd): per row,
// g_theta = gout^T df/dtheta, g_x = gout^T df/dx, g_u = gout^T df/du, all at the
// CLAMPED u (df/du = 0 where the clamp is active, as autograd through
// torch.clamp gives).  g_theta is written per row; the caller sums.
template <class Model>
__global__ void __launch_bounds__(kBlock) k_dynamics_vjp(int N, const float* __restrict__ theta,
                                                         const float* __restrict__ x, const float* __restrict__ u,
                                                         const float* __restrict__ gout, float* __restrict__ gtheta,
                                                         float* __restrict__ gx, float* __restrict__ gu) {
  constexpr int n = Model::N, m = Model::M, p = Model::P;
  using D2 = typename D2Of<Model>::type;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  Model md; md.load(theta);
  float xi[n], ui[m], uc[m], go[n];
  ld(xi, x + (size_t)i * n); ld(ui, u + (size_t)i * m); ld(go, gout + (size_t)i * n);
#pragma unroll
  for (int a = 0; a < m; ++a) uc[a] = fminf(fmaxf(ui[a], -Model::ULIM), Model::ULIM);
  float D[n][n + m], Ft[n][p];
  md.jacobian(xi, uc, D);
  D2::f_theta(theta, xi, uc, Ft);
  float gt[p], gxi[n], gui[m];
#pragma unroll
  for (int k = 0; k < p; ++k) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < n; ++r) s += go[r] * Ft[r][k];
    gt[k] = s;
  }
#pragma unroll
  for (int j = 0; j < n + m; ++j) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < n; ++r) s += go[r] * D[r][j];
    if (j < n) gxi[j] = s;
    else gui[j - n] = (ui[j - n] >= -Model::ULIM && ui[j - n] <= Model::ULIM) ? s : 0.f;
  }
  st(gtheta + (size_t)i * p, gt);
  if (gx) st(gx + (size_t)i * n, gxi);
  if (gu) st(gu + (size_t)i * m, gui);
}

template <class Model>
__global__ void __launch_bounds__(kBlock) k_linear_dyn(int N, const float* __restrict__ theta,
                                                       const float* __restrict__ x, const float* __restrict__ u,
                                                       float* __restrict__ Dout) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  Model md; md.load(theta);
  float xi[n], ui[m], D[n][d];
  ld(xi, x + (size_t)i * n); ld(ui, u + (size_t)i * m);
  md.jacobian(xi, ui, D);
  st2(Dout + (size_t)i * n * d, D);
}

// util.get_traj (util.py:104-127)
template <class Model>
__global__ void __launch_bounds__(kBlock) k_rollout(int T, int B, const float* __restrict__ theta,
                                                    const float* __restrict__ x_init, const float* __restrict__ u,
                                                    float* __restrict__ x_out) {
  constexpr int n = Model::N, m = Model::M;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Model md; md.load(theta);
  float xt[n];
  ld(xt, x_init + (size_t)b * n);
  st(x_out + (size_t)b * n, xt);
  for (int t = 0; t < T - 1; ++t) {
    float ut[m], xn[n];
    ld(ut, u + ((size_t)t * B + b) * m);
    md.forward(xt, ut, xn);
#pragma unroll
    for (int i = 0; i < n; ++i) xt[i] = xn[i];
    st(x_out + ((size_t)(t + 1) * B + b) * n, xt);
  }
}

// LinDx rollout: x_{t+1} = F_t [x_t;u_t] + f_t
template <int n, int m>
__global__ void __launch_bounds__(kBlock) k_rollout_lin(int T, int B, const float* __restrict__ F,
                                                        const float* __restrict__ f, const float* __restrict__ x_init,
                                                        const float* __restrict__ u, float* __restrict__ x_out) {
  constexpr int d = n + m;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float xt[n];
  ld(xt, x_init + (size_t)b * n);
  st(x_out + (size_t)b * n, xt);
  for (int t = 0; t < T - 1; ++t) {
    size_t tb = (size_t)t * B + b;
    float ut[m], Ft[n][d], xn[n];
    ld(ut, u + tb * m); ld2(Ft, F + tb * n * d);
#pragma unroll
    for (int i = 0; i < n; ++i) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < n; ++j) s += Ft[i][j] * xt[j];
#pragma unroll
      for (int j = 0; j < m; ++j) s += Ft[i][n + j] * ut[j];
      xn[i] = s;
    }
    if (f) {
      float ft[n]; ld(ft, f + tb * n);
#pragma unroll
      for (int i = 0; i < n; ++i) xn[i] += ft[i];
    }
#pragma unroll
    for (int i = 0; i < n; ++i) xt[i] = xn[i];
    st(x_out + ((size_t)(t + 1) * B + b) * n, xt);
  }
}

// MPC.linearize_dynamics ANALYTIC (mpc_explicit.py:516-546)
template <class Model>
__global__ void __launch_bounds__(kBlock) k_linearize(int T, int B, const float* __restrict__ theta,
                                                      const float* __restrict__ x, const float* __restrict__ u,
                                                      float* __restrict__ F, float* __restrict__ f) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)(T - 1) * B) return;
  Model md; md.load(theta);
  float xi[n], ui[m], D[n][d], xn[n], fo[n];
  ld(xi, x + (size_t)i * n); ld(ui, u + (size_t)i * m);
  md.forward(xi, ui, xn);
  md.jacobian(xi, ui, D);
#pragma unroll
  for (int r = 0; r < n; ++r) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < n; ++j) s += D[r][j] * xi[j];
#pragma unroll
    for (int j = 0; j < m; ++j) s += D[r][n + j] * ui[j];
    fo[r] = xn[r] - s;
  }
  st2(F + (size_t)i * n * d, D);
  st(f + (size_t)i * n, fo);
}

// ============================================================ quirk du-norm
__global__ void __launch_bounds__(kBlock) k_quirk_norm(int TM, int B, const float* __restrict__ du_sq,
                                                       float* __restrict__ out) {
  int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  float s = 0.f;
  const float* p = du_sq + (size_t)r * TM;
  for (int i = 0; i < TM; ++i) s += p[i];
  out[r] = sqrtf(s);
}

// ============================================================ standalone pnqp
// pnqp.py:5-82 for one problem per lane (the reference at batch size 1):
// min 1/2 x^T H x + q^T x, lower <= x <= upper, warm start x_init (nullable:
// the unconstrained solve, pnqp.py:14-19).  Outputs x, the free mask If, the
// masked matrix H_ of the last iteration (pnqp.py:44-48) and the iteration
// index at exit (pnqp.py:59 / 82).
template <int m>
__global__ void __launch_bounds__(kBlock) k_pnqp(int B, const float* __restrict__ H, const float* __restrict__ q,
                                                 Bounds bd, const float* __restrict__ x_init, float* __restrict__ x,
                                                 float* __restrict__ If, float* __restrict__ Hf_out,
                                                 int* __restrict__ n_iter) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float Hr[m][m], qr[m], lb[m], ub[m], xr[m], Ir[m], Hf[m][m];
  ld2(Hr, H + (size_t)b * m * m);
  ld(qr, q + (size_t)b * m);
#pragma unroll
  for (int a = 0; a < m; ++a) {
    lb[a] = bound_lo(bd, (long long)b * m + a);
    ub[a] = bound_hi(bd, (long long)b * m + a);
    xr[a] = x_init ? x_init[(size_t)b * m + a] : 0.f;
  }
  const int it = pnqp<m>(Hr, qr, lb, ub, x_init != nullptr, xr, Ir, Hf);
  st(x + (size_t)b * m, xr);
  if (If) st(If + (size_t)b * m, Ir);
  if (Hf_out) st2(Hf_out + (size_t)b * m * m, Hf);
  if (n_iter) n_iter[b] = it;
}

}  // namespace dilqr

using namespace dilqr;

extern "C" {

int dilqr_version(void) { return 9; }

// hash of csrc/ + include/dilqr.h at build time (Makefile); _native checks it
// against the tree so a stale prebuilt library cannot be loaded silently
const char* dilqr_build_id(void) { return DILQR_BUILD_ID; }

int dilqr_model_num_ctrl(int model) {
  switch (model) {
    case DILQR_MODEL_PENDULUM: return Pendulum::M;
    case DILQR_MODEL_CARTPOLE: return Cartpole::M;
    case DILQR_MODEL_ROCKET: return Rocket::M;
    case DILQR_MODEL_PENDULUM_COMPLEX: return PendulumComplex::M;
    default: return -1;
  }
}

int dilqr_model_num_params(int model) {
  switch (model) {
    case DILQR_MODEL_PENDULUM: return Pendulum::P;
    case DILQR_MODEL_CARTPOLE: return Cartpole::P;
    case DILQR_MODEL_ROCKET: return Rocket::P;
    case DILQR_MODEL_PENDULUM_COMPLEX: return PendulumComplex::P;
    default: return -1;
  }
}

int dilqr_dynamics_f32(int model, int N, const float* theta, const float* x, const float* u, float* out,
                       void* stream) {
  if (N < 0 || !theta || !x || !u || !out) return DILQR_E_ARG;
  if (N == 0) return 0;
  MODEL_SWITCH(model, (k_dynamics<MD><<<grid_for(N), kBlock, 0, S(stream)>>>(N, theta, x, u, out)));
  return launched();
}

int dilqr_dynamics_vjp_f32(int model, int N, const float* theta, const float* x, const float* u, const float* gout,
                           float* gtheta, float* gx, float* gu, void* stream) {
  if (N < 0 || !theta || !x || !u || !gout || !gtheta) return DILQR_E_ARG;
  if (N == 0) return 0;
  MODEL_SWITCH_TPP_D2(model, (k_dynamics_vjp<MD><<<grid_for(N), kBlock, 0, S(stream)>>>(N, theta, x, u, gout, gtheta,
                                                                                       gx, gu)));
  return launched();
}

int dilqr_linear_dyn_f32(int model, int N, const float* theta, const float* x, const float* u, float* D,
                         void* stream) {
  if (N < 0 || !theta || !x || !u || !D) return DILQR_E_ARG;
  if (N == 0) return 0;
  MODEL_SWITCH(model, (k_linear_dyn<MD><<<grid_for(N), kBlock, 0, S(stream)>>>(N, theta, x, u, D)));
  return launched();
}

int dilqr_rollout_f32(int model, int n, int m, int T, int B, const float* theta, const float* F, const float* f,
                      const float* x_init, const float* u, float* x_out, void* stream) {
  if (T < 1 || B < 0 || !x_init || !u || !x_out) return DILQR_E_ARG;
  if (!al16(F) || !al16(f) || !al16(x_init) || !al16(u) || !al16(x_out)) return DILQR_E_ARG;
  if (B == 0) return 0;
  if (model == DILQR_MODEL_LINDX) {
    if (!F && T > 1) return DILQR_E_ARG;
#define X(N_, M_) \
    if (n == N_ && m == M_) { k_rollout_lin<N_, M_><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, F, f, x_init, u, x_out); return launched(); }
    DILQR_FOR_ALL_SHAPES(X)
#undef X
    return DILQR_E_SHAPE;
  }
  if (!theta) return DILQR_E_ARG;
  MODEL_SWITCH(model, (k_rollout<MD><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, theta, x_init, u, x_out)));
  return launched();
}

int dilqr_linearize_f32(int model, int T, int B, const float* theta, const float* x, const float* u, float* F,
                        float* f, void* stream) {
  if (T < 1 || B < 0 || !theta || !x || !u || !F || !f) return DILQR_E_ARG;
  long long N = (long long)(T - 1) * B;
  if (N == 0) return 0;
  MODEL_SWITCH(model, (k_linearize<MD><<<grid_for(N), kBlock, 0, S(stream)>>>(T, B, theta, x, u, F, f)));
  return launched();
}

int dilqr_pnqp_f32(int m, int B, const float* H, const float* q, dilqr_bounds bounds, const float* x_init, float* x,
                   float* If, float* Hfree, int* n_iter, void* stream) {
  if (m < 1 || B < 0 || !H || !q || !x) return DILQR_E_ARG;
  if (bounds.mode == DILQR_BOUNDS_NONE || bad_bounds(bounds)) return DILQR_E_ARG;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  switch (m) {
    case 1: k_pnqp<1><<<grid_for(B), kBlock, 0, S(stream)>>>(B, H, q, bd, x_init, x, If, Hfree, n_iter); break;
    case 2: k_pnqp<2><<<grid_for(B), kBlock, 0, S(stream)>>>(B, H, q, bd, x_init, x, If, Hfree, n_iter); break;
    case 3: k_pnqp<3><<<grid_for(B), kBlock, 0, S(stream)>>>(B, H, q, bd, x_init, x, If, Hfree, n_iter); break;
    case 4: k_pnqp<4><<<grid_for(B), kBlock, 0, S(stream)>>>(B, H, q, bd, x_init, x, If, Hfree, n_iter); break;
    default: return DILQR_E_SHAPE;
  }
  return launched();
}

int dilqr_quirk_norm_f32(int T, int m, int B, const float* du_sq, float* out, void* stream) {
  if (T < 1 || m < 1 || B < 0 || !du_sq || !out) return DILQR_E_ARG;
  if (B == 0) return 0;
  k_quirk_norm<<<grid_for(B), kBlock, 0, S(stream)>>>(T * m, B, du_sq, out);
  return launched();
}

}  // extern "C"
