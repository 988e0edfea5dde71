// dilqr_kernels.hip — HIP kernels + C-ABI of the batched differentiable iLQR
// hot path, gfx950.  See include/dilqr.h for the contract and DESIGN.md for the
// data layout / roofline of each kernel.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dilqr_device.h"
#include "dilqr_models.h"

namespace dilqr {

constexpr int kBlock = 64;   // one wave per workgroup: 64 problems, 4 workgroups per CU
                             // at B=65536, freely distributed over the 8 XCDs.
constexpr size_t kLdsPerCU = 160 * 1024;   // CDNA4 LDS per CU
#ifndef DILQR_NO_LDS_GAINS
#define DILQR_NO_LDS_GAINS 0
#endif
constexpr bool kNoLdsGains = DILQR_NO_LDS_GAINS;   // test builds: gain records in HBM always

static inline int grid_for(long long n) { return (int)((n + kBlock - 1) / kBlock); }

// Diagnostic build only (-DDILQR_STAMPS, tools/phase_stamps.py; never the
// shipped library): lane 0 of every wave of the fused MPC iteration writes
// s_memtime at its phase boundaries (kernel entry, after the stop-rule
// prologue, after the sweep, after the line search, exit) and s_memrealtime
// at entry/exit into a buffer of its own that nothing else reads.
#ifdef DILQR_STAMPS
constexpr int kStampSlots = 8, kStampWaves = 4096;
__device__ unsigned long long g_stamps[kStampWaves * kStampSlots];
#define DILQR_STAMP(k)                                                                     \
  do {                                                                                     \
    const unsigned w_ = (blockIdx.x * blockDim.x + threadIdx.x) / 64u;                     \
    if ((threadIdx.x & 63u) == 0 && w_ < (unsigned)kStampWaves)                             \
      g_stamps[w_ * kStampSlots + (k)] = (k) >= 6 ? __builtin_amdgcn_s_memrealtime()       \
                                                  : __builtin_amdgcn_s_memtime();          \
  } while (0)
#else
#define DILQR_STAMP(k) do {} while (0)
#endif

DEV float bound_lo(const Bounds& bd, long long idx) { return bd.mode == DILQR_BOUNDS_TENSOR ? bd.lo_t[idx] : bd.lo; }
DEV float bound_hi(const Bounds& bd, long long idx) { return bd.mode == DILQR_BOUNDS_TENSOR ? bd.hi_t[idx] : bd.hi; }
}  // namespace dilqr

#include "dilqr_group.h"   // 16-lanes-per-problem kernels (rocket-sized d <= 16)
#include "dilqr_implicit_group.h"   // the implicit backward for those models

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

// ============================================================ Riccati sweep
// lqr_backward (lqr_step_explicit.py:54-162) with the delta-space c_back of
// 630-636 fused.  F [T-1,B,n,d] is read from HBM.
template <int n, int m, int MODE>
__global__ void __launch_bounds__(kBlock) k_lqr_backward(int T, int B, const float* __restrict__ C,
                                                         const float* __restrict__ c, const float* __restrict__ x,
                                                         const float* __restrict__ u, const float* __restrict__ F,
                                                         Bounds bd, const unsigned char* __restrict__ zI,
                                                         float* __restrict__ K, float* __restrict__ k,
                                                         int* __restrict__ n_qp) {
  constexpr int d = n + m;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  RiccatiState<n, m> rs;
  rs.init();
  bool symsofar = true;
  // per-step inputs, software-pipelined one step ahead (see ilqr_problem)
  struct In {
    float C[d][d], c[d], F[n][d], x[n], u[m];
    DEV void load(const float* Cp, const float* cp, const float* Fp, const float* xp, const float* up, int t, int T,
                  int B, int b) {
      size_t tb = (size_t)t * B + b;
      ld2(C, Cp + tb * d * d);
      ld(c, cp + tb * d);
      size_t tf = (size_t)(t < T - 1 ? t : (T > 1 ? T - 2 : 0)) * B + b;   // F[T-1] does not exist
      if (T > 1) ld2(F, Fp + tf * n * d);
      if (xp) ld(x, xp + tb * n);
      if (up) ld(u, up + tb * m);
    }
  } cur, nxt;
#pragma unroll
  for (int i = 0; i < n; ++i) cur.x[i] = nxt.x[i] = 0.f;
#pragma unroll
  for (int a = 0; a < m; ++a) cur.u[a] = nxt.u[a] = 0.f;
  cur.load(C, c, F, x, u, T - 1, T, B, b);
  for (int t = T - 1; t >= 0; --t) {
    size_t tb = (size_t)t * B + b;
    nxt.load(C, c, F, x, u, t > 0 ? t - 1 : 0, T, B, b);
    float cb[d];
#pragma unroll
    for (int i = 0; i < d; ++i) cb[i] = cur.c[i];
    if (x) {
      float tau[d];
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = cur.x[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = cur.u[a];
#pragma unroll
      for (int i = 0; i < d; ++i) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < d; ++j) s += cur.C[i][j] * tau[j];
        cb[i] = s + cb[i];
      }
    }
    if (t == T - 1) {
#pragma unroll
      for (int i = 0; i < n; ++i)
#pragma unroll
        for (int j = 0; j < d; ++j) cur.F[i][j] = 0.f;
    }
    float zIt[m], lb[m], ub[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      zIt[a] = 0.f; lb[a] = 0.f; ub[a] = 0.f;
      if constexpr (MODE == GAIN_ZERO_I) zIt[a] = zI[tb * m + a] ? 1.f : 0.f;
      if constexpr (MODE == GAIN_BOX) {
        lb[a] = bound_lo(bd, tb * m + a) - cur.u[a];
        ub[a] = bound_hi(bd, tb * m + a) - cur.u[a];
      }
    }
    float Kt[m][n], kt[m];
    symsofar &= bitwise_symmetric(cur.C);              // the fused sweep's rule (RiccatiState SYM)
    if (symsofar) rs.template step<MODE, DenseF, false, true>(cur.C, cb, cur.F, zIt, lb, ub, Kt, kt);
    else rs.template step<MODE>(cur.C, cb, cur.F, zIt, lb, ub, Kt, kt);
    st2(K + tb * m * n, Kt);
    st(k + tb * m, kt);
    cur = nxt;
  }
  if (n_qp) n_qp[b] = rs.n_qp;
}

// ============================================================ forward / line search
// lqr_forward (lqr_step_explicit.py:166-263), one problem per lane, the batch's
// `while any(cost > old_cost)` loop evaluated per problem (each problem's alpha
// depends only on its own cost, so this is the reference's result).
struct NoModel {};

template <int n, int m, class Model>
struct Dyn {
  Model md;
  const float* F;
  const float* f;
  int B;
  DEV void step(int t, int b, const float (&x)[n], const float (&uu)[m], float (&o)[n]) const {
    if constexpr (std::is_same_v<Model, NoModel>) {
      size_t tb = (size_t)t * B + b;
      float Ft[n][n + m];
      ld2(Ft, F + tb * n * (n + m));
#pragma unroll
      for (int i = 0; i < n; ++i) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Ft[i][j] * x[j];
#pragma unroll
        for (int j = 0; j < m; ++j) s += Ft[i][n + j] * uu[j];
        o[i] = s;
      }
      if (f) {
        float ft[n]; ld(ft, f + tb * n);
#pragma unroll
        for (int i = 0; i < n; ++i) o[i] += ft[i];
      }
    } else {
      md.forward(x, uu, o);
    }
  }
};

// One rollout pass with step size alpha.  Gains come from (K,k) [T,B,m,n]/[T,B,m]
// (GREC == 0) or from the fused kernel's per-lane gain records (GREC floats per
// (t,b): K, k, obj_t of the current trajectory).  Returns the new cost; if
// old_cost_out != nullptr it also returns the current trajectory's cost summed
// in time order from the records.
template <int n, int m, int GREC, class DynT>
DEV float forward_pass(const DynT& dyn, int T, int B, int b, float alpha, const float* __restrict__ x_init,
                       const float* __restrict__ C, const float* __restrict__ c, const float* __restrict__ x,
                       const float* __restrict__ u, const float* __restrict__ K, const float* __restrict__ k,
                       const float* __restrict__ grec, const Bounds& bd, const unsigned char* __restrict__ zI,
                       float* __restrict__ x_out, float* __restrict__ u_out, float* __restrict__ du_sq,
                       float* old_cost_out) {
  constexpr int d = n + m;
  float xn[n], dx[n];
  ld(xn, x_init + (size_t)b * n);
#pragma unroll
  for (int i = 0; i < n; ++i) dx[i] = 0.f;
  st(x_out + (size_t)b * n, xn);
  float cost = 0.f, oldc = 0.f;
  for (int t = 0; t < T; ++t) {
    size_t tb = (size_t)t * B + b;
    float Kt[m][n], kt[m], ut[m];
    if constexpr (GREC > 0) {
      float g[GREC];
      ld(g, grec + tb * GREC);
#pragma unroll
      for (int a = 0; a < m; ++a) {
#pragma unroll
        for (int j = 0; j < n; ++j) Kt[a][j] = g[a * n + j];
        kt[a] = g[m * n + a];
      }
      oldc += g[m * n + m];
    } else {
      ld2(Kt, K + tb * m * n);
      ld(kt, k + tb * m);
    }
    ld(ut, u + tb * m);
    float nu[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < n; ++j) s += Kt[a][j] * dx[j];
      nu[a] = (s + ut[a]) + alpha * kt[a];
      if (zI && zI[tb * m + a]) nu[a] = 0.f;
      if (bd.mode != DILQR_BOUNDS_NONE) nu[a] = eclamp(nu[a], bound_lo(bd, tb * m + a), bound_hi(bd, tb * m + a));
    }
    st(u_out + tb * m, nu);
    if (du_sq) {
#pragma unroll
      for (int a = 0; a < m; ++a) {
        float e = ut[a] - nu[a];
        du_sq[((size_t)t * m + a) * B + b] = e * e;
      }
    }
    float Ct[d][d], ct[d], tau[d];
    ld2(Ct, C + tb * d * d);
    ld(ct, c + tb * d);
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xn[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = nu[a];
    cost += quad_cost(Ct, ct, tau);
    if (t < T - 1) {
      float xnext[n], xcur[n];
      dyn.step(t, b, xn, nu, xnext);
      ld(xcur, x + (tb + B) * n);
#pragma unroll
      for (int i = 0; i < n; ++i) {
        dx[i] = xnext[i] - xcur[i];
        xn[i] = xnext[i];
      }
      st(x_out + (tb + B) * n, xn);
    }
  }
  if (old_cost_out) *old_cost_out = oldc;
  return cost;
}

// The current trajectory's cost (lqr_step_explicit.py:171), formed and summed
// exactly as the fused iteration forms it inside its backward sweep (stage
// costs as tau . (C tau) + c . tau, summed over t = T-1..0), so the fused and
// unfused pipelines take the same line-search decisions bit for bit.
template <int n, int m>
DEV float traj_cost(int T, int B, int b, const float* __restrict__ C, const float* __restrict__ c,
                    const float* __restrict__ x, const float* __restrict__ u) {
  constexpr int d = n + m;
  float cost = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    size_t tb = (size_t)t * B + b;
    float Ct[d][d], ct[d], tau[d], xt[n], ut[m], Ctau[d];
    ld2(Ct, C + tb * d * d); ld(ct, c + tb * d); ld(xt, x + tb * n); ld(ut, u + tb * m);
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
    cost += quad_cost(Ct, ct, tau, Ctau);
  }
  return cost;
}

template <int n, int m, class Model>
__global__ void __launch_bounds__(kBlock) k_lqr_forward(int T, int B, const float* __restrict__ theta,
                                                        const float* __restrict__ F, const float* __restrict__ f,
                                                        const float* __restrict__ x_init, const float* __restrict__ C,
                                                        const float* __restrict__ c, const float* __restrict__ x,
                                                        const float* __restrict__ u, const float* __restrict__ K,
                                                        const float* __restrict__ k, Bounds bd,
                                                        const unsigned char* __restrict__ zI, float decay, int max_ls,
                                                        float* __restrict__ x_out, float* __restrict__ u_out,
                                                        float* __restrict__ cost_out, float* __restrict__ du_sq,
                                                        float* __restrict__ alpha_out,
                                                        const float* __restrict__ old_cost_in) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Dyn<n, m, Model> dyn;
  if constexpr (!std::is_same_v<Model, NoModel>) dyn.md.load(theta);
  dyn.F = F; dyn.f = f; dyn.B = B;
  // lqr_step_explicit.py:171, or the caller's value of the same cost (an MPC
  // loop passes what its previous line search computed for this trajectory)
  const float old_cost = old_cost_in ? old_cost_in[b] : traj_cost<n, m>(T, B, b, C, c, x, u);
  float alpha = 1.f, cost = 0.f;
  for (int ls = 0; ls < max_ls; ++ls) {
    cost = forward_pass<n, m, 0>(dyn, T, B, b, alpha, x_init, C, c, x, u, K, k, nullptr, bd, zI, x_out, u_out,
                                 ls == 0 ? du_sq : nullptr, nullptr);
    if (!(cost > old_cost) || ls == max_ls - 1) break;
    alpha *= decay;                                             // lqr_step_explicit.py:249
  }
  cost_out[b] = cost;
  if (alpha_out) alpha_out[b] = alpha;                          // 254: the last pass's alpha
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

// ============================================================ fused iLQR iteration
// One MPC iteration body (mpc_explicit.py:249-263) for ONE problem (this lane):
// linearise at the current trajectory on the fly, Riccati sweep (+pnqp), the
// current cost, and the line-search rollout.  F never touches HBM; K/k go to
// per-lane gain records (LDS in the MPC kernel) that the rollout re-reads.
//
// Latency: at B=65536 there is one wave per SIMD, so every loop software-
// pipelines its loads one step ahead in registers (the step t-1 / t+1 inputs
// are in flight while step t computes).
// Private workspaces of per-(t,b) values the kernel re-reads column by column
// (gain records in HBM, the packed cost copy) are component-major: element j
// of record (t,b) is at [(t*K + j)*B + b] in float4/float2/float planes, so a
// wave's 64 lanes touch one contiguous run per access.  The MPC trajectory
// slots hold whole [x_t; u_t] records per lane instead (TRAJ_REC, below):
// fewer, wider accesses where the count of memory instructions, not bytes,
// is what the one-wave-per-SIMD kernel pays for.
// records of K floats stored as column planes of the widest vector loads:
// K/4 float4 planes, then a float2 plane if K%4 >= 2, then a float plane if K
// is odd (plane q of width w: w*[(t*nq + q)*B + b] floats from its base).
// Fewer, wider load instructions than K scalar planes (measured: 27 dword
// planes ran the fused kernel 8% slower than 7 float4 planes).
template <int K>
struct SoaRec {
  static constexpr int Q4 = K / 4, R2 = (K % 4) >= 2 ? 1 : 0, R1 = K % 2;
  static DEV size_t off2(int T, int B) { return (size_t)T * B * Q4 * 4; }
  static DEV size_t off1(int T, int B) { return off2(T, B) + (size_t)T * B * 2 * R2; }
  static DEV void load(float (&r)[K], const float* __restrict__ p, int T, size_t t, int B, int b) {
    const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int j = 0; j < Q4; ++j) {
      float4 v = q[(t * Q4 + j) * B + b];
      r[4 * j] = v.x; r[4 * j + 1] = v.y; r[4 * j + 2] = v.z; r[4 * j + 3] = v.w;
    }
    if constexpr (R2) {
      float2 v = reinterpret_cast<const float2*>(p + off2(T, B))[t * B + b];
      r[4 * Q4] = v.x; r[4 * Q4 + 1] = v.y;
    }
    if constexpr (R1) r[K - 1] = (p + off1(T, B))[t * B + b];
  }
  static DEV void store(float* __restrict__ p, const float (&r)[K], int T, size_t t, int B, int b) {
    float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
    for (int j = 0; j < Q4; ++j) q[(t * Q4 + j) * B + b] = make_float4(r[4 * j], r[4 * j + 1], r[4 * j + 2], r[4 * j + 3]);
    if constexpr (R2) reinterpret_cast<float2*>(p + off2(T, B))[t * B + b] = make_float2(r[4 * Q4], r[4 * Q4 + 1]);
    if constexpr (R1) (p + off1(T, B))[t * B + b] = r[K - 1];
  }
};

// Trajectory layouts of the fused kernels:
//  TRAJ_AOS — the caller's x [T,B,n] and u [T,B,m] (the reference's layout);
//  TRAJ_REC — the MPC slots of the thread-per-problem models: one record
//    [x_t; u_t] of d = n+m floats per (t, b), [T,B,d].  A lane moves its
//    record with two wide accesses (cartpole: dwordx4 + dwordx2) instead of d
//    dword accesses; the line search stores record t of each candidate once
//    both x_t and u_t are known.  (The earlier component-major slots took 13
//    dword stores per line-search step.)
constexpr int TRAJ_AOS = 0, TRAJ_REC = 1;

template <int TL, int n, int m>
DEV void ld_xu(float (&x)[n], float (&u)[m], const float* __restrict__ xp, const float* __restrict__ up, size_t t,
               int B, int b) {
  const size_t tb = t * B + b;
  if constexpr (TL == TRAJ_REC) {
    float r[n + m];
    // lane part and (uniform) step part of the address kept apart: the step's
    // offset is scalar arithmetic, the lane adds it with one 64-bit add
    ld(r, (xp + (size_t)b * (n + m)) + t * (size_t)B * (n + m));
#pragma unroll
    for (int i = 0; i < n; ++i) x[i] = r[i];
#pragma unroll
    for (int a = 0; a < m; ++a) u[a] = r[n + a];
  } else {
    ld(x, xp + tb * n);
    ld(u, up + tb * m);
  }
}

template <int TL, int n, int m>
DEV void st_xu(float* __restrict__ xp, float* __restrict__ up, const float (&x)[n], const float (&u)[m], size_t t,
               int B, int b) {
  const size_t tb = t * B + b;
  if constexpr (TL == TRAJ_REC) {
    float r[n + m];
#pragma unroll
    for (int i = 0; i < n; ++i) r[i] = x[i];
#pragma unroll
    for (int a = 0; a < m; ++a) r[n + a] = u[a];
    st(xp + tb * (n + m), r);
  } else {
    st(xp + tb * n, x);
    st(up + tb * m, u);
  }
}

// Where the fused kernels read the stage cost from: the caller's C [T,B,d,d] and
// c [T,B,d], or the solve's packed copy of a symmetric C, written by the solve's
// iteration 0: per (t,b) the diagonal of C, then c, then the strict upper
// triangle row-major (float4-column layout).  A problem whose C_t are all
// diagonal (every off-diagonal entry +0.0 bit for bit — the reference's own
// callers pass diag(q), il_env.py:159-162) reads only the leading 2d floats and
// holds literal zeros off the diagonal.  All variants fill the same full
// registers with the same values, so the arithmetic is identical.
template <int d>
struct CostFull {
  static constexpr bool kDiag = false;
  static constexpr bool kSym = false;      // symmetry is tested per step at run time
  const float* __restrict__ C;
  const float* __restrict__ c;
  DEV void load(float (&Cr)[d][d], float (&cr)[d], size_t t, int B, int b) const {
    const size_t tb = t * B + b;
    ld2(Cr, C + tb * d * d); ld(cr, c + tb * d);
  }
};

template <int d>
constexpr int packed_cost_floats() { return d * (d + 1) / 2 + d; }
// the diagonal-only read needs the leading 2d floats to be whole float4 planes
template <int d>
constexpr bool packed_diag_ok() { return (2 * d) % 4 == 0; }

// cost_sym[b] flags written by iteration 0.  kCostTinv: the packed record is
// the same, bit for bit, at every t (the reference's callers repeat one
// diag(q), p over the horizon: il_env.py:159-162, mpc_explicit.py:203-224)
constexpr unsigned char kCostSym = 1, kCostDiag = 2, kCostTinv = 4;

template <int d>
DEV void pack_cost(const float (&C)[d][d], const float (&c)[d], float (&buf)[packed_cost_floats<d>()], bool& sym,
                   bool& diag) {
  int k = 0;
#pragma unroll
  for (int i = 0; i < d; ++i) buf[k++] = C[i][i];
#pragma unroll
  for (int i = 0; i < d; ++i) buf[k++] = c[i];
#pragma unroll
  for (int i = 0; i < d; ++i)
#pragma unroll
    for (int j = i + 1; j < d; ++j) {
      sym &= __float_as_uint(C[i][j]) == __float_as_uint(C[j][i]);
      diag &= __float_as_uint(C[i][j]) == 0u && __float_as_uint(C[j][i]) == 0u;
      buf[k++] = C[i][j];
    }
}

// TINV: a time-invariant cost (flag kCostTinv) whose copy holds ONE record,
// t = T-1 (iteration 0 writes the others only once the cost changes over t);
// every step reads that record.
template <int d, bool DIAG = false, bool TINV = false>
struct CostPacked {
  static constexpr bool kDiag = DIAG;
  static constexpr bool kSym = true;
  const float* __restrict__ P;
  int T;
  DEV void load(float (&Cr)[d][d], float (&cr)[d], size_t t_, int B, int b) const {
    constexpr int PK = packed_cost_floats<d>();
    const size_t t = TINV ? (size_t)(T - 1) : t_;
    if constexpr (DIAG) {
      static_assert(packed_diag_ok<d>(), "diagonal read needs whole float4 planes");
      constexpr int Q4 = SoaRec<PK>::Q4;
      const float4* q = reinterpret_cast<const float4*>(P);
      float buf[2 * d];
#pragma unroll
      for (int j = 0; j < 2 * d / 4; ++j) {
        float4 v = q[(t * Q4 + j) * B + b];
        buf[4 * j] = v.x; buf[4 * j + 1] = v.y; buf[4 * j + 2] = v.z; buf[4 * j + 3] = v.w;
      }
      const float z = 0.f;
#pragma unroll
      for (int i = 0; i < d; ++i) {
#pragma unroll
        for (int j = 0; j < d; ++j) Cr[i][j] = z;
        Cr[i][i] = buf[i];
        cr[i] = buf[d + i];
      }
    } else {
      float buf[PK];
      SoaRec<PK>::load(buf, P, T, t, B, b);
      int k = 2 * d;
#pragma unroll
      for (int i = 0; i < d; ++i) {
        Cr[i][i] = buf[i];
        cr[i] = buf[d + i];
      }
#pragma unroll
      for (int i = 0; i < d; ++i)
#pragma unroll
        for (int j = i + 1; j < d; ++j) { Cr[i][j] = buf[k]; Cr[j][i] = buf[k]; ++k; }
    }
  }
};

// A diagonal cost that is the same at every t (flags kCostDiag | kCostTinv):
// its 2d floats are read once per problem (the copy's one record, t = T-1) or
// handed over from registers by the iteration that built the copy, and every
// step's load() hands out those registers — the values the per-step read would
// return, so the arithmetic is unchanged, with no HBM traffic for the cost.
template <int d>
struct CostDiagConst {
  static constexpr bool kDiag = true;
  static constexpr bool kSym = true;
  float dg[d], cc[d];
  DEV void init(const float* __restrict__ P, int T, int B, int b) {
    float Cr[d][d], cr[d];
    CostPacked<d, true>{P, T}.load(Cr, cr, T - 1, B, b);
#pragma unroll
    for (int i = 0; i < d; ++i) { dg[i] = Cr[i][i]; cc[i] = cr[i]; }
  }
  // from a packed record held in registers (diag, then c, ...)
  template <int PK>
  DEV void set(const float (&pk)[PK]) {
#pragma unroll
    for (int i = 0; i < d; ++i) { dg[i] = pk[i]; cc[i] = pk[d + i]; }
  }
  DEV void load(float (&Cr)[d][d], float (&cr)[d], size_t, int, int) const {
    const float z = 0.f;
#pragma unroll
    for (int i = 0; i < d; ++i) {
#pragma unroll
      for (int j = 0; j < d; ++j) Cr[i][j] = z;
      Cr[i][i] = dg[i];
      cr[i] = cc[i];
    }
  }
};

// The box bounds as a compile-time mode (DILQR_BOUNDS_*): scalar bounds are
// kernel arguments and per-(t,b) bounds are loaded with the step's other data,
// so no conditional load exists in the step (a conditional load makes the
// compiler drain every outstanding load, i.e. the prefetch, at the merge).
template <int m, int BM>
struct StepBounds {
  float lo[m], hi[m];
  DEV void load(const Bounds& bd, int t, int B, int b) {
    if constexpr (BM == DILQR_BOUNDS_TENSOR) {
      const size_t tb = (size_t)t * B + b;
      ld(lo, bd.lo_t + tb * m); ld(hi, bd.hi_t + tb * m);
    }
  }
  DEV float l(const Bounds& bd, int a) const {
    if constexpr (BM == DILQR_BOUNDS_TENSOR) return lo[a];
    else return bd.lo;
  }
  DEV float h(const Bounds& bd, int a) const {
    if constexpr (BM == DILQR_BOUNDS_TENSOR) return hi[a];
    else return bd.hi;
  }
};

template <int n, int m, int TL, int BM>
struct SweepIn {
  static constexpr int d = n + m;
  float C[d][d], c[d], x[n], u[m];
  StepBounds<m, BM> bnd;
  template <class CostT>
  DEV void load(const CostT& cs, const float* __restrict__ xp, const float* __restrict__ up, const Bounds& bd, int t,
                int B, int b) {
    cs.load(C, c, t, B, b); ld_xu<TL>(x, u, xp, up, t, B, b); bnd.load(bd, t, B, b);
  }
};

// Where the fused iteration keeps its gain records (K_t, k_t), written by the
// sweep and read back by the line search: a float4-column workspace in HBM
// (stride B, index b), or the workgroup's LDS (stride 64, index = lane) — each
// lane reads only what it wrote, so no barrier is involved.
struct GainRecs {
  float* p;
  int B, b;
};

// Inputs of line-search step t: gains, u_t and x_{t+1} of the current
// trajectory, the stage cost, bounds.  TRAJ_REC reads record t+1 whole (x_{t+1}
// and u_{t+1}); u_t is carried over from the previous step's record (the
// caller sets `u` of step 0 and copies `unext` forward).
template <int n, int m, int GREC, int TL, int BM>
struct FwdIn {
  static constexpr int d = n + m;
  float g[GREC], u[m], C[d][d], c[d], xnext[n], unext[m];
  StepBounds<m, BM> bnd;
  template <class CostT>
  DEV void load(const GainRecs& gr, const float* __restrict__ up, const CostT& cs,
                const float* __restrict__ xp, const Bounds& bd, int T, int t, int t1, int B, int b) {
    SoaRec<GREC>::load(g, gr.p, T, t, gr.B, gr.b); cs.load(C, c, t, B, b); bnd.load(bd, t, B, b);
    if constexpr (TL == TRAJ_REC) {
      ld_xu<TL>(xnext, unext, xp, up, t1, B, b);
    } else {
      ld(u, up + ((size_t)t * B + b) * m);
      ld(xnext, xp + ((size_t)t1 * B + b) * n);
    }
  }
};

// Prefetch distance of the fused sweep and line search, in steps.  At B =
// 65536 the one-problem-per-lane kernels run ONE wave per SIMD, so the only
// latency cover is the loads already in flight.  Two steps ahead measured no
// faster than one (0.0702 vs 0.0695 ms per iteration, config 2), so 1.
#ifndef DILQR_PF
#define DILQR_PF 1
#endif
constexpr int kPF = DILQR_PF;
#ifndef DILQR_PF_LS
#define DILQR_PF_LS 2
#endif
constexpr int kPFL = DILQR_PF_LS;                   // the line search's prefetch distance

// ---------------- forward: the line search (lqr_step_explicit.py:166-263).
// Pass p uses alpha_p = decay^p and is accepted when its cost <= old cost or
// it is the last pass.  Passes 2r and 2r+1 roll out TOGETHER (candidates A
// and B), sharing every load of the step; the first accepted candidate wins,
// which is exactly the sequential search.  A wave otherwise pays a whole
// second latency-bound pass whenever any of its 64 problems backtracks.
template <class Model, int BM, int TL, class CostT>
DEV int line_search(int T, int B, int b, const Model md, const float* __restrict__ x_init, const CostT& cs,
                    const float* __restrict__ x, const float* __restrict__ u, const Bounds& bd, float decay,
                    int max_ls, const GainRecs& ws, float* __restrict__ xa_out,
                    float* __restrict__ ua_out, float* __restrict__ xb_out, float* __restrict__ ub_out,
                    float* __restrict__ du_sq, float old_cost, float& cost_out, float& alpha_out,
                    bool b_in_gains = false) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  constexpr int GREC = m * n + m;                    // gain record: K, k (component-major)
  // b_in_gains (one round of candidates, gain records in LDS): candidate B's
  // record t overwrites gain record t, consumed by then (m = 1: both are d
  // floats), and only the problems whose B wins copy it to xb_out at the end —
  // instead of every problem writing both candidates to HBM.
  static_assert(TL != TRAJ_REC || GREC == d, "B records in the gain slots need m = 1");
  float alpha = 1.f, cost = 0.f;
  int win = 0;
  // Candidates A and B travel as the two components of f2 values: every
  // arithmetic step of the pair is one packed instruction (v_pk_fma_f32 /
  // v_pk_mul_f32 / v_pk_add_f32), and each component rounds exactly like the
  // scalar rollout of that candidate.  (Measured alternatives that were
  // slower on MI355X: unrolling the step loop twice over two prefetch buffers
  // and making every store unconditional, +3 us per iteration; unrolling it
  // three times with the three prefetch buffers rotating roles instead of
  // being copied — 13 fewer v_mov per step in the listing — +4 us.)
  for (int p = 0; p < max_ls; p += 2) {
    const bool twoB = p + 1 < max_ls;                       // uniform
    const float aA = alpha, aB = alpha * decay;
    const f2 al = {aA, aB};
    f2 xp[n], dp[n];
    {
      float x0[n];
      ld(x0, x_init + (size_t)b * n);
#pragma unroll
      for (int i = 0; i < n; ++i) { xp[i] = f2{x0[i], x0[i]}; dp[i] = f2{0.f, 0.f}; }
      if constexpr (TL == TRAJ_AOS) {
        st(xa_out + (size_t)b * n, x0);
        if (twoB) st(xb_out + (size_t)b * n, x0);
      }
    }
    f2 cp = {0.f, 0.f};
    // step s's record holds x_{s+1} of the current trajectory; indices clamp at T-1
    auto cl = [T](int s) { return s < T ? s : T - 1; };
    FwdIn<n, m, GREC, TL, BM> cur, n1, n2;
    cur.load(ws, u, cs, x, bd, T, 0, cl(1), B, b);
    if constexpr (TL == TRAJ_REC) {                     // u_0 from record 0
      float x0r[n];
      ld_xu<TL>(x0r, cur.u, x, u, 0, B, b);
    }
    if constexpr (kPFL >= 2) n1.load(ws, u, cs, x, bd, T, cl(1), cl(2), B, b);
    for (int t = 0; t < T; ++t) {
      if constexpr (kPFL >= 2) n2.load(ws, u, cs, x, bd, T, cl(t + 2), cl(t + 3), B, b);   // prefetch step t+2
      else n1.load(ws, u, cs, x, bd, T, cl(t + 1), cl(t + 2), B, b);                      // prefetch step t+1
      f2 nu[m];
#pragma unroll
      for (int a = 0; a < m; ++a) {
        f2 sp = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < n; ++j) sp += cur.g[a * n + j] * dp[j];
        nu[a] = (sp + cur.u[a]) + al * cur.g[m * n + a];
        if constexpr (BM != DILQR_BOUNDS_NONE) {
          const float lo = cur.bnd.l(bd, a), hi = cur.bnd.h(bd, a);
          nu[a] = f2{eclamp(nu[a].x, lo, hi), eclamp(nu[a].y, lo, hi)};
        }
      }
      {
        float ua[m], ub[m];
#pragma unroll
        for (int a = 0; a < m; ++a) { ua[a] = nu[a].x; ub[a] = nu[a].y; }
        if constexpr (TL == TRAJ_REC) {               // record t of each candidate: x_t, u_t
          float xa[n], xb[n];
#pragma unroll
          for (int i = 0; i < n; ++i) { xa[i] = xp[i].x; xb[i] = xp[i].y; }
          st_xu<TL>(xa_out, nullptr, xa, ua, t, B, b);
          if (twoB) {
            if (b_in_gains) {
              float rb[d];
#pragma unroll
              for (int i = 0; i < n; ++i) rb[i] = xb[i];
#pragma unroll
              for (int a = 0; a < m; ++a) rb[n + a] = ub[a];
              SoaRec<d>::store(ws.p, rb, T, t, ws.B, ws.b);
            } else {
              st_xu<TL>(xb_out, nullptr, xb, ub, t, B, b);
            }
          }
        } else {
          st(ua_out + ((size_t)t * B + b) * m, ua);
          if (twoB) st(ub_out + ((size_t)t * B + b) * m, ub);
        }
      }
      if (p == 0) {
#pragma unroll
        for (int a = 0; a < m; ++a) {
          float e = cur.u[a] - nu[a].x;
          du_sq[((size_t)t * m + a) * B + b] = e * e;
        }
      }
      f2 tau[d];
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = xp[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = nu[a];
      cp += quad_cost<d, CostT::kDiag>(cur.C, cur.c, tau);
      if (t < T - 1) {
        f2 xnext[n];
        md.forward(xp, nu, xnext);
        float xa[n], xb[n];
#pragma unroll
        for (int i = 0; i < n; ++i) {
          dp[i] = xnext[i] - cur.xnext[i];
          xp[i] = xnext[i];
          xa[i] = xnext[i].x;
          xb[i] = xnext[i].y;
        }
        if constexpr (TL == TRAJ_AOS) {
          st(xa_out + ((size_t)(t + 1) * B + b) * n, xa);
          if (twoB) st(xb_out + ((size_t)(t + 1) * B + b) * n, xb);
        }
      }
      if constexpr (TL == TRAJ_REC) {
#pragma unroll
        for (int a = 0; a < m; ++a) n1.u[a] = cur.unext[a];     // u_{t+1}
      }
      cur = n1;
      if constexpr (kPFL >= 2) n1 = n2;
    }
    const float cA = cp.x, cB = cp.y;
    if (!(cA > old_cost) || p == max_ls - 1) { cost = cA; alpha = aA; win = 0; break; }
    if (!(cB > old_cost) || p + 1 == max_ls - 1) { cost = cB; alpha = aB; win = 1; break; }
    alpha = aB * decay;                                     // lqr_step_explicit.py:249
  }
  if constexpr (TL == TRAJ_REC) {
    if (b_in_gains && win == 1) {                           // B won: its records from LDS to its slot
      for (int t = 0; t < T; ++t) {
        float rb[d], xt[n], ut[m];
        SoaRec<d>::load(rb, ws.p, T, t, ws.B, ws.b);
#pragma unroll
        for (int i = 0; i < n; ++i) xt[i] = rb[i];
#pragma unroll
        for (int a = 0; a < m; ++a) ut[a] = rb[n + a];
        st_xu<TL>(xb_out, nullptr, xt, ut, t, B, b);
      }
    }
  }
  cost_out = cost;
  alpha_out = alpha;
  return win;
}

// x, u (current trajectory) and the candidate outputs in layout TL; the gain
// records in ws and the packed cost are always float4-column.  ROLLOUT: x is a
// rollout of the model under u (the MPC slots are), so x_{t+1} = forward(x_t,
// u_t) bit for bit and models with kJacFromNext take part of the Jacobian from it.
// pack_out (iteration 0 of a solve): build the packed cost copy while the sweep
// reads C.  A time-invariant cost is stored as its t = T-1 record only (the
// records a later change of the cost proves necessary are written then, from
// the registers holding that record), and a time-invariant diagonal cost is
// handed to this iteration's line search in registers, so C is read once.
// PREV: the current trajectory's cost is prev_cost[b], the cost the previous
// MPC iteration's line search computed for it (the accepted candidate), so the
// sweep forms only C tau for c_back and not the stage costs again.
template <class Model, int BM, int TL, bool ROLLOUT, class CostT, bool PREV = false>
DEV int ilqr_problem(int T, int B, int b, const Model md, const float* __restrict__ x_init, const CostT& cs,
                     float* __restrict__ pack_out, unsigned char* __restrict__ sym_out, const float* __restrict__ x,
                     const float* __restrict__ u, const Bounds& bd, float decay, int max_ls,
                     const GainRecs& ws, float* __restrict__ xa_out, float* __restrict__ ua_out,
                     float* __restrict__ xb_out, float* __restrict__ ub_out, float* __restrict__ du_sq,
                     float& cost_out, float& alpha_out, bool b_in_gains = false,
                     const float* __restrict__ prev_cost = nullptr) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  constexpr int MODE = BM == DILQR_BOUNDS_NONE ? GAIN_UNC : GAIN_BOX;
  constexpr int GREC = m * n + m;                    // gain record: K, k (component-major)
  constexpr int PK = packed_cost_floats<d>();
  float old_cost = 0.f;                               // the current trajectory's cost, from the sweep
  if constexpr (PREV) old_cost = prev_cost[b];        // ... or from the previous line search
  bool sym = true, diag = true, tinv = true;
  bool symsofar = true;                               // C_t' bitwise symmetric for all t' >= t (RiccatiState SYM)
  float pk_last[PK];                                  // step T-1's packed record (tinv test)
  // ---------------- backward: linearise + Riccati + stage costs of the current trajectory
  {
    RiccatiState<n, m> rs;
    rs.init();
    float xn[n];                                        // x_{t+1} (ROLLOUT)
#pragma unroll
    for (int i = 0; i < n; ++i) xn[i] = 0.f;
    // inputs of step t, t-1 (and t-2 at kPF = 2) in flight together
    SweepIn<n, m, TL, BM> cur, n1, n2;
    cur.load(cs, x, u, bd, T - 1, B, b);
    if constexpr (kPF >= 2) n1.load(cs, x, u, bd, T > 1 ? T - 2 : 0, B, b);
    // step T-1 (F = 0, V = 0) is peeled off the loop, so the loop body always
    // computes the Jacobian (no zero-F defaults materialised at every step;
    // -1 us per fused iteration).  (Rotating the prefetch buffers by role
    // through the lambda's arguments instead of copying them measured +6 us.)
    using SI = SweepIn<n, m, TL, BM>;
    // one step on the inputs in `cur`: linearise, Riccati, stage cost; the
    // step's gain record is left in g (the caller stores it)
    auto sweep_body = [&](int t, auto last_c, const SI& cur, float (&g)[GREC]) {
      constexpr bool LAST = decltype(last_c)::value;
      float tau[d], Ctau[d], cb[d];
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = cur.x[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = cur.u[a];
      if (pack_out) {                                   // first iteration: build the packed copy
        float buf[PK];
        pack_cost(cur.C, cur.c, buf, sym, diag);
        if constexpr (LAST) {
          SoaRec<PK>::store(pack_out, buf, T, t, B, b);
#pragma unroll
          for (int k = 0; k < PK; ++k) pk_last[k] = buf[k];
        } else {
          bool same = true;
#pragma unroll
          for (int k = 0; k < PK; ++k) same &= __float_as_uint(buf[k]) == __float_as_uint(pk_last[k]);
          if (tinv && !same)                            // records t+1 .. T-2 were skipped: all equal step T-1's
            for (int s = t + 1; s < T - 1; ++s) SoaRec<PK>::store(pack_out, pk_last, T, s, B, b);
          tinv &= same;
          if (!tinv) SoaRec<PK>::store(pack_out, buf, T, t, B, b);
        }
      }
      float obj = 0.f;
      if constexpr (PREV) c_tau<d, CostT::kDiag>(cur.C, tau, Ctau);
      else obj = quad_cost<d, CostT::kDiag>(cur.C, cur.c, tau, Ctau);
#pragma unroll
      for (int i = 0; i < d; ++i) cb[i] = Ctau[i] + cur.c[i];
      float Ft[n][d];
      if constexpr (!LAST) {
        if constexpr (ROLLOUT && Model::kJacFromNext) md.jacobian_next(cur.x, cur.u, xn, Ft);
        else md.jacobian(cur.x, cur.u, Ft);
      } else {
#pragma unroll
        for (int i = 0; i < n; ++i)
#pragma unroll
          for (int j = 0; j < d; ++j) Ft[i][j] = 0.f;
      }
      float zIt[m], lb[m], ub[m];
#pragma unroll
      for (int a = 0; a < m; ++a) {
        zIt[a] = 0.f; lb[a] = 0.f; ub[a] = 0.f;
        if constexpr (MODE == GAIN_BOX) {
          lb[a] = cur.bnd.l(bd, a) - cur.u[a];
          ub[a] = cur.bnd.h(bd, a) - cur.u[a];
        }
      }
      float Kt[m][n], kt[m];
      using FS = typename Model::FSparsity;
      if constexpr (CostT::kSym) {
        rs.template step<MODE, FS, CostT::kDiag, true>(cur.C, cb, Ft, zIt, lb, ub, Kt, kt);
      } else {
        symsofar &= bitwise_symmetric(cur.C);
        if (symsofar) rs.template step<MODE, FS, CostT::kDiag, true>(cur.C, cb, Ft, zIt, lb, ub, Kt, kt);
        else rs.template step<MODE, FS, CostT::kDiag, false>(cur.C, cb, Ft, zIt, lb, ub, Kt, kt);
      }
#pragma unroll
      for (int a = 0; a < m; ++a) {
#pragma unroll
        for (int j = 0; j < n; ++j) g[a * n + j] = Kt[a][j];
        g[m * n + a] = kt[a];
      }
      if constexpr (!PREV) old_cost += obj;   // summed over t = T-1..0 (the reference's torch sum has its own order)
#pragma unroll
      for (int i = 0; i < n; ++i) xn[i] = cur.x[i];
    };
    auto sweep_step = [&](int t, auto last_c) {
      if constexpr (kPF >= 2) n2.load(cs, x, u, bd, t > 1 ? t - 2 : 0, B, b);   // prefetch step t-2
      else n1.load(cs, x, u, bd, t > 0 ? t - 1 : 0, B, b);                       // prefetch step t-1
      float g[GREC];
      sweep_body(t, last_c, cur, g);
      SoaRec<GREC>::store(ws.p, g, T, t, ws.B, ws.b);
      cur = n1;
      if constexpr (kPF >= 2) n1 = n2;
    };
    sweep_step(T - 1, std::true_type{});
#pragma unroll 2
    for (int t = T - 2; t >= 0; --t) sweep_step(t, std::false_type{});
    if (sym_out)
      sym_out[b] = sym ? (unsigned char)(kCostSym | (diag && packed_diag_ok<d>() ? kCostDiag : 0) |
                                         (tinv ? kCostTinv : 0))
                       : 0;
  }
  DILQR_STAMP(2);
  if constexpr (!CostT::kDiag && packed_diag_ok<d>()) {
    if (pack_out && sym && diag && tinv) {              // iteration 0 of a diag(q), p over t cost
      CostDiagConst<d> cc;
      cc.set(pk_last);
      return line_search<Model, BM, TL>(T, B, b, md, x_init, cc, x, u, bd, decay, max_ls, ws, xa_out, ua_out,
                                         xb_out, ub_out, du_sq, old_cost, cost_out, alpha_out, b_in_gains);
    }
  }
  return line_search<Model, BM, TL>(T, B, b, md, x_init, cs, x, u, bd, decay, max_ls, ws, xa_out, ua_out, xb_out,
                                     ub_out, du_sq, old_cost, cost_out, alpha_out, b_in_gains);
}

template <class Model, int BM>
__global__ void __launch_bounds__(kBlock) k_ilqr_iterate(int T, int B, const float* __restrict__ theta,
                                                         const float* __restrict__ x_init, const float* __restrict__ C,
                                                         const float* __restrict__ c, const float* __restrict__ x,
                                                         const float* __restrict__ u, Bounds bd, float decay, int max_ls,
                                                         float* __restrict__ ws, float* __restrict__ x_out,
                                                         float* __restrict__ u_out, float* __restrict__ cost_out,
                                                         float* __restrict__ du_sq, float* __restrict__ alpha_out,
                                                         const dilqr_mpc_ctrl* __restrict__ ctrl) {
  if (ctrl && ctrl->stopped) return;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  constexpr int n = Model::N, m = Model::M;
  constexpr int GREC = m * n + m;
  Model md; md.load(theta);
  float cost, alpha;
  // line-search candidate B rolls out into the workspace tail and is copied
  // over (x_out, u_out) when it wins
  float* xb = ws + (size_t)T * B * GREC;
  float* ub = xb + (size_t)T * B * n;
  const int win = ilqr_problem<Model, BM, TRAJ_AOS, false>(T, B, b, md, x_init, CostFull<n + m>{C, c}, nullptr, nullptr, x, u,
                                                   bd, decay,
                                            max_ls, GainRecs{ws, B, b},
                                            x_out, u_out, xb, ub, du_sq, cost, alpha);
  if (win) {
    for (int t = 0; t < T; ++t) {
      const size_t tb = (size_t)t * B + b;
      float xt[n], ut[m];
      ld(xt, xb + tb * n); ld(ut, ub + tb * m);
      st(x_out + tb * n, xt); st(u_out + tb * m, ut);
    }
  }
  cost_out[b] = cost;
  alpha_out[b] = alpha;
}

// ---------------- the device-resident MPC loop with per-problem trajectory slots
// Four trajectory buffers per problem ([4,T,B,n] / [4,T,B,m]); each problem
// keeps the index of its current and best slot, and the line search's two
// candidates roll out into the two free ones, so "accept candidate" and "best
// = this iterate" (mpc_explicit.py:277-283) are index updates, never copies.
using MpcState = dilqr_mpc_state;
constexpr int kSlots = 4;

DEV bool mpc_decide(const MpcState& S, int B, int k, int G, float eps, int not_improved_lim);

// the two lowest slot indices not in {cur, best}
// (selects only: the earlier counter-indexed form became a stack array)
DEV void free_slots(int cur, int best, int& sa, int& sb) {
  sa = -1;
  sb = -1;
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    const bool fr = s != cur && s != best;
    sb = (fr && sa >= 0 && sb < 0) ? s : sb;
    sa = (fr && sa < 0) ? s : sa;
  }
}

// LG: the gain records live in this workgroup's LDS (dynamic, T*64*GREC floats;
// dilqr_mpc_step_f32 picks it when 4 workgroups per CU still fit the 160 KB),
// instead of a workspace round trip through HBM/MALL every iteration.
// FIRST: iteration 0 of the solve (reads the caller's C, c and builds the
// packed copy) — its own instantiation, so the steady-state kernel carries no
// copy-building code and profiles separately.
template <class Model, int BM, bool LG, bool FIRST>
__global__ void __launch_bounds__(kBlock) k_mpc_iterate(int T, int B, const float* __restrict__ theta,
                                                        const float* __restrict__ x_init, const float* __restrict__ C,
                                                        const float* __restrict__ c, Bounds bd, float decay, int max_ls,
                                                        int iteration, float best_cost_eps, float eps,
                                                        int not_improved_lim, int G, MpcState S) {
  constexpr int n = Model::N, m = Model::M;
  constexpr bool first = FIRST;                             // == (iteration == 0), chosen by the host
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  // the problem's slot indices and cost flags are read together with the stop
  // rule's inputs (one memory latency in the prologue, not three)
  const int bl = b < B ? b : B - 1;
  const int cur = S.slot[bl], best = S.slot[B + bl];
  const unsigned char pk = (!FIRST && S.Cpk) ? S.cost_sym[bl] : 0;
  DILQR_STAMP(0);
  DILQR_STAMP(6);
  if (mpc_decide(S, B, iteration, G, eps, not_improved_lim)) return;
  if (b >= B) return;
  DILQR_STAMP(1);
  Model md; md.load(theta);
  const size_t TBd = (size_t)T * B * (n + m);               // one slot: [T,B,d] records
  int sa, sb;
  free_slots(cur, best, sa, sb);
  const float* xcur = S.Xs + cur * TBd;
  float* xsa = S.Xs + sa * TBd;
  float* xsb = S.Xs + sb * TBd;
  float cost, alpha;
  int win;
  extern __shared__ __attribute__((aligned(16))) float lds_gains[];
  const GainRecs gr = LG ? GainRecs{lds_gains, kBlock, (int)threadIdx.x} : GainRecs{S.ws, B, b};
  // the solve's packed symmetric cost: built by iteration 0's sweep (which reads
  // C, c), used from iteration 1 on by every problem whose C_t are all bitwise
  // symmetric, reading only diag(C_t) and c_t when they are all diagonal too
  // (per-lane flags; a wave normally takes one side of the branch)
  const CostFull<n + m> full{C, c};
  // one round of line-search candidates: B's records go to the consumed gain
  // slots in LDS and only B-winners copy them out (line_search)
  const bool b_lds = LG && max_ls <= 2;
  if constexpr (FIRST) {
    win = ilqr_problem<Model, BM, TRAJ_REC, true>(T, B, b, md, x_init, full, S.Cpk, S.Cpk ? S.cost_sym : nullptr,
                                                  xcur, nullptr, bd, decay, max_ls, gr, xsa, nullptr, xsb, nullptr,
                                                  S.du_sq, cost, alpha, b_lds);
  } else {
    if ((pk & (kCostDiag | kCostTinv)) == (kCostDiag | kCostTinv)) {
      if constexpr (packed_diag_ok<n + m>()) {
        CostDiagConst<n + m> cc;
        cc.init(S.Cpk, T, B, b);
        win = ilqr_problem<Model, BM, TRAJ_REC, true, CostDiagConst<n + m>, true>(T, B, b, md, x_init, cc, nullptr, nullptr, xcur, nullptr, bd,
                                                      decay, max_ls, gr, xsa, nullptr, xsb, nullptr, S.du_sq, cost,
                                                      alpha, b_lds, S.cost);
      } else {
        __builtin_unreachable();
      }
#ifdef DILQR_ONLY_DIAGCONST                // ISA-listing builds only (tools/loop_stats.py)
    } else {
      __builtin_unreachable();
    }
#else
    } else if (pk & kCostDiag) {           // set by iteration 0 only when packed_diag_ok
      if constexpr (packed_diag_ok<n + m>())
        win = ilqr_problem<Model, BM, TRAJ_REC, true, CostPacked<n + m, true>, true>(T, B, b, md, x_init, CostPacked<n + m, true>{S.Cpk, T}, nullptr,
                                                      nullptr, xcur, nullptr, bd, decay, max_ls, gr, xsa, nullptr, xsb,
                                                      nullptr, S.du_sq, cost, alpha, b_lds, S.cost);
      else
        __builtin_unreachable();
    } else if ((pk & (kCostSym | kCostTinv)) == (kCostSym | kCostTinv))
      win = ilqr_problem<Model, BM, TRAJ_REC, true, CostPacked<n + m, false, true>, true>(T, B, b, md, x_init, CostPacked<n + m, false, true>{S.Cpk, T},
                                                    nullptr, nullptr, xcur, nullptr, bd, decay, max_ls, gr, xsa, nullptr,
                                                    xsb, nullptr, S.du_sq, cost, alpha, b_lds, S.cost);
    else if (pk & kCostSym)
      win = ilqr_problem<Model, BM, TRAJ_REC, true, CostPacked<n + m>, true>(T, B, b, md, x_init, CostPacked<n + m>{S.Cpk, T}, nullptr, nullptr,
                                                    xcur, nullptr, bd, decay, max_ls, gr, xsa, nullptr, xsb, nullptr,
                                                    S.du_sq, cost, alpha, b_lds, S.cost);
    else
      win = ilqr_problem<Model, BM, TRAJ_REC, true, CostFull<n + m>, true>(T, B, b, md, x_init, full, nullptr, nullptr, xcur, nullptr, bd,
                                                    decay, max_ls, gr, xsa, nullptr, xsb, nullptr, S.du_sq, cost,
                                                    alpha, b_lds, S.cost);
#endif
  }
  DILQR_STAMP(3);
  const int nw = win ? sb : sa;
  S.cost[b] = cost;
  S.alpha[b] = alpha;
  bool better = !first && (cost <= S.best_cost[b] + best_cost_eps);      // mpc_explicit.py:278
  if (first || better) {
    S.best_cost[b] = cost;
    S.slot[B + b] = (unsigned char)nw;
  }
  S.improved[b] = (first || better) ? (better ? 2 : 1) : 0;
  if (S.best_iter && (first || better)) S.best_iter[b] = iteration;       // fixed-count solves
  S.slot[b] = (unsigned char)nw;
  DILQR_STAMP(4);
  DILQR_STAMP(7);
}

// the same two kernels for the 16-lanes-per-problem models (dilqr_group.h)
template <class Model, int MODE>
__global__ void __launch_bounds__(64) k_ilqr_iterate_group(int T, int B, const float* __restrict__ theta,
                                                           const float* __restrict__ x_init,
                                                           const float* __restrict__ C, const float* __restrict__ c,
                                                           const float* __restrict__ x, const float* __restrict__ u,
                                                           Bounds bd, float decay, int max_ls, float* __restrict__ ws,
                                                           float* __restrict__ x_out, float* __restrict__ u_out,
                                                           float* __restrict__ cost_out, float* __restrict__ du_sq,
                                                           float* __restrict__ alpha_out,
                                                           const dilqr_mpc_ctrl* __restrict__ ctrl) {
  __shared__ GroupLds<Model::N, Model::M> Ls[kGPW];
  if (ctrl && ctrl->stopped) return;
  const int r = threadIdx.x & (kG - 1), gp = threadIdx.x / kG;
  const int b0 = blockIdx.x * kGPW + gp;
  const bool valid = b0 < B;
  const int b = valid ? b0 : B - 1;          // idle groups shadow problem B-1 (same wave), writing nothing
  Model md; md.load(theta);
  float cost, alpha;
  int win;
  group_ilqr_problem<Model, MODE>(Ls[gp], T, B, b, r, valid, md, x_init, C, c, x, u, bd, decay, max_ls, ws, x_out,
                                  u_out, nullptr, nullptr, du_sq, cost, alpha, win);
  if (valid && r == 0) {
    cost_out[b] = cost;
    alpha_out[b] = alpha;
  }
}

template <class Model, int MODE>
__global__ void __launch_bounds__(64, kGroupWavesPerSimd) k_mpc_iterate_group(int T, int B, const float* __restrict__ theta,
                                                          const float* __restrict__ x_init,
                                                          const float* __restrict__ C, const float* __restrict__ c,
                                                          Bounds bd, float decay, int max_ls, int iteration,
                                                          float best_cost_eps, float eps, int not_improved_lim, int G,
                                                          MpcState S) {
  constexpr int n = Model::N, m = Model::M;
  __shared__ GroupLds<n, m> Ls[kGPW];
  if (mpc_decide(S, B, iteration, G, eps, not_improved_lim)) return;
  const int first = iteration == 0;
  const int r = threadIdx.x & (kG - 1), gp = threadIdx.x / kG;
  const int b0 = blockIdx.x * kGPW + gp;
  const bool valid = b0 < B;
  const int b = valid ? b0 : B - 1;
  Model md; md.load(theta);
  const size_t TBn = (size_t)T * B * n, TBm = (size_t)T * B * m;
  const int cur = S.slot[b], best = S.slot[B + b];
  int sa, sb;
  free_slots(cur, best, sa, sb);
  float cost, alpha;
  int win;
  group_ilqr_problem<Model, MODE>(Ls[gp], T, B, b, r, valid, md, x_init, C, c, S.Xs + cur * TBn, S.Us + cur * TBm,
                                  bd, decay, max_ls, S.ws, S.Xs + sa * TBn, S.Us + sa * TBm, S.Xs + sb * TBn,
                                  S.Us + sb * TBm, S.du_sq, cost, alpha, win);
  const int nw = win ? sb : sa;
  if (valid && r == 0) {
    S.cost[b] = cost;
    S.alpha[b] = alpha;
    const bool better = !first && (cost <= S.best_cost[b] + best_cost_eps);   // mpc_explicit.py:278
    if (first || better) {
      S.best_cost[b] = cost;
      S.slot[B + b] = (unsigned char)nw;
    }
    S.improved[b] = (first || better) ? (better ? 2 : 1) : 0;
    if (S.best_iter && (first || better)) S.best_iter[b] = iteration;     // fixed-count solves
    S.slot[b] = (unsigned char)nw;
  }
}

// ---------------- the stop rule (mpc_explicit.py:264, 279, 297-299), split so
// that no launch waits on a grid-wide fan-in:
//  * k_mpc_norm_rows (after iteration k): full_du_norm with the reference's
//    batch-mixing rows (the .transpose(1,2).contiguous().view(n_batch,-1) quirk,
//    lqr_step_explicit.py:245-247), best_du of the problems that took iteration
//    k, and per-workgroup partials (max row norm, any "improved") into plane
//    k&1 of the sync area.  Plain stores only.
//  * mpc_decide, in the prologue of iteration k+1 (every workgroup, redundantly,
//    identically): reduce the partials of iteration k, apply the stop rule to the
//    control state S_k -> S_{k+1}; workgroup 0 publishes S_{k+1} in ctrl[(k+1)&1].
//    The kernel boundary orders everything, so no fences or atomics are needed
//    (measured: the former last-workgroup fan-in cost 8 of 14 us per iteration).
// Sync area (uints): [16 + (2*par + 0)*G_MAX + blk] max bits, [16 + (2*par+1)*G_MAX
// + blk] any, G_MAX = ceil(B/64).
DEV int sync_gmax(int B) { return (B + 63) / 64; }

template <bool STAGE>
__global__ void __launch_bounds__(256) k_mpc_norm_rows(int TM, int B, int iteration, MpcState S) {
  // the block's rows are one contiguous span of TM*blockDim floats: stage it
  // through LDS with coalesced loads, then each thread sums its row (stride TM
  // words; TM odd -> conflict-free, TM even -> at most 2-way).  Every global
  // load (the control flag, improved[r], the span) is issued before the first
  // one is waited on: the kernel is one HBM latency, not three in a row.
  extern __shared__ __attribute__((aligned(16))) float sdu[];
  __shared__ unsigned red_max[4];
  __shared__ int red_any[4];
  const int stopped = S.ctrl[iteration & 1].stopped;   // iteration `iteration` did not run: acted on below
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int imp = r < B ? S.improved[r] : 0;
  if constexpr (STAGE) {
    const size_t base = (size_t)blockIdx.x * blockDim.x * TM;
    const size_t total = (size_t)B * TM;
    const int span = blockDim.x * TM;
    const int have = (int)((total - base) < (size_t)span ? total - base : (size_t)span);
    if ((span & 3) == 0 && (have & 3) == 0) {          // base is then 16-byte aligned too
      // up to 8 float4 loads in flight per thread (span <= 64 KiB = 4096 float4)
      constexpr int U = 8;
      const float4* src = reinterpret_cast<const float4*>(S.du_sq + base);
      float4* dst = reinterpret_cast<float4*>(sdu);
      const int n4 = span >> 2, h4 = have >> 2;
      for (int i0 = threadIdx.x; i0 < n4; i0 += blockDim.x * U) {
        float4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
          const int i = i0 + j * blockDim.x;
          v[j] = i < h4 ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
          const int i = i0 + j * blockDim.x;
          if (i < n4) dst[i] = v[j];
        }
      }
    } else {
      // up to 32 independent loads in flight per thread before the first LDS
      // store (a load->store loop would serialise one HBM latency per element)
      constexpr int U = 32;
      for (int i0 = threadIdx.x; i0 < span; i0 += blockDim.x * U) {
        float v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
          const int i = i0 + j * blockDim.x;
          v[j] = i < have ? S.du_sq[base + i] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
          const int i = i0 + j * blockDim.x;
          if (i < span) sdu[i] = v[j];
        }
      }
    }
    if (stopped) return;                               // uniform over the grid
    __syncthreads();
  } else {
    if (stopped) return;
  }
  unsigned mx = 0u;
  int any = 0;
  if (r < B) {
    float s = 0.f;
    const float* p = STAGE ? sdu + (size_t)threadIdx.x * TM : S.du_sq + (size_t)r * TM;
    for (int i = 0; i < TM; ++i) s += p[i];
    float fdn = sqrtf(s);
    S.full_du_norm[r] = fdn;
    mx = __float_as_uint(fdn);              // fdn >= 0: float order == uint order
    if (imp) S.best_du[r] = fdn;
    any = imp == 2;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    unsigned o = __shfl_xor(mx, off, 64);
    mx = o > mx ? o : mx;
    any |= __shfl_xor(any, off, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red_max[w] = mx; red_any[w] = any; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) { mx = red_max[i] > mx ? red_max[i] : mx; any |= red_any[i]; }
    const int gm = sync_gmax(B), par = iteration & 1;
    S.done_counter[16 + (2 * par) * gm + blockIdx.x] = mx;
    S.done_counter[16 + (2 * par + 1) * gm + blockIdx.x] = (unsigned)any;
  }
}

// ---------------- fixed-count solves (eps <= 0 and not_improved_lim >= the
// iteration count: the stop rule provably never fires, mpc_explicit.py:297-299).
// No stop-rule launch per iteration: each iteration writes its du rows into its
// own plane of du_sq ([iters,T,m,B]) and records, per problem, the last
// iteration that took the best-iterate branch (best_iter).  At the end this
// kernel forms best_du — the quirk row (lqr_step_explicit.py:245-247) of that
// iteration, summed in the same order as k_mpc_norm_rows, so the same bits —
// and publishes the iteration count in both control words.
__global__ void __launch_bounds__(256) k_mpc_fixed_finish(int TM, int B, int iterations, MpcState S) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < B) {
    const int k = S.best_iter[r];
    const float* p = S.du_sq + ((size_t)k * B + r) * TM;
    float s = 0.f;
    for (int i = 0; i < TM; ++i) s += p[i];
    S.best_du[r] = sqrtf(s);
  }
  if (r < 2) {
    dilqr_mpc_ctrl c = S.ctrl[r];
    c.iter = iterations;
    c.stopped = 0;
    S.ctrl[r] = c;
  }
}

// Prologue of iteration k >= 1 (one 64-lane wave per workgroup): the stop rule
// for iteration k-1.  Returns true when the solve has stopped (the wave exits).
DEV bool mpc_decide(const MpcState& S, int B, int k, int G, float eps, int not_improved_lim) {
  if (k == 0) return false;                            // S_0: begin zeroed ctrl[0..1]
  if (G < 0) return false;                             // fixed-count solve: the rule cannot fire
  // Every load is issued before the first is waited on — the control word and
  // all partials (valid memory whether or not the solve stopped) — so the
  // prologue costs one memory latency; the partials go in as uint4 when the
  // planes are 16-byte aligned (B % 256 == 0).
  const int gm = sync_gmax(B), par = (k - 1) & 1;
  const unsigned* pm = S.done_counter + 16 + (2 * par) * gm;
  const unsigned* pa = S.done_counter + 16 + (2 * par + 1) * gm;
  const int lane = threadIdx.x & 63;
  const dilqr_mpc_ctrl in = S.ctrl[(k - 1) & 1];        // S_{k-1}
  unsigned mx = 0u;
  int any = 0;
  if ((gm & 3) == 0 && G <= 1024) {
    const uint4* pm4 = reinterpret_cast<const uint4*>(pm);
    const uint4* pa4 = reinterpret_cast<const uint4*>(pa);
    uint4 vm[4], va[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = lane + 64 * j;
      const bool ok = 4 * i < G;
      vm[j] = ok ? pm4[i] : make_uint4(0u, 0u, 0u, 0u);
      va[j] = ok ? pa4[i] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i0 = 4 * (lane + 64 * j);
      const unsigned e[4] = {vm[j].x, vm[j].y, vm[j].z, vm[j].w};
      const unsigned f[4] = {va[j].x, va[j].y, va[j].z, va[j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (i0 + q < G) {
          mx = e[q] > mx ? e[q] : mx;
          any |= (int)f[q];
        }
      }
    }
  } else {
    for (int i = lane; i < G; i += 64) {
      unsigned v = pm[i];
      mx = v > mx ? v : mx;
      any |= (int)pa[i];
    }
  }
  dilqr_mpc_ctrl out = in;
  if (!in.stopped) {
    // wave-uniform decisions by ballot: max < eps <=> every lane's max < eps
    // (fdn >= 0, so uint order is float order; a NaN fails `< eps` in its lane
    // as it fails it as the max)
    const bool all_below = __ballot(!(__uint_as_float(mx) < eps)) == 0ull;
    const bool any_imp = __ballot(any != 0) != 0ull;
    out.iter = in.iter + 1;
    out.n_not_improved = any_imp ? 0 : in.n_not_improved + 1;     // mpc_explicit.py:264, 279
    if (all_below || out.n_not_improved > not_improved_lim) out.stopped = 1;   // 297-299
    if (blockIdx.x == 0) {                              // the published max (informational)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        unsigned o = __shfl_xor(mx, off, 64);
        mx = o > mx ? o : mx;
      }
      out.max_du_bits = mx;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) S.ctrl[k & 1] = out;
  return out.stopped != 0;
}

// slot layout: [T,B,d] records for the thread-per-problem models (TRAJ_REC;
// the state's Us is unused), the caller's [T,B,n] / [T,B,m] for the
// 16-lanes-per-problem ones
template <class Model>
constexpr int slot_layout() { return Model::N + Model::M <= 8 ? TRAJ_REC : TRAJ_AOS; }
constexpr int slot_layout_nm(int n, int m) { return n + m <= 8 ? TRAJ_REC : TRAJ_AOS; }

// rollout of u_init into slot 0 (util.get_traj) + reset of slots/ctrl.
// u_init: the caller's [T,B,m] controls, or null for zeros (the MPC default):
// read once, written into the slot with the states in the same pass.
template <class Model>
__global__ void __launch_bounds__(kBlock) k_mpc_begin(int T, int B, const float* __restrict__ theta,
                                                      const float* __restrict__ x_init,
                                                      const float* __restrict__ u_init, MpcState S) {
  constexpr int n = Model::N, m = Model::M;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b == 0) {
    dilqr_mpc_ctrl z = {};
    S.ctrl[0] = z;
    S.ctrl[1] = z;
#pragma unroll
    for (int i = 0; i < 9; ++i) S.done_counter[i] = 0u;
  }
  if (b >= B) return;
  Model md; md.load(theta);
  S.slot[b] = 0; S.slot[B + b] = 0;
  constexpr int TL = slot_layout<Model>();
  float xt[n];
  ld(xt, x_init + (size_t)b * n);
  for (int t = 0; t < T; ++t) {
    float ut[m], xn[n];
    if (u_init) {
      ld(ut, u_init + ((size_t)t * B + b) * m);
    } else {
#pragma unroll
      for (int a = 0; a < m; ++a) ut[a] = 0.f;
    }
    st_xu<TL>(S.Xs, S.Us, xt, ut, t, B, b);
    if (t < T - 1) {
      md.forward(xt, ut, xn);
#pragma unroll
      for (int i = 0; i < n; ++i) xt[i] = xn[i];
    }
  }
}

template <int n, int m>
__global__ void __launch_bounds__(kBlock) k_mpc_gather(int T, int B, MpcState S, float* __restrict__ x_out,
                                                       float* __restrict__ u_out) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int best = S.slot[B + b];
  constexpr int TL = slot_layout_nm(n, m);
  const float* X = S.Xs + (size_t)best * T * B * (TL == TRAJ_REC ? n + m : n);
  const float* U = S.Us + (size_t)best * T * B * m;
  for (int t = 0; t < T; ++t) {
    size_t tb = (size_t)t * B + b;
    float xt[n], ut[m];
    ld_xu<TL>(xt, ut, X, U, t, B, b);
    st(x_out + tb * n, xt); st(u_out + tb * m, ut);
  }
}

// ============================================================ MPC bookkeeping
// mpc_explicit.py:264-283: full_du_norm (quirk rows), best-iterate update.
template <int n, int m>
__global__ void __launch_bounds__(kBlock) k_mpc_best(int T, int B, int first, float best_cost_eps,
                                                     const float* __restrict__ x, const float* __restrict__ u,
                                                     const float* __restrict__ cost, const float* __restrict__ du_sq,
                                                     float* __restrict__ full_du_norm, float* __restrict__ best_x,
                                                     float* __restrict__ best_u, float* __restrict__ best_cost,
                                                     float* __restrict__ best_du, dilqr_mpc_ctrl* __restrict__ ctrl) {
  if (ctrl->stopped) return;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int TM = T * m;
  float s = 0.f;
  const float* p = du_sq + (size_t)b * TM;
  for (int i = 0; i < TM; ++i) s += p[i];
  float fdn = sqrtf(s);
  full_du_norm[b] = fdn;
  atomicMax(&ctrl->max_du_bits, __float_as_uint(fdn));
  float cb = cost[b];
  bool take = first != 0;
  if (!take && cb <= best_cost[b] + best_cost_eps) {
    take = true;
    atomicOr(&ctrl->any_improved, 1);
  }
  if (take) {
    best_cost[b] = cb;
    best_du[b] = fdn;
    for (int t = 0; t < T; ++t) {
      size_t tb = (size_t)t * B + b;
      float xt[n], ut[m];
      ld(xt, x + tb * n); ld(ut, u + tb * m);
      st(best_x + tb * n, xt); st(best_u + tb * m, ut);
    }
  }
}

// mpc_explicit.py:264, 279, 297-299
__global__ void k_mpc_control(int first, float eps, int not_improved_lim, dilqr_mpc_ctrl* ctrl) {
  if (ctrl->stopped) return;
  ctrl->iter += 1;
  ctrl->n_not_improved += 1;
  if (!first && ctrl->any_improved) ctrl->n_not_improved = 0;
  float mx = __uint_as_float(ctrl->max_du_bits);
  if (mx < eps || ctrl->n_not_improved > not_improved_lim) ctrl->stopped = 1;
  ctrl->any_improved = 0;
  ctrl->max_du_bits = 0u;
}

// ============================================================ classic adjoint
// lqr_step.py:312-407 for one problem per lane:
//   phase 1: Riccati sweep of the adjoint problem (c_back = -r, u_zero_I = active set)
//   phase 2: its LinDx rollout from 0 with the default line search (decay 0.2, 10
//            passes; old cost 0), d tau stored as dc = -d tau
//   phase 3: costates lam, dlam backwards; dC, dF, df, dx_init.
template <int n, int m, int MODE>
__global__ void __launch_bounds__(kBlock) k_lqr_adjoint(int T, int B, const float* __restrict__ C,
                                                        const float* __restrict__ c, const float* __restrict__ F,
                                                        const float* __restrict__ x, const float* __restrict__ u,
                                                        const float* __restrict__ dl_dx, const float* __restrict__ dl_du,
                                                        Bounds bd, float* __restrict__ ws, float* __restrict__ dx_init,
                                                        float* __restrict__ dC, float* __restrict__ dc,
                                                        float* __restrict__ dF, float* __restrict__ df) {
  constexpr int d = n + m;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  // active set (lqr_step.py:321-325)
  auto active = [&](size_t tb, int a) -> bool {
    if (bd.mode == DILQR_BOUNDS_NONE) return false;
    float ua = u[tb * m + a];
    return fabsf(ua - bound_lo(bd, tb * m + a)) <= 1e-8f || fabsf(ua - bound_hi(bd, tb * m + a)) <= 1e-8f;
  };
  // ---- phase 1
  RiccatiState<n, m> rs;
  rs.init();
  for (int t = T - 1; t >= 0; --t) {
    size_t tb = (size_t)t * B + b;
    float Ct[d][d], cb[d], rx[n], ru[m];
    ld2(Ct, C + tb * d * d);
    ld(rx, dl_dx + tb * n); ld(ru, dl_du + tb * m);
#pragma unroll
    for (int i = 0; i < n; ++i) cb[i] = -rx[i];
#pragma unroll
    for (int a = 0; a < m; ++a) cb[n + a] = -ru[a];
    float Ft[n][d];
    if (t < T - 1) {
      ld2(Ft, F + tb * n * d);
    } else {
#pragma unroll
      for (int i = 0; i < n; ++i)
#pragma unroll
        for (int j = 0; j < d; ++j) Ft[i][j] = 0.f;
    }
    float zIt[m], lb[m], ub[m];
    bool any = false;
#pragma unroll
    for (int a = 0; a < m; ++a) {
      zIt[a] = active(tb, a) ? 1.f : 0.f;
      any |= zIt[a] != 0.f;
      lb[a] = ub[a] = 0.f;
    }
    float Kt[m][n], kt[m];
    if (bd.mode != DILQR_BOUNDS_NONE) rs.template step<GAIN_ZERO_I>(Ct, cb, Ft, zIt, lb, ub, Kt, kt);
    else rs.template step<MODE>(Ct, cb, Ft, zIt, lb, ub, Kt, kt);
    (void)any;
    st2(ws + tb * (m * n + m), Kt);
    st(ws + tb * (m * n + m) + m * n, kt);
  }
  // ---- phase 2: rollout of the adjoint LQR from zero with line search
  float alpha = 1.f;
  for (int ls = 0; ls < 10; ++ls) {
    float xn[n], cost = 0.f;
#pragma unroll
    for (int i = 0; i < n; ++i) xn[i] = 0.f;
    for (int t = 0; t < T; ++t) {
      size_t tb = (size_t)t * B + b;
      float Kt[m][n], kt[m], nu[m];
      ld2(Kt, ws + tb * (m * n + m));
      ld(kt, ws + tb * (m * n + m) + m * n);
#pragma unroll
      for (int a = 0; a < m; ++a) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Kt[a][j] * xn[j];       // dx = new_x - 0
        nu[a] = (s + 0.f) + alpha * kt[a];
        if (active(tb, a)) nu[a] = 0.f;
      }
      float tau[d], Ct[d][d], rr[d];
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = xn[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = nu[a];
      float ndt[d];
#pragma unroll
      for (int i = 0; i < d; ++i) ndt[i] = -tau[i];
      st(dc + tb * d, ndt);
      ld2(Ct, C + tb * d * d);
      {
        float rx[n], ru[m];
        ld(rx, dl_dx + tb * n); ld(ru, dl_du + tb * m);
#pragma unroll
        for (int i = 0; i < n; ++i) rr[i] = -rx[i];
#pragma unroll
        for (int a = 0; a < m; ++a) rr[n + a] = -ru[a];
      }
      cost += quad_cost(Ct, rr, tau);
      if (t < T - 1) {
        float Ft[n][d];
        ld2(Ft, F + tb * n * d);
        float xnext[n];
#pragma unroll
        for (int i = 0; i < n; ++i) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) s += Ft[i][j] * tau[j];
          xnext[i] = s;
        }
#pragma unroll
        for (int i = 0; i < n; ++i) xn[i] = xnext[i];
      }
    }
    if (!(cost > 0.f) || ls == 9) break;
    alpha *= 0.2f;
  }
  // ---- phase 3: costates and gradients (lqr_step.py:352-405)
  float lam[n], dlam[n];
#pragma unroll
  for (int i = 0; i < n; ++i) lam[i] = dlam[i] = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    size_t tb = (size_t)t * B + b;
    float Ct[d][d], ctt[d], xt[n], ut[m], tau[d], dtau[d], rx[n];
    ld2(Ct, C + tb * d * d); ld(ctt, c + tb * d); ld(xt, x + tb * n); ld(ut, u + tb * m);
    ld(dtau, dc + tb * d);
    ld(rx, dl_dx + tb * n);
#pragma unroll
    for (int i = 0; i < d; ++i) dtau[i] = -dtau[i];
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
    // dC_t = -0.5 (dtau tau^T + tau dtau^T)
    float dCt[d][d];
#pragma unroll
    for (int i = 0; i < d; ++i)
#pragma unroll
      for (int j = 0; j < d; ++j) dCt[i][j] = -0.5f * (dtau[i] * tau[j] + tau[i] * dtau[j]);
    st2(dC + tb * d * d, dCt);
    if (t < T - 1) {
      // dF_t = -(dlam_{t+1} tau_t^T + lam_{t+1} dtau_t^T); df_t = -dlam_{t+1}
      float dFt[n][d], dft[n];
#pragma unroll
      for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int j = 0; j < d; ++j) dFt[i][j] = -(dlam[i] * tau[j] + lam[i] * dtau[j]);
        dft[i] = -dlam[i];
      }
      st2(dF + tb * n * d, dFt);
      if (df) st(df + tb * n, dft);
    }
    // lam_t = Cxx x + Cxu u + c_x + F_x^T lam_{t+1}; dlam likewise with dtau and -r_x
    float nl[n], ndl[n];
#pragma unroll
    for (int i = 0; i < n; ++i) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < n; ++j) { s1 += Ct[i][j] * xt[j]; s2 += Ct[i][j] * dtau[j]; }
      float s3 = 0.f, s4 = 0.f;
#pragma unroll
      for (int a = 0; a < m; ++a) { s3 += Ct[i][n + a] * ut[a]; s4 += Ct[i][n + a] * dtau[n + a]; }
      nl[i] = (s1 + s3) + ctt[i];
      ndl[i] = (s2 + s4) - rx[i];
    }
    if (t < T - 1) {
      float Ft[n][d];
      ld2(Ft, F + tb * n * d);
#pragma unroll
      for (int i = 0; i < n; ++i) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int l = 0; l < n; ++l) { s1 += Ft[l][i] * lam[l]; s2 += Ft[l][i] * dlam[l]; }
        nl[i] += s1;
        ndl[i] += s2;
      }
    }
#pragma unroll
    for (int i = 0; i < n; ++i) { lam[i] = nl[i]; dlam[i] = ndl[i]; }
  }
  float dxi[n];
#pragma unroll
  for (int i = 0; i < n; ++i) dxi[i] = -dlam[i];
  st(dx_init + (size_t)b * n, dxi);
}


// ============================================================ DiLQR implicit backward
// lqr_step_explicit.py:653-712 + fix_point_equ 458-598, by the algebra of
// oracle/adjoint.py implicit_backward_fast (validated against the literal
// restatement to 1e-14 in fp64): the reference's (T d)^2 system A^T w = g is one
// extra LQR solve with cost C_t + M_t^T, M_t = sum_i lam_{t+1,i} d D_t[i] / d tau
// (the Lagrangian Hessian of the dynamics), after which dC, dc, dtheta are the
// KKT gradients of the adjoint solve with r = w, whose trajectory is that same
// solve's y.  Per problem (one lane), four passes over T:
//   A (t up)   : gradx_t (grad_input's closed-loop d x_t / d theta, with the
//                reference's reversed-K and x_grad_xtm1 quirks) -> ws
//   B (t down) : primal costates lam_t -> ws; M_t; Riccati step with C_t + M_t^T,
//                c_back = -g_t, active set masked (u_zero_I engine) -> ws
//   C (t up)   : rollout y (no line search) -> ws
//   D (t down) : w_t = g_t - M_t^T y_t, dlam; dC_t, dc_t out; dtheta accumulated.
template <class Model> struct ImplicitWs {
  static constexpr int n = Model::N, m = Model::M, p = Model::P, d = n + m;
  static constexpr int GX = 0, LAM = n * p, KG = LAM + n, Y = KG + m * n + m;
  static constexpr int REC = ((Y + d) + 3) / 4 * 4;
};

template <class Model>
__global__ void __launch_bounds__(kBlock) k_implicit_backward(
    int T, int B, const float* __restrict__ theta, const float* __restrict__ C, const float* __restrict__ c,
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ K,
    const float* __restrict__ dl_dx, const float* __restrict__ dl_du, Bounds bd, float* __restrict__ ws,
    float* __restrict__ dC, float* __restrict__ dc, float* __restrict__ dtheta) {
  using D2 = typename D2Of<Model>::type;
  using W = ImplicitWs<Model>;
  constexpr int n = Model::N, m = Model::M, p = Model::P, d = n + m, R = W::REC;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Model md; md.load(theta);
  auto rec = [&](int t) { return ws + ((size_t)t * B + b) * R; };
  auto active = [&](size_t tb, int a, float ua) -> bool {
    if (bd.mode == DILQR_BOUNDS_NONE) return false;
    return fabsf(ua - bound_lo(bd, tb * m + a)) <= 1e-8f || fabsf(ua - bound_hi(bd, tb * m + a)) <= 1e-8f;
  };
  // ---------------- A: gradx_t, t = 0..T-1  (cartpole.py:755-769)
  {
    float gx[n][p];
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
      for (int k = 0; k < p; ++k) gx[i][k] = 0.f;
    st2(rec(0) + W::GX, gx);
    for (int t = 1; t < T; ++t) {
      size_t tb = (size_t)t * B + b;
      float xt[n], ut[m], D[n][d], ft[n][p], Kq[m][n];
      ld(xt, x + tb * n); ld(ut, u + tb * m);
      md.jacobian(xt, ut, D);
      D2::f_theta(theta, xt, ut, ft);
      ld2(Kq, K + ((size_t)(T - t) * B + b) * m * n);     // K[t-1] of the reversed stack = K_{T-t}
      float A[n][n];
#pragma unroll
      for (int i = 0; i < n; ++i)
#pragma unroll
        for (int l = 0; l < n; ++l) {
          float s = D[i][l];
          if (D2Of<Model>::XX00_ZERO && i == 0 && l == 0) s = 0.f;
#pragma unroll
          for (int a = 0; a < m; ++a) s += D[i][n + a] * Kq[a][l];
          A[i][l] = s;
        }
      float ng[n][p];
#pragma unroll
      for (int i = 0; i < n; ++i)
#pragma unroll
        for (int k = 0; k < p; ++k) {
          float s = 0.f;
#pragma unroll
          for (int l = 0; l < n; ++l) s += A[i][l] * gx[l][k];
          ng[i][k] = ft[i][k] + s;
        }
#pragma unroll
      for (int i = 0; i < n; ++i)
#pragma unroll
        for (int k = 0; k < p; ++k) gx[i][k] = ng[i][k];
      st2(rec(t) + W::GX, gx);
    }
  }
  // ---------------- B: costates, M_t, Riccati of the C + M^T problem
  {
    RiccatiState<n, m> rs;
    rs.init();
    float lam[n];
#pragma unroll
    for (int i = 0; i < n; ++i) lam[i] = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      size_t tb = (size_t)t * B + b;
      float Ct[d][d], ct[d], xt[n], ut[m], gxx[n], gu[m];
      ld2(Ct, C + tb * d * d); ld(ct, c + tb * d); ld(xt, x + tb * n); ld(ut, u + tb * m);
      ld(gxx, dl_dx + tb * n); ld(gu, dl_du + tb * m);
      float D[n][d];
      float Mt[d][d];
      if (t < T - 1) {
        md.jacobian(xt, ut, D);
        D2::lag_hess(theta, xt, ut, lam, Mt);             // lam = lam_{t+1}
      } else {
#pragma unroll
        for (int i = 0; i < n; ++i)
#pragma unroll
          for (int j = 0; j < d; ++j) D[i][j] = 0.f;
#pragma unroll
        for (int i = 0; i < d; ++i)
#pragma unroll
          for (int j = 0; j < d; ++j) Mt[i][j] = 0.f;
      }
      float Cp[d][d], cb[d];
#pragma unroll
      for (int i = 0; i < d; ++i)
#pragma unroll
        for (int j = 0; j < d; ++j) Cp[i][j] = Ct[i][j] + Mt[j][i];
#pragma unroll
      for (int i = 0; i < n; ++i) cb[i] = -gxx[i];
#pragma unroll
      for (int a = 0; a < m; ++a) cb[n + a] = -gu[a];
      float zI[m], lb[m], ub[m];
#pragma unroll
      for (int a = 0; a < m; ++a) { zI[a] = active(tb, a, ut[a]) ? 1.f : 0.f; lb[a] = ub[a] = 0.f; }
      float Kt[m][n], kt[m];
      if (bd.mode != DILQR_BOUNDS_NONE) rs.template step<GAIN_ZERO_I>(Cp, cb, D, zI, lb, ub, Kt, kt);
      else rs.template step<GAIN_UNC>(Cp, cb, D, zI, lb, ub, Kt, kt);
      float* r = rec(t);
      st2(r + W::KG, Kt);
#pragma unroll
      for (int a = 0; a < m; ++a) r[W::KG + m * n + a] = kt[a];
      // lam_t = Cxx x + Cxu u + c_x + F_x^T lam_{t+1}   (lqr_step_explicit.py:305-319)
      float nl[n];
#pragma unroll
      for (int i = 0; i < n; ++i) {
        float s = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Ct[i][j] * xt[j];
#pragma unroll
        for (int a = 0; a < m; ++a) s2 += Ct[i][n + a] * ut[a];
        float s3 = 0.f;
#pragma unroll
        for (int l = 0; l < n; ++l) s3 += D[l][i] * lam[l];
        nl[i] = ((s + s2) + ct[i]) + s3;
      }
#pragma unroll
      for (int i = 0; i < n; ++i) { lam[i] = nl[i]; r[W::LAM + i] = nl[i]; }
    }
  }
  // ---------------- C: rollout y of the modified problem (linear, alpha = 1)
  {
    float yx[n];
#pragma unroll
    for (int i = 0; i < n; ++i) yx[i] = 0.f;
    for (int t = 0; t < T; ++t) {
      size_t tb = (size_t)t * B + b;
      float* r = rec(t);
      float Kt[m][n], kt[m], ut[m];
      ld2(Kt, r + W::KG);
#pragma unroll
      for (int a = 0; a < m; ++a) kt[a] = r[W::KG + m * n + a];
      ld(ut, u + tb * m);
      float y[d];
#pragma unroll
      for (int i = 0; i < n; ++i) y[i] = yx[i];
#pragma unroll
      for (int a = 0; a < m; ++a) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Kt[a][j] * yx[j];
        y[n + a] = active(tb, a, ut[a]) ? 0.f : (s + 0.f) + kt[a];
      }
#pragma unroll
      for (int i = 0; i < d; ++i) r[W::Y + i] = y[i];
      if (t < T - 1) {
        float xt[n], D[n][d];
        ld(xt, x + tb * n);
        md.jacobian(xt, ut, D);
#pragma unroll
        for (int i = 0; i < n; ++i) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) s += D[i][j] * y[j];
          yx[i] = s;
        }
      }
    }
  }
  // ---------------- D: w, dlam, dC, dc, dtheta
  {
    float dlam[n], gx1[n][p], dth[p];
#pragma unroll
    for (int i = 0; i < n; ++i) {
      dlam[i] = 0.f;
#pragma unroll
      for (int k = 0; k < p; ++k) gx1[i][k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < p; ++k) dth[k] = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      size_t tb = (size_t)t * B + b;
      float* r = rec(t);
      float Ct[d][d], xt[n], ut[m], gxx[n], gu[m], y[d], gx[n][p];
      ld2(Ct, C + tb * d * d); ld(xt, x + tb * n); ld(ut, u + tb * m);
      ld(gxx, dl_dx + tb * n); ld(gu, dl_du + tb * m);
#pragma unroll
      for (int i = 0; i < d; ++i) y[i] = r[W::Y + i];
      ld2(gx, r + W::GX);
      float tau[d];
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
      // dC_t = -0.5 (y tau^T + tau y^T), dc_t = -y   (lqr_step_explicit.py:296-303)
      float dCt[d][d], dct[d];
#pragma unroll
      for (int i = 0; i < d; ++i) {
#pragma unroll
        for (int j = 0; j < d; ++j) dCt[i][j] = -0.5f * (y[i] * tau[j] + tau[i] * y[j]);
        dct[i] = -y[i];
      }
      st2(dC + tb * d * d, dCt);
      st(dc + tb * d, dct);
      float wx[n];
      float D[n][d];
      if (t < T - 1) {
        float lam1[n], Mt[d][d], Mp[d][p], Kq[m][n];
#pragma unroll
        for (int i = 0; i < n; ++i) lam1[i] = rec(t + 1)[W::LAM + i];
        md.jacobian(xt, ut, D);
        D2::lag_hess(theta, xt, ut, lam1, Mt);
        D2::lag_dparam(theta, xt, ut, lam1, Mp);
        ld2(Kq, K + ((size_t)(T - 1 - t) * B + b) * m * n);   // K[t] of the reversed stack
        // w_t = g_t - M_t^T y_t
#pragma unroll
        for (int k = 0; k < n; ++k) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) s += Mt[j][k] * y[j];
          wx[k] = gxx[k] - s;
        }
        // dtheta_t = -(y^T Mp) - (y^T (M_x + M_u Kq)) gradx_t - dlam_{t+1}^T gradx_{t+1}
        //            + dlam_{t+1}^T (D_x + D_u Kq) gradx_t
        float hx[n], hp[p];
#pragma unroll
        for (int k = 0; k < p; ++k) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) s += y[j] * Mp[j][k];
          hp[k] = s;
        }
#pragma unroll
        for (int l = 0; l < n; ++l) {
          float s = 0.f, s2 = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) {
            float ml = Mt[j][l];
#pragma unroll
            for (int a = 0; a < m; ++a) ml += Mt[j][n + a] * Kq[a][l];
            s += y[j] * ml;
          }
#pragma unroll
          for (int i = 0; i < n; ++i) {
            float dl = D[i][l];
#pragma unroll
            for (int a = 0; a < m; ++a) dl += D[i][n + a] * Kq[a][l];
            s2 += dlam[i] * dl;
          }
          hx[l] = s2 - s;
        }
#pragma unroll
        for (int k = 0; k < p; ++k) {
          float s = -hp[k];
#pragma unroll
          for (int l = 0; l < n; ++l) s += hx[l] * gx[l][k] - dlam[l] * gx1[l][k];
          dth[k] += s;
        }
      } else {
#pragma unroll
        for (int k = 0; k < n; ++k) wx[k] = gxx[k];
#pragma unroll
        for (int i = 0; i < n; ++i)
#pragma unroll
          for (int j = 0; j < d; ++j) D[i][j] = 0.f;
      }
      // dlam_t = Cxx y_x + Cxu y_u - w_x + F_x^T dlam_{t+1}   (lqr_step_explicit.py:321-335)
      float nd[n];
#pragma unroll
      for (int i = 0; i < n; ++i) {
        float s = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Ct[i][j] * y[j];
#pragma unroll
        for (int a = 0; a < m; ++a) s2 += Ct[i][n + a] * y[n + a];
#pragma unroll
        for (int l = 0; l < n; ++l) s3 += D[l][i] * dlam[l];
        nd[i] = ((s + s2) - wx[i]) + s3;
      }
#pragma unroll
      for (int i = 0; i < n; ++i) {
        dlam[i] = nd[i];
#pragma unroll
        for (int k = 0; k < p; ++k) gx1[i][k] = gx[i][k];
      }
    }
    st(dtheta + (size_t)b * p, dth);
  }
}

}  // namespace dilqr

// ====================================================================== C-ABI
using namespace dilqr;

#ifdef DILQR_STAMPS
// diagnostic build only: copy the phase stamps of the last fused MPC iteration
extern "C" int dilqr_debug_stamps(unsigned long long* host, int n) {
  if (n > kStampWaves * kStampSlots) n = kStampWaves * kStampSlots;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : -1;
}
#endif

namespace {

inline int herr(hipError_t e) { return e == hipSuccess ? 0 : -(int)e; }
inline int launched() { return herr(hipGetLastError()); }
inline bool al16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline Bounds mkb(const dilqr_bounds& b) { return Bounds{b.mode, b.lo, b.hi, b.lo_t, b.hi_t}; }
inline bool bad_bounds(const dilqr_bounds& b) {
  if (b.mode == DILQR_BOUNDS_TENSOR) return !b.lo_t || !b.hi_t;
  return b.mode != DILQR_BOUNDS_NONE && b.mode != DILQR_BOUNDS_SCALAR;
}

// (n, m) shapes compiled for the generic (LinDx / Riccati / adjoint) kernels.
// Model kernels use their own fixed shapes.
#define DILQR_FOR_EACH_SHAPE(X) X(3, 1) X(5, 1) X(4, 3) X(4, 1) X(2, 1) X(4, 2) X(6, 2) X(6, 1)
// shapes served by the 16-lanes-per-problem kernels (dilqr_group.h)
#define DILQR_FOR_EACH_GROUP_SHAPE(X) X(13, 3)
#define DILQR_FOR_ALL_SHAPES(X) DILQR_FOR_EACH_SHAPE(X) DILQR_FOR_EACH_GROUP_SHAPE(X)

// the stop-rule kernel with its rows staged in LDS when a block's span fits
// (64 KiB), else read in place
// k_mpc_norm_rows geometry: rows staged in LDS when a block's span fits 64 KiB
struct NormGeom {
  int threads, blocks;
  bool stage;
};
inline NormGeom norm_geom(int TM, int B) {
  int threads = 256;
  while (threads > 64 && (size_t)threads * TM * sizeof(float) > 65536) threads >>= 1;
  const bool stage = (size_t)threads * TM * sizeof(float) <= 65536;
  if (!stage) threads = 256;
  return {threads, (B + threads - 1) / threads, stage};
}

inline int launch_norm_rows(int TM, int B, int iteration, const MpcState& st, hipStream_t stream) {
  const NormGeom g = norm_geom(TM, B);
  if (g.stage)
    k_mpc_norm_rows<true><<<g.blocks, g.threads, (size_t)g.threads * TM * sizeof(float), stream>>>(TM, B, iteration,
                                                                                                   st);
  else
    k_mpc_norm_rows<false><<<g.blocks, g.threads, 0, stream>>>(TM, B, iteration, st);
  return launched();
}

}  // namespace

extern "C" {

int dilqr_version(void) { return 4; }

int dilqr_model_num_ctrl(int model) {
  switch (model) {
    case DILQR_MODEL_PENDULUM: return Pendulum::M;
    case DILQR_MODEL_CARTPOLE: return Cartpole::M;
    case DILQR_MODEL_ROCKET: return Rocket::M;
    default: return -1;
  }
}

int dilqr_model_num_params(int model) {
  switch (model) {
    case DILQR_MODEL_PENDULUM: return Pendulum::P;
    case DILQR_MODEL_CARTPOLE: return Cartpole::P;
    case DILQR_MODEL_ROCKET: return Rocket::P;
    default: return -1;
  }
}

// every model (per-problem kernels whose state fits a lane: dynamics,
// Jacobians, rollouts)
#define MODEL_SWITCH(model, CALL)                       \
  switch (model) {                                      \
    case DILQR_MODEL_PENDULUM: { using MD = Pendulum; CALL; break; } \
    case DILQR_MODEL_CARTPOLE: { using MD = Cartpole; CALL; break; } \
    case DILQR_MODEL_ROCKET: { using MD = Rocket; CALL; break; }     \
    default: return DILQR_E_SHAPE;                      \
  }
// models whose Riccati state fits one lane (thread-per-problem kernels)
#define MODEL_SWITCH_TPP(model, CALL)                   \
  switch (model) {                                      \
    case DILQR_MODEL_PENDULUM: { using MD = Pendulum; CALL; break; } \
    case DILQR_MODEL_CARTPOLE: { using MD = Cartpole; CALL; break; } \
    default: return DILQR_E_SHAPE;                      \
  }
static inline int grid_group(long long B) { return (int)((B + kGPW - 1) / kGPW); }

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
  MODEL_SWITCH_TPP(model, (k_dynamics_vjp<MD><<<grid_for(N), kBlock, 0, S(stream)>>>(N, theta, x, u, gout, gtheta,
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

int dilqr_lqr_backward_f32(int n, int m, int T, int B, const float* C, const float* c, const float* x,
                           const float* u, const float* F, dilqr_bounds bounds, const unsigned char* u_zero_I,
                           int m_solver, float* K, float* k, int* n_qp_iter, void* stream) {
  if (T < 1 || B < 0 || !C || !c || !K || !k || (T > 1 && !F)) return DILQR_E_ARG;
  if (x && !u) return DILQR_E_ARG;   // u alone: c is already c_back, u only shifts the bounds
  if (!al16(C) || !al16(c) || !al16(x) || !al16(u) || !al16(F) || !al16(K) || !al16(k)) return DILQR_E_ARG;
  if (bad_bounds(bounds)) return DILQR_E_ARG;
  if (bounds.mode != DILQR_BOUNDS_NONE && (u_zero_I || !u)) return DILQR_E_MODE;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  int mode = bounds.mode != DILQR_BOUNDS_NONE ? GAIN_BOX
             : u_zero_I ? GAIN_ZERO_I
             : (m_solver == DILQR_SOLVE_CHOL && m > 1) ? GAIN_CHOL : GAIN_UNC;
#define LAUNCH(N_, M_, MODE_) \
  k_lqr_backward<N_, M_, MODE_><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, C, c, x, u, F, bd, u_zero_I, K, k, n_qp_iter)
#define X(N_, M_)                                              \
  if (n == N_ && m == M_) {                                    \
    switch (mode) {                                            \
      case GAIN_UNC: LAUNCH(N_, M_, GAIN_UNC); break;          \
      case GAIN_CHOL: LAUNCH(N_, M_, GAIN_CHOL); break;        \
      case GAIN_ZERO_I: LAUNCH(N_, M_, GAIN_ZERO_I); break;    \
      default: LAUNCH(N_, M_, GAIN_BOX); break;                \
    }                                                          \
    return launched();                                         \
  }
  DILQR_FOR_EACH_SHAPE(X)
#undef LAUNCH
#define LAUNCH(N_, M_, MODE_)                                                                                     \
  k_lqr_backward_group<N_, M_, MODE_><<<grid_group(B), 64, 0, S(stream)>>>(T, B, C, c, x, u, F, bd, u_zero_I, K, k, \
                                                                           n_qp_iter)
  DILQR_FOR_EACH_GROUP_SHAPE(X)
#undef X
#undef LAUNCH
  return DILQR_E_SHAPE;
}

int dilqr_lqr_forward_f32(int model, int n, int m, int T, int B, const float* theta, const float* F, const float* f,
                          const float* x_init, const float* C, const float* c, const float* x, const float* u,
                          const float* K, const float* k, dilqr_bounds bounds, const unsigned char* u_zero_I,
                          float linesearch_decay, int max_linesearch_iter, float* x_out, float* u_out, float* cost,
                          float* du_sq, float* alpha, const float* old_cost, void* stream) {
  if (T < 1 || B < 0 || max_linesearch_iter < 1) return DILQR_E_ARG;
  if (!x_init || !C || !c || !x || !u || !K || !k || !x_out || !u_out || !cost) return DILQR_E_ARG;
  const void* ps[] = {F, f, x_init, C, c, x, u, K, k, x_out, u_out};
  for (const void* p : ps) if (!al16(p)) return DILQR_E_ARG;
  if (bad_bounds(bounds)) return DILQR_E_ARG;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  if (model == DILQR_MODEL_LINDX) {
    if (!F && T > 1) return DILQR_E_ARG;
#define X(N_, M_)                                                                                             \
    if (n == N_ && m == M_) {                                                                                  \
      k_lqr_forward<N_, M_, NoModel><<<grid_for(B), kBlock, 0, S(stream)>>>(                                   \
          T, B, theta, F, f, x_init, C, c, x, u, K, k, bd, u_zero_I, linesearch_decay, max_linesearch_iter,     \
          x_out, u_out, cost, du_sq, alpha, old_cost);                                                         \
      return launched();                                                                                       \
    }
    DILQR_FOR_EACH_SHAPE(X)
#undef X
    if (old_cost) return DILQR_E_MODE;                 // the 16-lane kernels form it themselves
#define X(N_, M_)                                                                                             \
    if (n == N_ && m == M_) {                                                                                  \
      k_lqr_forward_group<N_, M_, GroupNoModel><<<grid_group(B), 64, 0, S(stream)>>>(                          \
          T, B, theta, F, f, x_init, C, c, x, u, K, k, bd, u_zero_I, linesearch_decay, max_linesearch_iter,     \
          x_out, u_out, cost, du_sq, alpha);                                                                   \
      return launched();                                                                                       \
    }
    DILQR_FOR_EACH_GROUP_SHAPE(X)
#undef X
    return DILQR_E_SHAPE;
  }
  if (!theta) return DILQR_E_ARG;
  if (model == DILQR_MODEL_ROCKET) {
    if (n != Rocket::N || m != Rocket::M) return DILQR_E_SHAPE;
    if (old_cost) return DILQR_E_MODE;
    k_lqr_forward_group<Rocket::N, Rocket::M, Rocket><<<grid_group(B), 64, 0, S(stream)>>>(
        T, B, theta, F, f, x_init, C, c, x, u, K, k, bd, u_zero_I, linesearch_decay, max_linesearch_iter, x_out,
        u_out, cost, du_sq, alpha);
    return launched();
  }
  MODEL_SWITCH_TPP(model, ({
    if (n != MD::N || m != MD::M) return DILQR_E_SHAPE;
    k_lqr_forward<MD::N, MD::M, MD><<<grid_for(B), kBlock, 0, S(stream)>>>(
        T, B, theta, F, f, x_init, C, c, x, u, K, k, bd, u_zero_I, linesearch_decay, max_linesearch_iter, x_out,
        u_out, cost, du_sq, alpha, old_cost);
  }));
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

int dilqr_ilqr_iterate_f32(int model, int T, int B, const float* theta, const float* x_init, const float* C,
                           const float* c, const float* x, const float* u, dilqr_bounds bounds,
                           float linesearch_decay, int max_linesearch_iter, float* ws_gains, float* x_out,
                           float* u_out, float* cost, float* du_sq, float* alpha, dilqr_mpc_ctrl* ctrl,
                           void* stream) {
  if (T < 1 || B < 0 || max_linesearch_iter < 1) return DILQR_E_ARG;
  if (!theta || !x_init || !C || !c || !x || !u || !ws_gains || !x_out || !u_out || !cost || !du_sq || !alpha)
    return DILQR_E_ARG;
  const void* ps[] = {x_init, C, c, x, u, ws_gains, x_out, u_out};
  for (const void* p : ps) if (!al16(p)) return DILQR_E_ARG;
  if (bad_bounds(bounds)) return DILQR_E_ARG;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  bool box = bounds.mode != DILQR_BOUNDS_NONE;
  if (model == DILQR_MODEL_ROCKET) {
    if (box)
      k_ilqr_iterate_group<Rocket, GAIN_BOX><<<grid_group(B), 64, 0, S(stream)>>>(
          T, B, theta, x_init, C, c, x, u, bd, linesearch_decay, max_linesearch_iter, ws_gains, x_out, u_out, cost,
          du_sq, alpha, ctrl);
    else
      k_ilqr_iterate_group<Rocket, GAIN_UNC><<<grid_group(B), 64, 0, S(stream)>>>(
          T, B, theta, x_init, C, c, x, u, bd, linesearch_decay, max_linesearch_iter, ws_gains, x_out, u_out, cost,
          du_sq, alpha, ctrl);
    return launched();
  }
#define LAUNCH_IT(BM_)                                                                                              \
  k_ilqr_iterate<MD, BM_><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, theta, x_init, C, c, x, u, bd, linesearch_decay, \
                                                                max_linesearch_iter, ws_gains, x_out, u_out, cost,  \
                                                                du_sq, alpha, ctrl)
  MODEL_SWITCH_TPP(model, ({
    if (bounds.mode == DILQR_BOUNDS_TENSOR) LAUNCH_IT(DILQR_BOUNDS_TENSOR);
    else if (box) LAUNCH_IT(DILQR_BOUNDS_SCALAR);
    else LAUNCH_IT(DILQR_BOUNDS_NONE);
  }));
#undef LAUNCH_IT
  return launched();
}

int dilqr_mpc_update_best_f32(int n, int m, int T, int B, int first, float best_cost_eps, float eps,
                              int not_improved_lim, const float* x, const float* u, const float* cost,
                              const float* du_sq, float* full_du_norm, float* best_x, float* best_u,
                              float* best_cost, float* best_du, dilqr_mpc_ctrl* ctrl, void* stream) {
  if (T < 1 || B < 0 || !x || !u || !cost || !du_sq || !full_du_norm || !best_x || !best_u || !best_cost ||
      !best_du || !ctrl)
    return DILQR_E_ARG;
  if (!al16(x) || !al16(u) || !al16(best_x) || !al16(best_u)) return DILQR_E_ARG;
  if (B > 0) {
    bool ok = false;
#define X(N_, M_)                                                                                        \
    if (!ok && n == N_ && m == M_) {                                                                      \
      k_mpc_best<N_, M_><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, first, best_cost_eps, x, u, cost, du_sq, \
                                                                full_du_norm, best_x, best_u, best_cost,  \
                                                                best_du, ctrl);                           \
      ok = true;                                                                                          \
    }
    DILQR_FOR_ALL_SHAPES(X)
#undef X
    if (!ok) return DILQR_E_SHAPE;
    int e = launched();
    if (e) return e;
  }
  k_mpc_control<<<1, 1, 0, S(stream)>>>(first, eps, not_improved_lim, ctrl);
  return launched();
}

int dilqr_lqr_adjoint_f32(int n, int m, int T, int B, const float* C, const float* c, const float* F,
                          const float* x, const float* u, const float* dl_dx, const float* dl_du, dilqr_bounds bounds,
                          int m_solver, float* ws, float* dx_init, float* dC, float* dc, float* dF, float* df,
                          void* stream) {
  if (T < 1 || B < 0 || !C || !c || !x || !u || !dl_dx || !dl_du || !ws || !dx_init || !dC || !dc) return DILQR_E_ARG;
  if (T > 1 && (!F || !dF)) return DILQR_E_ARG;
  const void* ps[] = {C, c, F, x, u, dl_dx, dl_du, ws, dx_init, dC, dc, dF, df};
  for (const void* p : ps) if (!al16(p)) return DILQR_E_ARG;
  if (bad_bounds(bounds)) return DILQR_E_ARG;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  bool chol = m_solver == DILQR_SOLVE_CHOL && m > 1;
#define X(N_, M_)                                                                                           \
  if (n == N_ && m == M_) {                                                                                  \
    if (chol)                                                                                                \
      k_lqr_adjoint<N_, M_, GAIN_CHOL><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, C, c, F, x, u, dl_dx,    \
                                                                             dl_du, bd, ws, dx_init, dC, dc, \
                                                                             dF, df);                        \
    else                                                                                                     \
      k_lqr_adjoint<N_, M_, GAIN_UNC><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, C, c, F, x, u, dl_dx,     \
                                                                            dl_du, bd, ws, dx_init, dC, dc,  \
                                                                            dF, df);                         \
    return launched();                                                                                       \
  }
  DILQR_FOR_EACH_SHAPE(X)
#undef X
  return DILQR_E_SHAPE;
}


int dilqr_implicit_ws_floats(int model) {
  switch (model) {
    case DILQR_MODEL_PENDULUM: return ImplicitWs<Pendulum>::REC;
    case DILQR_MODEL_CARTPOLE: return ImplicitWs<Cartpole>::REC;
    case DILQR_MODEL_ROCKET: return ImplicitGroupWs<Rocket>::REC;
    default: return -1;
  }
}

int dilqr_implicit_backward_f32(int model, int T, int B, const float* theta, const float* C, const float* c,
                                const float* x, const float* u, const float* K, const float* dl_dx,
                                const float* dl_du, dilqr_bounds bounds, float* ws, float* dC, float* dc,
                                float* dtheta, void* stream) {
  if (T < 1 || B < 0) return DILQR_E_ARG;
  if (!theta || !C || !c || !x || !u || !K || !dl_dx || !dl_du || !ws || !dC || !dc || !dtheta) return DILQR_E_ARG;
  const void* ps[] = {C, c, x, u, K, dl_dx, dl_du, ws, dC, dc, dtheta};
  for (const void* q : ps) if (!al16(q)) return DILQR_E_ARG;
  if (bad_bounds(bounds)) return DILQR_E_ARG;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  if (model == DILQR_MODEL_ROCKET) {
    if (bd.mode == DILQR_BOUNDS_NONE)
      k_implicit_backward_group<Rocket, gen::RocketD2, GAIN_UNC><<<grid_group(B), 64, 0, S(stream)>>>(
          T, B, theta, C, c, x, u, K, dl_dx, dl_du, bd, ws, dC, dc, dtheta);
    else
      k_implicit_backward_group<Rocket, gen::RocketD2, GAIN_ZERO_I><<<grid_group(B), 64, 0, S(stream)>>>(
          T, B, theta, C, c, x, u, K, dl_dx, dl_du, bd, ws, dC, dc, dtheta);
    return launched();
  }
  MODEL_SWITCH_TPP(model, (k_implicit_backward<MD><<<grid_for(B), kBlock, 0, S(stream)>>>(
                          T, B, theta, C, c, x, u, K, dl_dx, dl_du, bd, ws, dC, dc, dtheta)));
  return launched();
}


static bool bad_state(const dilqr_mpc_state& st) {
  return !st.Xs || !st.Us || !st.slot || !st.best_cost || !st.best_du || !st.improved || !st.cost || !st.alpha ||
         !st.du_sq || !st.full_du_norm || !st.ws || !st.ctrl || !st.done_counter || !al16(st.Xs) || !al16(st.Us) ||
         !al16(st.ws) || (st.Cpk && (!st.cost_sym || !al16(st.Cpk)));
}

int dilqr_mpc_packed_cost_floats(int n, int m) {
  const int d = n + m;
  return d < 1 ? -1 : d * (d + 1) / 2 + d;
}

int dilqr_mpc_begin_f32(int model, int T, int B, const float* theta, const float* x_init, const float* u_init,
                        dilqr_mpc_state st, void* stream) {
  if (T < 1 || B < 0 || !theta || !x_init || !al16(x_init) || bad_state(st)) return DILQR_E_ARG;
  if (u_init && ((uintptr_t)u_init & 3u)) return DILQR_E_ARG;
  MODEL_SWITCH(model, (k_mpc_begin<MD><<<grid_for(B > 0 ? B : 1), kBlock, 0, S(stream)>>>(T, B, theta, x_init, u_init,
                                                                                          st)));
  return launched();
}

// the fused iteration's launch; fixed: a fixed-count solve (no stop rule,
// this iteration's du rows into plane `iteration` of du_sq, best_iter kept)
static int mpc_step(int model, int T, int B, const float* theta, const float* x_init, const float* C, const float* c,
                    dilqr_bounds bounds, float linesearch_decay, int max_linesearch_iter, int iteration,
                    float best_cost_eps, float eps, int not_improved_lim, dilqr_mpc_state st, bool fixed,
                    void* stream) {
  if (T < 1 || B < 0 || max_linesearch_iter < 1 || iteration < 0 || !theta || !x_init || !C || !c) return DILQR_E_ARG;
  if (!al16(x_init) || !al16(C) || !al16(c) || bad_state(st) || bad_bounds(bounds)) return DILQR_E_ARG;
  if (fixed && !st.best_iter) return DILQR_E_ARG;
  if (B == 0) return 0;
  const int m = dilqr_model_num_ctrl(model);
  if (m < 1) return DILQR_E_SHAPE;
  // G: partials of the previous iteration's rows; < 0: fixed-count solve
  const int G = fixed ? -1 : norm_geom(T * m, B).blocks;
  if (fixed) st.du_sq += (size_t)iteration * T * m * B;
  else st.best_iter = nullptr;
  const int lim = not_improved_lim;
  Bounds bd = mkb(bounds);
  bool box = bounds.mode != DILQR_BOUNDS_NONE;
  if (model == DILQR_MODEL_ROCKET) {
    if (box)
      k_mpc_iterate_group<Rocket, GAIN_BOX><<<grid_group(B), 64, 0, S(stream)>>>(
          T, B, theta, x_init, C, c, bd, linesearch_decay, max_linesearch_iter, iteration, best_cost_eps, eps, lim,
          G, st);
    else
      k_mpc_iterate_group<Rocket, GAIN_UNC><<<grid_group(B), 64, 0, S(stream)>>>(
          T, B, theta, x_init, C, c, bd, linesearch_decay, max_linesearch_iter, iteration, best_cost_eps, eps, lim,
          G, st);
  } else {
#define LAUNCH_IT(BM_, LG_, FIRST_, LDS_)                                                                   \
  k_mpc_iterate<MD, BM_, LG_, FIRST_><<<grid_for(B), kBlock, LDS_, S(stream)>>>(                             \
      T, B, theta, x_init, C, c, bd, linesearch_decay, max_linesearch_iter, iteration, best_cost_eps, eps, lim, \
      G, st)
#define LAUNCH_MPC(BM_)                                                                                      \
  do {                                                                                                       \
    const size_t lds = (size_t)T * kBlock * (MD::N * MD::M + MD::M) * sizeof(float);                        \
    const bool lg = lds * 4 <= kLdsPerCU && !kNoLdsGains;                                                   \
    if (iteration == 0 && lg) LAUNCH_IT(BM_, true, true, lds);                                               \
    else if (iteration == 0) LAUNCH_IT(BM_, false, true, 0);                                                 \
    else if (lg) LAUNCH_IT(BM_, true, false, lds);                                                           \
    else LAUNCH_IT(BM_, false, false, 0);                                                                    \
  } while (0)
    MODEL_SWITCH_TPP(model, ({
      if (bounds.mode == DILQR_BOUNDS_TENSOR) LAUNCH_MPC(DILQR_BOUNDS_TENSOR);
      else if (box) LAUNCH_MPC(DILQR_BOUNDS_SCALAR);
      else LAUNCH_MPC(DILQR_BOUNDS_NONE);
    }));
#undef LAUNCH_MPC
#undef LAUNCH_IT
  }
  return launched();
}

int dilqr_mpc_step_f32(int model, int T, int B, const float* theta, const float* x_init, const float* C,
                       const float* c, dilqr_bounds bounds, float linesearch_decay, int max_linesearch_iter,
                       int iteration, float best_cost_eps, float eps, int not_improved_lim, dilqr_mpc_state st,
                       void* stream) {
  return mpc_step(model, T, B, theta, x_init, C, c, bounds, linesearch_decay, max_linesearch_iter, iteration,
                  best_cost_eps, eps, not_improved_lim, st, false, stream);
}

int dilqr_mpc_iterate_fixed_f32(int model, int T, int B, const float* theta, const float* x_init, const float* C,
                                const float* c, dilqr_bounds bounds, float linesearch_decay, int max_linesearch_iter,
                                int iteration, float best_cost_eps, dilqr_mpc_state st, void* stream) {
  return mpc_step(model, T, B, theta, x_init, C, c, bounds, linesearch_decay, max_linesearch_iter, iteration,
                  best_cost_eps, 0.f, 0, st, true, stream);
}

int dilqr_mpc_finish_fixed_f32(int T, int m, int B, int iterations, dilqr_mpc_state st, void* stream) {
  if (T < 1 || m < 1 || B < 0 || iterations < 1 || bad_state(st) || !st.best_iter) return DILQR_E_ARG;
  if (B == 0) return 0;
  k_mpc_fixed_finish<<<(B + 255) / 256, 256, 0, S(stream)>>>(T * m, B, iterations, st);
  return launched();
}

int dilqr_mpc_stop_rule_f32(int T, int m, int B, int iteration, dilqr_mpc_state st, void* stream) {
  if (T < 1 || m < 1 || B < 0 || iteration < 0 || bad_state(st)) return DILQR_E_ARG;
  if (B == 0) return 0;
  return launch_norm_rows(T * m, B, iteration, st, S(stream));
}

int dilqr_mpc_iterate_f32(int model, int T, int B, const float* theta, const float* x_init, const float* C,
                          const float* c, dilqr_bounds bounds, float linesearch_decay, int max_linesearch_iter,
                          int iteration, float best_cost_eps, float eps, int not_improved_lim, dilqr_mpc_state st,
                          void* stream) {
  const int m = dilqr_model_num_ctrl(model);
  if (m < 1) return DILQR_E_SHAPE;
  int e = dilqr_mpc_step_f32(model, T, B, theta, x_init, C, c, bounds, linesearch_decay, max_linesearch_iter,
                             iteration, best_cost_eps, eps, not_improved_lim, st, stream);
  if (e) return e;
  return dilqr_mpc_stop_rule_f32(T, m, B, iteration, st, stream);
}

int dilqr_mpc_gather_best_f32(int n, int m, int T, int B, dilqr_mpc_state st, float* x_out, float* u_out,
                              void* stream) {
  if (T < 1 || B < 0 || !x_out || !u_out || !al16(x_out) || !al16(u_out) || bad_state(st)) return DILQR_E_ARG;
  if (B == 0) return 0;
#define X(N_, M_) \
  if (n == N_ && m == M_) { k_mpc_gather<N_, M_><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, st, x_out, u_out); return launched(); }
  DILQR_FOR_ALL_SHAPES(X)
#undef X
  return DILQR_E_SHAPE;
}

}  // extern "C"
