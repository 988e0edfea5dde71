// tu_implicit.hip — the DiLQR implicit backward for the one-problem-per-lane
// models (pendulum, cartpole); rocket's 16-lane kernel is in tu_implicit_rocket.hip.
#include "dilqr_common.h"
#include "dilqr_launch.h"

namespace dilqr {

// ============================================================ DiLQR implicit backward
// lqr_step_explicit.py:653-712 + fix_point_equ 458-598, by the algebra of
// oracle/adjoint.py implicit_backward_fast (validated against the literal
// restatement to 1e-14 in fp64): the reference's (T d)^2 system A^T w = g is one
// extra LQR solve with cost C_t + M_t^T, M_t = sum_i lam_{t+1,i} d D_t[i] / d tau
// (the Lagrangian Hessian of the dynamics), after which dC, dc, dtheta are the
// KKT gradients of the adjoint solve with r = w, whose trajectory is that same
// solve's y.  Per problem (one lane), three passes over T:
//   B (t down): primal costates lam_t (registers); M_t; Riccati step with
//               C_t + M_t^T, c_back = -g_t, active set masked (u_zero_I engine);
//               the gains (K_t, k_t) -> ws
//   C (t up)  : the rollout y of the modified problem (linear, alpha = 1) -> ws
//   D (t down): lam_t again (the same recursion as B: nothing stored), w_t =
//               g_t - M_t^T y_t, dlam; dC_t, dc_t out; dtheta.
// dtheta = sum_t [-y_t^T Mp_t + h_t^T gradx_t] where gradx_t is grad_input's
// closed-loop d x_t / d theta (cartpole.py:755-769: gradx_t = f_theta,t +
// A_t gradx_{t-1}, A_t = D_x,t + D_u,t Krev_t, with the reference's reversed-K
// and x_grad_xtm1 quirks).  Rather than roll gradx up (n*p floats per step
// stored and re-read), pass D carries its adjoint mu_t = h_t + A_{t+1}^T
// mu_{t+1} down and adds f_theta,t^T mu_t: the same sum, O(n) state, no
// storage.  The workspace is two component-major records per (t, b), the
// gains and y (SoaRec planes: a wave's loads are 1-KiB runs); the caller's
// tensors are the only other traffic.
template <class Model> struct ImplicitWs {
  static constexpr int n = Model::N, m = Model::M, d = n + m;
  static constexpr int G = m * n + m;                  // K_t, k_t of the modified Riccati step
  // floats per (t, b): the gain planes, the y planes, slack so the y region
  // starts 16-byte aligned whatever T*B is
  static constexpr int REC = G + d + 4;
  static DEV size_t y_off(int T, int B) { return ((size_t)T * B * G + 3) / 4 * 4; }
};

// lam_t = Cxx x + Cxu u + c_x + F_x^T lam_{t+1}   (lqr_step_explicit.py:305-319);
// D is zero at t = T-1.  Passes B and D run this same function on the same
// inputs, so they hold the same bits.
template <int n, int m, class FS = DenseF>
DEV void costate_step(const float (&Ct)[n + m][n + m], const float (&cx)[n], const float (&xt)[n],
                      const float (&ut)[m], const float (&D)[n][n + m], float (&lam)[n]) {
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
    for (int l = 0; l < n; ++l)
      if (FS::nz(l, i)) s3 += D[l][i] * lam[l];
    nl[i] = ((s + s2) + cx[i]) + s3;
  }
#pragma unroll
  for (int i = 0; i < n; ++i) lam[i] = nl[i];
}

// DILQR_IMPL_SKIP: timing-only builds (tools/ab.sh variants, never the shipped
// library) that leave out pass C (bit 0) and/or pass D (bit 1), to split the
// kernel's time by pass as rocket's group kernel does, or pass D's generated
// pieces (bit 2 lag_hess, bit 3 lag_dparam, bit 4 f_theta_cs: zeros instead)
#ifndef DILQR_IMPL_SKIP
#define DILQR_IMPL_SKIP 0
#endif
#ifndef DILQR_IMPL_PFD
#define DILQR_IMPL_PFD 1
#endif
#ifndef DILQR_IMPL_PFB
#define DILQR_IMPL_PFB 1
#endif
#ifndef DILQR_IMPL_PFC
#define DILQR_IMPL_PFC 0
#endif

// One wave's records of K floats for problems b0 .. b0+63 of one step are one
// contiguous run of 64*K floats ([t, b, K] layout).  Each lane writes its record
// to LDS and the wave stores the run coalesced (a 1-KiB dwordx4 run per
// instruction) instead of each lane storing its own 144-byte record: per-lane
// record stores ran at half the HBM write rate of coalesced ones
// (tools/microbench/store_patterns.hip).  One wave per workgroup
// (kBlock = 64): its LDS accesses complete in program order, so the wave
// barriers (scheduling only) are the whole synchronisation.  Lane strides of K
// dwords (K/4 float4, K/2 float2) keep the b128 / b64 writes bank-conflict free
// for the K used here (16, 36; 4, 6).
template <int K>
DEV void wave_store_records(float* __restrict__ base, const float (&r)[K], float* __restrict__ lds, int lane,
                            int nvalid) {
  static_assert(K % 2 == 0, "records of an even number of floats");
  __builtin_amdgcn_wave_barrier();                 // the previous step's reads of lds precede these writes
  if constexpr (K % 4 == 0) {
    constexpr int Q = K / 4;
    float4* L = reinterpret_cast<float4*>(lds);
#pragma unroll
    for (int i = 0; i < Q; ++i) L[lane * Q + i] = make_float4(r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]);
    __builtin_amdgcn_wave_barrier();
    float4* g = reinterpret_cast<float4*>(base);
    const int nv = nvalid * Q;
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const int i = lane + 64 * j;
      if (i < nv) g[i] = L[i];
    }
  } else {
    constexpr int Q = K / 2;
    float2* L = reinterpret_cast<float2*>(lds);
#pragma unroll
    for (int i = 0; i < Q; ++i) L[lane * Q + i] = make_float2(r[2 * i], r[2 * i + 1]);
    __builtin_amdgcn_wave_barrier();
    float2* g = reinterpret_cast<float2*>(base);
    const int nv = nvalid * Q;
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const int i = lane + 64 * j;
      if (i < nv) g[i] = L[i];
    }
  }
}

template <class Model>
__global__ void __launch_bounds__(kBlock) k_implicit_backward(
    int T, int B, const float* __restrict__ theta, const float* __restrict__ C, const float* __restrict__ c,
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ K,
    const float* __restrict__ dl_dx, const float* __restrict__ dl_du, Bounds bd, float* __restrict__ ws,
    float* __restrict__ dC, float* __restrict__ dc, float* __restrict__ dtheta) {
  using D2 = typename D2Of<Model>::type;
  using DZ = D2Of<Model>;                          // structural zeros of the generated pieces
  using FS = typename Model::FSparsity;            // ... and of the Jacobian
  using W = ImplicitWs<Model>;
  constexpr int n = Model::N, m = Model::M, p = Model::P, d = n + m, G = W::G;
  // every lane of the wave runs (pass D stores the wave's dC, dc records
  // together); lanes past the batch shadow problem B-1 and store nothing
  const int lane = threadIdx.x, b0 = blockIdx.x * kBlock;
  const int nvalid = B - b0 < kBlock ? B - b0 : kBlock;
  const bool valid = lane < nvalid;
  const int b = valid ? b0 + lane : B - 1;
  __shared__ __attribute__((aligned(16))) float s_dC[kBlock * d * d];
  __shared__ __attribute__((aligned(16))) float s_dc[kBlock * d];
  Model md; md.load(theta);
  float* const wsG = ws;
  float* const wsY = ws + W::y_off(T, B);
  auto active = [&](size_t tb, int a, float ua) -> bool {
    if (bd.mode == DILQR_BOUNDS_NONE) return false;
    return fabsf(ua - bound_lo(bd, tb * m + a)) <= 1e-8f || fabsf(ua - bound_hi(bd, tb * m + a)) <= 1e-8f;
  };
  auto zero_D = [](float (&D)[n][d]) {
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
      for (int j = 0; j < d; ++j) D[i][j] = 0.f;
  };
  // Pass B also tests whether the problem's C_t are one diagonal matrix for all
  // t (every off-diagonal word +0.0, the diagonals equal to step T-1's bit for
  // bit — the reference's callers pass diag(q) repeated over t) and whether the
  // c_t are one vector: pass D then takes them from these registers instead of
  // reading them again (the same values, so the same arithmetic).
  float cdiag[d], cvec[d];
  unsigned c_offd = 0u, c_dif = 0u, cv_dif = 0u;
  // ---------------- B: costates, M_t, Riccati of the C + M^T problem
  {
    RiccatiState<n, m> rs;
    rs.init();
    float lam[n];
#pragma unroll
    for (int i = 0; i < n; ++i) lam[i] = 0.f;
#if DILQR_IMPL_PFB
    // step t-1's x, u and loss gradients loaded while step t computes (1, the
    // shipped setting: config 4 0.220 -> 0.207 ms; 2, C_t and c_t too: 28
    // AGPRs, 0.213 ms — profiles/r06/ab_implicit_cartpole_prefetch.txt)
    struct BIn {
      float x[n], u[m], gx[n], gu[m];
#if DILQR_IMPL_PFB > 1
      float C[d][d], c[d];
#endif
    };
    auto load_b = [&](int t, BIn& in) {
      const size_t tb = (size_t)t * B + b;
      ld(in.x, x + tb * n); ld(in.u, u + tb * m); ld(in.gx, dl_dx + tb * n); ld(in.gu, dl_du + tb * m);
#if DILQR_IMPL_PFB > 1
      ld2(in.C, C + tb * d * d); ld(in.c, c + tb * d);
#endif
    };
    BIn bin;
    load_b(T - 1, bin);
#endif
    for (int t = T - 1; t >= 0; --t) {
      size_t tb = (size_t)t * B + b;
      float Ct[d][d], ct[d], xt[n], ut[m], gxx[n], gu[m];
#if DILQR_IMPL_PFB
      BIn bnx;
      load_b(t > 0 ? t - 1 : 0, bnx);
#pragma unroll
      for (int i = 0; i < n; ++i) { xt[i] = bin.x[i]; gxx[i] = bin.gx[i]; }
#pragma unroll
      for (int a = 0; a < m; ++a) { ut[a] = bin.u[a]; gu[a] = bin.gu[a]; }
#if DILQR_IMPL_PFB > 1
#pragma unroll
      for (int i = 0; i < d; ++i) {
        ct[i] = bin.c[i];
#pragma unroll
        for (int j = 0; j < d; ++j) Ct[i][j] = bin.C[i][j];
      }
#else
      ld2(Ct, C + tb * d * d); ld(ct, c + tb * d);
#endif
      bin = bnx;
#else
      ld2(Ct, C + tb * d * d); ld(ct, c + tb * d); ld(xt, x + tb * n); ld(ut, u + tb * m);
      ld(gxx, dl_dx + tb * n); ld(gu, dl_du + tb * m);
#endif
      if (t == T - 1) {
#pragma unroll
        for (int i = 0; i < d; ++i) { cdiag[i] = Ct[i][i]; cvec[i] = ct[i]; }
      }
#pragma unroll
      for (int i = 0; i < d; ++i) {
        c_dif |= __float_as_uint(Ct[i][i]) ^ __float_as_uint(cdiag[i]);
        cv_dif |= __float_as_uint(ct[i]) ^ __float_as_uint(cvec[i]);
#pragma unroll
        for (int j = 0; j < d; ++j)
          if (j != i) c_offd |= __float_as_uint(Ct[i][j]);
      }
      float D[n][d];
      float Mt[d][d];
      if (t < T - 1) {
        float cn, sn;                                     // the integrated angle, once per step
        md.next_cs(xt, ut, cn, sn);
        md.jacobian_sc(xt, ut, cn, sn, D);
        D2::lag_hess(theta, xt, ut, lam, cn, sn, Mt);     // lam = lam_{t+1}
      } else {
        zero_D(D);
#pragma unroll
        for (int i = 0; i < d; ++i)
#pragma unroll
          for (int j = 0; j < d; ++j) Mt[i][j] = 0.f;
      }
      float Cp[d][d], cb[d];
#pragma unroll
      for (int i = 0; i < d; ++i)
#pragma unroll
        for (int j = 0; j < d; ++j) Cp[i][j] = DZ::hess_nz(j, i) ? Ct[i][j] + Mt[j][i] : Ct[i][j];
#pragma unroll
      for (int i = 0; i < n; ++i) cb[i] = -gxx[i];
#pragma unroll
      for (int a = 0; a < m; ++a) cb[n + a] = -gu[a];
      float zI[m], lb[m], ub[m];
#pragma unroll
      for (int a = 0; a < m; ++a) { zI[a] = active(tb, a, ut[a]) ? 1.f : 0.f; lb[a] = ub[a] = 0.f; }
      float Kt[m][n], kt[m];
      if (bd.mode != DILQR_BOUNDS_NONE) rs.template step<GAIN_ZERO_I, FS>(Cp, cb, D, zI, lb, ub, Kt, kt);
      else rs.template step<GAIN_UNC, FS>(Cp, cb, D, zI, lb, ub, Kt, kt);
      float gr[G];
#pragma unroll
      for (int a = 0; a < m; ++a) {
#pragma unroll
        for (int j = 0; j < n; ++j) gr[a * n + j] = Kt[a][j];
        gr[m * n + a] = kt[a];
      }
      if (valid) SoaRec<G>::store(wsG, gr, T, t, B, b);
      float cx[n];
#pragma unroll
      for (int i = 0; i < n; ++i) cx[i] = ct[i];
      costate_step<n, m, FS>(Ct, cx, xt, ut, D, lam);
    }
  }
  const bool c_regs = c_offd == 0u && c_dif == 0u, cv_regs = cv_dif == 0u;
  // ---------------- C (t up): the rollout y of the modified problem (linear,
  // alpha = 1, active controls zeroed)
  {
    float yx[n];
#pragma unroll
    for (int i = 0; i < n; ++i) yx[i] = 0.f;
#if DILQR_IMPL_PFC
    struct CIn {
      float x[n], u[m], g[G];
    };
    auto load_c = [&](int t, CIn& in) {
      const size_t tb = (size_t)t * B + b;
      ld(in.x, x + tb * n); ld(in.u, u + tb * m);
      SoaRec<G>::load(in.g, wsG, T, t, B, b);
    };
    CIn cpre;
    load_c(0, cpre);
#endif
    for (int t = 0; t < ((DILQR_IMPL_SKIP & 1) ? 0 : T); ++t) {
      size_t tb = (size_t)t * B + b;
      float xt[n], ut[m], gr[G];
#if DILQR_IMPL_PFC
      CIn cnx;
      load_c(t + 1 < T ? t + 1 : t, cnx);
#pragma unroll
      for (int i = 0; i < n; ++i) xt[i] = cpre.x[i];
#pragma unroll
      for (int a = 0; a < m; ++a) ut[a] = cpre.u[a];
#pragma unroll
      for (int i = 0; i < G; ++i) gr[i] = cpre.g[i];
      cpre = cnx;
#else
      ld(xt, x + tb * n); ld(ut, u + tb * m);
      SoaRec<G>::load(gr, wsG, T, t, B, b);
#endif
      float y[d];
#pragma unroll
      for (int i = 0; i < n; ++i) y[i] = yx[i];
#pragma unroll
      for (int a = 0; a < m; ++a) {
        float s_ = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s_ += gr[a * n + j] * yx[j];
        y[n + a] = active(tb, a, ut[a]) ? 0.f : (s_ + 0.f) + gr[m * n + a];
      }
      if (valid) SoaRec<d>::store(wsY, y, T, t, B, b);
      if (t < T - 1) {
        float D[n][d];
        md.jacobian(xt, ut, D);
#pragma unroll
        for (int i = 0; i < n; ++i) {
          float s_ = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j)
            if (FS::nz(i, j)) s_ += D[i][j] * y[j];
          yx[i] = s_;
        }
      }
    }
  }
  // ---------------- D: lam, w, dlam, dC, dc, dtheta (t down)
  {
    float lam[n], dlam[n], mu[n], ax[n], au[m], dth[p];
#pragma unroll
    for (int i = 0; i < n; ++i) { lam[i] = 0.f; dlam[i] = 0.f; mu[i] = 0.f; ax[i] = 0.f; }
#pragma unroll
    for (int a = 0; a < m; ++a) au[a] = 0.f;
#pragma unroll
    for (int k = 0; k < p; ++k) dth[k] = 0.f;
#if DILQR_IMPL_PFD
    // step t-1's per-step inputs are loaded while step t computes (one wave per
    // SIMD: nothing else covers the loads' latency); the index clamps at 0, so
    // the load is unconditional (a conditional one drains the queue at its merge).
    // Config 4: 0.227 -> 0.221 ms (profiles/r06/ab_implicit_cartpole_prefetch.txt)
    struct DIn {
      float x[n], u[m], gx[n], gu[m], y[d], K[m][n];
    };
    auto load_in = [&](int t, DIn& in) {
      const size_t tb = (size_t)t * B + b;
      ld(in.x, x + tb * n); ld(in.u, u + tb * m);
      ld(in.gx, dl_dx + tb * n); ld(in.gu, dl_du + tb * m);
      SoaRec<d>::load(in.y, wsY, T, t, B, b);
      ld2(in.K, K + ((size_t)(T - 1 - t) * B + b) * m * n);
    };
    DIn cin;
    load_in(T - 1, cin);
#endif
    for (int t = (DILQR_IMPL_SKIP & 2) ? -1 : T - 1; t >= 0; --t) {
      size_t tb = (size_t)t * B + b;
      float Ct[d][d], ct[d], xt[n], ut[m], gxx[n], gu[m], y[d];
#if DILQR_IMPL_PFD
      DIn nin;
      load_in(t > 0 ? t - 1 : 0, nin);
#endif
      if (c_regs) {
#pragma unroll
        for (int i = 0; i < d; ++i)
#pragma unroll
          for (int j = 0; j < d; ++j) Ct[i][j] = i == j ? cdiag[i] : 0.f;
      } else {
        ld2(Ct, C + tb * d * d);
      }
      if (cv_regs) {
#pragma unroll
        for (int i = 0; i < d; ++i) ct[i] = cvec[i];
      } else {
        ld(ct, c + tb * d);
      }
#if DILQR_IMPL_PFD
#pragma unroll
      for (int i = 0; i < n; ++i) { xt[i] = cin.x[i]; gxx[i] = cin.gx[i]; }
#pragma unroll
      for (int a = 0; a < m; ++a) { ut[a] = cin.u[a]; gu[a] = cin.gu[a]; }
#pragma unroll
      for (int i = 0; i < d; ++i) y[i] = cin.y[i];
#else
      ld(xt, x + tb * n); ld(ut, u + tb * m);
      ld(gxx, dl_dx + tb * n); ld(gu, dl_du + tb * m);
      SoaRec<d>::load(y, wsY, T, t, B, b);
#endif
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
      wave_store_records<d * d>(dC + ((size_t)t * B + b0) * d * d,
                                *reinterpret_cast<const float(*)[d * d]>(&dCt[0][0]), s_dC, lane, nvalid);
      wave_store_records<d>(dc + ((size_t)t * B + b0) * d, dct, s_dc, lane, nvalid);
      float D[n][d], wx[n], hx[n], cn, sn;
      md.next_cs(xt, ut, cn, sn);         // the integrated angle, once per step
      md.jacobian_sc(xt, ut, cn, sn, D);  // D_t (t = T-1: only for A_{T-1} of the mu carry)
      // the carry A_{t+1}^T mu_{t+1} = (D_x,t+1)^T mu_{t+1} + Krev^T (D_u,t+1)^T mu_{t+1},
      // Krev = K[t] of the reversed stack = K_{T-1-t}: the gain grad_input pairs with step t+1
      if (t < T - 1) {
        float Kq[m][n], Mt[d][d], Mp[d][p];
#if DILQR_IMPL_PFD
#pragma unroll
        for (int a = 0; a < m; ++a)
#pragma unroll
          for (int j = 0; j < n; ++j) Kq[a][j] = cin.K[a][j];
#else
        ld2(Kq, K + ((size_t)(T - 1 - t) * B + b) * m * n);
#endif
#if DILQR_IMPL_SKIP & 4
#pragma unroll
        for (int i = 0; i < d; ++i)
#pragma unroll
          for (int j = 0; j < d; ++j) Mt[i][j] = 0.f;
#else
        D2::lag_hess(theta, xt, ut, lam, cn, sn, Mt);  // lam = lam_{t+1}
#endif
#if DILQR_IMPL_SKIP & 8
#pragma unroll
        for (int i = 0; i < d; ++i)
#pragma unroll
          for (int j = 0; j < p; ++j) Mp[i][j] = 0.f;
#else
        D2::lag_dparam(theta, xt, ut, lam, cn, sn, Mp);
#endif
        // w_t = g_t - M_t^T y_t
#pragma unroll
        for (int k = 0; k < n; ++k) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j)
            if (DZ::hess_nz(j, k)) s += Mt[j][k] * y[j];
          wx[k] = gxx[k] - s;
        }
        // dtheta_t = -(y^T Mp) + h_t^T gradx_t - dlam_{t+1}^T gradx_{t+1} with
        // h_t = dlam_{t+1}^T (D_x + D_u Kq) - y^T (M_x + M_u Kq)
#pragma unroll
        for (int k = 0; k < p; ++k) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j)
            if (DZ::dparam_nz(j, k)) s += y[j] * Mp[j][k];
          dth[k] -= s;
        }
#pragma unroll
        for (int l = 0; l < n; ++l) {
          float s = 0.f, s2 = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) {
            bool any = DZ::hess_nz(j, l);
            float ml = any ? Mt[j][l] : 0.f;
#pragma unroll
            for (int a = 0; a < m; ++a)
              if (DZ::hess_nz(j, n + a)) { ml += Mt[j][n + a] * Kq[a][l]; any = true; }
            if (any) s += y[j] * ml;
          }
#pragma unroll
          for (int i = 0; i < n; ++i) {
            bool any = FS::nz(i, l);
            float dl = any ? D[i][l] : 0.f;
#pragma unroll
            for (int a = 0; a < m; ++a)
              if (FS::nz(i, n + a)) { dl += D[i][n + a] * Kq[a][l]; any = true; }
            if (any) s2 += dlam[i] * dl;
          }
          hx[l] = s2 - s;
        }
        // mu carry from step t+1 (A_{t+1} pairs D_{t+1} with this step's Kq)
#pragma unroll
        for (int l = 0; l < n; ++l) {
          float s = ax[l];
#pragma unroll
          for (int a = 0; a < m; ++a) s += Kq[a][l] * au[a];
          hx[l] += s;
        }
      } else {
#pragma unroll
        for (int k = 0; k < n; ++k) { wx[k] = gxx[k]; hx[k] = 0.f; }
      }
      // dlam_t = Cxx y_x + Cxu y_u - w_x + F_x^T dlam_{t+1}   (lqr_step_explicit.py:321-335);
      // lam_t by the pass-B recursion (F_t = D_t for t < T-1, zero at T-1)
      float cx[n];
#pragma unroll
      for (int i = 0; i < n; ++i) cx[i] = ct[i];
      {
        float Dl[n][d];
        if (t < T - 1) {
#pragma unroll
          for (int i = 0; i < n; ++i)
#pragma unroll
            for (int j = 0; j < d; ++j) Dl[i][j] = D[i][j];
        } else {
          zero_D(Dl);
        }
        float nd[n];
#pragma unroll
        for (int i = 0; i < n; ++i) {
          float s = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
          for (int j = 0; j < n; ++j) s += Ct[i][j] * y[j];
#pragma unroll
          for (int a = 0; a < m; ++a) s2 += Ct[i][n + a] * y[n + a];
#pragma unroll
          for (int l = 0; l < n; ++l)
            if (FS::nz(l, i)) s3 += Dl[l][i] * dlam[l];
          nd[i] = ((s + s2) - wx[i]) + s3;
        }
#pragma unroll
        for (int i = 0; i < n; ++i) dlam[i] = nd[i];
        costate_step<n, m, FS>(Ct, cx, xt, ut, Dl, lam);
      }
      if (t >= 1) {
        // mu_t = h_t - dlam_t (+ the carry, folded into h_t above); dtheta += f_theta,t^T mu_t
#pragma unroll
        for (int l = 0; l < n; ++l) mu[l] = hx[l] - dlam[l];
        float ft[n][p];
#if DILQR_IMPL_SKIP & 16
#pragma unroll
        for (int i = 0; i < n; ++i)
#pragma unroll
          for (int j = 0; j < p; ++j) ft[i][j] = 0.f;
#else
        D2::f_theta_cs(theta, xt, ut, cn, sn, ft);
#endif
#pragma unroll
        for (int k = 0; k < p; ++k) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < n; ++i)
            if (DZ::ftheta_nz(i, k)) s += ft[i][k] * mu[i];
          dth[k] += s;
        }
        // the next step's carry: (D_x,t)^T mu_t (the x_grad_xtm1 quirk: no D[0][0]) and (D_u,t)^T mu_t
#pragma unroll
        for (int l = 0; l < n; ++l) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < n; ++i)
            if (FS::nz(i, l) && !(D2Of<Model>::XX00_ZERO && i == 0 && l == 0)) s += D[i][l] * mu[i];
          ax[l] = s;
        }
#pragma unroll
        for (int a = 0; a < m; ++a) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < n; ++i)
            if (FS::nz(i, n + a)) s += D[i][n + a] * mu[i];
          au[a] = s;
        }
      }
#if DILQR_IMPL_PFD
      cin = nin;
#endif
    }
    if (valid) st(dtheta + (size_t)b * p, dth);
  }
}

}  // namespace dilqr

using namespace dilqr;

extern "C" {

int dilqr_implicit_ws_floats(int model) {
  switch (model) {
    case DILQR_MODEL_PENDULUM: return ImplicitWs<Pendulum>::REC;
    case DILQR_MODEL_CARTPOLE: return ImplicitWs<Cartpole>::REC;
    case DILQR_MODEL_ROCKET: return implicit_rocket_ws_floats();
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
  if (model == DILQR_MODEL_ROCKET)
    return launch_implicit_rocket(ImplicitArgs{T, B, theta, C, c, x, u, K, dl_dx, dl_du, bd, ws, dC, dc, dtheta,
                                               S(stream)});
  MODEL_SWITCH_TPP_D2(model, (k_implicit_backward<MD><<<grid_for(B), kBlock, 0, S(stream)>>>(
                          T, B, theta, C, c, x, u, K, dl_dx, dl_du, bd, ws, dC, dc, dtheta)));
  return launched();
}

}  // extern "C"
