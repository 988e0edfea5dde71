// dilqr_implicit_group.h — the DiLQR implicit backward (k_implicit_backward,
// tu_implicit.hip) for the 16-lanes-per-problem models (rocket, d = 16).
// Included by tu_implicit_rocket.hip after dilqr_group.h.
//
// Same three passes (B down, C up, D down) and the same algebra as the one-lane kernel
// (oracle/adjoint.py implicit_backward_fast; lqr_step_explicit.py:653-712 with
// rocket's grad_input, rocket.py:263-323, and its build_batched_* tables,
// rocket.py:541-820), distributed by rows: lane r owns row r of every d x d or
// n x p quantity.  The pieces come from the generated RocketD2:
//   mcol(r)   column r of M_t = sum_i lam_{t+1,i} dD_t[i]/dtau   (so row r of
//             the modified cost C_t + M_t^T is C_t[r] + mcol(r))
//   mp_row(r) row r of sum_i lam_{t+1,i} dD_t[i]/dtheta
//   xx_row(r) row r of the reference's x_grad_xtm1 builder
//   xth_row(r) row r of dx_{t+1}/dtheta
// and Model::jac_row(r) (row r of D_t, which is also x_grad_utm1's source).
// Vectors every lane needs in full (lam, dlam, y, the adjoint carry) go through LDS; the
// Riccati step of the modified problem is the sweeps' transposed step
// (group_riccati_step_c, DILQR_IMPL_BT).
#pragma once

#include "dilqr_group.h"

#ifndef DILQR_IMPL_SKIP
#define DILQR_IMPL_SKIP 0
#endif
#ifndef DILQR_IMPL_C_PF
#define DILQR_IMPL_C_PF 1
#endif
// DILQR_IMPL_NT: dC, dc written with non-temporal stores (A/B: ~2 % slower,
// profiles/r06/ab_implicit_rocket_nt_stores.txt)
#ifndef DILQR_IMPL_NT
#define DILQR_IMPL_NT 0
#endif
// DILQR_IMPL_GPFB / GPFD: passes B / D loading step t-1's inputs one step
// ahead (A/B only: 1.16-1.25 ms with either, both or neither, within the
// noise; profiles/r06/ab_implicit_rocket_prefetch_BD.txt)
#ifndef DILQR_IMPL_GPFB
#define DILQR_IMPL_GPFB 0
#endif
#ifndef DILQR_IMPL_GPFD
#define DILQR_IMPL_GPFD 0
#endif

namespace dilqr {

// per-(t,b) workspace record (floats), written lane-contiguous: what pass C
// and pass D cannot recompute — the modified Riccati step's gains (B -> C) and
// the rollout y (C -> D).  The costates are recomputed by pass D and gradx is
// replaced by its adjoint (tu_implicit.hip), so neither is stored.
template <class Model> struct ImplicitGroupWs {
  static constexpr int n = Model::N, m = Model::M, p = Model::P;
  static constexpr int KG = 0;                 // [m][16]: K[a][r] at r < n, k[a] at n
  static constexpr int Y = KG + m * kG;        // y_t, [16]
  static constexpr int REC = Y + kG;
};

template <int n, int p>
struct ImplicitGroupLds {
  // rows of the gradx-adjoint carry: row i = mu_i * x_grad_xtm1[i][:] (lane i
  // writes its row, lane l sums column l); odd row stride for the column reads
  float ax[n][n + 2];
  float vec[kG];                               // lam_{t+1} (B) / y_t (C)
  float lam[kG];                               // lam_{t+1} (D)
  float dlam[kG];                              // dlam_{t+1} (D)
};

// DILQR_IMPL_BT (default 1): pass B's Riccati step in the sweeps' transposed
// form (group_riccati_step_c: V_{t+1} column r in lane r's registers, W = V^T F
// and Q's rows exchanged through LDS, both products over the Jacobian's
// structural nonzeros, Rocket::FSparsity 69 of 208, read from the F rows the
// costates need in LDS anyway; the unconstrained value update in Schur form)
// instead of the rows-of-V step (group_riccati_step: two dense 13x13x16
// products on V and F rows from LDS).  0 keeps the old step (A/B only).
#ifndef DILQR_IMPL_BT
#define DILQR_IMPL_BT 1
#endif
// LDS of one problem for the transposed step: W^T and Q share their words (a
// workgroup is one wave, whose LDS accesses complete in program order: every
// lane's read of its W column precedes the Q row writes), F rows beside them;
// padded to 16 words mod 32 so the two problems of a half-wave read disjoint
// banks (as GroupLdsT)
template <int n, int m>
struct ImplicitStepLds {
  static constexpr int d = n + m;
  static constexpr int W = 16;
  static constexpr int QS = W + 4;
  static constexpr int RS = GroupLds<n, m>::RS;
  union {
    float Wt[n + 1][W];
    float Q[d][QS];
  };
  float Kk[m][W];
  float F[n][RS];
  static constexpr int kWords = ((n + 1) * W > d * QS ? (n + 1) * W : d * QS) + m * W + n * RS;
  float pad[((16 - kWords % 32) % 32 + 32) % 32];
};
static_assert(sizeof(ImplicitStepLds<13, 3>) / 4 % 32 == 16, "bank offset between groups");
template <class LdsT>
struct FRowsLds {
  const LdsT& L;
  DEV float at(int k, int j) const { return L.F[k][j]; }
};

// PASSES: which of the passes this launch runs (1 = B, 2 = C, 4 = D; 7 = all in
// one launch).  Split launches run the same code per pass; what pass B hands
// pass D in registers when they share a launch — whether each lane's cost row
// and c_t entry are the same diagonal row for all t (crow_regs, cv_regs) and
// their values — is kept as one flag word per problem in a spare word of the
// t = 0 workspace record (KG column 14: no gain lives there, pass C never reads
// it) and re-read from C's step T-1 row in pass D.  A pass alone needs fewer
// registers than the three together: 3 waves per SIMD instead of 2 for passes
// B and C.  Not the default (tu_implicit_rocket.hip DILQR_IMPL_SPLIT: no gain).
#ifndef DILQR_IMPL_SPLIT_WAVES
#define DILQR_IMPL_SPLIT_WAVES 3
#endif
#ifndef DILQR_IMPL_D_WAVES
#define DILQR_IMPL_D_WAVES 2                 // at 3 pass D spills (168 VGPRs + 104 B scratch)
#endif
template <class Model, class D2, int MODE, int PASSES = 7>
__global__ void __launch_bounds__(64, PASSES == 7   ? kGroupWavesPerSimd
                                      : PASSES == 4 ? DILQR_IMPL_D_WAVES
                                                    : DILQR_IMPL_SPLIT_WAVES) k_implicit_backward_group(
    int T, int B, const float* __restrict__ theta, const float* __restrict__ C, const float* __restrict__ c,
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ K,
    const float* __restrict__ dl_dx, const float* __restrict__ dl_du, Bounds bd, float* __restrict__ ws,
    float* __restrict__ dC, float* __restrict__ dc, float* __restrict__ dtheta) {
  constexpr int n = Model::N, m = Model::M, p = Model::P, d = n + m;
  static_assert(d <= kG, "one row per lane");
  using W = ImplicitGroupWs<Model>;
#if DILQR_IMPL_BT
  using LdsB = ImplicitStepLds<n, m>;
#else
  using LdsB = GroupLds<n, m>;
#endif
  __shared__ LdsB Ls[kGPW];
  __shared__ ImplicitGroupLds<n, p> Is[kGPW];
  const int r = threadIdx.x & (kG - 1);
  const int gp = threadIdx.x / kG;
  const int b0 = blockIdx.x * kGPW + gp;
  const bool valid = b0 < B;
  const int b = valid ? b0 : B - 1;           // a padding group recomputes problem B-1, writes nothing
  LdsB& L = Ls[gp];
  ImplicitGroupLds<n, p>& I = Is[gp];
  Model md;
  md.load(theta);
  // 1/theta_k, once per launch: the generated pieces divide only by
  // parameters, so the divisions become products with these wave-uniform
  // reciprocals (scalar registers via readfirstlane); the Jacobian rows take
  // the model's per-launch coefficients (Rocket::load)
  float ith[p];
#pragma unroll
  for (int k = 0; k < p; ++k)
    ith[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(1.0f / theta[k])));
  auto rec = [&](int t) { return ws + ((size_t)t * B + b) * W::REC; };
  auto active = [&](size_t tb, int a, float ua) -> bool {
    if (bd.mode == DILQR_BOUNDS_NONE) return false;
    return fabsf(ua - bound_lo(bd, tb * m + a)) <= 1e-8f || fabsf(ua - bound_hi(bd, tb * m + a)) <= 1e-8f;
  };
  auto load_tau = [&](size_t tb, float (&xt)[n], float (&ut)[m]) {   // the group's lanes read the same bytes
#pragma unroll
    for (int i = 0; i < n; ++i) xt[i] = x[tb * n + i];
#pragma unroll
    for (int a = 0; a < m; ++a) ut[a] = u[tb * m + a];
  };
  // Pass B also tests, per lane, whether row r of C_t is the same diagonal row
  // for every t (off-diagonal words +0.0, the diagonal equal to step T-1's bit
  // for bit) and whether c_t[r] is: pass D then takes them from registers (the
  // reference's callers pass diag(q), p repeated over t; the same values, so
  // the same arithmetic, and C is read once instead of twice).
  float cdg = 0.f, cvr = 0.f;
  unsigned c_offd = 0u, c_dif = 0u, cv_dif = 0u;
  // ---------------- B: costates, M_t, Riccati of the C + M^T problem (active set masked)
  if constexpr ((PASSES & 1) != 0) {
#if DILQR_IMPL_BT
    float U[n];                                        // column r of V_{t+1} (lane n: v_{t+1})
#pragma unroll
    for (int i = 0; i < n; ++i) U[i] = 0.f;
#else
    if (r < n) {
#pragma unroll
      for (int kk = 0; kk < GroupLds<n, m>::W; ++kk) L.V[r][kk] = 0.f;
      L.v[r] = 0.f;
    }
#endif
    if (r < kG) I.vec[r] = 0.f;
    float prev_k[m];
#pragma unroll
    for (int a = 0; a < m; ++a) prev_k[a] = 0.f;
    bool have_prev = false;
    int nqp = 0;
    __syncthreads();
    // DILQR_IMPL_GPFB: step t-1's inputs (x, u, the cost row, c, the loss
    // gradient) loaded while step t computes
    struct BIn {
      float x[n], u[m], C[d], c, g;
    };
    auto load_b = [&](int t, BIn& in) {
      const size_t tb = (size_t)t * B + b;
      load_tau(tb, in.x, in.u);
#pragma unroll
      for (int j = 0; j < d; ++j) in.C[j] = 0.f;
      in.c = in.g = 0.f;
      if (r < d) {
        ld(in.C, C + (tb * d + r) * d);
        in.c = c[tb * d + r];
        in.g = r < n ? dl_dx[tb * n + r] : dl_du[tb * m + (r - n)];
      }
    };
    BIn nx;
    if (DILQR_IMPL_GPFB) load_b(T - 1, nx);
    for (int t = T - 1; t >= 0; --t) {
      const size_t tb = (size_t)t * B + b;
      float xt[n], ut[m], Crow[d], cr = 0.f, gr = 0.f;
      {
        BIn cur;
        if (DILQR_IMPL_GPFB) {
          cur = nx;
          if (t > 0) load_b(t - 1, nx);
        } else {
          load_b(t, cur);
        }
#pragma unroll
        for (int i = 0; i < n; ++i) xt[i] = cur.x[i];
#pragma unroll
        for (int a = 0; a < m; ++a) ut[a] = cur.u[a];
#pragma unroll
        for (int j = 0; j < d; ++j) Crow[j] = cur.C[j];
        cr = cur.c;
        gr = cur.g;
      }
      float cdr = 0.f;
#pragma unroll
      for (int j = 0; j < d; ++j) {
        cdr = (j == r) ? Crow[j] : cdr;
        if (j != r) c_offd |= __float_as_uint(Crow[j]);
      }
      if (t == T - 1) { cdg = cdr; cvr = cr; }
      c_dif |= __float_as_uint(cdr) ^ __float_as_uint(cdg);
      cv_dif |= __float_as_uint(cr) ^ __float_as_uint(cvr);
      float lam1[n];
#pragma unroll
      for (int i = 0; i < n; ++i) lam1[i] = I.vec[i];     // lam_{t+1} (0 at t = T-1)
      float Mc[d];
      if (t < T - 1) {
#if DILQR_IMPL_SKIP & 64                                   // timing only: no M_t column in pass B
#pragma unroll
        for (int j = 0; j < d; ++j) Mc[j] = 0.f * lam1[j % n];
#else
        D2::mcol(r, theta, ith, xt, ut, lam1, Mc);
#endif
        if (r < n) {
          float Fr[d];
          md.jac_row_sel(r, xt, ut, Fr);
#pragma unroll
          for (int j = 0; j < d; ++j) L.F[r][j] = Fr[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < d; ++j) Mc[j] = 0.f;
        if (r < n) {
#pragma unroll
          for (int j = 0; j < d; ++j) L.F[r][j] = 0.f;
        }
      }
      __syncthreads();
      float Cp[d];
#pragma unroll
      for (int j = 0; j < d; ++j) Cp[j] = r < d ? Crow[j] + Mc[j] : 0.f;
      float zI[m], lb[m], ub[m];
#pragma unroll
      for (int a = 0; a < m; ++a) {
        zI[a] = active(tb, a, ut[a]) ? 1.f : 0.f;
        lb[a] = ub[a] = 0.f;
      }
      float Kt[m][n], kt[m];
#if DILQR_IMPL_SKIP & 32                                   // timing only: no Riccati step (Cp kept live)
      {
        float s = -gr;
#pragma unroll
        for (int j = 0; j < d; ++j) s += Cp[j];
        if (r < n) L.Kk[0][r] = s;
        __syncthreads();
      }
#elif DILQR_IMPL_BT
      // t = T-1 through the general step: F's rows and U are zero there, so W = 0
      // and Q = Cp + 0, q = -g + 0, the LAST step's values bit for bit
      float col[m];
      group_riccati_step_c<n, m, MODE, typename Model::FSparsity, false>(
          L, r, FRowsLds<LdsB>{L}, U, CostRegs<d>{Cp, -gr}, zI, lb, ub, col, prev_k, have_prev, nqp);
      (void)Kt; (void)kt;
#else
      group_riccati_step<n, m, MODE>(L, r, Cp, -gr, zI, lb, ub, Kt, kt, prev_k, have_prev, nqp);
#endif
      // lam_t = Cxx x + Cxu u + c_x + F_x^T lam_{t+1}   (lqr_step_explicit.py:305-319)
      float lam_r = 0.f;
      if (r < n) {
        float s = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Crow[j] * xt[j];
#pragma unroll
        for (int a = 0; a < m; ++a) s2 += Crow[n + a] * ut[a];
#pragma unroll
        for (int l = 0; l < n; ++l) s3 += L.F[l][r] * lam1[l];
        lam_r = ((s + s2) + cr) + s3;
      }
      if (valid) {
        float* R0 = rec(t);
#if DILQR_IMPL_BT && !(DILQR_IMPL_SKIP & 32)
        if (r <= n) {                                      // lane r < n: K[:, r]; lane n: k
#pragma unroll
          for (int a = 0; a < m; ++a) R0[W::KG + a * kG + r] = col[a];
        }
#else
        if (r < n) {
#pragma unroll
          for (int a = 0; a < m; ++a) R0[W::KG + a * kG + r] = L.Kk[a][r];
        } else if (r == n) {
#pragma unroll
          for (int a = 0; a < m; ++a) R0[W::KG + a * kG + n] = L.Kk[a][GroupLds<n, m>::W];
        }
#endif
      }
      __syncthreads();                                     // every lane is done with lam_{t+1}, F, Kk
      if (r < n) I.vec[r] = lam_r;
      __syncthreads();
    }
  }
  // per lane: row r of C and c_t[r] from registers in pass D
  bool crow_regs = c_offd == 0u && c_dif == 0u, cv_regs = cv_dif == 0u;
  constexpr int kFlagSlot = W::KG + 14;            // t = 0 record, gain column 14: unused (r < n = 13 and k at n)
  static_assert(Model::N + 1 < 15, "the flag word needs a free gain column");
  if constexpr ((PASSES & 1) != 0 && (PASSES & 4) == 0) {
    // hand the flags to the pass-D launch: bit r = crow_regs of lane r, bit 16 + r = cv_regs
    const unsigned long long bc = __ballot(crow_regs), bv = __ballot(cv_regs);
    const int sh = threadIdx.x & ~(kG - 1);
    const unsigned word = (unsigned)((bc >> sh) & 0xFFFFull) | ((unsigned)((bv >> sh) & 0xFFFFull) << 16);
    if (valid && r == 0) rec(0)[kFlagSlot] = __uint_as_float(word);
  }
  if constexpr ((PASSES & 4) != 0 && (PASSES & 1) == 0) {
    const unsigned word = __float_as_uint(rec(0)[kFlagSlot]);
    crow_regs = (word >> r) & 1u;
    cv_regs = (word >> (16 + r)) & 1u;
    // the register row and value pass B kept: step T-1's (equal at every t when the flag is set)
    if (r < d) {
      const size_t tb = (size_t)(T - 1) * B + b;
      if (crow_regs) cdg = C[(tb * d + r) * d + r];
      if (cv_regs) cvr = c[tb * d + r];
    }
  }
  // ---------------- C (t up): the rollout y of the modified problem (linear, alpha = 1)
  // (DILQR_IMPL_SKIP: timing-only builds that leave out pass C (bit 1) or pass D
  // (bit 2) to split the kernel's time by pass, or in pass D the dC/dc stores
  // (4), mcol + mp_row (8), xth_row + xx_row (16); in pass B the Riccati step
  // (32) or mcol (64); never the shipped library)
  if constexpr ((PASSES & 2) != 0) {
    float yx = 0.f;                                        // lane r < n: y_t[r]
    // DILQR_IMPL_C_PF: step t+1's inputs (x, u, this lane's gain column, k)
    // loaded while step t computes — pass C is a short chain per step behind its
    // loads, and its live set is far below the kernel's peak (passes B and D)
    float xq[n], uq[m], Kcq[m], kq[m];
    auto load_c = [&](int t, float (&xs)[n], float (&us)[m], float (&Kc)[m], float (&kt)[m]) {
      load_tau((size_t)t * B + b, xs, us);
      const float* R0 = rec(t);
#pragma unroll
      for (int a = 0; a < m; ++a) {
        Kc[a] = r < n ? R0[W::KG + a * kG + r] : 0.f;
        kt[a] = R0[W::KG + a * kG + n];
      }
    };
    if (DILQR_IMPL_C_PF) load_c(0, xq, uq, Kcq, kq);
    for (int t = 0; t < ((DILQR_IMPL_SKIP & 1) ? 0 : T); ++t) {
      const size_t tb = (size_t)t * B + b;
      float* R0 = rec(t);
      float xt[n], ut[m], Kc[m], kt[m];
      if (DILQR_IMPL_C_PF) {
#pragma unroll
        for (int i = 0; i < n; ++i) xt[i] = xq[i];
#pragma unroll
        for (int a = 0; a < m; ++a) { ut[a] = uq[a]; Kc[a] = Kcq[a]; kt[a] = kq[a]; }
        if (t + 1 < T) load_c(t + 1, xq, uq, Kcq, kq);
      } else {
        load_c(t, xt, ut, Kc, kt);
      }
      // y_t from y_t's state part (the previous step's D y)
      float yr = r < n ? yx : 0.f;
#pragma unroll
      for (int a = 0; a < m; ++a) {
        const float s = group_sum(Kc[a] * (r < n ? yx : 0.f));
        const float ya = active(tb, a, ut[a]) ? 0.f : (s + 0.f) + kt[a];
        yr = (r == n + a) ? ya : yr;
      }
      if (valid && r < d) R0[W::Y + r] = yr;
      if (t < T - 1) {                                     // uniform
        if (r < d) I.vec[r] = yr;
        __syncthreads();
        if (r < n) {
          float Dr[d];
          md.jac_row_sel(r, xt, ut, Dr);
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) s += Dr[j] * I.vec[j];
          yx = s;
        }
        __syncthreads();
      }
    }
  }
  // ---------------- D: lam, w, dlam, dC, dc, dtheta (t down)
  if constexpr ((PASSES & 4) != 0) {
    float acc[p];
#pragma unroll
    for (int k = 0; k < p; ++k) acc[k] = 0.f;
    float au[m];                                           // (D_u,t+1)^T mu_{t+1}
#pragma unroll
    for (int a = 0; a < m; ++a) au[a] = 0.f;
    if (r < kG) { I.dlam[r] = 0.f; I.lam[r] = 0.f; }
    __syncthreads();
    // DILQR_IMPL_GPFD: step t-1's x, u, y and loss gradient loaded while step t computes
    struct DIn {
      float x[n], u[m], y[d], g;
    };
    auto load_d = [&](int t, DIn& in) {
      const size_t tb = (size_t)t * B + b;
      load_tau(tb, in.x, in.u);
      const float* R0 = rec(t);
#pragma unroll
      for (int j = 0; j < d; ++j) in.y[j] = R0[W::Y + j];
      in.g = 0.f;
      if (r < d) in.g = r < n ? dl_dx[tb * n + r] : dl_du[tb * m + (r - n)];
    };
    DIn dnx;
    if (DILQR_IMPL_GPFD && !(DILQR_IMPL_SKIP & 2)) load_d(T - 1, dnx);
    for (int t = (DILQR_IMPL_SKIP & 2) ? -1 : T - 1; t >= 0; --t) {
      const size_t tb = (size_t)t * B + b;
      float xt[n], ut[m], y[d], Crow[d], cr = 0.f, gr = 0.f;
      {
        DIn cur;
        if (DILQR_IMPL_GPFD) {
          cur = dnx;
          if (t > 0) load_d(t - 1, dnx);
        } else {
          load_d(t, cur);
        }
#pragma unroll
        for (int i = 0; i < n; ++i) xt[i] = cur.x[i];
#pragma unroll
        for (int a = 0; a < m; ++a) ut[a] = cur.u[a];
#pragma unroll
        for (int j = 0; j < d; ++j) { y[j] = cur.y[j]; Crow[j] = 0.f; }
        gr = cur.g;
      }
      if (r < d) {
        if (crow_regs) {
#pragma unroll
          for (int j = 0; j < d; ++j) Crow[j] = j == r ? cdg : 0.f;
        } else {
          ld(Crow, C + (tb * d + r) * d);
        }
        cr = cv_regs ? cvr : c[tb * d + r];
      }
      float tau[d];
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
      float yr = 0.f, taur = 0.f;
#pragma unroll
      for (int j = 0; j < d; ++j) { yr = (j == r) ? y[j] : yr; taur = (j == r) ? tau[j] : taur; }
      // dC_t row r = -0.5 (y_r tau^T + tau_r y^T), dc_t = -y   (lqr_step_explicit.py:296-303)
      // (Round 6: these rows staged through LDS and stored as the wave's
      // contiguous 4-KiB run, 64 contiguous 16-byte chunks per instruction:
      // 1.375 -> 1.386 ms, no gain — the stores' cost is the 1 GB of dC itself
      // at the write rate, 0.17 ms (DILQR_IMPL_SKIP & 4),
      // profiles/r06/ab_implicit_rocket_split.txt)
      if (valid && r < d && !(DILQR_IMPL_SKIP & 4)) {
        float dCr[d];
#pragma unroll
        for (int j = 0; j < d; ++j) dCr[j] = -0.5f * (yr * tau[j] + taur * y[j]);
        if (DILQR_IMPL_NT) {
          st_nt(dC + (tb * d + r) * d, dCr);
          __builtin_nontemporal_store(-yr, dc + tb * d + r);
        } else {
          st(dC + (tb * d + r) * d, dCr);
          dc[tb * d + r] = -yr;
        }
      }
      // row r of D_t -> LDS (t = T-1: only for the carry's D_u, F_{T-1} is zero)
      if (r < n) {
        float Fr[d];
#if DILQR_IMPL_SKIP & 128                                  // timing only: no Jacobian in pass D
#pragma unroll
        for (int j = 0; j < d; ++j) Fr[j] = 0.f * xt[j % n];
#else
        md.jac_row_sel(r, xt, ut, Fr);
#endif
#pragma unroll
        for (int j = 0; j < d; ++j) L.F[r][j] = Fr[j];
      }
      float wr = gr, Dtd = 0.f, Dtl = 0.f;                 // w_t[r]; (D^T dlam_{t+1})[r], (D^T lam_{t+1})[r]
      float hx = 0.f;                                      // lane r < n: h_t[r] + (A_{t+1}^T mu_{t+1})[r]
      if (t < T - 1) {
        float Mc[d], Mp[p];
        {
          float lam1[n];
#pragma unroll
          for (int i = 0; i < n; ++i) lam1[i] = I.lam[i];  // lam_{t+1}
#if DILQR_IMPL_SKIP & 8
#pragma unroll
          for (int j = 0; j < d; ++j) Mc[j] = 0.f * lam1[j % n];
#pragma unroll
          for (int k = 0; k < p; ++k) Mp[k] = 0.f * lam1[k];
#else
          D2::mcol(r, theta, ith, xt, ut, lam1, Mc);
          D2::mp_row(r, theta, ith, xt, ut, lam1, Mp);
#endif
        }
        __syncthreads();
        float z = 0.f;                                     // (M_t^T y_t)[r]
#pragma unroll
        for (int j = 0; j < d; ++j) z += Mc[j] * y[j];
        if (r < d) {
#if DILQR_IMPL_SKIP & 256                                  // timing only: no D^T dlam, D^T lam column sums
          Dtd = I.dlam[r & 7]; Dtl = I.lam[r & 7];
#else
#pragma unroll
          for (int i = 0; i < n; ++i) { Dtd += L.F[i][r] * I.dlam[i]; Dtl += L.F[i][r] * I.lam[i]; }
#endif
        }
        wr = gr - z;
        // dtheta_t = -(y^T Mp) + h_t^T gradx_t - dlam_{t+1}^T gradx_{t+1},
        // h_t = dlam_{t+1}^T (D_x + D_u Kq) - y^T (M_x + M_u Kq)   (oracle/adjoint.py implicit_backward_fast)
        float zu[m], du[m];
#pragma unroll
        for (int a = 0; a < m; ++a) {
          zu[a] = __shfl(z, n + a, kG);
          du[a] = __shfl(Dtd, n + a, kG);
        }
        if (r < d) {
#pragma unroll
          for (int k = 0; k < p; ++k) acc[k] -= yr * Mp[k];
        }
        if (r < n) {
          const float* Kp = K + ((size_t)(T - 1 - t) * B + b) * m * n;   // K[t] of the reversed stack
          float sx = z, s2 = Dtd, cu = 0.f;
#pragma unroll
          for (int a = 0; a < m; ++a) {
            const float Kal = Kp[a * n + r];
            sx += zu[a] * Kal;
            s2 += du[a] * Kal;
            cu += au[a] * Kal;
          }
          // the carry A_{t+1}^T mu_{t+1}: column r of the rows step t+1 left in LDS,
          // plus Krev^T (D_u,t+1)^T mu_{t+1} (A_{t+1} pairs D_{t+1} with this step's Kq)
          float cx = 0.f;
#pragma unroll
          for (int i = 0; i < n; ++i) cx += I.ax[i][r];
          hx = (s2 - sx) + (cx + cu);
        }
      }
      // dlam_t = Cxx y_x + Cxu y_u - w_x + F_x^T dlam_{t+1}   (lqr_step_explicit.py:321-335)
      // lam_t  = Cxx x + Cxu u + c_x + F_x^T lam_{t+1}        (pass B's recursion, 305-319)
      float nd = 0.f, nl = 0.f;
      if (r < n) {
        float s = 0.f, s2 = 0.f, q = 0.f, q2 = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) { s += Crow[j] * y[j]; q += Crow[j] * xt[j]; }
#pragma unroll
        for (int a = 0; a < m; ++a) { s2 += Crow[n + a] * y[n + a]; q2 += Crow[n + a] * ut[a]; }
        nd = ((s + s2) - wr) + Dtd;
        nl = ((q + q2) + cr) + Dtl;
      }
      // mu_t = h_t - dlam_t (+ the carry); dtheta += f_theta,t^T mu_t; this
      // step's carry rows for step t-1: mu_t[i] * x_grad_xtm1[i][:], (D_u,t)^T mu_t
      float mu = 0.f;
      if (t >= 1) {                                        // uniform
        float axr[n];
        if (r < n) {
          mu = hx - nd;
          float ft[p];
#if DILQR_IMPL_SKIP & 16
#pragma unroll
          for (int k = 0; k < p; ++k) ft[k] = 0.f * xt[k];
#pragma unroll
          for (int l = 0; l < n; ++l) axr[l] = 0.f * xt[l];
#else
          D2::xth_row(r, theta, ith, xt, ut, ft);
#endif
#pragma unroll
          for (int k = 0; k < p; ++k) acc[k] += ft[k] * mu;
#if !(DILQR_IMPL_SKIP & 16)
          D2::xx_row(r, theta, ith, xt, ut, axr);
#endif
        }
#pragma unroll
        for (int a = 0; a < m; ++a) au[a] = group_sum(r < n ? L.F[r][n + a] * mu : 0.f);
        __syncthreads();                                   // every lane is done with dlam, lam, ax of t+1
        if (r < n) {
#pragma unroll
          for (int l = 0; l < n; ++l) I.ax[r][l] = axr[l] * mu;
        }
      } else {
        __syncthreads();
      }
      if (r < n) { I.dlam[r] = nd; I.lam[r] = nl; }
      __syncthreads();
    }
    float dth = 0.f;
#pragma unroll
    for (int k = 0; k < p; ++k) {
      const float s = group_sum(acc[k]);
      dth = (r == k) ? s : dth;
    }
    if (valid && r < p) dtheta[(size_t)b * p + r] = dth;
  }
}

}  // namespace dilqr
