// dilqr_group.h — 16 lanes per problem for the larger models (d = n+m <= 16,
// rocket: n=13 m=3).  Included by dilqr_kernels.hip.
//
// One lane per problem stops fitting once a step's matrices (C 16x16, F 13x16,
// V 13x13) exceed the register file, so here a problem is a 16-lane group of a
// wave (4 problems per wave, one wave per workgroup) and lane r owns ROW r:
// C row r streams from HBM (64 contiguous bytes per lane, 1 KiB per problem),
// V, v, F and the u-rows of Q are exchanged through the workgroup's LDS, and
// the m x m gain solve (and pnqp) runs redundantly in every lane of the group,
// so every lane holds K and k in registers.  Cross-lane sums use 16-lane xor
// shuffles.  Same math as RiccatiState::step (lqr_step_explicit.py:63-160).
#pragma once
#include <type_traits>

#include "dilqr_device.h"

namespace dilqr {

constexpr int kG = 16;          // lanes per problem
constexpr int kGPW = 64 / kG;   // problems per wave (= per workgroup)
// Occupancy floor of the implicit group kernel (waves per SIMD, i.e. at most
// 512/N VGPRs).  Round 4's pass D (the costates recomputed, the gradx adjoint
// carried down, ws records of 64 floats instead of 160) needs 205 VGPRs: at a
// floor of 3 (168) it spills ~130 VGPRs, at 2 it spills none — and config 3
// (B = 32768: 2048 waves) has two waves per SIMD to give anyway.
#ifndef DILQR_GROUP_WAVES
#define DILQR_GROUP_WAVES 2
#endif
constexpr int kGroupWavesPerSimd = DILQR_GROUP_WAVES;

struct GroupNoModel {           // LinDx dynamics (F, f given)
  DEV void load(const float*) {}
};

// Sum over the 16 lanes of a group in four DPP adds (no LDS crossbar, unlike
// __shfl_xor's ds_bpermute): lane^1 and lane^2 within each quad (quad_perm),
// then the other quad of the half-row (row_half_mirror: lane i <-> 7-i) and the
// other half of the row (row_mirror: i <-> 15-i).  Every step adds two partial
// sums that their two lanes hold in swapped order, so all 16 lanes end with the
// bitwise-identical total (group-uniform decisions depend on that).
template <int CTRL>
DEV float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
DEV float group_sum(float v) {
  v += dpp_mov<0xB1>(v);      // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);      // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);     // row_half_mirror
  v += dpp_mov<0x140>(v);     // row_mirror
  return v;
}

template <int n, int m>
struct GroupLds {
  static constexpr int d = n + m;
  static constexpr int W = 16;                 // padded row width (b128 reads)
  // V and F rows 20 words apart: a lane's 16-byte row stores then start on 8
  // distinct 4-bank sets across the 8 lanes of a store group (a 16-word stride
  // put 4 lanes on each of 2 sets: 26 % of the implicit backward's LDS cycles
  // were bank conflicts)
#ifndef DILQR_GROUP_RS
#define DILQR_GROUP_RS 20
#endif
  static constexpr int RS = DILQR_GROUP_RS;
  float V[n][RS];
  float v[W];
  float F[n][RS];
  float Qu[m][W + 4];                          // u rows of Q, q_u at [.][W]
  float Kk[m][W + 4];                          // gains K, k at [.][W]
  float tau[W];
  // tau2: the paired line search's second candidate; its tail pads the struct
  // to 16 words mod 32, so the two groups of a half-wave read columns from
  // disjoint LDS banks (see GroupLdsT)
  static constexpr int kWords = 2 * n * RS + W + 2 * m * (W + 4) + 2 * W;
  float tau2[W + ((16 - kWords % 32) % 32 + 32) % 32];
};

// Gains from the u-rows of Q (modes as RiccatiState::step), distributed over
// the group: lane j solves right-hand side j — Q_ux column j for j < n, q_u for
// j = n — against the same m x m matrix (elimination and pivots depend only on
// the matrix, so each column's arithmetic is exactly the multi-RHS solve's).
// pnqp (box mode) needs all of q_u and runs in every lane.  Lane j < n returns
// K[:, j] in col; lane n returns k.
template <int n, int m, int MODE>
DEV void group_gains_col(int j, const float (&Quu)[m][m], const float (&rhs)[m], const float (&qu)[m],
                         const float (&zI)[m], const float (&lb)[m], const float (&ub)[m], float (&col)[m],
                         float (&prev_k)[m], bool& have_prev, int& n_qp) {
  if constexpr (MODE == GAIN_UNC || MODE == GAIN_CHOL) {
    float A[m][m], X[m][1];
#pragma unroll
    for (int a = 0; a < m; ++a) {
#pragma unroll
      for (int b = 0; b < m; ++b) A[a][b] = Quu[a][b] + ((MODE == GAIN_CHOL && a == b) ? 1e-6f : 0.f);
      X[a][0] = rhs[a];
    }
    if constexpr (MODE == GAIN_CHOL) chol_solve<m, 1>(A, X);
    else gauss_solve<m, 1, true>(A, X);
#pragma unroll
    for (int a = 0; a < m; ++a) col[a] = -X[a][0];
  } else if constexpr (MODE == GAIN_ZERO_I) {
    float A[m][m], X[m][1];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      bool Ia = zI[a] != 0.f;
#pragma unroll
      for (int b = 0; b < m; ++b) {
        bool fr = (zI[a] == 0.f) && (zI[b] == 0.f);
        A[a][b] = (fr ? Quu[a][b] : 0.f) + ((a == b && Ia) ? 1e-8f : 0.f);
      }
      X[a][0] = Ia ? 0.f : rhs[a];
    }
    gauss_solve<m, 1>(A, X);
#pragma unroll
    for (int a = 0; a < m; ++a) col[a] = -X[a][0];
  } else {                                        // GAIN_BOX: pnqp, then the free-block solve
    float x[m], If[m], Hf[m][m];
#pragma unroll
    for (int a = 0; a < m; ++a) x[a] = prev_k[a];
    int it = pnqp<m>(Quu, qu, lb, ub, have_prev, x, If, Hf);
    n_qp += 1 + it;
#pragma unroll
    for (int a = 0; a < m; ++a) prev_k[a] = x[a];
    have_prev = true;
    float X[m][1];
#pragma unroll
    for (int a = 0; a < m; ++a) X[a][0] = If[a] != 0.f ? rhs[a] : 0.f;
    gauss_solve<m, 1>(Hf, X);
#pragma unroll
    for (int a = 0; a < m; ++a) col[a] = j < n ? -X[a][0] : x[a];
  }
}

// One backward Riccati step for the group's problem; lane r owns rows r of
// C/Q/P/V.  Crow: C_t row r, cb_r: c_back_t[r] (both only meaningful for r < d).
// F_t rows are already in L.F (zero for t = T-1), V/v of step t+1 in L.V / L.v.
// On return the gains are in K/k (all lanes) and L.Kk, V/v of step t in L.
template <int n, int m, int MODE>
DEV void group_riccati_step(GroupLds<n, m>& L, int r, const float (&Crow)[n + m], float cb_r,
                            const float (&zI)[m], const float (&lb)[m], const float (&ub)[m], float (&K)[m][n],
                            float (&k)[m], float (&prev_k)[m], bool& have_prev, int& n_qp) {
  constexpr int d = n + m;
  constexpr int n2 = (n + 1) / 2, d2 = (d + 1) / 2;   // column pairs (the pad columns of V and F are 0)
  static_assert(2 * d2 <= GroupLds<n, m>::W, "pairs stay inside the padded rows");
  const bool row = r < d;
  // P row r = F[:, r]^T V ; q_r = cb_r + F[:, r] . v.  The dense products run
  // on column pairs (v_pk_fma_f32: two FMAs per lane per instruction); each
  // element still accumulates in the same order with one fma per term, so the
  // rounding is that of the scalar loop.
  float Fcol[n];
#pragma unroll
  for (int l = 0; l < n; ++l) Fcol[l] = row ? L.F[l][r] : 0.f;
  f2 P2[n2];
#pragma unroll
  for (int i = 0; i < n2; ++i) P2[i] = f2{0.f, 0.f};
#pragma unroll
  for (int l = 0; l < n; ++l) {
    const f2* Vl = reinterpret_cast<const f2*>(&L.V[l][0]);
#pragma unroll
    for (int i = 0; i < n2; ++i) P2[i] = P2[i] + Fcol[l] * Vl[i];
  }
  float qr = 0.f;
#pragma unroll
  for (int l = 0; l < n; ++l) qr += Fcol[l] * L.v[l];
  qr = cb_r + qr;
  // Q row r = C row r + P row r F
  f2 S2[d2];
#pragma unroll
  for (int i = 0; i < d2; ++i) S2[i] = f2{0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < n; ++kk) {
    const f2* Fk = reinterpret_cast<const f2*>(&L.F[kk][0]);
    const float p = (kk & 1) ? P2[kk / 2].y : P2[kk / 2].x;
#pragma unroll
    for (int i = 0; i < d2; ++i) S2[i] = S2[i] + p * Fk[i];
  }
  float Q[d];
#pragma unroll
  for (int j = 0; j < d; ++j) Q[j] = Crow[j] + ((j & 1) ? S2[j / 2].y : S2[j / 2].x);
  if (r >= n && r < d) {
#pragma unroll
    for (int j = 0; j < d; ++j) L.Qu[r - n][j] = Q[j];
    L.Qu[r - n][GroupLds<n, m>::W] = qr;
  }
  __syncthreads();
  float Quu[m][m], qu[m], rhs[m];
  const int jc = r <= n ? r : n;                 // this lane's right-hand side (lanes > n repeat k's)
#pragma unroll
  for (int a = 0; a < m; ++a) {
#pragma unroll
    for (int b = 0; b < m; ++b) Quu[a][b] = L.Qu[a][n + b];
    qu[a] = L.Qu[a][GroupLds<n, m>::W];
    rhs[a] = jc < n ? L.Qu[a][jc] : qu[a];
  }
  float col[m];
  group_gains_col<n, m, MODE>(jc, Quu, rhs, qu, zI, lb, ub, col, prev_k, have_prev, n_qp);
  if (r < n) {
#pragma unroll
    for (int a = 0; a < m; ++a) L.Kk[a][r] = col[a];
  } else if (r == n) {
#pragma unroll
    for (int a = 0; a < m; ++a) L.Kk[a][GroupLds<n, m>::W] = col[a];
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < m; ++a) {
#pragma unroll
    for (int jj = 0; jj < n; ++jj) K[a][jj] = L.Kk[a][jj];
    k[a] = L.Kk[a][GroupLds<n, m>::W];
  }
  if (r < n) {
    float Kc[m];
#pragma unroll
    for (int a = 0; a < m; ++a) Kc[a] = L.Kk[a][r];
    float KcQuu[m];
#pragma unroll
    for (int b = 0; b < m; ++b) {
      float s = 0.f;
#pragma unroll
      for (int a = 0; a < m; ++a) s += Kc[a] * Quu[a][b];
      KcQuu[b] = s;
    }
    // V row r on column pairs, K and Q_ux pairs straight from LDS (the pad
    // column n of the last pair is computed and dropped)
    f2 V2[n2];
#pragma unroll
    for (int i = 0; i < n2; ++i) {
      f2 s1 = f2{0.f, 0.f}, s2 = f2{0.f, 0.f}, s3 = f2{0.f, 0.f};
#pragma unroll
      for (int a = 0; a < m; ++a) {
        const f2 Ka = reinterpret_cast<const f2*>(&L.Kk[a][0])[i];
        const f2 Qa = reinterpret_cast<const f2*>(&L.Qu[a][0])[i];
        s1 = s1 + Q[n + a] * Ka;
        s2 = s2 + Kc[a] * Qa;
        s3 = s3 + KcQuu[a] * Ka;
      }
      V2[i] = ((f2{Q[2 * i], Q[2 * i + 1]} + s1) + s2) + s3;
    }
    float Vr[n];
#pragma unroll
    for (int kk = 0; kk < n; ++kk) Vr[kk] = (kk & 1) ? V2[kk / 2].y : V2[kk / 2].x;
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
    for (int a = 0; a < m; ++a) {
      s1 += Q[n + a] * k[a];
      s2 += Kc[a] * qu[a];
      s3 += KcQuu[a] * k[a];
    }
    float vr = ((qr + s1) + s2) + s3;
    // every lane has finished reading the old V (first barrier above)
#pragma unroll
    for (int kk = 0; kk < n; ++kk) L.V[r][kk] = Vr[kk];
    L.v[r] = vr;
  }
}

// ---------------------------------------------------------------- transposed step
// The Riccati step of the sweeps (k_lqr_backward_group, the fused MPC sweep)
// with V_{t+1} held in registers, TRANSPOSED: lane l < n keeps column l of
// V_{t+1} (= row l of V^T), lane n keeps v_{t+1}.  Then
//   W  = V^T F   (lane l: its row times F; lane n: v^T F)     — one LDS exchange
//   lane j reads column j of W and forms column j of F^T W = F^T V^T F, which
//   is ROW j of P = F^T V F; its extra row n gives (F^T v)_j,
// so lane j holds row j of Q = C + F^T V F and q_j = c_back_j + (F^T v)_j (the
// reference's Q, q, lqr_step_explicit.py:96-101), and the new V_t column j /
// v_t come from Q's columns (one more exchange).  Both products run over F's
// nonzeros only when F's structure is known at compile time (the model's
// Jacobian in registers, FS = Model::FSparsity: rocket 69 of 208 entries):
// a zero term adds exactly nothing to an fma chain started at +0 (such a chain
// never holds -0), so the dense F of the unfused path (FS = DenseF, rows in
// LDS, DenseF of dilqr_device.h) gives the same bits on finite data.  Replaces per step the old rows-of-V
// step's two dense 13x13x16 products and its V/F row broadcasts (group_riccati_step).
template <int n, int m, bool HAS_F, bool HAS_TAU>
struct GroupLdsT {
  static constexpr int d = n + m;
  static constexpr int W = 16;                   // padded row width (b128 accesses)
  // Q row r: Q[r][0..d), q_r at [d].  Row stride: 16-byte aligned (W + 4) for
  // the fused sweep (its u-column reads are one b128 per row), odd (d + 1) for
  // the F-from-HBM sweep — measured at config 3 shapes, each layout is the
  // faster one for its kernel (fused 0.407 vs 0.451 ms per MPC iteration,
  // standalone 0.47 vs 0.56 ms)
  static constexpr int QS = HAS_F ? d + 1 : W + 4;
  float Wt[n + 1][W];                            // rows of V^T F, then v^T F
  float Q[d][QS];
  float Kk[m][W];                                // gains K (box / pinverse modes: every lane needs all of K)
  float F[HAS_F ? n : 1][W];                     // F rows (F from HBM)
  // The 4 groups of a wave use consecutive structs; a half-wave (32 lanes, the
  // LDS's 32 banks) holds two of them, whose column reads (lane j: word j of a
  // row) share banks unless the two bases differ by 16 words mod 32 (measured:
  // the fused sweep 0.45 -> 0.41 ms per MPC iteration).  The padding is the
  // tail of tau2, so a struct already at 16 mod 32 grows by nothing (the LDS
  // per workgroup sets how many fit a CU).
  static constexpr int kWords = (n + 1) * W + d * QS + m * W + (HAS_F ? n : 1) * W + 2 * (HAS_TAU ? W : 1);
  static constexpr int kPad = ((16 - kWords % 32) % 32 + 32) % 32;
  float tau[HAS_TAU ? W : 1];                    // tau / the line search's states
  float tau2[(HAS_TAU ? W : 1) + kPad];
};
static_assert(sizeof(GroupLdsT<13, 3, false, false>) / 4 % 32 == 16, "bank offset between groups");
static_assert(sizeof(GroupLdsT<13, 3, true, true>) / 4 % 32 == 16, "bank offset between groups");

// F as a lane sees it: registers (the model's Jacobian, every lane the whole
// matrix) or the rows in LDS
template <int n, int d>
struct FRegs {
  const float (&f)[n][d];
  DEV float at(int k, int j) const { return f[k][j]; }
};
template <int n, int m>
struct FRows {
  const GroupLdsT<n, m, true, true>& L;
  DEV float at(int k, int j) const { return L.F[k][j]; }
};

// One step.  U: this lane's column of V_{t+1} (lane n: v_{t+1}), replaced by
// V_t's.  LAST (t = T-1): V_{t+1} = 0 and F = 0, so Q = C + 0, q = c_back + 0.
// col: this lane's gain column (lane j < n: K[:, j], lanes >= n: k).
// The cost row reaches the step through `cost(Crow, cb_r)`, called where the
// row is first needed (after the W^T exchange): a caller that loads it from HBM
// there keeps it out of the registers live across V^T F and its load off the
// step's top (the standalone sweep: 0.476 -> 0.469 ms at config 3);
// CostRegs passes a row already in registers.
template <int d>
struct CostRegs {
  const float (&C)[d];
  float cb;
  DEV void operator()(float (&o)[d], float& ocb) const {
#pragma unroll
    for (int j = 0; j < d; ++j) o[j] = C[j];
    ocb = cb;
  }
};

template <int n, int m, int MODE, class FS, bool LAST, class FA, class LdsT, class CP>
DEV void group_riccati_step_c(LdsT& L, int r, const FA& F, float (&U)[n], const CP& cost, const float (&zI)[m],
                              const float (&lb)[m], const float (&ub)[m], float (&col)[m], float (&prev_k)[m],
                              bool& have_prev, int& n_qp) {
  constexpr int d = n + m;
  float Q[d], qr;
  if constexpr (LAST) {
    float Crow[d], cb_r;
    cost(Crow, cb_r);
#pragma unroll
    for (int j = 0; j < d; ++j) Q[j] = Crow[j] + 0.f;
    qr = cb_r + 0.f;
  } else {
    if (r <= n) {                                  // row r of V^T F (lane n: v^T F)
      float Wr[d];
#pragma unroll
      for (int j = 0; j < d; ++j) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < n; ++k)
          if (FS::nz(k, j)) s += U[k] * F.at(k, j);
        Wr[j] = s;
      }
#pragma unroll
      for (int j = 0; j < d; ++j) L.Wt[r][j] = Wr[j];
    }
    __syncthreads();
    float Wc[n + 1];
#pragma unroll
    for (int l = 0; l <= n; ++l) Wc[l] = L.Wt[l][r];
    float Crow[d], cb_r;
    cost(Crow, cb_r);
#pragma unroll
    for (int i = 0; i < d; ++i) {                  // row r of F^T V F = column r of F^T (V^T F)
      float s = 0.f;
#pragma unroll
      for (int l = 0; l < n; ++l)
        if (FS::nz(l, i)) s += F.at(l, i) * Wc[l];
      Q[i] = Crow[i] + s;
    }
    qr = cb_r + Wc[n];
  }
#pragma unroll
  for (int j = 0; j < d; ++j) L.Q[r][j] = Q[j];
  L.Q[r][d] = qr;
  __syncthreads();
  float Quu[m][m], qu[m], rhs[m];
  const int jc = r <= n ? r : n;                   // this lane's right-hand side (lanes > n repeat k's)
#pragma unroll
  for (int a = 0; a < m; ++a) {
#pragma unroll
    for (int b = 0; b < m; ++b) Quu[a][b] = L.Q[n + a][n + b];
    qu[a] = L.Q[n + a][d];
    rhs[a] = jc < n ? L.Q[n + a][jc] : qu[a];
  }
  group_gains_col<n, m, MODE>(jc, Quu, rhs, qu, zI, lb, ub, col, prev_k, have_prev, n_qp);
  // V_t column r (lane n: v_t), from column r of Q (lane n: q) and Q's u columns:
  //   V[i][c] = ((Q[i][c] + sum_a Q[i][n+a] K[a][c]) + sum_a K[a][i] Q[n+a][c]) + sum_a K[a][i] (Quu K)[a][c]
  // (lqr_step_explicit.py:157-160), v the same with q and k.  Unconstrained, K
  // = -Quu^-1 Qux makes the last two terms cancel (K^T (Qux + Quu K) = 0): V =
  // Qxx + Qxu K, v = q_x + Qxu k, and only this lane's own gain column is needed.
  constexpr bool SCHUR = MODE == GAIN_UNC;
  float Kall[m][n];
  if constexpr (!SCHUR) {
    if (r < n) {
#pragma unroll
      for (int a = 0; a < m; ++a) L.Kk[a][r] = col[a];
    }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < m; ++a)
#pragma unroll
      for (int i = 0; i < n; ++i) Kall[a][i] = L.Kk[a][i];
  }
  if (r <= n) {
    const int cx = r < n ? r : d;
    float z[m], Qnc[m];
    if constexpr (!SCHUR) {
#pragma unroll
      for (int a = 0; a < m; ++a) {
        float s = 0.f;
#pragma unroll
        for (int b = 0; b < m; ++b) s += Quu[a][b] * col[b];
        z[a] = s;
        Qnc[a] = L.Q[n + a][cx];
      }
    }
#pragma unroll
    for (int i = 0; i < n; ++i) {
      float s1 = 0.f;
#pragma unroll
      for (int a = 0; a < m; ++a) s1 += L.Q[i][n + a] * col[a];
      float vi = L.Q[i][cx] + s1;
      if constexpr (!SCHUR) {
        float s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int a = 0; a < m; ++a) {
          s2 += Kall[a][i] * Qnc[a];
          s3 += Kall[a][i] * z[a];
        }
        vi = (vi + s2) + s3;
      }
      U[i] = vi;
    }
  }
}

template <int n, int m, int MODE, class FS, bool LAST, class FA, class LdsT>
DEV void group_riccati_step_t(LdsT& L, int r, const FA& F, float (&U)[n], const float (&Crow)[n + m], float cb_r,
                              const float (&zI)[m], const float (&lb)[m], const float (&ub)[m], float (&col)[m],
                              float (&prev_k)[m], bool& have_prev, int& n_qp) {
  group_riccati_step_c<n, m, MODE, FS, LAST>(L, r, F, U, CostRegs<n + m>{Crow, cb_r}, zI, lb, ub, col, prev_k,
                                             have_prev, n_qp);
}

// standalone sweep, F from HBM (the LinDx / classic path and the north-star
// kernel for rocket shapes): F's rows through LDS, dense
template <int n, int m, int MODE>
__global__ void __launch_bounds__(64) k_lqr_backward_group(int T, int B, const float* __restrict__ C,
                                                           const float* __restrict__ c, const float* __restrict__ x,
                                                           const float* __restrict__ u, const float* __restrict__ F,
                                                           Bounds bd, const unsigned char* __restrict__ zI,
                                                           float* __restrict__ K, float* __restrict__ k,
                                                           int* __restrict__ n_qp, int* __restrict__ n_qp_step) {
  constexpr int d = n + m;
  using LdsT = GroupLdsT<n, m, true, true>;
  __shared__ LdsT Ls[kGPW];
  const int r = threadIdx.x & (kG - 1);
  const int gp = threadIdx.x / kG;
  const int b = blockIdx.x * kGPW + gp;
  const bool valid = b < B;
  const int bb = valid ? b : 0;
  LdsT& L = Ls[gp];
  float U[n];
#pragma unroll
  for (int i = 0; i < n; ++i) U[i] = 0.f;
  float prev_k[m];
#pragma unroll
  for (int a = 0; a < m; ++a) prev_k[a] = 0.f;
  bool have_prev = false;
  int nqp = 0;
  auto step = [&](int t, auto last_c) {
    constexpr bool LAST = decltype(last_c)::value;
    const size_t tb = (size_t)t * B + bb;
    float tau_r = 0.f;
    if (r < d && x) tau_r = r < n ? x[tb * n + r] : u[tb * m + (r - n)];
    if constexpr (!LAST) {
      if (r < n) {
        float Fr[d];
        ld(Fr, F + (tb * n + r) * d);
#pragma unroll
        for (int j = 0; j < d; ++j) L.F[r][j] = Fr[j];
      }
    }
    if (r < d) L.tau[r] = tau_r;
    __syncthreads();
    // the cost row and c_back = c + C tau, loaded where the step first needs them
    auto cost = [&](float (&Crow)[d], float& cb) {
#pragma unroll
      for (int j = 0; j < d; ++j) Crow[j] = 0.f;
      cb = 0.f;
      if (r < d) {
        ld(Crow, C + (tb * d + r) * d);
        cb = c[tb * d + r];
        if (x) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) s += Crow[j] * L.tau[j];
          cb = s + cb;
        }
      }
    };
    float zIt[m], lb[m], ub[m], ut[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      ut[a] = u ? u[tb * m + a] : 0.f;
      zIt[a] = (MODE == GAIN_ZERO_I && zI[tb * m + a]) ? 1.f : 0.f;
      lb[a] = ub[a] = 0.f;
      if constexpr (MODE == GAIN_BOX) {
        lb[a] = bound_lo(bd, tb * m + a) - ut[a];
        ub[a] = bound_hi(bd, tb * m + a) - ut[a];
      }
    }
    float col[m];
    const int qp_before = nqp;
    group_riccati_step_c<n, m, MODE, DenseF, LAST>(L, r, FRows<n, m>{L}, U, cost, zIt, lb, ub, col, prev_k,
                                                   have_prev, nqp);
    if (MODE == GAIN_BOX && valid && n_qp_step && r == 0) atomicMax(n_qp_step + t, nqp - qp_before - 1);
    if (valid) {
      if (r < n) {
#pragma unroll
        for (int a = 0; a < m; ++a) K[tb * m * n + a * n + r] = col[a];
      }
      if (r == n) {
#pragma unroll
        for (int a = 0; a < m; ++a) k[tb * m + a] = col[a];
      }
    }
    __syncthreads();
  };
  step(T - 1, std::true_type{});
  for (int t = T - 2; t >= 0; --t) step(t, std::false_type{});
  if (valid && n_qp && r == 0) n_qp[b] = nqp;
}

// ---------------------------------------------------------------- forward pass
// forward_pass (dilqr_kernels.hip) for a 16-lane group: lane r < n carries
// state component r, K . dx is a 16-lane shuffle sum, the full state for the
// dynamics and the stage cost is exchanged through LDS, and the stage cost is
// shuffle-reduced from the per-row terms tau_r (C_r . tau) / 2 + c_r tau_r.
// Dynamics: Model::forward_row (model rollout) or, with md == nullptr, the
// LinDx step x' = F_t tau + f_t with F row r read by lane r.
template <int n, int m, int GREC, class Model, class LdsT>
DEV float group_forward_pass(LdsT& L, const Model* md, const float* __restrict__ F,
                             const float* __restrict__ f, int T, int B, int b, int r, bool valid, float alpha,
                             const float* __restrict__ x_init, const float* __restrict__ C,
                             const float* __restrict__ c, const float* __restrict__ x, const float* __restrict__ u,
                             const float* __restrict__ K, const float* __restrict__ k,
                             const float* __restrict__ grec, const Bounds& bd, const unsigned char* __restrict__ zI,
                             float* __restrict__ x_out, float* __restrict__ u_out, float* __restrict__ du_sq,
                             float* old_cost_out) {
  constexpr int d = n + m;
  float xr = (r < n) ? x_init[(size_t)b * n + r] : 0.f;      // this lane's state component
  float dxr = 0.f;
  if (valid && r < n) x_out[(size_t)b * n + r] = xr;
  float cst = 0.f, oldc = 0.f;
  for (int t = 0; t < T; ++t) {
    const size_t tb = (size_t)t * B + b;
    float ut[m], kt[m], Kc[m];
    if constexpr (GREC > 0) {
      const float* rec = grec + tb * GREC;
#pragma unroll
      for (int a = 0; a < m; ++a) {
        kt[a] = rec[m * n + a];
        Kc[a] = r < n ? rec[a * n + r] : 0.f;
      }
      oldc += rec[m * n + m];
    } else {
#pragma unroll
      for (int a = 0; a < m; ++a) {
        kt[a] = k[tb * m + a];
        Kc[a] = r < n ? K[(tb * m + a) * n + r] : 0.f;
      }
    }
#pragma unroll
    for (int a = 0; a < m; ++a) ut[a] = u[tb * m + a];
    float nu[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      float s = group_sum(Kc[a] * dxr);
      nu[a] = (s + ut[a]) + alpha * kt[a];
      if (zI && zI[tb * m + a]) nu[a] = 0.f;
      if (bd.mode != DILQR_BOUNDS_NONE) nu[a] = eclamp(nu[a], bound_lo(bd, tb * m + a), bound_hi(bd, tb * m + a));
    }
    float nur = 0.f, uur = 0.f;
#pragma unroll
    for (int a = 0; a < m; ++a) {
      nur = (r == n + a) ? nu[a] : nur;
      uur = (r == n + a) ? ut[a] : uur;
    }
    if (valid && r >= n && r < d) {
      u_out[tb * m + (r - n)] = nur;
      if (du_sq) {
        float e = uur - nur;
        du_sq[((size_t)t * m + (r - n)) * B + b] = e * e;
      }
    }
    // the full new state through LDS
    if (r < n) L.tau[r] = xr;
    __syncthreads();
    float xf[n];
#pragma unroll
    for (int i = 0; i < n; ++i) xf[i] = L.tau[i];
    __syncthreads();
    const float taur = r < n ? xr : nur;
    float part = 0.f;
    if (r < d) {
      float Crow[d];
      ld(Crow, C + (tb * d + r) * d);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < n; ++j) s += Crow[j] * xf[j];
#pragma unroll
      for (int a = 0; a < m; ++a) s += Crow[n + a] * nu[a];
      part = 0.5f * (taur * s) + taur * c[tb * d + r];
    }
    cst += group_sum(part);                                  // all 16 lanes shuffle
    if (t < T - 1 && r < n) {
      float xnext;
      if constexpr (std::is_same_v<Model, GroupNoModel>) {
        float Fr[d];
        ld(Fr, F + (tb * n + r) * d);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Fr[j] * xf[j];
#pragma unroll
        for (int a = 0; a < m; ++a) s += Fr[n + a] * nu[a];
        xnext = f ? s + f[tb * n + r] : s;
      } else {
        xnext = md->forward_row(r, xf, nu);
      }
      dxr = xnext - x[(tb + B) * n + r];
      xr = xnext;
      if (valid) x_out[(tb + B) * n + r] = xr;
    }
  }
  if (old_cost_out) *old_cost_out = oldc;
  return cst;
}

// Where a group's stage cost comes from.  Lane r needs row r of C_t and c_t.
// Either the caller's C [T,B,d,d], c [T,B,d] (one 64-byte row per lane per
// step), or — for a problem whose cost the solve's iteration 0 found to be
// diagonal (every off-diagonal entry +0.0 bit for bit) and the same at every t
// (the reference's own callers: diag(q), p repeated, il_env.py:159-162) — two
// registers per lane, C[r][r] and c[r].  row() fills Crow with exactly the
// values the load returns, so the arithmetic is unchanged, bit for bit; only
// the bytes are not read (the dense rows were 30 KB per problem and pass).
struct GroupCost {
  const float* __restrict__ C;
  const float* __restrict__ c;
  bool dconst;
  float cd, cc;
  template <int d>
  DEV void row(size_t tb, int r, float (&Crow)[d], float& cr) const {
    if (dconst) {
#pragma unroll
      for (int j = 0; j < d; ++j) Crow[j] = (j == r) ? cd : 0.f;
      cr = cc;
    } else if (r < d) {
      ld(Crow, C + (tb * d + r) * d);
      cr = c[tb * d + r];
    } else {
#pragma unroll
      for (int j = 0; j < d; ++j) Crow[j] = 0.f;
      cr = 0.f;
    }
  }
};

// Two step sizes rolled out together (the fused MPC kernel's paired line
// search, see ilqr_problem): candidates A (alpha aA) and B (aB, if twoB) share
// the step's loads; each keeps its own state component, controls and cost.
template <int n, int m, int GREC, class Model, class LdsT>
DEV void group_forward_pair(LdsT& L, const Model& md, int T, int B, int b, int r, bool valid, float aA,
                            float aB, bool twoB, const float* __restrict__ x_init, const GroupCost& cs,
                            const float* __restrict__ x, const float* __restrict__ u,
                            const float* __restrict__ grec, const Bounds& bd, float* __restrict__ xa_out,
                            float* __restrict__ ua_out, float* __restrict__ xb_out, float* __restrict__ ub_out,
                            float* __restrict__ du_sq, float& cA, float& cB, float& old_cost) {
  constexpr int d = n + m;
  float xA = (r < n) ? x_init[(size_t)b * n + r] : 0.f, xB = xA;
  float dA = 0.f, dB = 0.f;
  if (valid && r < n) {
    xa_out[(size_t)b * n + r] = xA;
    if (twoB) xb_out[(size_t)b * n + r] = xB;
  }
  float sA = 0.f, sB = 0.f, oldc = 0.f;
  for (int t = 0; t < T; ++t) {
    const size_t tb = (size_t)t * B + b;
    const float* rec = grec + tb * GREC;
    float ut[m], kt[m], Kc[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      kt[a] = rec[m * n + a];
      Kc[a] = r < n ? rec[a * n + r] : 0.f;
      ut[a] = u[tb * m + a];
    }
    oldc += rec[m * n + m];
    float nuA[m], nuB[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      const float pa = group_sum(Kc[a] * dA), pb = group_sum(Kc[a] * dB);
      nuA[a] = (pa + ut[a]) + aA * kt[a];
      nuB[a] = (pb + ut[a]) + aB * kt[a];
      if (bd.mode != DILQR_BOUNDS_NONE) {
        const float lo = bound_lo(bd, tb * m + a), hi = bound_hi(bd, tb * m + a);
        nuA[a] = eclamp(nuA[a], lo, hi);
        nuB[a] = eclamp(nuB[a], lo, hi);
      }
    }
    float nrA = 0.f, nrB = 0.f, uur = 0.f;
#pragma unroll
    for (int a = 0; a < m; ++a) {
      nrA = (r == n + a) ? nuA[a] : nrA;
      nrB = (r == n + a) ? nuB[a] : nrB;
      uur = (r == n + a) ? ut[a] : uur;
    }
    if (valid && r >= n && r < d) {
      ua_out[tb * m + (r - n)] = nrA;
      if (twoB) ub_out[tb * m + (r - n)] = nrB;
      if (du_sq) {
        float e = uur - nrA;
        du_sq[((size_t)t * m + (r - n)) * B + b] = e * e;
      }
    }
    if (r < n) { L.tau[r] = xA; L.tau2[r] = xB; }
    __syncthreads();
    float fA[n], fB[n];
#pragma unroll
    for (int i = 0; i < n; ++i) { fA[i] = L.tau[i]; fB[i] = L.tau2[i]; }
    __syncthreads();
    float pA = 0.f, pB = 0.f;
    if (r < d) {
      float Crow[d], cr;
      cs.row(tb, r, Crow, cr);
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < n; ++j) { s1 += Crow[j] * fA[j]; s2 += Crow[j] * fB[j]; }
#pragma unroll
      for (int a = 0; a < m; ++a) { s1 += Crow[n + a] * nuA[a]; s2 += Crow[n + a] * nuB[a]; }
      const float tA = r < n ? xA : nrA, tB = r < n ? xB : nrB;
      pA = 0.5f * (tA * s1) + tA * cr;
      pB = 0.5f * (tB * s2) + tB * cr;
    }
    sA += group_sum(pA);
    sB += group_sum(pB);
    if (t < T - 1 && r < n) {
      const float xo = x[(tb + B) * n + r];
      const float nA = md.forward_row(r, fA, nuA);
      dA = nA - xo;
      xA = nA;
      if (valid) xa_out[(tb + B) * n + r] = xA;
      if (twoB) {
        const float nB = md.forward_row(r, fB, nuB);
        dB = nB - xo;
        xB = nB;
        if (valid) xb_out[(tb + B) * n + r] = xB;
      }
    }
  }
  cA = sA;
  cB = sB;
  old_cost = oldc;
}

// the line search's accept test (lqr_step_explicit.py:244-252) for a group.  The
// 16 lanes of a group hold the same cost, so `done` is group-uniform; the wave
// keeps looping until every group accepted (its barriers stay balanced), and a
// group that already accepted re-runs its pass at the same alpha, reproducing
// the same trajectory.  Returns true when the wave may leave the loop.
DEV bool group_ls_done(float cost, float old_cost, int ls, int max_ls, bool valid, float& alpha, float decay) {
  const bool done = !(cost > old_cost) || ls == max_ls - 1;
  if (__all(done || !valid)) return true;
  if (!done) alpha *= decay;
  return false;
}

// current trajectory cost (lqr_step_explicit.py:171) for a group
template <int n, int m>
DEV float group_traj_cost(int T, int B, int b, int r, const float* __restrict__ C, const float* __restrict__ c,
                          const float* __restrict__ x, const float* __restrict__ u) {
  constexpr int d = n + m;
  float cost = 0.f;
  for (int t = 0; t < T; ++t) {
    const size_t tb = (size_t)t * B + b;
    float part = 0.f;
    if (r < d) {
      float xt[n], ut[m], Crow[d];
      ld(xt, x + tb * n); ld(ut, u + tb * m); ld(Crow, C + (tb * d + r) * d);
      float s = 0.f, taur = 0.f;
#pragma unroll
      for (int j = 0; j < n; ++j) { s += Crow[j] * xt[j]; taur = (j == r) ? xt[j] : taur; }
#pragma unroll
      for (int a = 0; a < m; ++a) { s += Crow[n + a] * ut[a]; taur = (r == n + a) ? ut[a] : taur; }
      part = 0.5f * (taur * s) + taur * c[tb * d + r];
    }
    cost += group_sum(part);
  }
  return cost;
}

// standalone line search (lqr_forward, lqr_step_explicit.py:166-263) for a group
template <int n, int m, class Model>
__global__ void __launch_bounds__(64) k_lqr_forward_group(int T, int B, const float* __restrict__ theta,
                                                          const float* __restrict__ F, const float* __restrict__ f,
                                                          const float* __restrict__ x_init,
                                                          const float* __restrict__ C, const float* __restrict__ c,
                                                          const float* __restrict__ x, const float* __restrict__ u,
                                                          const float* __restrict__ K, const float* __restrict__ k,
                                                          Bounds bd, const unsigned char* __restrict__ zI,
                                                          float decay, int max_ls, float* __restrict__ x_out,
                                                          float* __restrict__ u_out, float* __restrict__ cost_out,
                                                          float* __restrict__ du_sq, float* __restrict__ alpha_out) {
  __shared__ GroupLds<n, m> Ls[kGPW];
  const int r = threadIdx.x & (kG - 1);
  const int gp = threadIdx.x / kG;
  const int b0 = blockIdx.x * kGPW + gp;
  const bool valid = b0 < B;
  const int b = valid ? b0 : B - 1;
  Model md;
  if constexpr (!std::is_same_v<Model, GroupNoModel>) md.load(theta);
  const float old_cost = group_traj_cost<n, m>(T, B, b, r, C, c, x, u);
  float alpha = 1.f, cost = 0.f;
  for (int ls = 0; ls < max_ls; ++ls) {
    cost = group_forward_pass<n, m, 0>(Ls[gp], &md, F, f, T, B, b, r, valid, alpha, x_init, C, c, x, u, K, k,
                                       nullptr, bd, zI, x_out, u_out, ls == 0 ? du_sq : nullptr, nullptr);
    if (group_ls_done(cost, old_cost, ls, max_ls, valid, alpha, decay)) break;
  }
  if (valid && r == 0) {
    cost_out[b] = cost;
    if (alpha_out) alpha_out[b] = alpha;
  }
}

// ---------------------------------------------------------------- fused iteration
// The backward half of ilqr_problem (dilqr_fused.h) for a 16-lane group:
// on-the-fly Jacobian rows (Model::jac_row), Riccati + the current stage costs;
// gain records (K_t, k_t, stage cost) go to ws [T,B,GREC].
// cs: the cost source (GroupCost).  cpk_out / sym_out (the solve's iteration 0,
// reading the caller's C): decide per problem whether its cost is diagonal and
// time-invariant (flag 7 in sym_out[b], else 0) and, if so, store its row
// values [B][2d] (diag, then c) in cpk_out and switch cs to them, so that a line
// search of this same iteration already takes them from registers.
template <class Model>
constexpr int group_grec() { return ((Model::M * Model::N + Model::M + 1) + 3) / 4 * 4; }

template <class Model, int MODE, class LdsT>
DEV void group_sweep(LdsT& L, int T, int B, int b, int r, bool valid, const Model& md,
                     GroupCost& cs, const float* __restrict__ x, const float* __restrict__ u, const Bounds& bd,
                     float* __restrict__ ws, float* __restrict__ cpk_out = nullptr,
                     unsigned char* __restrict__ sym_out = nullptr) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  bool ok_diag = true, ok_tinv = true;     // this lane's row: off-diagonal +0.0, equal to step T-1's
  float cd_last = 0.f, cc_last = 0.f;
  constexpr int GREC = group_grec<Model>();
  float U[n];                              // column r of V_{t+1} (lane n: v_{t+1}), group_riccati_step_t
#pragma unroll
  for (int i = 0; i < n; ++i) U[i] = 0.f;
  float prev_k[m];
#pragma unroll
  for (int a = 0; a < m; ++a) prev_k[a] = 0.f;
  bool have_prev = false;
  int nqp = 0;
  auto step = [&](int t, auto last_c) {
    constexpr bool LAST = decltype(last_c)::value;
    const size_t tb = (size_t)t * B + b;
    float Crow[d], cr = 0.f, xt[n], ut[m];
    ld(xt, x + tb * n);                              // the group's 16 lanes read the same 64 B
    ld(ut, u + tb * m);
    cs.row(tb, r, Crow, cr);
    if (cpk_out) {                                   // iteration 0: is the cost a time-invariant diagonal?
      float dg = 0.f;
#pragma unroll
      for (int j = 0; j < d; ++j) {
        if (j == r) dg = Crow[j];
        else ok_diag &= __float_as_uint(Crow[j]) == 0u;
      }
      if (LAST) { cd_last = dg; cc_last = cr; }
      ok_tinv &= __float_as_uint(dg) == __float_as_uint(cd_last) && __float_as_uint(cr) == __float_as_uint(cc_last);
    }
    float tau[d];
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
    float Ct = 0.f;
#pragma unroll
    for (int j = 0; j < d; ++j) Ct += Crow[j] * tau[j];
    static_assert(d == kG, "lane r owns tau_r");
    const float taur = r < n ? x[tb * n + r] : u[tb * m + (r - n)];   // tau[r], one load (no select chain)
    const float obj = group_sum(0.5f * (taur * Ct) + taur * cr);
    const float cb = Ct + cr;
    float zIt[m], lb[m], ub[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      zIt[a] = 0.f; lb[a] = ub[a] = 0.f;
      if constexpr (MODE == GAIN_BOX) {
        lb[a] = bound_lo(bd, tb * m + a) - ut[a];
        ub[a] = bound_hi(bd, tb * m + a) - ut[a];
      }
    }
    float col[m];
    // F_t = the model's Jacobian at (x_t, u_t), the whole matrix in every lane
    // (uniform code; its structural zeros drop out of the products)
    float Fu[n][d];
    if constexpr (!LAST) md.jacobian(xt, ut, Fu);
    group_riccati_step_t<n, m, MODE, typename Model::FSparsity, LAST>(L, r, FRegs<n, d>{Fu}, U, Crow, cb, zIt, lb, ub,
                                                                     col, prev_k, have_prev, nqp);
    if (valid) {
      float* rec = ws + tb * GREC;
      if (r < n) {
#pragma unroll
        for (int a = 0; a < m; ++a) rec[a * n + r] = col[a];
      }
      if (r == n) {
#pragma unroll
        for (int a = 0; a < m; ++a) rec[m * n + a] = col[a];
      }
      if (r == 0) rec[m * n + m] = obj;
    }
    __syncthreads();
  };
  step(T - 1, std::true_type{});
  for (int t = T - 2; t >= 0; --t) step(t, std::false_type{});
  if (cpk_out) {
    // the group's verdict (all 16 rows), then the record and the flag; this
    // iteration's line search reads the registers already
    const unsigned long long bad = __ballot(!(ok_diag && ok_tinv));
    const bool grp = ((bad >> (threadIdx.x & ~(kG - 1))) & ((1ull << kG) - 1)) == 0ull;
    if (valid) {
      cpk_out[(size_t)b * 2 * d + r] = cd_last;
      cpk_out[(size_t)b * 2 * d + d + r] = cc_last;
      if (r == 0) sym_out[b] = grp ? 7 : 0;
    }
    if (grp) { cs.dconst = true; cs.cd = cd_last; cs.cc = cc_last; }
  }
}

// ilqr_problem (dilqr_fused.h) for a 16-lane group: group_sweep, then the
// line-search rollout with row-distributed dynamics (Model::forward_row) and
// shuffle-reduced costs.  (The rocket MPC iteration runs its line search one
// problem per lane instead: dilqr_lane_search.h.)
template <class Model, int MODE, class LdsT>
DEV void group_ilqr_problem(LdsT& L, int T, int B, int b, int r, bool valid,
                            const Model& md, const float* __restrict__ x_init, GroupCost cs,
                            const float* __restrict__ x, const float* __restrict__ u,
                            const Bounds& bd, float decay, int max_ls, float* __restrict__ ws,
                            float* __restrict__ x_out, float* __restrict__ u_out, float* __restrict__ xb_out,
                            float* __restrict__ ub_out, float* __restrict__ du_sq, float& cost_out, float& alpha_out,
                            int& win_out) {
  constexpr int n = Model::N, m = Model::M;
  constexpr int GREC = group_grec<Model>();
  group_sweep<Model, MODE>(L, T, B, b, r, valid, md, cs, x, u, bd, ws);
  // ---------------- forward line search
  float alpha = 1.f, cost = 0.f, old_cost = 0.f;
  int win = 0;
  if (xb_out) {
    // passes 2r and 2r+1 together (first accepted wins = the sequential search);
    // the wave leaves when every group accepted
    bool done = false;
    for (int p = 0; p < max_ls; p += 2) {
      const bool twoB = p + 1 < max_ls;
      float cA, cB, oc;
      const float aA = alpha, aB = alpha * decay;
      // a group that already accepted keeps rolling (its barriers) but writes nothing
      group_forward_pair<n, m, GREC>(L, md, T, B, b, r, valid && !done, aA, aB, twoB, x_init, cs, x, u, ws, bd,
                                     x_out,
                                     u_out, xb_out, ub_out, p == 0 ? du_sq : nullptr, cA, cB, oc);
      if (p == 0) old_cost = oc;
      if (!done) {
        if (!(cA > old_cost) || p == max_ls - 1) { cost = cA; alpha = aA; win = 0; done = true; }
        else if (!(cB > old_cost) || p + 1 == max_ls - 1) { cost = cB; alpha = aB; win = 1; done = true; }
        else alpha = aB * decay;
      }
      if (__all(done || !valid)) break;
    }
  } else {
    for (int ls = 0; ls < max_ls; ++ls) {
      float oldc;
      cost = group_forward_pass<n, m, GREC>(L, &md, nullptr, nullptr, T, B, b, r, valid, alpha, x_init, cs.C, cs.c, x, u,
                                            nullptr, nullptr, ws, bd, nullptr, x_out, u_out,
                                            ls == 0 ? du_sq : nullptr, &oldc);
      if (ls == 0) old_cost = oldc;
      if (group_ls_done(cost, old_cost, ls, max_ls, valid, alpha, decay)) break;
    }
  }
  cost_out = cost;
  alpha_out = alpha;
  win_out = win;
}

}  // namespace dilqr
