// dilqr_group8.h — the MPC sweep of the d = 16 models (rocket: n=13 m=3) on
// EIGHT lanes per problem, two rows per lane.
//
// The 16-lane group kernels (dilqr_group.h) give every lane one row of Q and one
// column of V, and every lane of a group also evaluates the problem's whole
// Jacobian (69 structural nonzeros) and the m x m gain solve: per wave-step
// ~500 VALU instructions, of which ~140 are this per-problem work repeated in
// 16 lanes.  With lane l owning rows l and l+8 of Q (columns l, l+8 of V)
// the repeated part is paid for 8 problems per wave instead of 4 while the
// row/column products (the part that scales with the rows) are unchanged per
// problem.
//
// Bits: every entry is computed by the same expression, in the same order, as
// group_riccati_step_t computes it in the lane that owns that row there (the
// multi-right-hand-side gain solve gives each column the single-column
// arithmetic, and the stage cost's 16-row sum is group_sum's butterfly over
// each half of the rows, then the two halves), so this sweep and
// k_lqr_backward_group agree exactly (test_rocket_fused_vs_unfused).
//
// LDS banks: lane l stores rows l and l+8 at a row stride of 17 words (see
// Group8Lds; rows 2l, 2l+1 at stride 16 put all 8 lanes on the same banks).
#pragma once
#include "dilqr_fused.h"
#include "dilqr_group.h"

namespace dilqr {

// DILQR_G8_SKIP: timing-only builds (never the shipped library) that replace
// the per-problem work every lane of a group repeats with stand-ins: bit 0 the
// Jacobian, bit 1 the 3 x 3 gain solve (VERDICT r05 item 3's pricing)
// DILQR_G8_PK (A/B builds; default 0): each lane's two rows (ra, rb) carried
// as packed pairs through the step's products (bits: 1 V^T F, 2 F^T W, 4 the
// value update, 8 C tau), so one v_pk_fma_f32 forms both rows' term with the
// shared factor broadcast from one half; each half is the scalar fma chain of
// the same terms in the same order (the same bits).  Measured at config 3
// (profiles/r06/ab_rocket_sweep_g8_packed.txt): the value update alone (4)
// 0.268-0.270 vs 0.267-0.268 ms per iteration, every other set slower
// (0.288-0.339): the broadcast operands of the packed products need aligned
// register pairs, and the unconstrained register-cost kernel leaves its
// 128-VGPR budget (4 waves per SIMD) for AGPR copies and spills.
#ifndef DILQR_G8_PK
#define DILQR_G8_PK 0
#endif
#define G8PK_U ((DILQR_G8_PK & 5) != 0)
#ifndef DILQR_G8_SKIP
#define DILQR_G8_SKIP 0
#endif
constexpr int kG8 = 8;            // lanes per problem
constexpr int kG8PW = 64 / kG8;   // problems per wave (= per workgroup)
// Group8Lds's W/Q union relies on a workgroup being exactly one wave64 (LDS
// operations of one wave complete in program order): the kernels launch
// kG8PW * kG8 = 64 threads per workgroup, and gfx950 runs wave64
static_assert(kG8PW * kG8 == 64, "a group-8 workgroup must be exactly one wave64");

// group_sum's tree over 16 rows with rows l and l+8 in lane l of an 8-lane
// group: the pairs, quads and half-rows of rows 0-7 (pa) and of rows 8-15 (pb)
// by the same three DPP stages, then the two halves.
DEV float group8_sum(float pa, float pb) {
  pa += dpp_mov<0xB1>(pa);    // quad_perm [1,0,3,2]
  pb += dpp_mov<0xB1>(pb);
  pa += dpp_mov<0x4E>(pa);    // quad_perm [2,3,0,1]
  pb += dpp_mov<0x4E>(pb);
  pa += dpp_mov<0x141>(pa);   // row_half_mirror
  pb += dpp_mov<0x141>(pb);
  return pa + pb;
}

// Q / W row stride 17 (odd): 4-byte stores, but a problem's block is 280
// words instead of 376, so 4 workgroups (waves) per SIMD fit the LDS and the
// register-cost kernel's 121 VGPRs — 4 096 waves in one round instead of 1.33
// rounds at 3 per SIMD.  Bank-conflict-free: lane l's row starts 17 l words
// in, blocks 8 mod 16 words apart.  Measured at config 3 (A/B on one box,
// 3 rounds): MPC iteration 0.345-0.352 -> 0.321-0.327 ms against stride 20.
#ifndef DILQR_G8_QS
#define DILQR_G8_QS 17
#endif
template <int n, int m, bool KK = true>
struct Group8Lds {
  static constexpr int d = n + m;
  static constexpr int W = 16;
  static constexpr int QS = DILQR_G8_QS;         // Q row stride, q_r at [d]
  // W^T rows and Q share the words: a workgroup is one wave, whose LDS
  // accesses complete in program order, so Q's stores (after every lane's
  // W column reads) cannot overtake them.
  union {
    float Wt[n + 1][QS];                         // rows of V^T F, then v^T F
    float Q[d][QS];
  };
  float Kk[KK ? m : 1][W];                       // gains K (box mode: every lane needs all of K)
  // The 4 problems of a half-wave (a b32 read's lane group) read the same
  // relative words; struct strides of 8 mod 16 words put them on 4 disjoint
  // 8-bank sets (16 mod 32 paired them: a 2-way conflict on every column read,
  // 40 % of the sweep's LDS cycles in SQ_LDS_BANK_CONFLICT)
  static constexpr int kWords = d * QS + (KK ? m : 1) * W;
  float pad[(8 - kWords % 16 + 16) % 16];
};
static_assert(sizeof(Group8Lds<13, 3>) / 4 % 16 == 8, "bank offset between problems");
static_assert(sizeof(Group8Lds<13, 3, false>) / 4 % 16 == 8, "bank offset between problems");

// Two right-hand sides of group_gains_col at once (columns ja, jb of the gain
// matrix; j = n is k): the same elimination, each column's own substitution.
template <int n, int m, int MODE>
DEV void group_gains_col2(int ja, int jb, const float (&Quu)[m][m], const float (&ra)[m], const float (&rb)[m],
                          const float (&qu)[m], const float (&lb)[m], const float (&ub)[m], float (&ca)[m],
                          float (&cb)[m], float (&prev_k)[m], bool& have_prev) {
  static_assert(MODE == GAIN_UNC || MODE == GAIN_BOX, "MPC sweep modes");
  if constexpr (MODE == GAIN_UNC) {
    float A[m][m], X[m][2];
#pragma unroll
    for (int a = 0; a < m; ++a) {
#pragma unroll
      for (int b = 0; b < m; ++b) A[a][b] = Quu[a][b] + 0.f;
      X[a][0] = ra[a];
      X[a][1] = rb[a];
    }
    gauss_solve<m, 2, true>(A, X);
#pragma unroll
    for (int a = 0; a < m; ++a) { ca[a] = -X[a][0]; cb[a] = -X[a][1]; }
  } else {
    float x[m], If[m], Hf[m][m];
#pragma unroll
    for (int a = 0; a < m; ++a) x[a] = prev_k[a];
    pnqp<m>(Quu, qu, lb, ub, have_prev, x, If, Hf);
#pragma unroll
    for (int a = 0; a < m; ++a) prev_k[a] = x[a];
    have_prev = true;
    float X[m][2];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      X[a][0] = If[a] != 0.f ? ra[a] : 0.f;
      X[a][1] = If[a] != 0.f ? rb[a] : 0.f;
    }
    gauss_solve<m, 2>(Hf, X);
#pragma unroll
    for (int a = 0; a < m; ++a) {
      ca[a] = ja < n ? -X[a][0] : x[a];
      cb[a] = jb < n ? -X[a][1] : x[a];
    }
  }
}

// The cost rows of one lane (rows ra, rb): the caller's C_t, c_t rows, or the
// time-invariant diagonal held in registers (cd, cc per row)
struct Group8Cost {
  const float* __restrict__ C;
  const float* __restrict__ c;
  bool dconst;
  float cd[2], cc[2];
  template <bool DCONST, int d>
  DEV void row(size_t tb, int r, int k, float (&Crow)[d], float& cr) const {
    if constexpr (DCONST) {
#pragma unroll
      for (int j = 0; j < d; ++j) Crow[j] = (j == r) ? cd[k] : 0.f;
      cr = cc[k];
    } else {
      ld(Crow, C + (tb * d + r) * d);
      cr = c[tb * d + r];
    }
  }
};

// group_sweep (dilqr_group.h) on 8 lanes per problem.  UA/UB: columns ra, rb of
// V_{t+1} (row n: v_{t+1}).  cpk_out / sym_out: iteration 0's cost analysis.
// DCONST: every problem of the wave holds a time-invariant diagonal cost in
// registers (its own instantiation: the caller's rows would keep 32 more
// registers live across the step)
template <class Model, int MODE, bool DCONST, class LdsT>
DEV bool group8_sweep(LdsT& L, int T, int B, int b, int l, bool valid, const Model& md,
                      Group8Cost& cs, const float* __restrict__ x, const float* __restrict__ u, const Bounds& bd,
                      float* __restrict__ ws, float* __restrict__ cpk_out, unsigned char* __restrict__ sym_out) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  static_assert(d == 2 * kG8, "two rows per lane");
  using FS = typename Model::FSparsity;
  constexpr int GREC = group_grec<Model>();
  constexpr bool SCHUR = MODE == GAIN_UNC;
  const int ra = l, rb = l + kG8;                  // ra < n in every lane; rb <= n (a V column or v) in lanes 0-5
  bool ok = true;                                  // iteration 0: this lane's rows diagonal and time-invariant
  float cd_last[2] = {0.f, 0.f}, cc_last[2] = {0.f, 0.f};
#if G8PK_U
  f2 U2[n];                                        // (column ra, column rb) of V_{t+1}, one pair per row
#pragma unroll
  for (int i = 0; i < n; ++i) U2[i] = f2{0.f, 0.f};
#else
  float UA[n], UB[n];
#pragma unroll
  for (int i = 0; i < n; ++i) { UA[i] = 0.f; UB[i] = 0.f; }
#endif
  float prev_k[m];
#pragma unroll
  for (int a = 0; a < m; ++a) prev_k[a] = 0.f;
  bool have_prev = false;
  auto step = [&](int t, auto last_c) {
    constexpr bool LAST = decltype(last_c)::value;
    const size_t tb = (size_t)t * B + b;
    float xt[n], ut[m];
    ld(xt, x + tb * n);
    ld(ut, u + tb * m);
    float CA[d], CB[d], cra, crb;
    cs.row<DCONST>(tb, ra, 0, CA, cra);
    cs.row<DCONST>(tb, rb, 1, CB, crb);
    if (!DCONST && cpk_out) {
      float dga = 0.f, dgb = 0.f;
#pragma unroll
      for (int j = 0; j < d; ++j) {
        if (j == ra) dga = CA[j]; else ok &= __float_as_uint(CA[j]) == 0u;
        if (j == rb) dgb = CB[j]; else ok &= __float_as_uint(CB[j]) == 0u;
      }
      if (LAST) { cd_last[0] = dga; cc_last[0] = cra; cd_last[1] = dgb; cc_last[1] = crb; }
      ok &= __float_as_uint(dga) == __float_as_uint(cd_last[0]) && __float_as_uint(cra) == __float_as_uint(cc_last[0]);
      ok &= __float_as_uint(dgb) == __float_as_uint(cd_last[1]) && __float_as_uint(crb) == __float_as_uint(cc_last[1]);
    }
    float tau[d];
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
#if DILQR_G8_PK & 8
    float Cta, Ctb;
    {
      f2 ct = f2{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < d; ++j) ct = ct + f2{CA[j], CB[j]} * tau[j];
      Cta = ct.x;
      Ctb = ct.y;
    }
#else
    float Cta = 0.f, Ctb = 0.f;
#pragma unroll
    for (int j = 0; j < d; ++j) { Cta += CA[j] * tau[j]; Ctb += CB[j] * tau[j]; }
#endif
    const float taua = ra < n ? x[tb * n + ra] : u[tb * m + (ra - n)];   // tau[ra], tau[rb]: loads, no select chains
    const float taub = rb < n ? x[tb * n + rb] : u[tb * m + (rb - n)];
    const float obj = group8_sum(0.5f * (taua * Cta) + taua * cra, 0.5f * (taub * Ctb) + taub * crb);
    const float cba = Cta + cra, cbb = Ctb + crb;
    float QA[d], QB[d], qa, qb;
    if constexpr (LAST) {
#pragma unroll
      for (int j = 0; j < d; ++j) { QA[j] = CA[j] + 0.f; QB[j] = CB[j] + 0.f; }
      qa = cba + 0.f;
      qb = cbb + 0.f;
    } else {
      float F[n][d];
#if DILQR_G8_SKIP & 1
      // timing-only build: a stand-in for the Jacobian (one product per
      // structural nonzero) to price the per-problem Jacobian every lane repeats
#pragma unroll
      for (int k = 0; k < n; ++k)
#pragma unroll
        for (int j = 0; j < d; ++j) F[k][j] = FS::nz(k, j) ? xt[(k + j) % n] * 0.001f : 0.f;
#else
      md.jacobian(xt, ut, F);
#endif
      {                                            // rows ra, rb of V^T F (row n: v^T F)
        float Wa[d], Wb[d];
#pragma unroll
        for (int j = 0; j < d; ++j) {
#if DILQR_G8_PK & 1
          f2 s2 = f2{0.f, 0.f};
#pragma unroll
          for (int k = 0; k < n; ++k)
            if (FS::nz(k, j)) s2 = s2 + U2[k] * F[k][j];
          Wa[j] = s2.x;
          Wb[j] = s2.y;
#else
          float sa = 0.f, sb = 0.f;
#pragma unroll
          for (int k = 0; k < n; ++k)
            if (FS::nz(k, j)) {
#if G8PK_U
              sa += U2[k].x * F[k][j];
              sb += U2[k].y * F[k][j];
#else
              sa += UA[k] * F[k][j];
              sb += UB[k] * F[k][j];
#endif
            }
          Wa[j] = sa;
          Wb[j] = sb;
#endif
        }
#pragma unroll
        for (int j = 0; j < d; ++j) L.Wt[ra][j] = Wa[j];
        if (rb <= n) {
#pragma unroll
          for (int j = 0; j < d; ++j) L.Wt[rb][j] = Wb[j];
        }
      }
      __syncthreads();
#if DILQR_G8_PK & 2
      f2 Wc2[n + 1];
#pragma unroll
      for (int k = 0; k <= n; ++k) Wc2[k] = f2{L.Wt[k][ra], L.Wt[k][rb]};
#pragma unroll
      for (int i = 0; i < d; ++i) {                // rows ra, rb of F^T V F
        f2 s2 = f2{0.f, 0.f};
#pragma unroll
        for (int k = 0; k < n; ++k)
          if (FS::nz(k, i)) s2 = s2 + F[k][i] * Wc2[k];
        const f2 q2 = f2{CA[i], CB[i]} + s2;
        QA[i] = q2.x;
        QB[i] = q2.y;
      }
      qa = cba + Wc2[n].x;
      qb = cbb + Wc2[n].y;
#else
      float Wca[n + 1], Wcb[n + 1];
#pragma unroll
      for (int k = 0; k <= n; ++k) { Wca[k] = L.Wt[k][ra]; Wcb[k] = L.Wt[k][rb]; }
#pragma unroll
      for (int i = 0; i < d; ++i) {                // rows ra, rb of F^T V F
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int k = 0; k < n; ++k)
          if (FS::nz(k, i)) { sa += F[k][i] * Wca[k]; sb += F[k][i] * Wcb[k]; }
        QA[i] = CA[i] + sa;
        QB[i] = CB[i] + sb;
      }
      qa = cba + Wca[n];
      qb = cbb + Wcb[n];
#endif
    }
    // Q overwrites W^T's words: every lane's W column reads above precede
    // these stores in the wave's program order (one wave per workgroup), and
    // the scheduling barrier keeps the compiler from moving them across
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < d; ++j) { L.Q[ra][j] = QA[j]; L.Q[rb][j] = QB[j]; }
    L.Q[ra][d] = qa;
    L.Q[rb][d] = qb;
    __syncthreads();
    float Quu[m][m], qu[m], rha[m], rhb[m];
    const int ja = ra <= n ? ra : n, jb = rb <= n ? rb : n;   // right-hand sides (rows > n repeat k's)
#pragma unroll
    for (int a = 0; a < m; ++a) {
#pragma unroll
      for (int c2 = 0; c2 < m; ++c2) Quu[a][c2] = L.Q[n + a][n + c2];
      qu[a] = L.Q[n + a][d];
      rha[a] = ja < n ? L.Q[n + a][ja] : qu[a];
      rhb[a] = jb < n ? L.Q[n + a][jb] : qu[a];
    }
    float lo[m], hi[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      lo[a] = hi[a] = 0.f;
      if constexpr (MODE == GAIN_BOX) {
        lo[a] = bound_lo(bd, tb * m + a) - ut[a];
        hi[a] = bound_hi(bd, tb * m + a) - ut[a];
      }
    }
    float cola[m], colb[m];
#if DILQR_G8_SKIP & 2
    // timing-only build: a diagonal stand-in for the 3x3 gain solve every lane repeats
#pragma unroll
    for (int a = 0; a < m; ++a) {
      const float ir = __builtin_amdgcn_rcpf(Quu[a][a]);
      cola[a] = -rha[a] * ir;
      colb[a] = -rhb[a] * ir;
    }
#else
    group_gains_col2<n, m, MODE>(ja, jb, Quu, rha, rhb, qu, lo, hi, cola, colb, prev_k, have_prev);
#endif
    // V_t columns ra, rb (row n's lane: v_t), group_riccati_step_t's expressions
    float Kall[m][n];
    if constexpr (!SCHUR) {
#pragma unroll
      for (int a = 0; a < m; ++a) {
        if (ra < n) L.Kk[a][ra] = cola[a];
        if (rb < n) L.Kk[a][rb] = colb[a];
      }
      __syncthreads();
#pragma unroll
      for (int a = 0; a < m; ++a)
#pragma unroll
        for (int i = 0; i < n; ++i) Kall[a][i] = L.Kk[a][i];
    }
    {
      const int cxa = ra, cxb = rb < n ? rb : d;
      float za[m], zb[m], Qna[m], Qnb[m];
      if constexpr (!SCHUR) {
#pragma unroll
        for (int a = 0; a < m; ++a) {
          float s = 0.f, s2 = 0.f;
#pragma unroll
          for (int c2 = 0; c2 < m; ++c2) { s += Quu[a][c2] * cola[c2]; s2 += Quu[a][c2] * colb[c2]; }
          za[a] = s;
          zb[a] = s2;
          Qna[a] = L.Q[n + a][cxa];
          Qnb[a] = L.Q[n + a][cxb];
        }
      }
#pragma unroll
      for (int i = 0; i < n; ++i) {
#if DILQR_G8_PK & 4
        f2 s1 = f2{0.f, 0.f};
#pragma unroll
        for (int a = 0; a < m; ++a) s1 = s1 + L.Q[i][n + a] * f2{cola[a], colb[a]};
        f2 v2 = f2{L.Q[i][cxa], L.Q[i][cxb]} + s1;
        if constexpr (!SCHUR) {
          f2 s2 = f2{0.f, 0.f}, s3 = f2{0.f, 0.f};
#pragma unroll
          for (int a = 0; a < m; ++a) {
            s2 = s2 + Kall[a][i] * f2{Qna[a], Qnb[a]};
            s3 = s3 + Kall[a][i] * f2{za[a], zb[a]};
          }
          v2 = (v2 + s2) + s3;
        }
        U2[i] = v2;
#else
        float s1a = 0.f, s1b = 0.f;
#pragma unroll
        for (int a = 0; a < m; ++a) {
          const float qi = L.Q[i][n + a];
          s1a += qi * cola[a];
          s1b += qi * colb[a];
        }
        float va = L.Q[i][cxa] + s1a, vb = L.Q[i][cxb] + s1b;
        if constexpr (!SCHUR) {
          float s2a = 0.f, s3a = 0.f, s2b = 0.f, s3b = 0.f;
#pragma unroll
          for (int a = 0; a < m; ++a) {
            s2a += Kall[a][i] * Qna[a];
            s3a += Kall[a][i] * za[a];
            s2b += Kall[a][i] * Qnb[a];
            s3b += Kall[a][i] * zb[a];
          }
          va = (va + s2a) + s3a;
          vb = (vb + s2b) + s3b;
        }
#if G8PK_U
        U2[i] = f2{va, vb};
#else
        UA[i] = va;
        UB[i] = vb;
#endif
#endif
      }
    }
    if (valid) {
      float* rec = ws + tb * GREC;
#pragma unroll
      for (int a = 0; a < m; ++a) {
        if (ra < n) rec[a * n + ra] = cola[a];
        if (rb < n) rec[a * n + rb] = colb[a];
        if (rb == n) rec[m * n + a] = colb[a];
      }
      if (l == 0) rec[m * n + m] = obj;
    }
    __syncthreads();
  };
  step(T - 1, std::true_type{});
  for (int t = T - 2; t >= 0; --t) step(t, std::false_type{});
  if (!DCONST && cpk_out) {
    const unsigned long long bad = __ballot(!ok);
    const bool grp = ((bad >> (threadIdx.x & ~(kG8 - 1))) & ((1ull << kG8) - 1)) == 0ull;
    if (valid) {
      cpk_out[(size_t)b * 2 * d + ra] = cd_last[0];
      cpk_out[(size_t)b * 2 * d + rb] = cd_last[1];
      cpk_out[(size_t)b * 2 * d + d + ra] = cc_last[0];
      cpk_out[(size_t)b * 2 * d + d + rb] = cc_last[1];
      if (l == 0) sym_out[b] = grp ? 7 : 0;
    }
    return !grp;                                   // iteration 0: this problem keeps the caller's cost
  }
  return false;
}

}  // namespace dilqr
