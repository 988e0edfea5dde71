// tu_riccati.hip — the standalone backward Riccati sweep (lqr_backward,
// lqr_step_explicit.py:54-162), one lane or one 16-lane group per problem.
#include "dilqr_common.h"

// DILQR_GROUP_SWEEP_SMALL (default 0; timing builds only): batches of at most
// this many cartpole problems take the 16-lane group sweep (dilqr_group.h,
// lane r owns row r) instead of one lane per problem — the small-batch mapping
// of DESIGN.md §6, measured in profiles/r06/small_sweep_mapping.txt
#ifndef DILQR_GROUP_SWEEP_SMALL
#define DILQR_GROUP_SWEEP_SMALL 0
#endif

namespace dilqr {

// ============================================================ Riccati sweep
// lqr_backward (lqr_step_explicit.py:54-162) with the delta-space c_back of
// 630-636 fused.  F [T-1,B,n,d] is read from HBM.
template <int n, int m, int MODE>
__global__ void __launch_bounds__(kBlock) k_lqr_backward(int T, int B, const float* __restrict__ C,
                                                         const float* __restrict__ c, const float* __restrict__ x,
                                                         const float* __restrict__ u, const float* __restrict__ F,
                                                         Bounds bd, const unsigned char* __restrict__ zI,
                                                         float* __restrict__ K, float* __restrict__ k,
                                                         int* __restrict__ n_qp, int* __restrict__ n_qp_step) {
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
    const int qp_before = rs.n_qp;
    if (symsofar) rs.template step<MODE, DenseF, false, true>(cur.C, cb, cur.F, zIt, lb, ub, Kt, kt);
    else rs.template step<MODE>(cur.C, cb, cur.F, zIt, lb, ub, Kt, kt);
    if (MODE == GAIN_BOX && n_qp_step) atomicMax(n_qp_step + t, rs.n_qp - qp_before - 1);
    st2(K + tb * m * n, Kt);
    st(k + tb * m, kt);
    cur = nxt;
  }
  if (n_qp) n_qp[b] = rs.n_qp;
}

}  // namespace dilqr

using namespace dilqr;

extern "C" {

int dilqr_lqr_backward_f32(int n, int m, int T, int B, const float* C, const float* c, const float* x,
                           const float* u, const float* F, dilqr_bounds bounds, const unsigned char* u_zero_I,
                           int m_solver, float* K, float* k, int* n_qp_iter, int* n_qp_step, void* stream) {
  if (T < 1 || B < 0 || !C || !c || !K || !k || (T > 1 && !F)) return DILQR_E_ARG;
  if (x && !u) return DILQR_E_ARG;   // u alone: c is already c_back, u only shifts the bounds
  if (!al16(C) || !al16(c) || !al16(x) || !al16(u) || !al16(F) || !al16(K) || !al16(k)) return DILQR_E_ARG;
  if (bad_bounds(bounds)) return DILQR_E_ARG;
  // bounds with u = NULL (then x = NULL too): the bounds are already relative,
  // lb = lower - u_t formed by the caller (e.g. clipped to +-delta_u,
  // lqr_step_explicit.py:132-135)
  if (bounds.mode != DILQR_BOUNDS_NONE && u_zero_I) return DILQR_E_MODE;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  int mode = bounds.mode != DILQR_BOUNDS_NONE ? GAIN_BOX
             : u_zero_I ? GAIN_ZERO_I
             : (m_solver == DILQR_SOLVE_CHOL && m > 1) ? GAIN_CHOL : GAIN_UNC;
#if DILQR_GROUP_SWEEP_SMALL
  // timing builds only (tools/small_sweep_mapping.py): cartpole's sweep on the
  // 16-lane row-per-lane group mapping for small batches, against the lane sweep
  if (n == 5 && m == 1 && B <= DILQR_GROUP_SWEEP_SMALL) {
#define GLAUNCH(MODE_)                                                                                       \
    k_lqr_backward_group<5, 1, MODE_><<<grid_group(B), 64, 0, S(stream)>>>(T, B, C, c, x, u, F, bd, u_zero_I, K, \
                                                                           k, n_qp_iter, n_qp_step)
    switch (mode) {
      case GAIN_UNC: GLAUNCH(GAIN_UNC); break;
      case GAIN_ZERO_I: GLAUNCH(GAIN_ZERO_I); break;
      default: GLAUNCH(GAIN_BOX); break;
    }
#undef GLAUNCH
    return launched();
  }
#endif
#define LAUNCH(N_, M_, MODE_) \
  k_lqr_backward<N_, M_, MODE_><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, C, c, x, u, F, bd, u_zero_I, K, k, n_qp_iter, \
                                                                       n_qp_step)
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
                                                                           n_qp_iter, n_qp_step)
  DILQR_FOR_EACH_GROUP_SHAPE(X)
#undef X
#undef LAUNCH
  return DILQR_E_SHAPE;
}

}  // extern "C"
