// tu_mpc_rocket.hip — the fused iteration for the 16-lanes-per-problem model
// (env_dx/rocket.py, n=13 m=3): standalone and device-resident MPC kernels.
#include "dilqr_group8.h"
#include "dilqr_lane_search.h"

namespace dilqr {

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
  __shared__ GroupLdsT<Model::N, Model::M, false, true> Ls[kGPW];
  if (ctrl && ctrl->stopped) return;
  const int r = threadIdx.x & (kG - 1), gp = threadIdx.x / kG;
  const int b0 = blockIdx.x * kGPW + gp;
  const bool valid = b0 < B;
  const int b = valid ? b0 : B - 1;          // idle groups shadow problem B-1 (same wave), writing nothing
  Model md; md.load(theta);
  float cost, alpha;
  int win;
  group_ilqr_problem<Model, MODE>(Ls[gp], T, B, b, r, valid, md, x_init, GroupCost{C, c, false, 0.f, 0.f}, x, u, bd,
                                  decay, max_ls, ws, x_out, u_out, nullptr, nullptr, du_sq, cost, alpha, win);
  if (valid && r == 0) {
    cost_out[b] = cost;
    alpha_out[b] = alpha;
  }
}

// The MPC iteration of the 16-lanes-per-problem models is two launches: the
// group sweep (stop-rule prologue, linearise + Riccati on 16 lanes per problem,
// gain records to S.ws, iteration 0's cost flags), then the line search one
// problem per lane (dilqr_lane_search.h) with the best-iterate bookkeeping.
// Measured at config 3 (rocket, B = 32768, T = 30): the single group kernel
// doing both took 1.08 ms per iteration, its row-distributed rollout being the
// larger half.
template <class Model, int MODE>
#ifndef DILQR_SWEEP_WAVES
#define DILQR_SWEEP_WAVES 3
#endif
__global__ void __launch_bounds__(64, DILQR_SWEEP_WAVES) k_mpc_sweep_group(int T, int B, const float* __restrict__ theta,
                                                          const float* __restrict__ C, const float* __restrict__ c,
                                                          Bounds bd, int iteration, float eps, int not_improved_lim,
                                                          int G, MpcState S) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  __shared__ GroupLdsT<n, m, false, false> Ls[kGPW];
  if (mpc_decide(S, B, iteration, G, eps, not_improved_lim)) return;
  const bool first = iteration == 0;
  const int r = threadIdx.x & (kG - 1), gp = threadIdx.x / kG;
  const int b0 = blockIdx.x * kGPW + gp;
  const bool valid = b0 < B;
  const int b = valid ? b0 : B - 1;
  Model md; md.load(theta);
  const size_t TBn = (size_t)T * B * n, TBm = (size_t)T * B * m;
  const int cur = S.slot[b];
  // the cost: the caller's rows, or (a time-invariant diagonal cost, flagged by
  // iteration 0) two registers per lane from the solve's record [B][2d]
  GroupCost cs{C, c, false, 0.f, 0.f};
  if (!first && S.Cpk && S.cost_sym[b] == 7) {
    cs.dconst = true;
    cs.cd = S.Cpk[(size_t)b * 2 * d + r];
    cs.cc = S.Cpk[(size_t)b * 2 * d + d + r];
  }
  group_sweep<Model, MODE>(Ls[gp], T, B, b, r, valid, md, cs, S.Xs + cur * TBn, S.Us + cur * TBm, bd, S.ws,
                           first ? S.Cpk : nullptr, first ? S.cost_sym : nullptr);
}

// The same sweep on 8 lanes per problem (dilqr_group8.h): 8 problems per wave,
// the per-problem work (Jacobian, gain solve) repeated in 8 lanes instead of
// 16.  Measured at config 3 (A/B on one box, tools/ab_rocket.py): MPC iteration
// 0.400 -> 0.360 ms, the steady sweep 255 -> 197 us.
#ifndef DILQR_SWEEP8_WAVES
#define DILQR_SWEEP8_WAVES 3
#endif
template <class Model, int MODE, bool DCONST>
__global__ void __launch_bounds__(64, MODE == GAIN_BOX ? 2 : DCONST ? DILQR_SWEEP8_WAVES : 3) k_mpc_sweep_g8(int T, int B, const float* __restrict__ theta,
                                                                         const float* __restrict__ C,
                                                                         const float* __restrict__ c, Bounds bd,
                                                                         int iteration, float eps, int not_improved_lim,
                                                                         int G, MpcState S) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  __shared__ Group8Lds<n, m, MODE != GAIN_UNC> Ls[kG8PW];
  if (mpc_decide(S, B, iteration, G, eps, not_improved_lim)) return;
  const bool first = iteration == 0;
  // the dense-cost instantiation after iteration 0, when iteration 0 found
  // every cost to be a time-invariant diagonal one: nothing to do (it is
  // launched on a grid capped at the chip's resident workgroups then, striding)
  if (!DCONST && !first && S.Cpk && S.done_counter[kDenseCount] == 0u) return;
  const int l = threadIdx.x & (kG8 - 1), gp = threadIdx.x / kG8;
  Model md; md.load(theta);
  const size_t TBn = (size_t)T * B * n, TBm = (size_t)T * B * m;
  const int nblk = (B + kG8PW - 1) / kG8PW;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {   // one pass unless the grid is small
    const int b0 = blk * kG8PW + gp;
    const bool valid = b0 < B;
    const int b = valid ? b0 : B - 1;
    const int cur = S.slot[b];
    // the register cost when every problem of the wave has one (wave-uniform);
    // the two kinds of wave run in two instantiations launched back to back,
    // each leaving the other's waves at once
    const bool dconst = !first && S.Cpk && S.cost_sym[b] == 7;
    if (__all(dconst) != DCONST) continue;
    Group8Cost cs{C, c, DCONST, {0.f, 0.f}, {0.f, 0.f}};
    if (DCONST) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        cs.cd[k] = S.Cpk[(size_t)b * 2 * d + l + kG8 * k];        // rows l, l + 8
        cs.cc[k] = S.Cpk[(size_t)b * 2 * d + d + l + kG8 * k];
      }
    }
    const bool dense = group8_sweep<Model, MODE, DCONST>(Ls[gp], T, B, b, l, valid, md, cs, S.Xs + cur * TBn,
                                                         S.Us + cur * TBm, bd, S.ws, first ? S.Cpk : nullptr,
                                                         first ? S.cost_sym : nullptr);
    if (!DCONST && first && S.Cpk) {                              // count the problems that stay dense
      const unsigned long long bal = __ballot(dense && valid && l == 0);
      if ((threadIdx.x & 63) == 0 && bal) atomicAdd(&S.done_counter[kDenseCount], (unsigned)__popcll(bal));
    }
  }
}

// DILQR_SWEEP_LANES: 8 (default) or 16 lanes per problem in the MPC sweep (the
// 16-lane kernel stays for A/B builds)
#ifndef DILQR_SWEEP_LANES
#define DILQR_SWEEP_LANES 8
#endif
// The dense-cost instantiations after iteration 0 usually find nothing to do
// (iteration 0 counted no dense-cost problem), but the host cannot see that
// count without a sync, so their grid must serve a batch of dense costs at full
// speed too: it is capped at the workgroups the chip keeps resident at once
// (CUs x the kernel's occupancy per CU), and the kernel strides over the rest.
// (Round 5 capped it at 256 workgroups, which left a dense batch at a quarter
// of a wave per SIMD, striding serially — ADVICE r05.)
template <class K>
int resident_workgroups(K kern, int threads, size_t lds) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, threads, lds) != hipSuccess || cus <= 0 || per <= 0)
    return 1 << 30;                                       // unknown: no cap
  return cus * per;
}

// DILQR_SEARCH_QUAD: the line search on a quad of lanes per problem (1, the
// default: every pass of a round at once, cost only) or on lane pairs (0)
#ifndef DILQR_SEARCH_QUAD
#define DILQR_SEARCH_QUAD 1
#endif
int launch_mpc_step_rocket(const MpcStepArgs& a) {
#if DILQR_SEARCH_QUAD
  const int gq = grid_for(4 * (long long)a.B);
#define SEARCH(BM_, DC_)                                                                                          \
  do {                                                                                                            \
    static const int cap = resident_workgroups(k_mpc_search_quad<Rocket, BM_, false>, kBlock, 0);                 \
    const int g = (DC_ || !a.st.Cpk) ? gq : (gq < cap ? gq : cap);                                                 \
    k_mpc_search_quad<Rocket, BM_, DC_><<<g, kBlock, 0, a.stream>>>(                                               \
        a.T, a.B, a.theta, a.x_init, a.C, a.c, a.bd, a.decay, a.max_ls, a.iteration, a.best_cost_eps, a.G, a.st);  \
  } while (0)
#else
#define SEARCH(BM_, DC_)                                                                                          \
  k_mpc_search_lane<Rocket, BM_, DC_><<<grid_for(2 * (long long)a.B), kBlock, 0, a.stream>>>(                     \
      a.T, a.B, a.theta, a.x_init, a.C, a.c, a.bd, a.decay, a.max_ls, a.iteration, a.best_cost_eps, a.G, a.st)
#endif
#if DILQR_SWEEP_LANES == 8
  // the dense-cost instantiations after iteration 0 (with a packed copy):
  // a small grid that strides over the problems, so that the usual empty pass
  // (every cost a time-invariant diagonal one) costs a few workgroups, not
  // B/8 of them
  const int g8 = (int)((a.B + kG8PW - 1) / kG8PW);
#define SWEEP8(MODE_, DC_)                                                                                        \
  do {                                                                                                            \
    static const int cap = resident_workgroups(k_mpc_sweep_g8<Rocket, MODE_, false>, 64, 0);                      \
    const int g = (DC_ || a.iteration == 0 || !a.st.Cpk) ? g8 : (g8 < cap ? g8 : cap);                           \
    k_mpc_sweep_g8<Rocket, MODE_, DC_><<<g, 64, 0, a.stream>>>(a.T, a.B, a.theta, a.C, a.c, a.bd, a.iteration,    \
                                                              a.eps, a.lim, a.G, a.st);                           \
  } while (0)
#define SWEEP(MODE_)                                                                                              \
  SWEEP8(MODE_, true);                                                                                            \
  SWEEP8(MODE_, false)
#else
#if DILQR_SEARCH_QUAD
#error "the quad search relies on the 8-lane sweep's count of dense-cost problems (kDenseCount)"
#endif
#define SWEEP(MODE_)                                                                                              \
  k_mpc_sweep_group<Rocket, MODE_><<<grid_group(a.B), 64, 0, a.stream>>>(                                         \
      a.T, a.B, a.theta, a.C, a.c, a.bd, a.iteration, a.eps, a.lim, a.G, a.st)
#endif
  if (a.bd.mode != DILQR_BOUNDS_NONE) {
    SWEEP(GAIN_BOX);
    SEARCH(DILQR_BOUNDS_SCALAR, true);
    SEARCH(DILQR_BOUNDS_SCALAR, false);
  } else {
    SWEEP(GAIN_UNC);
    SEARCH(DILQR_BOUNDS_NONE, true);
    SEARCH(DILQR_BOUNDS_NONE, false);
  }
#undef SEARCH
#undef SWEEP
#if DILQR_SWEEP_LANES == 8
#undef SWEEP8
#endif
  return launched();
}

int launch_ilqr_iterate_rocket(const IlqrIterArgs& a) {
  if (a.bd.mode != DILQR_BOUNDS_NONE)
    k_ilqr_iterate_group<Rocket, GAIN_BOX><<<grid_group(a.B), 64, 0, a.stream>>>(
        a.T, a.B, a.theta, a.x_init, a.C, a.c, a.x, a.u, a.bd, a.decay, a.max_ls, a.ws, a.x_out, a.u_out, a.cost,
        a.du_sq, a.alpha, a.ctrl);
  else
    k_ilqr_iterate_group<Rocket, GAIN_UNC><<<grid_group(a.B), 64, 0, a.stream>>>(
        a.T, a.B, a.theta, a.x_init, a.C, a.c, a.x, a.u, a.bd, a.decay, a.max_ls, a.ws, a.x_out, a.u_out, a.cost,
        a.du_sq, a.alpha, a.ctrl);
  return launched();
}

}  // namespace dilqr
