// dilqr_lane_search.h — the line search of the 16-lanes-per-problem models
// (rocket, d = 16) run ONE problem per lane.
//
// The group kernels need 16 lanes per problem for the Riccati sweep (a step's
// V, Q, F do not fit one lane's registers), but the rollout only carries a
// 13-vector: distributed over a group, its row-wise dynamics is a switch that
// every lane of the wave executes case by case, the state goes through LDS at
// every step, and the 4 problems of a wave pay 16 lanes of instructions each.
// Here a lane rolls one candidate of one problem out (Rocket::forward) from
// the gain records the group sweep left in HBM, so a wave does 32 problems'
// paired rollouts for the instructions the group kernel spent on 4.
//
// The arithmetic is the group line search's, bit for bit (group_forward_pair):
// a 16-lane group_sum is a fixed butterfly, restated as tree16 below; each
// row's cost product chain is the same sequence of fmas; the dynamics are
// forward_row's expressions.  So the MPC path (group sweep + this search) and
// the unfused k_lqr_forward_group agree exactly (test_rocket_fused_vs_unfused).
#pragma once
#include "dilqr_fused.h"
#include "dilqr_group.h"

namespace dilqr {

// The sum group_sum leaves in every lane of a 16-lane group, in one lane: its
// four DPP stages add lane pairs (i, i^1), then (i, i^2), then the mirrored
// quads of each half-row, then the two half-rows; float addition commutes, so
// every lane's total is this tree.
template <class V>
DEV V tree16(const V (&v)[16]) {
  const V q0 = (v[0] + v[1]) + (v[2] + v[3]);
  const V q1 = (v[4] + v[5]) + (v[6] + v[7]);
  const V q2 = (v[8] + v[9]) + (v[10] + v[11]);
  const V q3 = (v[12] + v[13]) + (v[14] + v[15]);
  return (q0 + q1) + (q2 + q3);
}

// Inputs of search step t: the gain record (K, k, the current stage cost), x_t
// and u_t of the current trajectory; loaded one step ahead.
template <int n, int m, int GREC>
struct LaneIn {
  float g[GREC], u[m], x[n];
  DEV void load(const float* __restrict__ ws, const float* __restrict__ x_, const float* __restrict__ u_, int t,
                int B, int b) {
    const size_t tb = (size_t)t * B + b;
    ld(g, ws + tb * GREC);
    ld(u, u_ + tb * m);
    ld(x, x_ + tb * n);
  }
};

// Stage cost of this lane's candidate, tau = [x; u], the rows summed as
// group_forward_pair does.  DCONST: the time-invariant diagonal cost held in
// registers (cd, cc) — row r's product chain there is fma(C[r][j], tau_j, .)
// over j with C[r][j] = +0 off the diagonal, which equals
// fma(cd_r, tau_r, probe) with probe = that chain's +0 (NaN if any tau_j is
// not finite: 0 * inf); otherwise the caller's C_t, c_t rows from HBM.
template <int d, bool DCONST>
DEV float lane_stage_cost(const float (&tau)[d], const float (&cd)[d], const float (&cc)[d],
                          const float* __restrict__ C, const float* __restrict__ c, size_t tb) {
  static_assert(d == 16, "the group sum covers 16 rows");
  float pr[d];
  if constexpr (DCONST) {
    float probe = 0.f;
#pragma unroll
    for (int j = 0; j < d; ++j) probe = __builtin_fmaf(0.f, tau[j], probe);
#pragma unroll
    for (int r = 0; r < d; ++r) {
      const float s = __builtin_fmaf(cd[r], tau[r], probe);
      pr[r] = 0.5f * (tau[r] * s) + tau[r] * cc[r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < d; ++r) {             // a dense cost: one row in registers at a time
      float Crow[d];
      ld(Crow, C + (tb * d + r) * d);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < d; ++j) s += Crow[j] * tau[j];
      pr[r] = 0.5f * (tau[r] * s) + tau[r] * c[tb * d + r];
    }
  }
  return tree16(pr);
}

// One pass of this lane's candidate (step size al; lane pair (A, B) of a
// problem: passes 2p and 2p+1 of the search), its stage costs summed into
// cost and the current trajectory's (from the gain records) into old_cost.
// DCONST: the whole wave's problems hold a time-invariant diagonal cost in
// registers (cd, cc), else every lane reads the caller's rows (a flagged
// problem's rows hold the same values).  Writes x/u to (xo, uo) when `wr`.
#ifndef DILQR_SEARCH_PFD
#define DILQR_SEARCH_PFD 1
#endif
template <class Model, int BM, bool DCONST, int PFD = DILQR_SEARCH_PFD>
DEV void lane_pass(int T, int B, int b, const Model& md, const float* __restrict__ x_init,
                   const float (&cd)[Model::N + Model::M], const float (&cc)[Model::N + Model::M],
                   const float* __restrict__ C, const float* __restrict__ c, const float* __restrict__ ws,
                   const float* __restrict__ x, const float* __restrict__ u, const Bounds& bd, float al, bool wr,
                   float* __restrict__ xo, float* __restrict__ uo, float* __restrict__ du_sq, float& cost,
                   float& old_cost) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  constexpr int GREC = group_grec<Model>();
  float xs[n];
  ld(xs, x_init + (size_t)b * n);
  if (wr) st(xo + (size_t)b * n, xs);
  float sc = 0.f, oldc = 0.f;
  auto body = [&](int t, const LaneIn<n, m, GREC>& in) {
    const size_t tb = (size_t)t * B + b;
    oldc += in.g[m * n + m];
    float nu[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      // K dx with dx_t = x_t(new) - x_t(current), dx_0 = 0 (the group's dA
      // starts at 0: K * 0 keeps its sign); rows n.. of the group hold 0 * 0
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float dx = t > 0 ? xs[r < n ? r : 0] - in.x[r < n ? r : 0] : 0.f;
        v[r] = r < n ? in.g[a * n + r] * dx : 0.f;
      }
      const float s = tree16(v);
      nu[a] = (s + in.u[a]) + al * in.g[m * n + a];
      if constexpr (BM != DILQR_BOUNDS_NONE)
        nu[a] = eclamp(nu[a], bound_lo(bd, tb * m + a), bound_hi(bd, tb * m + a));
    }
    if (wr) st(uo + tb * m, nu);
    if (du_sq) {
#pragma unroll
      for (int a = 0; a < m; ++a) {
        const float e = in.u[a] - nu[a];
        du_sq[((size_t)t * m + a) * B + b] = e * e;
      }
    }
    float tau[d];
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xs[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = nu[a];
    sc += lane_stage_cost<d, DCONST>(tau, cd, cc, C, c, tb);
    if (t < T - 1) {
      float xn[n];
      md.forward(xs, nu, xn);
#pragma unroll
      for (int i = 0; i < n; ++i) xs[i] = xn[i];
      if (wr) st(xo + (tb + B) * n, xs);
    }
  };
  // a ring of PFD + 1 input buffers: step t+PFD's loads in flight while step
  // t computes (the loop unrolled PFD + 1 times, so the buffers rotate by
  // name, no copies).  Measured at config 3 (tools/ab_rocket.py, one box):
  // PFD 1 0.339-0.351 ms per MPC iteration, 2 0.356-0.368, 3 0.358-0.364 —
  // a search round streams ~360 MB (gain records, the current trajectory, two
  // candidates out) at ~5 TB/s, so deeper prefetch only adds registers.
  constexpr int P = PFD + 1;
  LaneIn<n, m, GREC> ring[P];
#pragma unroll
  for (int i = 0; i < P - 1; ++i)
    if (i < T) ring[i].load(ws, x, u, i, B, b);
  for (int t = 0; t < T; t += P) {
#pragma unroll
    for (int j = 0; j < P; ++j) {
      if (t + j < T) {
        if (t + j + P - 1 < T) ring[(j + P - 1) % P].load(ws, x, u, t + j + P - 1, B, b);
        body(t + j, ring[j]);
      }
    }
  }
  cost = sc;
  old_cost = oldc;
}

// The MPC iteration's line search, one problem per LANE PAIR: lane 2b+0 rolls
// candidate A (alpha) of problem b, lane 2b+1 candidate B (alpha * decay) —
// passes 2p and 2p+1 of the search, as in group_ilqr_problem — into slots sa /
// sb; the pair swaps costs and both take the same decision; then lane A does
// the best-iterate bookkeeping of k_mpc_iterate.  (Both candidates as f2 in
// one lane measured slower: 512 waves for 1024 SIMDs at config 3, 54 % of
// wave time waiting on loads.)  Runs after the group sweep of the same
// iteration (k_mpc_sweep_group), which published the stop rule's decision
// (ctrl[iteration & 1]) and, at iteration 0, the cost flags.
template <class Model, int BM, bool DCONST>
__global__ void __launch_bounds__(64) k_mpc_search_lane(int T, int B, const float* __restrict__ theta,
                                                        const float* __restrict__ x_init,
                                                        const float* __restrict__ C, const float* __restrict__ c,
                                                        Bounds bd, float decay, int max_ls, int iteration,
                                                        float best_cost_eps, int G, MpcState S) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  if (iteration > 0 && G >= 0 && S.ctrl[iteration & 1].stopped) return;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = tid >> 1, cand = tid & 1;
  if (b >= B) return;                                          // both lanes of a pair
  Model md; md.load(theta);
  const bool first = iteration == 0;
  const size_t TBn = (size_t)T * B * n, TBm = (size_t)T * B * m;
  const int cur = S.slot[b], best = S.slot[B + b];
  int sa, sb;
  free_slots(cur, best, sa, sb);
  const int so = cand ? sb : sa;
  const float* x = S.Xs + cur * TBn;
  const float* u = S.Us + cur * TBm;
  float* xo = S.Xs + so * TBn;
  float* uo = S.Us + so * TBm;
  const bool dconst = S.Cpk && S.cost_sym[b] == 7;
  float cd[d], cc[d];
#pragma unroll
  for (int r = 0; r < d; ++r) { cd[r] = 0.f; cc[r] = 0.f; }
  if (dconst) {
    ld(cd, S.Cpk + (size_t)b * 2 * d);
    ld(cc, S.Cpk + (size_t)b * 2 * d + d);
  }
  // the register cost when every problem of the wave has one (wave-uniform);
  // the two kinds of wave run in two instantiations (launched back to back,
  // each leaves the other's waves at once), so that the dense-cost rollout's
  // registers do not weigh on the common one
  if (__all(dconst) != DCONST) return;
  float alpha = 1.f, cost = 0.f, old_cost = 0.f;
  int win = 0;
  for (int p = 0; p < max_ls; p += 2) {
    const bool twoB = p + 1 < max_ls;
    const float aA = alpha, aB = alpha * decay;
    const float al = cand ? aB : aA;
    const bool wr = !cand || twoB;                             // B rolls out only if pass p+1 exists
    float cm, oc;
    float* dq = (p == 0 && !cand) ? S.du_sq : nullptr;
    lane_pass<Model, BM, DCONST>(T, B, b, md, x_init, cd, cc, C, c, S.ws, x, u, bd, al, wr, xo, uo, dq, cm, oc);
    const float co = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(cm), 0xB1, 0xF, 0xF, false));
    const float cA = cand ? co : cm, cB = cand ? cm : co;
    if (p == 0) old_cost = oc;
    if (!(cA > old_cost) || p == max_ls - 1) { cost = cA; alpha = aA; win = 0; break; }
    if (!(cB > old_cost) || p + 1 == max_ls - 1) { cost = cB; alpha = aB; win = 1; break; }
    alpha = aB * decay;                                       // lqr_step_explicit.py:249
  }
  if (cand) return;
  const int nw = win ? sb : sa;
  S.cost[b] = cost;
  S.alpha[b] = alpha;
  const bool better = !first && (cost <= S.best_cost[b] + best_cost_eps);   // mpc_explicit.py:278
  if (first || better) {
    S.best_cost[b] = cost;
    S.slot[B + b] = (unsigned char)nw;
  }
  S.improved[b] = (first || better) ? (better ? 2 : 1) : 0;
  if (S.best_iter && (first || better)) S.best_iter[b] = iteration;       // fixed-count solves
  S.slot[b] = (unsigned char)nw;
}

// The same line search on a QUAD of lanes per problem (16 problems per wave):
// lane j of the quad rolls pass p = 4r + j of round r out for its COST only, so
// one round decides up to four passes and the gain records and the current
// trajectory are read once per round for all of them (the quad's lanes read
// the same addresses).  Pass 0 (lane 0) also writes its trajectory to slot sa,
// speculatively: it is the winner in most early iterations.  The last pass
// (p = max_ls - 1) is accepted whatever its cost (lqr_step_explicit.py:252), so
// it is never rolled out to be compared.  When the winner is not pass 0, lane 0
// of the quad rolls the winner's step size out again with writes (phase 2; the
// same function on the same inputs: the same bits).  So the search returns the
// sequential search's pass, cost, step size and trajectory bit for bit, like
// k_mpc_search_lane, with one round (and at most one rewrite) where the pairs
// took up to three rounds (max_ls = 5), two waves per SIMD at config 3 where
// the pairs had one, and no second candidate stream to HBM.
// the quad search's prefetch distance (0: its two waves per SIMD hide the loads)
// and its launch-bounds floor
#ifndef DILQR_QUAD_PFD
#define DILQR_QUAD_PFD 0
#endif
#ifndef DILQR_QUAD_WAVES
#define DILQR_QUAD_WAVES 2
#endif
template <class Model, int BM, bool DCONST>
DEV void search_quad_problem(int T, int B, int tid, const Model& md, const float* __restrict__ x_init,
                             const float* __restrict__ C, const float* __restrict__ c, const Bounds& bd, float decay,
                             int max_ls, int iteration, float best_cost_eps, const MpcState& S) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  const int b = tid >> 2, j = tid & 3;
  if (b >= B) return;                                          // a whole quad
  const bool first = iteration == 0;
  const size_t TBn = (size_t)T * B * n, TBm = (size_t)T * B * m;
  const int cur = S.slot[b], best = S.slot[B + b];
  int sa, sb;
  free_slots(cur, best, sa, sb);
  const float* x = S.Xs + cur * TBn;
  const float* u = S.Us + cur * TBm;
  float* xo = S.Xs + sa * TBn;
  float* uo = S.Us + sa * TBm;
  const bool dconst = S.Cpk && S.cost_sym[b] == 7;
  float cd[d], cc[d];
#pragma unroll
  for (int r = 0; r < d; ++r) { cd[r] = 0.f; cc[r] = 0.f; }
  if (dconst) {
    ld(cd, S.Cpk + (size_t)b * 2 * d);
    ld(cc, S.Cpk + (size_t)b * 2 * d + d);
  }
  if (__all(dconst) != DCONST) return;                         // wave-uniform, as k_mpc_search_lane
  const int q0 = (threadIdx.x & 63) & ~3;                      // the quad's first lane
  const int last = max_ls - 1;
  // alpha_p = decay^p by the sequential search's chain of products (249)
  float al = 1.f;
  for (int i = 0; i < j; ++i) al *= decay;
  float old_cost = 0.f, cost = 0.f;
  int win = -1;                                                // the accepted pass (quad-uniform)
  for (int p0 = 0;; p0 += 4) {
    const int p = p0 + j;
    // lane 0 of round 0 always rolls pass 0 out (with writes, and the du rows
    // of the reference's full_du_norm); other passes only to be compared
    const bool roll = (p == 0) || (p < last);
    float cm = 0.f, oc = 0.f;
    if (roll)
      lane_pass<Model, BM, DCONST, DILQR_QUAD_PFD>(T, B, b, md, x_init, cd, cc, C, c, S.ws, x, u, bd, al, p == 0,
                                                   xo, uo, p == 0 ? S.du_sq : nullptr, cm, oc);
    if (p0 == 0) old_cost = __shfl(oc, q0, 64);                // every pass sums the same old cost; lane 0's
    // the first pass of this round that is accepted: cost <= old, or the last
    const bool acc = p <= last && ((roll && !(cm > old_cost)) || p == last);
    const unsigned long long bal = __ballot(acc);
    const unsigned qb = (unsigned)(bal >> q0) & 15u;
    if (qb) {
      const int k = __builtin_ctz(qb);
      win = p0 + k;
      cost = __shfl(cm, q0 + k, 64);                           // a rolled pass's cost (the last: phase 2)
      break;
    }
    for (int i = 0; i < 4; ++i) al *= decay;                   // this lane's pass of the next round
  }
  // alpha of the accepted pass, the same chain
  float aw = 1.f;
  for (int i = 0; i < win; ++i) aw *= decay;
  if (j != 0) return;
  if (win != 0) {                                              // phase 2: the winner's trajectory
    float oc;
    lane_pass<Model, BM, DCONST, DILQR_QUAD_PFD>(T, B, b, md, x_init, cd, cc, C, c, S.ws, x, u, bd, aw, true, xo,
                                                 uo, nullptr, cost, oc);
  }
  S.cost[b] = cost;
  S.alpha[b] = aw;
  const bool better = !first && (cost <= S.best_cost[b] + best_cost_eps);   // mpc_explicit.py:278
  if (first || better) {
    S.best_cost[b] = cost;
    S.slot[B + b] = (unsigned char)sa;
  }
  S.improved[b] = (first || better) ? (better ? 2 : 1) : 0;
  if (S.best_iter && (first || better)) S.best_iter[b] = iteration;       // fixed-count solves
  S.slot[b] = (unsigned char)sa;
}

template <class Model, int BM, bool DCONST>
__global__ void __launch_bounds__(64, DCONST ? DILQR_QUAD_WAVES : 1) k_mpc_search_quad(int T, int B, const float* __restrict__ theta,
                                                        const float* __restrict__ x_init,
                                                        const float* __restrict__ C, const float* __restrict__ c,
                                                        Bounds bd, float decay, int max_ls, int iteration,
                                                        float best_cost_eps, int G, MpcState S) {
  if (iteration > 0 && G >= 0 && S.ctrl[iteration & 1].stopped) return;
  // the dense-cost instantiation when iteration 0 found no dense cost (launched
  // on a small grid then): nothing to do
  if (!DCONST && S.Cpk && S.done_counter[kDenseCount] == 0u) return;
  Model md; md.load(theta);
  const int nq = (int)(((long long)4 * B + blockDim.x - 1) / blockDim.x);
  for (int blk = blockIdx.x; blk < nq; blk += gridDim.x)    // one pass unless the grid is small
    search_quad_problem<Model, BM, DCONST>(T, B, blk * blockDim.x + threadIdx.x, md, x_init, C, c, bd, decay,
                                           max_ls, iteration, best_cost_eps, S);

}

}  // namespace dilqr
