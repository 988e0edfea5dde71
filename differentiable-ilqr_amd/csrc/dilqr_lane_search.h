// dilqr_lane_search.h — the line search of the 16-lanes-per-problem models
// (rocket, d = 16) run ONE problem per lane.
//
// The group kernels need 16 lanes per problem for the Riccati sweep (a step's
// V, Q, F do not fit one lane's registers), but the rollout only carries a
// 13-vector: distributed over a group, its row-wise dynamics is a switch that
// every lane of the wave executes case by case, the state goes through LDS at
// every step, and the 4 problems of a wave pay 16 lanes of instructions each.
// Here lane b rolls problem b's two candidates out (f2, Rocket::forward) from
// the gain records the group sweep left in HBM, so a wave does 64 problems'
// rollouts for the instructions the group kernel spent on 4.
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

// Stage cost of both candidates, tau = [x; u] (f2), the rows summed as
// group_forward_pair does.  dconst: the time-invariant diagonal cost held in
// registers (cd, cc) — row r's product chain there is fma(C[r][j], tau_j, .)
// over j with C[r][j] = +0 off the diagonal, which equals
// fma(cd_r, tau_r, probe) with probe = that chain's +0 (NaN if any tau_j is
// not finite: 0 * inf); otherwise the caller's C_t, c_t rows from HBM.
template <int d, bool DCONST>
DEV f2 lane_stage_cost(const f2 (&tau)[d], const float (&cd)[d], const float (&cc)[d],
                       const float* __restrict__ C, const float* __restrict__ c, size_t tb) {
  static_assert(d == 16, "the group sum covers 16 rows");
  f2 pr[d];
  if constexpr (DCONST) {
    f2 probe = f2{0.f, 0.f};
#pragma unroll
    for (int j = 0; j < d; ++j) probe = vfma(f2(0.f), tau[j], probe);
#pragma unroll
    for (int r = 0; r < d; ++r) {
      const f2 s = vfma(f2(cd[r]), tau[r], probe);
      pr[r] = 0.5f * (tau[r] * s) + tau[r] * cc[r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < d; ++r) {             // a dense cost: one row in registers at a time
      float Crow[d];
      ld(Crow, C + (tb * d + r) * d);
      f2 s = f2{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < d; ++j) s += Crow[j] * tau[j];
      pr[r] = 0.5f * (tau[r] * s) + tau[r] * c[tb * d + r];
    }
  }
  return tree16(pr);
}

// One pass pair of the search (candidates A = alpha, B = alpha * decay, if
// twoB), its stage costs summed into cA / cB and the current trajectory's
// (from the gain records) into old_cost.  DCONST: the whole wave's problems
// hold a time-invariant diagonal cost in registers (cd, cc), else every lane
// reads the caller's rows (a flagged problem's rows hold the same values).
template <class Model, int BM, bool DCONST>
DEV void lane_pass(int T, int B, int b, const Model& md, const float* __restrict__ x_init,
                   const float (&cd)[Model::N + Model::M], const float (&cc)[Model::N + Model::M],
                   const float* __restrict__ C, const float* __restrict__ c, const float* __restrict__ ws,
                   const float* __restrict__ x, const float* __restrict__ u, const Bounds& bd, float aA, float aB,
                   bool twoB, float* __restrict__ xa_out, float* __restrict__ ua_out, float* __restrict__ xb_out,
                   float* __restrict__ ub_out, float* __restrict__ du_sq, float& cA, float& cB, float& old_cost) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  constexpr int GREC = group_grec<Model>();
  const f2 al = f2{aA, aB};
  f2 xs[n];
  {
    float x0[n];
    ld(x0, x_init + (size_t)b * n);
    st(xa_out + (size_t)b * n, x0);
    if (twoB) st(xb_out + (size_t)b * n, x0);
#pragma unroll
    for (int i = 0; i < n; ++i) xs[i] = f2{x0[i], x0[i]};
  }
  f2 sc = f2{0.f, 0.f};
  float oldc = 0.f;
  LaneIn<n, m, GREC> in, nx;
  in.load(ws, x, u, 0, B, b);
  for (int t = 0; t < T; ++t) {
    const size_t tb = (size_t)t * B + b;
    nx.load(ws, x, u, t + 1 < T ? t + 1 : t, B, b);                  // step t+1's inputs in flight
    oldc += in.g[m * n + m];
    f2 nu[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      // K dx with dx_t = x_t(new) - x_t(current), dx_0 = 0 (the group's dA
      // starts at 0: K * 0 keeps its sign); rows n.. of the group hold 0 * 0
      f2 v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const f2 dx = t > 0 ? xs[r < n ? r : 0] - in.x[r < n ? r : 0] : f2{0.f, 0.f};
        v[r] = r < n ? in.g[a * n + r] * dx : f2{0.f, 0.f};
      }
      const f2 s = tree16(v);
      nu[a] = (s + in.u[a]) + al * in.g[m * n + a];
      if constexpr (BM != DILQR_BOUNDS_NONE) {
        const float lo = bound_lo(bd, tb * m + a), hi = bound_hi(bd, tb * m + a);
        nu[a] = f2{eclamp(nu[a].x, lo, hi), eclamp(nu[a].y, lo, hi)};
      }
    }
    {
      float ua[m], ub[m];
#pragma unroll
      for (int a = 0; a < m; ++a) { ua[a] = nu[a].x; ub[a] = nu[a].y; }
      st(ua_out + tb * m, ua);
      if (twoB) st(ub_out + tb * m, ub);
      if (du_sq) {
#pragma unroll
        for (int a = 0; a < m; ++a) {
          const float e = in.u[a] - ua[a];
          du_sq[((size_t)t * m + a) * B + b] = e * e;
        }
      }
    }
    f2 tau[d];
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xs[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = nu[a];
    sc += lane_stage_cost<d, DCONST>(tau, cd, cc, C, c, tb);
    if (t < T - 1) {
      f2 xn[n];
      md.forward(xs, nu, xn);
      float xa[n], xb[n];
#pragma unroll
      for (int i = 0; i < n; ++i) {
        xs[i] = xn[i];
        xa[i] = xn[i].x;
        xb[i] = xn[i].y;
      }
      st(xa_out + (tb + B) * n, xa);
      if (twoB) st(xb_out + (tb + B) * n, xb);
    }
    in = nx;
  }
  cA = sc.x;
  cB = sc.y;
  old_cost = oldc;
}

// The MPC iteration's line search for problem b (lane b): paired passes 2p and
// 2p+1 as in group_ilqr_problem, candidates into slots sa / sb, then the
// best-iterate bookkeeping of k_mpc_iterate.  Runs after the group sweep
// of the same iteration (k_mpc_sweep_group), which published the stop rule's
// decision (ctrl[iteration & 1]) and, at iteration 0, the cost flags.
template <class Model, int BM>
__global__ void __launch_bounds__(64) k_mpc_search_lane(int T, int B, const float* __restrict__ theta,
                                                        const float* __restrict__ x_init,
                                                        const float* __restrict__ C, const float* __restrict__ c,
                                                        Bounds bd, float decay, int max_ls, int iteration,
                                                        float best_cost_eps, int G, MpcState S) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  constexpr int GREC = group_grec<Model>();
  if (iteration > 0 && G >= 0 && S.ctrl[iteration & 1].stopped) return;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Model md; md.load(theta);
  const bool first = iteration == 0;
  const size_t TBn = (size_t)T * B * n, TBm = (size_t)T * B * m;
  const int cur = S.slot[b], best = S.slot[B + b];
  int sa, sb;
  free_slots(cur, best, sa, sb);
  const float* x = S.Xs + cur * TBn;
  const float* u = S.Us + cur * TBm;
  float* xa_out = S.Xs + sa * TBn;
  float* ua_out = S.Us + sa * TBm;
  float* xb_out = S.Xs + sb * TBn;
  float* ub_out = S.Us + sb * TBm;
  const bool dconst = S.Cpk && S.cost_sym[b] == 7;
  float cd[d], cc[d];
#pragma unroll
  for (int r = 0; r < d; ++r) { cd[r] = 0.f; cc[r] = 0.f; }
  if (dconst) {
    ld(cd, S.Cpk + (size_t)b * 2 * d);
    ld(cc, S.Cpk + (size_t)b * 2 * d + d);
  }
  // the register cost when every problem of the wave has one (wave-uniform)
  const bool wave_dconst = __all(dconst);
  float alpha = 1.f, cost = 0.f, old_cost = 0.f;
  int win = 0;
  for (int p = 0; p < max_ls; p += 2) {
    const bool twoB = p + 1 < max_ls;
    const float aA = alpha, aB = alpha * decay;
    float cA, cB, oc;
    float* dq = p == 0 ? S.du_sq : nullptr;
    if (wave_dconst)
      lane_pass<Model, BM, true>(T, B, b, md, x_init, cd, cc, C, c, S.ws, x, u, bd, aA, aB, twoB, xa_out, ua_out,
                                 xb_out, ub_out, dq, cA, cB, oc);
    else
      lane_pass<Model, BM, false>(T, B, b, md, x_init, cd, cc, C, c, S.ws, x, u, bd, aA, aB, twoB, xa_out, ua_out,
                                  xb_out, ub_out, dq, cA, cB, oc);
    if (p == 0) old_cost = oc;
    if (!(cA > old_cost) || p == max_ls - 1) { cost = cA; alpha = aA; win = 0; break; }
    if (!(cB > old_cost) || p + 1 == max_ls - 1) { cost = cB; alpha = aB; win = 1; break; }
    alpha = aB * decay;                                       // lqr_step_explicit.py:249
  }
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

}  // namespace dilqr
