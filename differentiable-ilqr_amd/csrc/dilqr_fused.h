// dilqr_fused.h — the fused iLQR iteration (linearise + Riccati sweep + line
// search in one pass per problem) and the device-resident MPC loop kernel for
// the one-problem-per-lane models (pendulum, cartpole), plus their launchers.
// Instantiated per model in tu_mpc_<model>.hip.  See DESIGN.md §2, §3, §5.
#pragma once
#include "dilqr_common.h"
#include "dilqr_launch.h"

namespace dilqr {

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

// (bitwise tests as xor/or reductions with one compare each, not a compare
// and a mask update per entry)
template <int d>
DEV void pack_cost(const float (&C)[d][d], const float (&c)[d], float (&buf)[packed_cost_floats<d>()], bool& sym,
                   bool& diag) {
  int k = 0;
#pragma unroll
  for (int i = 0; i < d; ++i) buf[k++] = C[i][i];
#pragma unroll
  for (int i = 0; i < d; ++i) buf[k++] = c[i];
  unsigned asym = 0u, offd = 0u;
#pragma unroll
  for (int i = 0; i < d; ++i)
#pragma unroll
    for (int j = i + 1; j < d; ++j) {
      asym |= __float_as_uint(C[i][j]) ^ __float_as_uint(C[j][i]);
      offd |= __float_as_uint(C[i][j]) | __float_as_uint(C[j][i]);
      buf[k++] = C[i][j];
    }
  sym &= asym == 0u;
  diag &= offd == 0u;
}

// every word of a and b equal, bit for bit
template <int K>
DEV bool same_bits(const float (&a)[K], const float (&b)[K]) {
  unsigned dif = 0u;
#pragma unroll
  for (int k = 0; k < K; ++k) dif |= __float_as_uint(a[k]) ^ __float_as_uint(b[k]);
  return dif == 0u;
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

// Prefetch distance of the fused sweep, in steps.  At B = 65536 the
// one-problem-per-lane kernels run ONE wave per SIMD, so the only latency
// cover is the loads already in flight.  Round 2 measured two steps ahead no
// faster than one (0.0702 vs 0.0695 ms per iteration, config 2) — on a GPU
// short of its clocks (bench's 5 warmup solves); warm, round 6: the headline
// 1.873-1.877e9 -> 1.917-1.923e9, the steady iteration 34.0 -> 33.5 us
// (profiles/r06/ab_sweep_prefetch2.txt), so 2.
#ifndef DILQR_PF
#define DILQR_PF 2
#endif
constexpr int kPF = DILQR_PF;
// The line search's: 2 was faster with SLP vectorisation on (round 2); in
// the no-SLP build 1 is (headline A/B, 4 rounds on one box: 1.742e9 ->
// 1.772e9 problem-iterations/s — one buffer copy per step instead of two);
// re-measured warm in round 6 (with the sweep at 2): 1.920e9 at 1 against
// 1.853e9 at 2 (profiles/r06/ab_ls_prefetch2.txt).
#ifndef DILQR_PF_LS
#define DILQR_PF_LS 1
#endif
constexpr int kPFL = DILQR_PF_LS;                   // the line search's prefetch distance
static_assert(kPFL == 1 || kPFL == 2, "the line search prefetches one or two steps ahead");

#ifndef DILQR_PHASE_SKIP
#define DILQR_PHASE_SKIP 0
#endif

// ---------------- forward: the line search (lqr_step_explicit.py:166-263).
// Pass p uses alpha_p = decay^p and is accepted when its cost <= old cost or
// it is the last pass.  Passes 2r and 2r+1 roll out TOGETHER (candidates A
// and B), sharing every load of the step; the first accepted candidate wins,
// which is exactly the sequential search.  A wave otherwise pays a whole
// second latency-bound pass whenever any of its 64 problems backtracks.
// PAIR: the common MPC case as its own instantiation — exactly one round of two
// candidates (max_ls == 2) with B's records in the gain slots — so the step
// loop carries no test of the round, of "is there a B", of "where does B go".
template <class Model, int BM, int TL, class CostT, bool PAIR = false>
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
  if constexpr (PAIR) {
    max_ls = 2;
    b_in_gains = true;
  }
  float alpha = 1.f, cost = 0.f;
  int win = 0;
  // Candidates A and B travel as the two components of f2 values: every
  // arithmetic step of the pair is one packed instruction (v_pk_fma_f32 /
  // v_pk_mul_f32 / v_pk_add_f32), and each component rounds exactly like the
  // scalar rollout of that candidate.  (Measured alternatives that were
  // slower on MI355X: unrolling the step loop twice over two prefetch buffers
  // and making every store unconditional, +3 us per iteration; unrolling it
  // three times with the three prefetch buffers rotating roles instead of
  // being copied — 13 fewer v_mov per step in the listing — +4 us.  Round 5,
  // after peeling step T-1 (1.759e9 -> 1.790e9 problem-iterations/s on one
  // box): the loop unrolled twice over two buffers swapping roles, 172 -> 158
  // VALU per step, no faster (1.781e9 vs 1.786e9); each candidate record
  // stored dword by dword from the packed pairs' halves, 12 fewer v_mov per
  // step, 9 % slower (1.60e9) — six narrow stores per record cost more than
  // the moves they save.)
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
    if constexpr (kPFL >= 2) {
      if (T > 1) n1.load(ws, u, cs, x, bd, T, 1, cl(2), B, b);
    }
    // step T-1 is peeled off the loop (LAST: no prefetch, no dynamics step), so
    // the loop body updates the candidate states unconditionally — no branch
    // whose join needs the old states copied into the new ones' registers
    // c: this step's inputs, nx: the next step's, loaded here (prefetch 1)
    auto step = [&](int t, auto last_c, auto& c, auto& nx) {
      constexpr bool LAST = decltype(last_c)::value;
      if constexpr (!LAST) {
        if constexpr (kPFL >= 2) {
          if (t + 2 < T) n2.load(ws, u, cs, x, bd, T, t + 2, cl(t + 3), B, b);    // prefetch step t+2
        } else {
          nx.load(ws, u, cs, x, bd, T, t + 1, cl(t + 2), B, b);                   // prefetch step t+1
        }
      }
      f2 nu[m];
#pragma unroll
      for (int a = 0; a < m; ++a) {
        f2 sp = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < n; ++j) sp += c.g[a * n + j] * dp[j];
        nu[a] = (sp + c.u[a]) + al * c.g[m * n + a];
        if constexpr (BM != DILQR_BOUNDS_NONE) {
          const float lo = c.bnd.l(bd, a), hi = c.bnd.h(bd, a);
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
          float e = c.u[a] - nu[a].x;
          du_sq[((size_t)t * m + a) * B + b] = e * e;
        }
      }
      f2 tau[d];
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = xp[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = nu[a];
      cp += quad_cost<d, CostT::kDiag>(c.C, c.c, tau);
      if constexpr (!LAST) {
        f2 xnext[n];
        md.forward(xp, nu, xnext);
        float xa[n], xb[n];
#pragma unroll
        for (int i = 0; i < n; ++i) {
          dp[i] = xnext[i] - c.xnext[i];
          xp[i] = xnext[i];
          xa[i] = xnext[i].x;
          xb[i] = xnext[i].y;
        }
        if constexpr (TL == TRAJ_AOS) {
          st(xa_out + ((size_t)(t + 1) * B + b) * n, xa);
          if (twoB) st(xb_out + ((size_t)(t + 1) * B + b) * n, xb);
        }
      }
      if constexpr (!LAST) {
        if constexpr (TL == TRAJ_REC) {
#pragma unroll
          for (int a = 0; a < m; ++a) nx.u[a] = c.unext[a];     // u_{t+1}
        }
      }
    };
    for (int t = 0; t < T - 1; ++t) {
      step(t, std::false_type{}, cur, n1);
      cur = n1;
      if constexpr (kPFL >= 2) n1 = n2;
    }
    step(T - 1, std::true_type{}, cur, n1);
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
// PREV: the current trajectory's cost is prev_cost, the cost the previous
// MPC iteration's line search computed for it (the accepted candidate), so the
// sweep forms only C tau for c_back and not the stage costs again.
template <class Model, int BM, int TL, bool ROLLOUT, class CostT, bool PREV = false>
DEV int ilqr_problem(int T, int B, int b, const Model md, const float* __restrict__ x_init, const CostT& cs,
                     float* __restrict__ pack_out, unsigned char* __restrict__ sym_out, const float* __restrict__ x,
                     const float* __restrict__ u, const Bounds& bd, float decay, int max_ls,
                     const GainRecs& ws, float* __restrict__ xa_out, float* __restrict__ ua_out,
                     float* __restrict__ xb_out, float* __restrict__ ub_out, float* __restrict__ du_sq,
                     float& cost_out, float& alpha_out, bool b_in_gains = false,
                     float prev_cost = 0.f, unsigned* flags_out = nullptr) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  constexpr int MODE = BM == DILQR_BOUNDS_NONE ? GAIN_UNC : GAIN_BOX;
  constexpr int GREC = m * n + m;                    // gain record: K, k (component-major)
  constexpr int PK = packed_cost_floats<d>();
  float old_cost = 0.f;                               // the current trajectory's cost, from the sweep
  if constexpr (PREV) old_cost = prev_cost;           // ... or from the previous line search
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
          const bool same = same_bits(buf, pk_last);
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
// unrolled twice (headline A/B in the no-SLP build, 4 rounds: 1 1.725e9,
// 2 1.755e9, 3 1.754e9 problem-iterations/s)
#ifndef DILQR_SWEEP_UNROLL
#define DILQR_SWEEP_UNROLL 2
#endif
#pragma unroll DILQR_SWEEP_UNROLL
    for (int t = T - 2; t >= 0; --t) sweep_step(t, std::false_type{});
    if (sym_out) {
      const unsigned char f = sym ? (unsigned char)(kCostSym | (diag && packed_diag_ok<d>() ? kCostDiag : 0) |
                                                    (tinv ? kCostTinv : 0))
                                  : 0;
      sym_out[b] = f;
      if (flags_out) *flags_out = f;                    // (a local of an inlined caller: a register)
    }
  }
  DILQR_STAMP(2);
#if DILQR_PHASE_SKIP & 1
  // timing-only builds (tools/small_phase_split.py; never the shipped library):
  // the iteration ends after the sweep, the trajectory kept, so every iteration
  // repeats the same sweep and the line search's share is the difference
  cost_out = old_cost;
  alpha_out = 1.f;
  return 0;
#endif
  if constexpr (!CostT::kDiag && packed_diag_ok<d>()) {
    if (pack_out && sym && diag && tinv) {              // iteration 0 of a diag(q), p over t cost
      CostDiagConst<d> cc;
      cc.set(pk_last);
      if (b_in_gains && max_ls == 2)
        return line_search<Model, BM, TL, CostDiagConst<d>, true>(T, B, b, md, x_init, cc, x, u, bd, decay, max_ls, ws,
                                                                  xa_out, ua_out, xb_out, ub_out, du_sq, old_cost,
                                                                  cost_out, alpha_out, b_in_gains);
      return line_search<Model, BM, TL>(T, B, b, md, x_init, cc, x, u, bd, decay, max_ls, ws, xa_out, ua_out,
                                         xb_out, ub_out, du_sq, old_cost, cost_out, alpha_out, b_in_gains);
    }
  }
  if (b_in_gains && max_ls == 2)
    return line_search<Model, BM, TL, CostT, true>(T, B, b, md, x_init, cs, x, u, bd, decay, max_ls, ws, xa_out,
                                                   ua_out, xb_out, ub_out, du_sq, old_cost, cost_out, alpha_out,
                                                   b_in_gains);
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

// One MPC iteration of problem b (this lane) on its trajectory slots: the
// fused linearise + sweep + line search into the two free slots.  The caller
// holds the problem's state — cur/best slot, its cost flags pk (steady
// iterations), the current trajectory's cost prev_cost (the previous line
// search's) — and does the best-iterate bookkeeping with the result.
// LG: the gain records live in this workgroup's LDS (dynamic, T*64*GREC floats;
// picked when 4 workgroups per CU still fit the 160 KB), instead of a workspace
// round trip through HBM/MALL every iteration.
// FIRST: iteration 0 of the solve (reads the caller's C, c and builds the
// packed copy; its cost flags come back in *flags_out).  Otherwise the cost is
// read as the flags pk say; PREV: the current trajectory's cost is prev_cost
// (iterations >= 1) — else the sweep sums it (iteration 0 of a whole-solve
// launch, whose begin already built the packed copy).
struct LaneIter {
  float cost, alpha;
  int slot;                                                 // the accepted candidate's slot
};

template <class Model, int BM, bool LG, bool FIRST, bool PREV = true, int GS = kBlock>
DEV LaneIter mpc_iteration_lane(int T, int B, int b, const Model md, const float* __restrict__ x_init,
                                const float* __restrict__ C, const float* __restrict__ c, const Bounds& bd,
                                float decay, int max_ls, const MpcState& S, float* __restrict__ du_sq,
                                float* __restrict__ lds_gains, int cur, int best, unsigned pk, float prev_cost,
                                unsigned* flags_out = nullptr) {
  constexpr int n = Model::N, m = Model::M;
  const size_t TBd = (size_t)T * B * (n + m);               // one slot: [T,B,d] records
  int sa, sb;
  free_slots(cur, best, sa, sb);
  const float* xcur = S.Xs + cur * TBd;
  float* xsa = S.Xs + sa * TBd;
  float* xsb = S.Xs + sb * TBd;
  float cost, alpha;
  int win;
  const GainRecs gr = LG ? GainRecs{lds_gains, GS, (int)threadIdx.x} : GainRecs{S.ws, B, b};
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
                                                  du_sq, cost, alpha, b_lds, 0.f, flags_out);
  } else {
    if ((pk & (kCostDiag | kCostTinv)) == (kCostDiag | kCostTinv)) {
      if constexpr (packed_diag_ok<n + m>()) {
        CostDiagConst<n + m> cc;
        cc.init(S.Cpk, T, B, b);
        win = ilqr_problem<Model, BM, TRAJ_REC, true, CostDiagConst<n + m>, PREV>(T, B, b, md, x_init, cc, nullptr, nullptr, xcur, nullptr, bd,
                                                      decay, max_ls, gr, xsa, nullptr, xsb, nullptr, du_sq, cost,
                                                      alpha, b_lds, prev_cost);
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
        win = ilqr_problem<Model, BM, TRAJ_REC, true, CostPacked<n + m, true>, PREV>(T, B, b, md, x_init, CostPacked<n + m, true>{S.Cpk, T}, nullptr,
                                                      nullptr, xcur, nullptr, bd, decay, max_ls, gr, xsa, nullptr, xsb,
                                                      nullptr, du_sq, cost, alpha, b_lds, prev_cost);
      else
        __builtin_unreachable();
    } else if ((pk & (kCostSym | kCostTinv)) == (kCostSym | kCostTinv))
      win = ilqr_problem<Model, BM, TRAJ_REC, true, CostPacked<n + m, false, true>, PREV>(T, B, b, md, x_init, CostPacked<n + m, false, true>{S.Cpk, T},
                                                    nullptr, nullptr, xcur, nullptr, bd, decay, max_ls, gr, xsa, nullptr,
                                                    xsb, nullptr, du_sq, cost, alpha, b_lds, prev_cost);
    else if (pk & kCostSym)
      win = ilqr_problem<Model, BM, TRAJ_REC, true, CostPacked<n + m>, PREV>(T, B, b, md, x_init, CostPacked<n + m>{S.Cpk, T}, nullptr, nullptr,
                                                    xcur, nullptr, bd, decay, max_ls, gr, xsa, nullptr, xsb, nullptr,
                                                    du_sq, cost, alpha, b_lds, prev_cost);
    else
      win = ilqr_problem<Model, BM, TRAJ_REC, true, CostFull<n + m>, PREV>(T, B, b, md, x_init, full, nullptr, nullptr, xcur, nullptr, bd,
                                                    decay, max_ls, gr, xsa, nullptr, xsb, nullptr, du_sq, cost,
                                                    alpha, b_lds, prev_cost);
#endif
  }
  return LaneIter{cost, alpha, win ? sb : sa};
}

// best-iterate test (mpc_explicit.py:277-283): iteration 0 always takes it
DEV bool mpc_takes_best(bool first, float cost, float best_cost, float best_cost_eps) {
  return first || cost <= best_cost + best_cost_eps;
}

// One launch per MPC iteration (the stop-rule path; fixed-count solves of the
// single-lane models run k_mpc_solve_fixed instead).  FIRST: iteration 0 — its
// own instantiation, so the steady-state kernel carries no copy-building code
// and profiles separately.
template <class Model, int BM, bool LG, bool FIRST>
__global__ void __launch_bounds__(kBlock) k_mpc_iterate(int T, int B, const float* __restrict__ theta,
                                                        const float* __restrict__ x_init, const float* __restrict__ C,
                                                        const float* __restrict__ c, Bounds bd, float decay, int max_ls,
                                                        int iteration, float best_cost_eps, float eps,
                                                        int not_improved_lim, int G, MpcState S) {
  constexpr bool first = FIRST;                             // == (iteration == 0), chosen by the host
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  // the problem's slot indices, cost flags and costs are read together with the
  // stop rule's inputs (one memory latency in the prologue, not several)
  const int bl = b < B ? b : B - 1;
  const int cur = S.slot[bl], best = S.slot[B + bl];
  const unsigned char pk = (!FIRST && S.Cpk) ? S.cost_sym[bl] : 0;
  const float prev = FIRST ? 0.f : S.cost[bl];
  const float best_cost = FIRST ? 0.f : S.best_cost[bl];
  DILQR_STAMP(0);
  DILQR_STAMP(6);
  if (mpc_decide(S, B, iteration, G, eps, not_improved_lim)) return;
  if (b >= B) return;
  DILQR_STAMP(1);
  Model md; md.load(theta);
  extern __shared__ __attribute__((aligned(16))) float lds_gains[];
  const LaneIter r = mpc_iteration_lane<Model, BM, LG, FIRST>(T, B, b, md, x_init, C, c, bd, decay, max_ls, S,
                                                              S.du_sq, lds_gains, cur, best, pk, prev);
  DILQR_STAMP(3);
  S.cost[b] = r.cost;
  S.alpha[b] = r.alpha;
  const bool take = mpc_takes_best(first, r.cost, best_cost, best_cost_eps);
  if (take) {
    S.best_cost[b] = r.cost;
    S.slot[B + b] = (unsigned char)r.slot;
  }
  S.improved[b] = take ? (first ? 1 : 2) : 0;
  if (S.best_iter && take) S.best_iter[b] = iteration;      // fixed-count solves
  S.slot[b] = (unsigned char)r.slot;
  DILQR_STAMP(4);
  DILQR_STAMP(7);
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

// get_traj(u_init) of problem b into slot 0 (util.py:104-127; u_init: the
// caller's [T,B,m] controls, or null for zeros, the MPC default) and its slot
// indices reset; the states and controls are written in one pass.
// the begin pass's cost prefetch distance in steps: 2, 3 and 4 measured no
// faster than 1 (solve 0.386-0.391 ms for each, A/B on one box; the pass
// streams C at ~5 TB/s, its loads and its slot-record stores interleaved)
#ifndef DILQR_BEGIN_PF
#define DILQR_BEGIN_PF 1
#endif
// ANALYSE (the whole-solve launch with a packed cost copy): the same pass also
// streams the caller's C_t, c_t (one step ahead in registers), builds the
// solve's packed copy and returns the problem's cost flags, exactly as
// iteration 0's sweep does otherwise (ilqr_problem pack_out: same records,
// the same single t = T-1 record for a time-invariant cost, same flags) — so
// the C stream overlaps the light rollout instead of the Riccati sweep, and
// iteration 0 runs on the packed copy like every later iteration.
template <class Model, bool ANALYSE = false>
DEV unsigned mpc_begin_lane(int T, int B, int b, const Model& md, const float* __restrict__ x_init,
                            const float* __restrict__ u_init, const MpcState& S,
                            const float* __restrict__ C = nullptr, const float* __restrict__ c = nullptr) {
  constexpr int n = Model::N, m = Model::M, d = n + m;
  constexpr int PK = packed_cost_floats<d>();
  S.slot[b] = 0; S.slot[B + b] = 0;
  constexpr int TL = slot_layout<Model>();
  const CostFull<d> full{C, c};
  // the inputs of steps t+1 .. t+PFB (cost and control) are in flight while
  // step t runs; the loop is unrolled by PFB so the buffers rotate by name, not
  // by copies.  The control is loaded with the cost, not after it: vmcnt counts
  // in issue order, so a control load issued behind the cost prefetch would
  // make its wait drain the prefetch too.
  constexpr int PFB = ANALYSE ? DILQR_BEGIN_PF : 1;
  float Cq[PFB][d][d], cq[PFB][d], uq[PFB][m];
  auto load_step = [&](int s, int t) {
    if (u_init) {
      ld(uq[s], u_init + ((size_t)t * B + b) * m);
    } else {
#pragma unroll
      for (int a = 0; a < m; ++a) uq[s][a] = 0.f;
    }
    if constexpr (ANALYSE) full.load(Cq[s], cq[s], t, B, b);
  };
#pragma unroll
  for (int s = 0; s < PFB; ++s) load_step(s, s < T ? s : T - 1);
  bool sym = true, diag = true, tinv = true;
  float pk_first[PK];                                       // step 0's packed record (tinv test)
  float xt[n];
  ld(xt, x_init + (size_t)b * n);
  for (int t0 = 0; t0 < T; t0 += PFB) {
#pragma unroll
    for (int s = 0; s < PFB; ++s) {
      const int t = t0 + s;
      if (t >= T) break;
      float ut[m], xn[n];
      float Cc[d][d], cc[d];
#pragma unroll
      for (int a = 0; a < m; ++a) ut[a] = uq[s][a];
      if constexpr (ANALYSE) {
#pragma unroll
        for (int i = 0; i < d; ++i) {
          cc[i] = cq[s][i];
#pragma unroll
          for (int j = 0; j < d; ++j) Cc[i][j] = Cq[s][i][j];
        }
      }
      const int tp = t + PFB < T ? t + PFB : T - 1;
      load_step(s, tp);
      st_xu<TL>(S.Xs, S.Us, xt, ut, t, B, b);
      if (t < T - 1) {
        md.forward(xt, ut, xn);
#pragma unroll
        for (int i = 0; i < n; ++i) xt[i] = xn[i];
      }
      if constexpr (ANALYSE) {
        float buf[PK];
        pack_cost(Cc, cc, buf, sym, diag);
        if (t == 0) {
#pragma unroll
          for (int k = 0; k < PK; ++k) pk_first[k] = buf[k];
        } else {
          const bool same = same_bits(buf, pk_first);
          if (tinv && !same)                                // records 0 .. t-1 were skipped: all equal step 0's
            for (int s_ = 0; s_ < t; ++s_) SoaRec<PK>::store(S.Cpk, pk_first, T, s_, B, b);
          tinv &= same;
          if (!tinv) SoaRec<PK>::store(S.Cpk, buf, T, t, B, b);
        }
      }
    }
  }
  if constexpr (ANALYSE) {
    if (tinv) SoaRec<PK>::store(S.Cpk, pk_first, T, T - 1, B, b);   // the one record a time-invariant copy keeps
    const unsigned char f = sym ? (unsigned char)(kCostSym | (diag && packed_diag_ok<d>() ? kCostDiag : 0) |
                                                  (tinv ? kCostTinv : 0))
                                : 0;
    S.cost_sym[b] = f;
    return f;
  }
  return 0u;
}

// done_counter[kDenseCount]: the problems whose cost iteration 0 found not to
// be a time-invariant diagonal one (the 16-lanes-per-problem models' dense-cost
// instantiations have nothing to do when it is 0)
constexpr int kDenseCount = 9;

// The control words and the stop rule's sync counters of a new solve.
DEV void mpc_reset_ctrl(const MpcState& S) {
  dilqr_mpc_ctrl z = {};
  S.ctrl[0] = z;
  S.ctrl[1] = z;
#pragma unroll
  for (int i = 0; i <= kDenseCount; ++i) S.done_counter[i] = 0u;
}

// ---------------- a whole fixed-count solve in ONE launch (thread-per-problem
// models).  With eps <= 0 and not_improved_lim >= the iteration count the stop
// rule cannot fire (mpc_explicit.py:297-299), so nothing couples two problems
// until the final best_du (k_mpc_fixed_finish, whose quirk rows mix the batch):
// each lane runs begin, iteration 0 and iterations 1..iters-1 of its problem
// back to back — the same per-lane code as k_mpc_begin + k_mpc_iterate<FIRST>
// + k_mpc_iterate<steady>, so the same bits — holding its slot indices, cost
// flags and costs in registers between iterations.  What this saves is the
// per-launch cost at one wave per SIMD: dispatch, ramp and the wait for the
// grid's slowest wave, once per iteration.  A lane reads back
// only trajectory records it wrote itself, and the gain records in LDS are its
// own, so no barrier is involved; every lane's loop runs exactly `iters`
// iterations and exits.
// Occupancy experiment builds only (tools/gpu_occupancy_exp.sh;
// never the shipped library): kSolveLpw problems per 64-lane wave (32: half the
// lanes idle, twice the waves) and a launch-bounds floor of DILQR_SOLVE_OCC
// waves per SIMD (2: at most 256 registers per lane), so that two waves of the
// same per-lane code are co-resident on a SIMD with their gain records in LDS.
#ifndef DILQR_SOLVE_LPW
#define DILQR_SOLVE_LPW 64
#endif
#ifndef DILQR_SOLVE_OCC
#define DILQR_SOLVE_OCC 1
#endif
constexpr int kSolveLpw = DILQR_SOLVE_LPW;

template <class Model, int BM, bool LG>
__global__ void __launch_bounds__(kBlock, DILQR_SOLVE_OCC) k_mpc_solve_fixed(int T, int B, const float* __restrict__ theta,
                                                            const float* __restrict__ x_init,
                                                            const float* __restrict__ u_init,
                                                            const float* __restrict__ C, const float* __restrict__ c,
                                                            Bounds bd, float decay, int max_ls, int iters,
                                                            float best_cost_eps, MpcState S) {
  constexpr int m = Model::M;
  const int b = blockIdx.x * kSolveLpw + threadIdx.x;
  // diagnostic stamps (tools/phase_stamps.py solve): 0/6 entry, 1 begin done,
  // 3 iteration 0 done, 4 last iteration starts, 2 its sweep done, 5/7 exit
  DILQR_STAMP(0);
  DILQR_STAMP(6);
  if (b == 0) mpc_reset_ctrl(S);
  if (b >= B || (int)threadIdx.x >= kSolveLpw) return;
  Model md; md.load(theta);
  extern __shared__ __attribute__((aligned(16))) float lds_gains[];
  // begin; with a packed copy it also reads C once and sets the cost flags, and
  // iteration 0 then reads the cost as every later iteration does (its sweep
  // sums the current trajectory's cost: nothing before it did); without one
  // (pk = 0) iteration 0 reads the caller's C like the per-launch path
  const unsigned pk = S.Cpk ? mpc_begin_lane<Model, true>(T, B, b, md, x_init, u_init, S, C, c)
                            : mpc_begin_lane<Model>(T, B, b, md, x_init, u_init, S);
  DILQR_STAMP(1);
  LaneIter r = mpc_iteration_lane<Model, BM, LG, false, false, kSolveLpw>(T, B, b, md, x_init, C, c, bd, decay,
                                                                          max_ls, S, S.du_sq, lds_gains, 0, 0, pk,
                                                                          0.f);
  int cur = r.slot, best = r.slot, best_iter = 0;
  float best_cost = r.cost;
  bool take = true;
  DILQR_STAMP(3);
  const size_t plane = (size_t)T * m * B;                   // one iteration's du rows
  for (int it = 1; it < iters; ++it) {
    if (it == iters - 1) DILQR_STAMP(4);
    r = mpc_iteration_lane<Model, BM, LG, false, true, kSolveLpw>(T, B, b, md, x_init, C, c, bd, decay, max_ls, S,
                                                                  S.du_sq + it * plane, lds_gains, cur, best, pk,
                                                                  r.cost);
    take = mpc_takes_best(false, r.cost, best_cost, best_cost_eps);
    if (take) { best_cost = r.cost; best = r.slot; best_iter = it; }
    cur = r.slot;
  }
  // the state the per-iteration launches leave behind
  S.cost[b] = r.cost;
  S.alpha[b] = r.alpha;
  S.best_cost[b] = best_cost;
  S.slot[b] = (unsigned char)cur;
  S.slot[B + b] = (unsigned char)best;
  S.improved[b] = take ? (iters == 1 ? 1 : 2) : 0;
  S.best_iter[b] = best_iter;
  DILQR_STAMP(5);
  DILQR_STAMP(7);
}

// ---------------- a whole stop-rule solve in ONE launch for a small batch
// (B <= kSmallMax: the IL loop's n_batch = 32, il_exp.py:44).  The stop rule
// (mpc_explicit.py:264-299) couples the batch only through the quirk rows of
// full_du_norm and two reductions (max row norm, "any improved"); with every
// problem in one workgroup those are a barrier and an LDS reduction, so the
// loop needs no launch per iteration and no host poll.  Each lane runs the
// same per-lane code as k_mpc_solve_fixed (begin, iteration 0 without PREV,
// then PREV), and after each iteration the workgroup forms the rows exactly as
// k_mpc_norm_rows does (same order of summation) and applies the rule exactly
// as mpc_decide does: the same iterates, costs, best_du, full_du_norm and
// stop iteration as the per-iteration launches
// (test_small_batch_solve_equals_per_iteration_launches).
// (256: four waves, one per SIMD of the CU — a larger workgroup would bound the
// per-lane iteration's registers at 512 / waves-per-SIMD and spill it; the first
// build at 1024 threads ran the IL step at B = 32 in 7.8 ms against 6.3 ms for
// the per-iteration launches)
constexpr int kSmallMax = 256;

template <class Model, int BM, bool LG>
__global__ void __launch_bounds__(kSmallMax) k_mpc_solve_small(int T, int B, const float* __restrict__ theta,
                                                               const float* __restrict__ x_init,
                                                               const float* __restrict__ u_init,
                                                               const float* __restrict__ C,
                                                               const float* __restrict__ c, Bounds bd, float decay,
                                                               int max_ls, int iters, float best_cost_eps, float eps,
                                                               int not_improved_lim, MpcState S) {
  constexpr int m = Model::M;
  __shared__ unsigned red_max[kSmallMax / 64];
  __shared__ int red_any[kSmallMax / 64];
  extern __shared__ __attribute__((aligned(16))) float lds_gains[];
  const int b = threadIdx.x;
  const bool act = b < B;
  const int nw = (int)(blockDim.x + 63) / 64, w = b >> 6;
  const int TM = T * m;
  Model md; md.load(theta);
  unsigned pk = 0u;
  LaneIter r{0.f, 0.f, 0};
  int cur = 0, best = 0, imp = 0;
  float best_cost = 0.f;
  if (act) {
    pk = S.Cpk ? mpc_begin_lane<Model, true>(T, B, b, md, x_init, u_init, S, C, c)
               : mpc_begin_lane<Model>(T, B, b, md, x_init, u_init, S);
    r = mpc_iteration_lane<Model, BM, LG, false, false, 64>(T, B, b, md, x_init, C, c, bd, decay, max_ls, S,
                                                            S.du_sq, lds_gains, 0, 0, pk, 0.f);
    cur = best = r.slot;
    best_cost = r.cost;
    imp = 1;
  }
  int done = 0, n_not_improved = 0, stopped = 0;
  unsigned mx_all = 0u, mx_prev = 0u;
  for (;;) {
    ++done;
    __syncthreads();                                       // every lane's du rows of this iteration are stored
    unsigned mx = 0u;
    int any = 0;
    if (act) {                                             // k_mpc_norm_rows, row b
      float s2 = 0.f;
      const float* p = S.du_sq + (size_t)b * TM;
      for (int i = 0; i < TM; ++i) s2 += p[i];
      const float fdn = sqrtf(s2);
      S.full_du_norm[b] = fdn;
      if (imp) S.best_du[b] = fdn;
      mx = __float_as_uint(fdn);
      any = imp == 2;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned o = __shfl_xor(mx, off, 64);
      mx = o > mx ? o : mx;
      any |= __shfl_xor(any, off, 64);
    }
    if ((b & 63) == 0) { red_max[w] = mx; red_any[w] = any; }
    __syncthreads();                                       // (also: every lane has read its row)
    mx = 0u;
    any = 0;
    for (int i = 0; i < nw; ++i) { mx = red_max[i] > mx ? red_max[i] : mx; any |= red_any[i]; }
    mx_prev = mx_all;
    mx_all = mx;
    if (done == iters) break;                              // the last iteration's rule is never applied
    n_not_improved = any ? 0 : n_not_improved + 1;         // mpc_explicit.py:264, 279 (mpc_decide)
    if (__uint_as_float(mx) < eps || n_not_improved > not_improved_lim) {   // 297-299
      stopped = 1;
      break;
    }
    if (act) {
      r = mpc_iteration_lane<Model, BM, LG, false, true, 64>(T, B, b, md, x_init, C, c, bd, decay, max_ls, S,
                                                             S.du_sq, lds_gains, cur, best, pk, r.cost);
      const bool take = mpc_takes_best(false, r.cost, best_cost, best_cost_eps);
      if (take) { best_cost = r.cost; best = r.slot; }
      imp = take ? 2 : 0;
      cur = r.slot;
    }
  }
  if (act) {                                               // the state the per-iteration launches leave
    S.cost[b] = r.cost;
    S.alpha[b] = r.alpha;
    S.best_cost[b] = best_cost;
    S.slot[b] = (unsigned char)cur;
    S.slot[B + b] = (unsigned char)best;
    S.improved[b] = imp;
  }
  if (b == 0) {
    // the control word the per-iteration launches leave: a stop is published by
    // the prologue of the iteration after the one that met the rule (iter =
    // iterations that ran, that iteration's max); without a stop the last
    // prologue ran before the last iteration (iter = iters - 1, the max of the
    // iteration before it)
    dilqr_mpc_ctrl o = {};
    o.iter = stopped ? done : done - 1;
    o.stopped = stopped;
    o.n_not_improved = n_not_improved;
    o.max_du_bits = stopped ? mx_all : mx_prev;
    S.ctrl[0] = o;
    S.ctrl[1] = o;
  }
}

// ---------------------------------------------------------------- launchers
// Gain records in LDS (lds bytes per 64-problem workgroup) when four
// workgroups per CU fit — one wave per SIMD at the headline's 65536 problems —
// or when the whole grid fits the chip's LDS in one round anyway (a small
// batch with a long horizon: the IL loop's T = 35, 4096 problems), and a
// workgroup's share stays within the 64 KiB a launch may take without opting in.
inline bool lds_gains_fit(size_t lds, int B) {
  if (kNoLdsGains || lds > 65536) return false;
  if (lds * 4 <= kLdsPerCU) return true;
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  return (size_t)grid_for(B) <= (size_t)cus * (kLdsPerCU / lds);
}
// the fused MPC iteration of one thread-per-problem model: bounds mode, gain
// records in LDS when four workgroups per CU still fit, iteration 0's own
// instantiation
template <class MD>
int launch_mpc_step_tpp(const MpcStepArgs& a) {
#define LAUNCH_IT(BM_, LG_, FIRST_, LDS_)                                                                     \
  k_mpc_iterate<MD, BM_, LG_, FIRST_><<<grid_for(a.B), kBlock, LDS_, a.stream>>>(                            \
      a.T, a.B, a.theta, a.x_init, a.C, a.c, a.bd, a.decay, a.max_ls, a.iteration, a.best_cost_eps, a.eps, a.lim, \
      a.G, a.st)
#define LAUNCH_MPC(BM_)                                                                                      \
  do {                                                                                                       \
    const size_t lds = (size_t)a.T * kBlock * (MD::N * MD::M + MD::M) * sizeof(float);                      \
    const bool lg = lds_gains_fit(lds, a.B);                                                                 \
    if (a.iteration == 0 && lg) LAUNCH_IT(BM_, true, true, lds);                                             \
    else if (a.iteration == 0) LAUNCH_IT(BM_, false, true, 0);                                               \
    else if (lg) LAUNCH_IT(BM_, true, false, lds);                                                           \
    else LAUNCH_IT(BM_, false, false, 0);                                                                    \
  } while (0)
  if (a.bd.mode == DILQR_BOUNDS_TENSOR) LAUNCH_MPC(DILQR_BOUNDS_TENSOR);
  else if (a.bd.mode != DILQR_BOUNDS_NONE) LAUNCH_MPC(DILQR_BOUNDS_SCALAR);
  else LAUNCH_MPC(DILQR_BOUNDS_NONE);
#undef LAUNCH_MPC
#undef LAUNCH_IT
  return launched();
}

// a whole fixed-count solve of one thread-per-problem model (k_mpc_solve_fixed)
template <class MD>
int launch_mpc_solve_tpp(const MpcSolveArgs& a) {
#define LAUNCH_SOLVE(BM_)                                                                                    \
  do {                                                                                                       \
    const size_t lds = (size_t)a.T * kSolveLpw * (MD::N * MD::M + MD::M) * sizeof(float);                   \
    const int grid = (int)(((long long)a.B + kSolveLpw - 1) / kSolveLpw);                                   \
    if (lds_gains_fit(lds * kBlock / kSolveLpw, a.B))                                                       \
      k_mpc_solve_fixed<MD, BM_, true><<<grid, kBlock, lds, a.stream>>>(                                      \
          a.T, a.B, a.theta, a.x_init, a.u_init, a.C, a.c, a.bd, a.decay, a.max_ls, a.iters, a.best_cost_eps, a.st); \
    else                                                                                                     \
      k_mpc_solve_fixed<MD, BM_, false><<<grid, kBlock, 0, a.stream>>>(                                       \
          a.T, a.B, a.theta, a.x_init, a.u_init, a.C, a.c, a.bd, a.decay, a.max_ls, a.iters, a.best_cost_eps, a.st); \
  } while (0)
  if (a.bd.mode == DILQR_BOUNDS_TENSOR) LAUNCH_SOLVE(DILQR_BOUNDS_TENSOR);
  else if (a.bd.mode != DILQR_BOUNDS_NONE) LAUNCH_SOLVE(DILQR_BOUNDS_SCALAR);
  else LAUNCH_SOLVE(DILQR_BOUNDS_NONE);
#undef LAUNCH_SOLVE
  return launched();
}

// a whole stop-rule solve of one thread-per-problem model in one workgroup
// (B <= kSmallMax; gain records in LDS for one wave when they fit)
template <class MD>
int launch_mpc_solve_small_tpp(const MpcSolveArgs& a, float eps, int lim) {
  if (a.B > kSmallMax) return DILQR_E_SHAPE;
  const int threads = (a.B + 63) / 64 * 64;
  const size_t lds = (size_t)a.T * 64 * (MD::N * MD::M + MD::M) * sizeof(float);
  const bool lg = threads == 64 && lds <= 65536 && !kNoLdsGains;
#define LAUNCH_SMALL(BM_)                                                                                    \
  do {                                                                                                       \
    if (lg)                                                                                                  \
      k_mpc_solve_small<MD, BM_, true><<<1, threads, lds, a.stream>>>(                                        \
          a.T, a.B, a.theta, a.x_init, a.u_init, a.C, a.c, a.bd, a.decay, a.max_ls, a.iters, a.best_cost_eps, eps, \
          lim, a.st);                                                                                        \
    else                                                                                                     \
      k_mpc_solve_small<MD, BM_, false><<<1, threads, 0, a.stream>>>(                                         \
          a.T, a.B, a.theta, a.x_init, a.u_init, a.C, a.c, a.bd, a.decay, a.max_ls, a.iters, a.best_cost_eps, eps, \
          lim, a.st);                                                                                        \
  } while (0)
  if (a.bd.mode == DILQR_BOUNDS_TENSOR) LAUNCH_SMALL(DILQR_BOUNDS_TENSOR);
  else if (a.bd.mode != DILQR_BOUNDS_NONE) LAUNCH_SMALL(DILQR_BOUNDS_SCALAR);
  else LAUNCH_SMALL(DILQR_BOUNDS_NONE);
#undef LAUNCH_SMALL
  return launched();
}

template <class MD>
int launch_ilqr_iterate_tpp(const IlqrIterArgs& a) {
#define LAUNCH_IT(BM_)                                                                                        \
  k_ilqr_iterate<MD, BM_><<<grid_for(a.B), kBlock, 0, a.stream>>>(a.T, a.B, a.theta, a.x_init, a.C, a.c, a.x, a.u, \
                                                                   a.bd, a.decay, a.max_ls, a.ws, a.x_out,     \
                                                                   a.u_out, a.cost, a.du_sq, a.alpha, a.ctrl)
  if (a.bd.mode == DILQR_BOUNDS_TENSOR) LAUNCH_IT(DILQR_BOUNDS_TENSOR);
  else if (a.bd.mode != DILQR_BOUNDS_NONE) LAUNCH_IT(DILQR_BOUNDS_SCALAR);
  else LAUNCH_IT(DILQR_BOUNDS_NONE);
#undef LAUNCH_IT
  return launched();
}

}  // namespace dilqr
