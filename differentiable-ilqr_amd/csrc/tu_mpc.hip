// tu_mpc.hip — the MPC loop's small kernels (begin, gather, stop rule,
// fixed-count finish, unfused best-iterate bookkeeping) and every MPC C-ABI
// entry point; the fused iterations are launched through dilqr_launch.h.
#include "dilqr_fused.h"

namespace dilqr {

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
    const float* q = S.du_sq + ((size_t)(iterations - 1) * B + r) * TM;
    float s = 0.f, s2 = 0.f;
    for (int i = 0; i < TM; ++i) { s += p[i]; s2 += q[i]; }
    S.best_du[r] = sqrtf(s);
    S.full_du_norm[r] = sqrtf(s2);          // the last iteration's rows, as the per-iteration rule leaves it
  }
  if (r < 2) {
    dilqr_mpc_ctrl c = S.ctrl[r];
    c.iter = iterations;
    c.stopped = 0;
    S.ctrl[r] = c;
  }
}

// rollout of u_init into slot 0 (util.get_traj) + reset of slots/ctrl
// (mpc_begin_lane; u_init null: zeros, the MPC default).
template <class Model>
__global__ void __launch_bounds__(kBlock) k_mpc_begin(int T, int B, const float* __restrict__ theta,
                                                      const float* __restrict__ x_init,
                                                      const float* __restrict__ u_init, MpcState S) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b == 0) mpc_reset_ctrl(S);
  if (b >= B) return;
  Model md; md.load(theta);
  mpc_begin_lane<Model>(T, B, b, md, x_init, u_init, S);
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

inline int launch_norm_rows(int TM, int B, int iteration, const MpcState& st, hipStream_t stream) {
  const NormGeom g = norm_geom(TM, B);
  if (g.stage)
    k_mpc_norm_rows<true><<<g.blocks, g.threads, (size_t)g.threads * TM * sizeof(float), stream>>>(TM, B, iteration,
                                                                                                   st);
  else
    k_mpc_norm_rows<false><<<g.blocks, g.threads, 0, stream>>>(TM, B, iteration, st);
  return launched();
}

}  // namespace dilqr

using namespace dilqr;

extern "C" {

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
  const IlqrIterArgs a{T, B, theta, x_init, C, c, x, u, mkb(bounds), linesearch_decay, max_linesearch_iter,
                       ws_gains, x_out, u_out, cost, du_sq, alpha, ctrl, S(stream)};
  switch (model) {
    case DILQR_MODEL_PENDULUM: return launch_ilqr_iterate_pendulum(a);
    case DILQR_MODEL_CARTPOLE: return launch_ilqr_iterate_cartpole(a);
    case DILQR_MODEL_ROCKET: return launch_ilqr_iterate_rocket(a);
    case DILQR_MODEL_PENDULUM_COMPLEX: return launch_ilqr_iterate_pendulum_complex(a);
    default: return DILQR_E_SHAPE;
  }
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
  const MpcStepArgs a{T, B, theta, x_init, C, c, mkb(bounds), linesearch_decay, max_linesearch_iter, iteration,
                      best_cost_eps, eps, not_improved_lim, G, st, S(stream)};
  switch (model) {
    case DILQR_MODEL_PENDULUM: return launch_mpc_step_pendulum(a);
    case DILQR_MODEL_CARTPOLE: return launch_mpc_step_cartpole(a);
    case DILQR_MODEL_ROCKET: return launch_mpc_step_rocket(a);
    case DILQR_MODEL_PENDULUM_COMPLEX: return launch_mpc_step_pendulum_complex(a);
    default: return DILQR_E_SHAPE;
  }
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

int dilqr_mpc_solve_fixed_f32(int model, int T, int B, const float* theta, const float* x_init, const float* u_init,
                              const float* C, const float* c, dilqr_bounds bounds, float linesearch_decay,
                              int max_linesearch_iter, int iterations, float best_cost_eps, dilqr_mpc_state st,
                              void* stream) {
  if (T < 1 || B < 0 || max_linesearch_iter < 1 || iterations < 1 || !theta || !x_init || !C || !c) return DILQR_E_ARG;
  if (!al16(x_init) || !al16(C) || !al16(c) || bad_state(st) || bad_bounds(bounds) || !st.best_iter)
    return DILQR_E_ARG;
  if (u_init && ((uintptr_t)u_init & 3u)) return DILQR_E_ARG;
  const int m = dilqr_model_num_ctrl(model);
  if (m < 1) return DILQR_E_SHAPE;
  if (B == 0) return 0;
  int e;
  if (model == DILQR_MODEL_PENDULUM || model == DILQR_MODEL_CARTPOLE || model == DILQR_MODEL_PENDULUM_COMPLEX) {
    const MpcSolveArgs a{T, B, theta, x_init, u_init, C, c, mkb(bounds), linesearch_decay, max_linesearch_iter,
                         iterations, best_cost_eps, st, S(stream)};
    e = model == DILQR_MODEL_CARTPOLE ? launch_mpc_solve_cartpole(a)
        : model == DILQR_MODEL_PENDULUM ? launch_mpc_solve_pendulum(a) : launch_mpc_solve_pendulum_complex(a);
  } else {
    // the 16-lanes-per-problem models change their lane mapping between the
    // sweep and the line search: one launch pair per iteration
    e = dilqr_mpc_begin_f32(model, T, B, theta, x_init, u_init, st, stream);
    for (int i = 0; !e && i < iterations; ++i)
      e = dilqr_mpc_iterate_fixed_f32(model, T, B, theta, x_init, C, c, bounds, linesearch_decay,
                                      max_linesearch_iter, i, best_cost_eps, st, stream);
  }
  if (e) return e;
  return dilqr_mpc_finish_fixed_f32(T, m, B, iterations, st, stream);
}

int dilqr_mpc_solve_small_f32(int model, int T, int B, const float* theta, const float* x_init, const float* u_init,
                              const float* C, const float* c, dilqr_bounds bounds, float linesearch_decay,
                              int max_linesearch_iter, int iterations, float best_cost_eps, float eps,
                              int not_improved_lim, dilqr_mpc_state st, void* stream) {
  if (T < 1 || B < 0 || max_linesearch_iter < 1 || iterations < 1 || !theta || !x_init || !C || !c) return DILQR_E_ARG;
  if (!al16(x_init) || !al16(C) || !al16(c) || bad_state(st) || bad_bounds(bounds)) return DILQR_E_ARG;
  if (u_init && ((uintptr_t)u_init & 3u)) return DILQR_E_ARG;
  if (B > kSmallMax) return DILQR_E_SHAPE;
  if (B == 0) return 0;
  const MpcSolveArgs a{T, B, theta, x_init, u_init, C, c, mkb(bounds), linesearch_decay, max_linesearch_iter,
                       iterations, best_cost_eps, st, S(stream)};
  switch (model) {
    case DILQR_MODEL_PENDULUM: return launch_mpc_solve_small_pendulum(a, eps, not_improved_lim);
    case DILQR_MODEL_CARTPOLE: return launch_mpc_solve_small_cartpole(a, eps, not_improved_lim);
    case DILQR_MODEL_PENDULUM_COMPLEX: return launch_mpc_solve_small_pendulum_complex(a, eps, not_improved_lim);
    default: return DILQR_E_SHAPE;            // rocket: its sweep and search use different lane mappings
  }
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

int dilqr_mpc_iterate_range_f32(int model, int T, int B, const float* theta, const float* x_init, const float* C,
                                const float* c, dilqr_bounds bounds, float linesearch_decay, int max_linesearch_iter,
                                int first_iteration, int count, float best_cost_eps, float eps, int not_improved_lim,
                                dilqr_mpc_state st, void* stream) {
  if (count < 0 || first_iteration < 0) return DILQR_E_ARG;
  for (int i = first_iteration; i < first_iteration + count; ++i) {
    const int e = dilqr_mpc_iterate_f32(model, T, B, theta, x_init, C, c, bounds, linesearch_decay,
                                        max_linesearch_iter, i, best_cost_eps, eps, not_improved_lim, st, stream);
    if (e) return e;
  }
  return 0;
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
