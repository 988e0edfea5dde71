// tu_forward.hip — the standalone rollout + line search (lqr_forward,
// lqr_step_explicit.py:166-263) and the classic adjoint (lqr_step.py:312-407).
#include "dilqr_common.h"

namespace dilqr {

// ============================================================ forward / line search
// lqr_forward (lqr_step_explicit.py:166-263), one problem per lane, the batch's
// `while any(cost > old_cost)` loop evaluated per problem (each problem's alpha
// depends only on its own cost, so this is the reference's result).
struct NoModel {};

template <int n, int m, class Model>
struct Dyn {
  Model md;
  const float* F;
  const float* f;
  int B;
  DEV void step(int t, int b, const float (&x)[n], const float (&uu)[m], float (&o)[n]) const {
    if constexpr (std::is_same_v<Model, NoModel>) {
      size_t tb = (size_t)t * B + b;
      float Ft[n][n + m];
      ld2(Ft, F + tb * n * (n + m));
#pragma unroll
      for (int i = 0; i < n; ++i) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Ft[i][j] * x[j];
#pragma unroll
        for (int j = 0; j < m; ++j) s += Ft[i][n + j] * uu[j];
        o[i] = s;
      }
      if (f) {
        float ft[n]; ld(ft, f + tb * n);
#pragma unroll
        for (int i = 0; i < n; ++i) o[i] += ft[i];
      }
    } else {
      md.forward(x, uu, o);
    }
  }
};

// One rollout pass with step size alpha.  Gains come from (K,k) [T,B,m,n]/[T,B,m]
// (GREC == 0) or from the fused kernel's per-lane gain records (GREC floats per
// (t,b): K, k, obj_t of the current trajectory).  Returns the new cost; if
// old_cost_out != nullptr it also returns the current trajectory's cost summed
// in time order from the records.
template <int n, int m, int GREC, class DynT>
DEV float forward_pass(const DynT& dyn, int T, int B, int b, float alpha, const float* __restrict__ x_init,
                       const float* __restrict__ C, const float* __restrict__ c, const float* __restrict__ x,
                       const float* __restrict__ u, const float* __restrict__ K, const float* __restrict__ k,
                       const float* __restrict__ grec, const Bounds& bd, const unsigned char* __restrict__ zI,
                       float* __restrict__ x_out, float* __restrict__ u_out, float* __restrict__ du_sq,
                       float* old_cost_out) {
  constexpr int d = n + m;
  float xn[n], dx[n];
  ld(xn, x_init + (size_t)b * n);
#pragma unroll
  for (int i = 0; i < n; ++i) dx[i] = 0.f;
  st(x_out + (size_t)b * n, xn);
  float cost = 0.f, oldc = 0.f;
  for (int t = 0; t < T; ++t) {
    size_t tb = (size_t)t * B + b;
    float Kt[m][n], kt[m], ut[m];
    if constexpr (GREC > 0) {
      float g[GREC];
      ld(g, grec + tb * GREC);
#pragma unroll
      for (int a = 0; a < m; ++a) {
#pragma unroll
        for (int j = 0; j < n; ++j) Kt[a][j] = g[a * n + j];
        kt[a] = g[m * n + a];
      }
      oldc += g[m * n + m];
    } else {
      ld2(Kt, K + tb * m * n);
      ld(kt, k + tb * m);
    }
    ld(ut, u + tb * m);
    float nu[m];
#pragma unroll
    for (int a = 0; a < m; ++a) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < n; ++j) s += Kt[a][j] * dx[j];
      nu[a] = (s + ut[a]) + alpha * kt[a];
      if (zI && zI[tb * m + a]) nu[a] = 0.f;
      if (bd.mode != DILQR_BOUNDS_NONE) nu[a] = eclamp(nu[a], bound_lo(bd, tb * m + a), bound_hi(bd, tb * m + a));
    }
    st(u_out + tb * m, nu);
    if (du_sq) {
#pragma unroll
      for (int a = 0; a < m; ++a) {
        float e = ut[a] - nu[a];
        du_sq[((size_t)t * m + a) * B + b] = e * e;
      }
    }
    float Ct[d][d], ct[d], tau[d];
    ld2(Ct, C + tb * d * d);
    ld(ct, c + tb * d);
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xn[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = nu[a];
    cost += quad_cost(Ct, ct, tau);
    if (t < T - 1) {
      float xnext[n], xcur[n];
      dyn.step(t, b, xn, nu, xnext);
      ld(xcur, x + (tb + B) * n);
#pragma unroll
      for (int i = 0; i < n; ++i) {
        dx[i] = xnext[i] - xcur[i];
        xn[i] = xnext[i];
      }
      st(x_out + (tb + B) * n, xn);
    }
  }
  if (old_cost_out) *old_cost_out = oldc;
  return cost;
}

// The current trajectory's cost (lqr_step_explicit.py:171), formed and summed
// exactly as the fused iteration forms it inside its backward sweep (stage
// costs as tau . (C tau) + c . tau, summed over t = T-1..0), so the fused and
// unfused pipelines take the same line-search decisions bit for bit.
template <int n, int m>
DEV float traj_cost(int T, int B, int b, const float* __restrict__ C, const float* __restrict__ c,
                    const float* __restrict__ x, const float* __restrict__ u) {
  constexpr int d = n + m;
  float cost = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    size_t tb = (size_t)t * B + b;
    float Ct[d][d], ct[d], tau[d], xt[n], ut[m], Ctau[d];
    ld2(Ct, C + tb * d * d); ld(ct, c + tb * d); ld(xt, x + tb * n); ld(ut, u + tb * m);
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
    cost += quad_cost(Ct, ct, tau, Ctau);
  }
  return cost;
}

template <int n, int m, class Model>
__global__ void __launch_bounds__(kBlock) k_lqr_forward(int T, int B, const float* __restrict__ theta,
                                                        const float* __restrict__ F, const float* __restrict__ f,
                                                        const float* __restrict__ x_init, const float* __restrict__ C,
                                                        const float* __restrict__ c, const float* __restrict__ x,
                                                        const float* __restrict__ u, const float* __restrict__ K,
                                                        const float* __restrict__ k, Bounds bd,
                                                        const unsigned char* __restrict__ zI, float decay, int max_ls,
                                                        float* __restrict__ x_out, float* __restrict__ u_out,
                                                        float* cost_out, float* __restrict__ du_sq,
                                                        float* __restrict__ alpha_out,
                                                        const float* old_cost_in) {
  // cost_out and old_cost_in may alias (an MPC loop passes its cost buffer as
  // both): each lane reads old_cost_in[b] before it writes cost_out[b]
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Dyn<n, m, Model> dyn;
  if constexpr (!std::is_same_v<Model, NoModel>) dyn.md.load(theta);
  dyn.F = F; dyn.f = f; dyn.B = B;
  // lqr_step_explicit.py:171, or the caller's value of the same cost (an MPC
  // loop passes what its previous line search computed for this trajectory)
  const float old_cost = old_cost_in ? old_cost_in[b] : traj_cost<n, m>(T, B, b, C, c, x, u);
  float alpha = 1.f, cost = 0.f;
  for (int ls = 0; ls < max_ls; ++ls) {
    cost = forward_pass<n, m, 0>(dyn, T, B, b, alpha, x_init, C, c, x, u, K, k, nullptr, bd, zI, x_out, u_out,
                                 ls == 0 ? du_sq : nullptr, nullptr);
    if (!(cost > old_cost) || ls == max_ls - 1) break;
    alpha *= decay;                                             // lqr_step_explicit.py:249
  }
  cost_out[b] = cost;
  if (alpha_out) alpha_out[b] = alpha;                          // 254: the last pass's alpha
}

// ============================================================ classic adjoint
// lqr_step.py:312-407 for one problem per lane:
//   phase 1: Riccati sweep of the adjoint problem (c_back = -r, u_zero_I = active set)
//   phase 2: its LinDx rollout from 0 with the default line search (decay 0.2, 10
//            passes; old cost 0), d tau stored as dc = -d tau
//   phase 3: costates lam, dlam backwards; dC, dF, df, dx_init.
template <int n, int m, int MODE>
__global__ void __launch_bounds__(kBlock) k_lqr_adjoint(int T, int B, const float* __restrict__ C,
                                                        const float* __restrict__ c, const float* __restrict__ F,
                                                        const float* __restrict__ x, const float* __restrict__ u,
                                                        const float* __restrict__ dl_dx, const float* __restrict__ dl_du,
                                                        Bounds bd, float* __restrict__ ws, float* __restrict__ dx_init,
                                                        float* __restrict__ dC, float* __restrict__ dc,
                                                        float* __restrict__ dF, float* __restrict__ df) {
  constexpr int d = n + m;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  // active set (lqr_step.py:321-325)
  auto active = [&](size_t tb, int a) -> bool {
    if (bd.mode == DILQR_BOUNDS_NONE) return false;
    float ua = u[tb * m + a];
    return fabsf(ua - bound_lo(bd, tb * m + a)) <= 1e-8f || fabsf(ua - bound_hi(bd, tb * m + a)) <= 1e-8f;
  };
  // ---- phase 1
  RiccatiState<n, m> rs;
  rs.init();
  for (int t = T - 1; t >= 0; --t) {
    size_t tb = (size_t)t * B + b;
    float Ct[d][d], cb[d], rx[n], ru[m];
    ld2(Ct, C + tb * d * d);
    ld(rx, dl_dx + tb * n); ld(ru, dl_du + tb * m);
#pragma unroll
    for (int i = 0; i < n; ++i) cb[i] = -rx[i];
#pragma unroll
    for (int a = 0; a < m; ++a) cb[n + a] = -ru[a];
    float Ft[n][d];
    if (t < T - 1) {
      ld2(Ft, F + tb * n * d);
    } else {
#pragma unroll
      for (int i = 0; i < n; ++i)
#pragma unroll
        for (int j = 0; j < d; ++j) Ft[i][j] = 0.f;
    }
    float zIt[m], lb[m], ub[m];
    bool any = false;
#pragma unroll
    for (int a = 0; a < m; ++a) {
      zIt[a] = active(tb, a) ? 1.f : 0.f;
      any |= zIt[a] != 0.f;
      lb[a] = ub[a] = 0.f;
    }
    float Kt[m][n], kt[m];
    if (bd.mode != DILQR_BOUNDS_NONE) rs.template step<GAIN_ZERO_I>(Ct, cb, Ft, zIt, lb, ub, Kt, kt);
    else rs.template step<MODE>(Ct, cb, Ft, zIt, lb, ub, Kt, kt);
    (void)any;
    st2(ws + tb * (m * n + m), Kt);
    st(ws + tb * (m * n + m) + m * n, kt);
  }
  // ---- phase 2: rollout of the adjoint LQR from zero with line search
  float alpha = 1.f;
  for (int ls = 0; ls < 10; ++ls) {
    float xn[n], cost = 0.f;
#pragma unroll
    for (int i = 0; i < n; ++i) xn[i] = 0.f;
    for (int t = 0; t < T; ++t) {
      size_t tb = (size_t)t * B + b;
      float Kt[m][n], kt[m], nu[m];
      ld2(Kt, ws + tb * (m * n + m));
      ld(kt, ws + tb * (m * n + m) + m * n);
#pragma unroll
      for (int a = 0; a < m; ++a) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) s += Kt[a][j] * xn[j];       // dx = new_x - 0
        nu[a] = (s + 0.f) + alpha * kt[a];
        if (active(tb, a)) nu[a] = 0.f;
      }
      float tau[d], Ct[d][d], rr[d];
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = xn[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = nu[a];
      float ndt[d];
#pragma unroll
      for (int i = 0; i < d; ++i) ndt[i] = -tau[i];
      st(dc + tb * d, ndt);
      ld2(Ct, C + tb * d * d);
      {
        float rx[n], ru[m];
        ld(rx, dl_dx + tb * n); ld(ru, dl_du + tb * m);
#pragma unroll
        for (int i = 0; i < n; ++i) rr[i] = -rx[i];
#pragma unroll
        for (int a = 0; a < m; ++a) rr[n + a] = -ru[a];
      }
      cost += quad_cost(Ct, rr, tau);
      if (t < T - 1) {
        float Ft[n][d];
        ld2(Ft, F + tb * n * d);
        float xnext[n];
#pragma unroll
        for (int i = 0; i < n; ++i) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) s += Ft[i][j] * tau[j];
          xnext[i] = s;
        }
#pragma unroll
        for (int i = 0; i < n; ++i) xn[i] = xnext[i];
      }
    }
    if (!(cost > 0.f) || ls == 9) break;
    alpha *= 0.2f;
  }
  // ---- phase 3: costates and gradients (lqr_step.py:352-405)
  float lam[n], dlam[n];
#pragma unroll
  for (int i = 0; i < n; ++i) lam[i] = dlam[i] = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    size_t tb = (size_t)t * B + b;
    float Ct[d][d], ctt[d], xt[n], ut[m], tau[d], dtau[d], rx[n];
    ld2(Ct, C + tb * d * d); ld(ctt, c + tb * d); ld(xt, x + tb * n); ld(ut, u + tb * m);
    ld(dtau, dc + tb * d);
    ld(rx, dl_dx + tb * n);
#pragma unroll
    for (int i = 0; i < d; ++i) dtau[i] = -dtau[i];
#pragma unroll
    for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
    for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
    // dC_t = -0.5 (dtau tau^T + tau dtau^T)
    float dCt[d][d];
#pragma unroll
    for (int i = 0; i < d; ++i)
#pragma unroll
      for (int j = 0; j < d; ++j) dCt[i][j] = -0.5f * (dtau[i] * tau[j] + tau[i] * dtau[j]);
    st2(dC + tb * d * d, dCt);
    if (t < T - 1) {
      // dF_t = -(dlam_{t+1} tau_t^T + lam_{t+1} dtau_t^T); df_t = -dlam_{t+1}
      float dFt[n][d], dft[n];
#pragma unroll
      for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int j = 0; j < d; ++j) dFt[i][j] = -(dlam[i] * tau[j] + lam[i] * dtau[j]);
        dft[i] = -dlam[i];
      }
      st2(dF + tb * n * d, dFt);
      if (df) st(df + tb * n, dft);
    }
    // lam_t = Cxx x + Cxu u + c_x + F_x^T lam_{t+1}; dlam likewise with dtau and -r_x
    float nl[n], ndl[n];
#pragma unroll
    for (int i = 0; i < n; ++i) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < n; ++j) { s1 += Ct[i][j] * xt[j]; s2 += Ct[i][j] * dtau[j]; }
      float s3 = 0.f, s4 = 0.f;
#pragma unroll
      for (int a = 0; a < m; ++a) { s3 += Ct[i][n + a] * ut[a]; s4 += Ct[i][n + a] * dtau[n + a]; }
      nl[i] = (s1 + s3) + ctt[i];
      ndl[i] = (s2 + s4) - rx[i];
    }
    if (t < T - 1) {
      float Ft[n][d];
      ld2(Ft, F + tb * n * d);
#pragma unroll
      for (int i = 0; i < n; ++i) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int l = 0; l < n; ++l) { s1 += Ft[l][i] * lam[l]; s2 += Ft[l][i] * dlam[l]; }
        nl[i] += s1;
        ndl[i] += s2;
      }
    }
#pragma unroll
    for (int i = 0; i < n; ++i) { lam[i] = nl[i]; dlam[i] = ndl[i]; }
  }
  float dxi[n];
#pragma unroll
  for (int i = 0; i < n; ++i) dxi[i] = -dlam[i];
  st(dx_init + (size_t)b * n, dxi);
}

}  // namespace dilqr

using namespace dilqr;

extern "C" {

int dilqr_lqr_forward_f32(int model, int n, int m, int T, int B, const float* theta, const float* F, const float* f,
                          const float* x_init, const float* C, const float* c, const float* x, const float* u,
                          const float* K, const float* k, dilqr_bounds bounds, const unsigned char* u_zero_I,
                          float linesearch_decay, int max_linesearch_iter, float* x_out, float* u_out, float* cost,
                          float* du_sq, float* alpha, const float* old_cost, void* stream) {
  if (T < 1 || B < 0 || max_linesearch_iter < 1) return DILQR_E_ARG;
  if (!x_init || !C || !c || !x || !u || !K || !k || !x_out || !u_out || !cost) return DILQR_E_ARG;
  const void* ps[] = {F, f, x_init, C, c, x, u, K, k, x_out, u_out};
  for (const void* p : ps) if (!al16(p)) return DILQR_E_ARG;
  if (bad_bounds(bounds)) return DILQR_E_ARG;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  if (model == DILQR_MODEL_LINDX) {
    if (!F && T > 1) return DILQR_E_ARG;
#define X(N_, M_)                                                                                             \
    if (n == N_ && m == M_) {                                                                                  \
      k_lqr_forward<N_, M_, NoModel><<<grid_for(B), kBlock, 0, S(stream)>>>(                                   \
          T, B, theta, F, f, x_init, C, c, x, u, K, k, bd, u_zero_I, linesearch_decay, max_linesearch_iter,     \
          x_out, u_out, cost, du_sq, alpha, old_cost);                                                         \
      return launched();                                                                                       \
    }
    DILQR_FOR_EACH_SHAPE(X)
#undef X
    if (old_cost) return DILQR_E_MODE;                 // the 16-lane kernels form it themselves
#define X(N_, M_)                                                                                             \
    if (n == N_ && m == M_) {                                                                                  \
      k_lqr_forward_group<N_, M_, GroupNoModel><<<grid_group(B), 64, 0, S(stream)>>>(                          \
          T, B, theta, F, f, x_init, C, c, x, u, K, k, bd, u_zero_I, linesearch_decay, max_linesearch_iter,     \
          x_out, u_out, cost, du_sq, alpha);                                                                   \
      return launched();                                                                                       \
    }
    DILQR_FOR_EACH_GROUP_SHAPE(X)
#undef X
    return DILQR_E_SHAPE;
  }
  if (!theta) return DILQR_E_ARG;
  if (model == DILQR_MODEL_ROCKET) {
    if (n != Rocket::N || m != Rocket::M) return DILQR_E_SHAPE;
    if (old_cost) return DILQR_E_MODE;
    k_lqr_forward_group<Rocket::N, Rocket::M, Rocket><<<grid_group(B), 64, 0, S(stream)>>>(
        T, B, theta, F, f, x_init, C, c, x, u, K, k, bd, u_zero_I, linesearch_decay, max_linesearch_iter, x_out,
        u_out, cost, du_sq, alpha);
    return launched();
  }
  MODEL_SWITCH_TPP(model, ({
    if (n != MD::N || m != MD::M) return DILQR_E_SHAPE;
    k_lqr_forward<MD::N, MD::M, MD><<<grid_for(B), kBlock, 0, S(stream)>>>(
        T, B, theta, F, f, x_init, C, c, x, u, K, k, bd, u_zero_I, linesearch_decay, max_linesearch_iter, x_out,
        u_out, cost, du_sq, alpha, old_cost);
  }));
  return launched();
}

int dilqr_lqr_adjoint_f32(int n, int m, int T, int B, const float* C, const float* c, const float* F,
                          const float* x, const float* u, const float* dl_dx, const float* dl_du, dilqr_bounds bounds,
                          int m_solver, float* ws, float* dx_init, float* dC, float* dc, float* dF, float* df,
                          void* stream) {
  if (T < 1 || B < 0 || !C || !c || !x || !u || !dl_dx || !dl_du || !ws || !dx_init || !dC || !dc) return DILQR_E_ARG;
  if (T > 1 && (!F || !dF)) return DILQR_E_ARG;
  const void* ps[] = {C, c, F, x, u, dl_dx, dl_du, ws, dx_init, dC, dc, dF, df};
  for (const void* p : ps) if (!al16(p)) return DILQR_E_ARG;
  if (bad_bounds(bounds)) return DILQR_E_ARG;
  if (B == 0) return 0;
  Bounds bd = mkb(bounds);
  bool chol = m_solver == DILQR_SOLVE_CHOL && m > 1;
#define X(N_, M_)                                                                                           \
  if (n == N_ && m == M_) {                                                                                  \
    if (chol)                                                                                                \
      k_lqr_adjoint<N_, M_, GAIN_CHOL><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, C, c, F, x, u, dl_dx,    \
                                                                             dl_du, bd, ws, dx_init, dC, dc, \
                                                                             dF, df);                        \
    else                                                                                                     \
      k_lqr_adjoint<N_, M_, GAIN_UNC><<<grid_for(B), kBlock, 0, S(stream)>>>(T, B, C, c, F, x, u, dl_dx,     \
                                                                            dl_du, bd, ws, dx_init, dC, dc,  \
                                                                            dF, df);                         \
    return launched();                                                                                       \
  }
  DILQR_FOR_EACH_SHAPE(X)
#undef X
  return DILQR_E_SHAPE;
}

}  // extern "C"
