// tu_grad_input.hip — the model protocol's second-order API: get_matrices
// (cartpole.py:105-716, pendulum.py:152-382, rocket.py:258-261 with its
// build_batched_* tables 541-820) and grad_input (cartpole.py:717-788,
// pendulum.py:383-443, rocket.py:263-323).  The implicit backward does not go
// through these (it contracts the same terms on the fly); they
// serve callers of the reference's model API.  One lane per row / problem.
#include "dilqr_common.h"

namespace dilqr {

// per row i: D [n][d] (the closed-form Jacobian), D_params [n][d][p],
// D_x [n][d][n], D_u [n][d][m], x_theta [n][p], x_xtm1 [n][n], x_utm1 [n][m].
// The second-order arrays are written sparsely (generated matrices(): only the
// structural nonzeros); the entry point zero-fills them first.
template <class Model, class D2>
__global__ void __launch_bounds__(kBlock) k_get_matrices(int N, const float* __restrict__ theta,
                                                         const float* __restrict__ x, const float* __restrict__ u,
                                                         float* __restrict__ D, float* __restrict__ Dp,
                                                         float* __restrict__ Dx, float* __restrict__ Du,
                                                         float* __restrict__ xth, float* __restrict__ xx,
                                                         float* __restrict__ xu) {
  constexpr int n = Model::N, m = Model::M, p = Model::P, d = n + m;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  Model md; md.load(theta);
  float xi[n], ui[m];
  ld(xi, x + (size_t)i * n); ld(ui, u + (size_t)i * m);
  float Dr[n][d];
  md.jacobian(xi, ui, Dr);
  float* Di = D + (size_t)i * n * d;
  float* xui = xu + (size_t)i * n * m;
#pragma unroll
  for (int r = 0; r < n; ++r) {
#pragma unroll
    for (int j = 0; j < d; ++j) Di[r * d + j] = Dr[r][j];
#pragma unroll
    for (int a = 0; a < m; ++a) xui[r * m + a] = Dr[r][n + a];
  }
  D2::matrices(theta, xi, ui, Dp + (size_t)i * n * d * p, Dx + (size_t)i * n * d * n, Du + (size_t)i * n * d * m,
               xth + (size_t)i * n * p, xx + (size_t)i * n * n);
}

// grad_input (cartpole.py:717-788) for problem b, over t = 0..T-1, from the
// get_matrices arrays of the T*B rows [T,B,...]:
//   gradx_t  = x_theta_t + (x_xtm1_t + x_utm1_t K_{t-1}) gradx_{t-1}       (t > 0)
//   grad_D_t = D_params_t + (D_x_t + D_u_t K_t) gradx_t                     (t < T-1)
//   grad_d_{t-1} = gradx_t - grad_D_{t-1} tau_{t-1} - D_{t-1} [gradx_{t-1}; K_{t-1} gradx_{t-1}]
//   d_x_t = -D_x_t tau_t, d_u_t = -D_u_t tau_t                              (t < T-1)
// K [T,B,m,n] consumed as K[t] (the caller passes the gains in the order the
// reference stacks them); NULL = zeros (grad_input(X, U) without K).
// grad_D_{t-1} is re-read from the output this lane wrote at step t-1.
template <class Model>
__global__ void __launch_bounds__(kBlock) k_grad_input(
    int T, int B, const float* __restrict__ X, const float* __restrict__ U, const float* __restrict__ K,
    const float* __restrict__ D, const float* __restrict__ Dp, const float* __restrict__ Dx,
    const float* __restrict__ Du, const float* __restrict__ xth, const float* __restrict__ xx,
    const float* __restrict__ xu, float* grad_D, float* __restrict__ grad_d, float* __restrict__ d_x,
    float* __restrict__ d_u) {
  constexpr int n = Model::N, m = Model::M, p = Model::P, d = n + m;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float gx[n][p], Km1[m][n];
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int k = 0; k < p; ++k) gx[i][k] = 0.f;
#pragma unroll
  for (int a = 0; a < m; ++a)
#pragma unroll
    for (int l = 0; l < n; ++l) Km1[a][l] = 0.f;
  float taum1[d];
#pragma unroll
  for (int j = 0; j < d; ++j) taum1[j] = 0.f;
  for (int t = 0; t < T; ++t) {
    const size_t tb = (size_t)t * B + b;
    float Kt[m][n];
    if (K) {
      ld2(Kt, K + tb * m * n);
    } else {
#pragma unroll
      for (int a = 0; a < m; ++a)
#pragma unroll
        for (int l = 0; l < n; ++l) Kt[a][l] = 0.f;
    }
    float tau[d];
    {
      float xt[n], ut[m];
      ld(xt, X + tb * n); ld(ut, U + tb * m);
#pragma unroll
      for (int i = 0; i < n; ++i) tau[i] = xt[i];
#pragma unroll
      for (int a = 0; a < m; ++a) tau[n + a] = ut[a];
    }
    float gxm1[n][p];
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
      for (int k = 0; k < p; ++k) gxm1[i][k] = gx[i][k];
    if (t > 0) {
      const float* xxt = xx + tb * n * n;
      const float* xut = xu + tb * n * m;
      const float* xtht = xth + tb * n * p;
#pragma unroll
      for (int i = 0; i < n; ++i) {
        float A[n];
#pragma unroll
        for (int l = 0; l < n; ++l) {
          float s = 0.f;
#pragma unroll
          for (int a = 0; a < m; ++a) s += xut[i * m + a] * Km1[a][l];
          A[l] = xxt[i * n + l] + s;
        }
#pragma unroll
        for (int k = 0; k < p; ++k) {
          float s = 0.f;
#pragma unroll
          for (int l = 0; l < n; ++l) s += A[l] * gxm1[l][k];
          gx[i][k] = xtht[i * p + k] + s;
        }
      }
    }
    if (t < T - 1) {
      const float* Dpt = Dp + tb * n * d * p;
      const float* Dxt = Dx + tb * n * d * n;
      const float* Dut = Du + tb * n * d * m;
      float* gDt = grad_D + tb * n * d * p;
      float* dxo = d_x + tb * n * n;
      float* duo = d_u + tb * n * m;
      for (int i = 0; i < n; ++i) {
        float ax[n], au[m];
#pragma unroll
        for (int k = 0; k < n; ++k) ax[k] = 0.f;
#pragma unroll
        for (int k = 0; k < m; ++k) au[k] = 0.f;
#pragma unroll
        for (int j = 0; j < d; ++j) {
          float A[n];
#pragma unroll
          for (int l = 0; l < n; ++l) {
            float s = 0.f;
#pragma unroll
            for (int a = 0; a < m; ++a) s += Dut[(i * d + j) * m + a] * Kt[a][l];
            A[l] = Dxt[(i * d + j) * n + l] + s;
            ax[l] += Dxt[(i * d + j) * n + l] * tau[j];
          }
#pragma unroll
          for (int a = 0; a < m; ++a) au[a] += Dut[(i * d + j) * m + a] * tau[j];
#pragma unroll
          for (int k = 0; k < p; ++k) {
            float s = 0.f;
#pragma unroll
            for (int l = 0; l < n; ++l) s += A[l] * gx[l][k];
            gDt[(i * d + j) * p + k] = Dpt[(i * d + j) * p + k] + s;
          }
        }
#pragma unroll
        for (int k = 0; k < n; ++k) dxo[i * n + k] = -ax[k];
#pragma unroll
        for (int a = 0; a < m; ++a) duo[i * m + a] = -au[a];
      }
    }
    if (t > 0) {
      const size_t tb1 = tb - B;                       // step t-1
      const float* gDm1 = grad_D + tb1 * n * d * p;    // written by this lane at step t-1
      const float* Dm1 = D + tb1 * n * d;
      float par[d][p];                                 // [gradx_{t-1}; K_{t-1} gradx_{t-1}]
#pragma unroll
      for (int k = 0; k < p; ++k) {
#pragma unroll
        for (int i = 0; i < n; ++i) par[i][k] = gxm1[i][k];
#pragma unroll
        for (int a = 0; a < m; ++a) {
          float s = 0.f;
#pragma unroll
          for (int l = 0; l < n; ++l) s += Km1[a][l] * gxm1[l][k];
          par[n + a][k] = s;
        }
      }
      float* gdo = grad_d + tb1 * n * p;
      for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < p; ++k) {
          float s1 = 0.f, s2 = 0.f;
#pragma unroll
          for (int j = 0; j < d; ++j) {
            s1 += gDm1[(i * d + j) * p + k] * taum1[j];
            s2 += Dm1[i * d + j] * par[j][k];
          }
          gdo[i * p + k] = (gx[i][k] - s1) - s2;
        }
      }
    }
#pragma unroll
    for (int a = 0; a < m; ++a)
#pragma unroll
      for (int l = 0; l < n; ++l) Km1[a][l] = Kt[a][l];
#pragma unroll
    for (int j = 0; j < d; ++j) taum1[j] = tau[j];
  }
}

}  // namespace dilqr

using namespace dilqr;

#define MODEL_SWITCH_D2(model, CALL)                                                       \
  switch (model) {                                                                         \
    case DILQR_MODEL_PENDULUM: { using MD = Pendulum; using MD2 = gen::PendulumD2; CALL; break; } \
    case DILQR_MODEL_CARTPOLE: { using MD = Cartpole; using MD2 = gen::CartpoleD2; CALL; break; } \
    case DILQR_MODEL_ROCKET: { using MD = Rocket; using MD2 = gen::RocketD2; CALL; break; }       \
    default: return DILQR_E_SHAPE;                                                         \
  }

extern "C" {

int dilqr_get_matrices_f32(int model, int N, const float* theta, const float* x, const float* u, float* D,
                           float* Dp, float* Dx, float* Du, float* xth, float* xx, float* xu, void* stream) {
  if (N < 0 || !theta || !x || !u || !D || !Dp || !Dx || !Du || !xth || !xx || !xu) return DILQR_E_ARG;
  if (dilqr_model_num_ctrl(model) < 0) return DILQR_E_SHAPE;
  if (N == 0) return 0;
  int e = 0;
  MODEL_SWITCH_D2(model, ({
    constexpr int nn = MD::N, mm = MD::M, pp = MD::P, dd = MD::N + MD::M;
    const size_t rows = (size_t)N;
    hipStream_t s = S(stream);
    e = herr(hipMemsetAsync(Dp, 0, rows * nn * dd * pp * sizeof(float), s));
    if (!e) e = herr(hipMemsetAsync(Dx, 0, rows * nn * dd * nn * sizeof(float), s));
    if (!e) e = herr(hipMemsetAsync(Du, 0, rows * nn * dd * mm * sizeof(float), s));
    if (!e) e = herr(hipMemsetAsync(xth, 0, rows * nn * pp * sizeof(float), s));
    if (!e) e = herr(hipMemsetAsync(xx, 0, rows * nn * nn * sizeof(float), s));
    if (e) return e;
    k_get_matrices<MD, MD2><<<grid_for(N), kBlock, 0, s>>>(N, theta, x, u, D, Dp, Dx, Du, xth, xx, xu);
  }));
  return launched();
}

int dilqr_grad_input_f32(int model, int T, int B, const float* X, const float* U, const float* K, const float* D,
                         const float* Dp, const float* Dx, const float* Du, const float* xth, const float* xx,
                         const float* xu, float* grad_D, float* grad_d, float* d_x, float* d_u, void* stream) {
  if (T < 1 || B < 0 || !X || !U || !D || !Dp || !Dx || !Du || !xth || !xx || !xu) return DILQR_E_ARG;
  if (T > 1 && (!grad_D || !grad_d || !d_x || !d_u)) return DILQR_E_ARG;
  if (!al16(K)) return DILQR_E_ARG;
  if (B == 0 || T == 1) return 0;
  MODEL_SWITCH(model, (k_grad_input<MD><<<grid_for(B), kBlock, 0, S(stream)>>>(
                          T, B, X, U, K, D, Dp, Dx, Du, xth, xx, xu, grad_D, grad_d, d_x, d_u)));
  return launched();
}

}  // extern "C"
