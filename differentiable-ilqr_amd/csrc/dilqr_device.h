// dilqr_device.h — device building blocks of the batched iLQR hot path (gfx950).
//
// Mapping: ONE PROBLEM PER LANE ("thread per problem", TPP).  The per-step
// matrices of a problem are tiny (cartpole: C 6x6, F 5x6, V 5x5), so a lane
// keeps its problem's V, v, Q, gains and trajectory state in VGPRs with every
// index a compile-time constant (all loops fully unrolled), and a wave runs 64
// independent problems in lock-step with no cross-lane traffic at all.  Each
// lane's per-step record in HBM ([T,B,...] time-major, as the reference lays it
// out) is contiguous, and the 64 records a wave touches at step t are adjacent,
// so a wave's loads of one step stream one contiguous span of HBM.
//
// Everything here restates the reference math (file:line cited per routine);
// only the batch mapping differs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dilqr.h"

#define DEV __device__ __forceinline__

namespace dilqr {

// two floats in a VGPR pair: arithmetic on it compiles to the packed fp32 VALU
// ops (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32), two FMAs per lane per issue
typedef float f2 __attribute__((ext_vector_type(2)));

// Scalar-generic elementary functions: the model code is written once for a
// float and for an f2 holding the same quantity of two independent
// trajectories (the line search's two candidates).  Each f2 component gets
// exactly the float operation (IEEE +,-,*,/ per component; the libm calls per
// component), so a packed evaluation rounds like two scalar ones.
DEV float vatan2(float y, float x) { return atan2f(y, x); }
DEV f2 vatan2(f2 y, f2 x) { return f2{atan2f(y.x, x.x), atan2f(y.y, x.y)}; }
DEV float vcos(float x) { return cosf(x); }
DEV f2 vcos(f2 x) { return f2{cosf(x.x), cosf(x.y)}; }
DEV float vsin(float x) { return sinf(x); }
DEV f2 vsin(f2 x) { return f2{sinf(x.x), sinf(x.y)}; }
// sin and cos of one angle with one argument reduction (ocml's sincos shares
// sin's and cos's reduction and polynomials: bit-identical to sinf/cosf —
// checked over 6.1e8 inputs spanning every exponent by
// tools/microbench/sincos_bits.hip on MI355X)
DEV void vsincos(float x, float& s, float& c) { sincosf(x, &s, &c); }
DEV void vsincos(f2 x, f2& s, f2& c) {
  float s0, c0, s1, c1;
  sincosf(x.x, &s0, &c0);
  sincosf(x.y, &s1, &c1);
  s = f2{s0, s1};
  c = f2{c0, c1};
}
DEV float vclamp(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
DEV f2 vclamp(f2 x, float lo, float hi) { return f2{fminf(fmaxf(x.x, lo), hi), fminf(fmaxf(x.y, lo), hi)}; }

// Hardware reciprocal / reciprocal square root (v_rcp_f32 / v_rsq_f32, 1 ulp)
// and explicit fused multiply-add, per component.
DEV float vrcp(float x) { return __builtin_amdgcn_rcpf(x); }
DEV f2 vrcp(f2 x) { return f2{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)}; }
DEV float vrsq(float x) { return __builtin_amdgcn_rsqf(x); }
DEV f2 vrsq(f2 x) { return f2{__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)}; }
DEV float vfma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
DEV f2 vfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// sin and cos of a moderate angle: Cody-Waite reduction by pi/2 (three-part
// constant, fma), minimax polynomials on [-pi/4, pi/4] (Cephes sinf/cosf
// coefficients), quadrant fix-up.  |d| > 8192, inf and NaN take ocml's sincosf.
// The polynomial part is written once for float and f2, so the two
// line-search candidates evaluate it as packed fp32 ops.
DEV void sincos_quadrant(int q, float s1, float c1, float& s, float& c) {
  const float ss = (q & 1) ? c1 : s1, cc = (q & 1) ? s1 : c1;
  s = (q & 2) ? -ss : ss;
  c = ((q + 1) & 2) ? -cc : cc;
}
// The sine and cosine chains written interleaved, step by step (the same
// operations, so the same bits): on gfx950 a packed-math result read by the
// next instruction costs a wait state (s_nop), and alternating the two
// independent chains gives each result one instruction of distance.
template <class S>
DEV void sincos_poly(S r, S& s1, S& c1) {
  const S z = r * r;
  S a = vfma(S(-1.9515295891e-4f), z, S(8.3321608736e-3f));
  S b = vfma(S(2.443315711809948e-5f), z, S(-1.388731625493765e-3f));
  a = vfma(a, z, S(-1.6666654611e-1f));
  b = vfma(b, z, S(4.166664568298827e-2f));
  const S zz = z * z;
  const S h = S(-0.5f) * z;
  a = a * z;
  b = vfma(b, zz, h);
  s1 = vfma(a, r, r);
  c1 = b + S(1.0f);
}
// The reduction-and-polynomial path runs unconditionally (branch-free);
// lanes whose argument is out of its range are patched afterwards in a branch
// that a wave skips when none of its lanes needs it.
DEV void sincos_fast(float d, float& s, float& c) {
  const float k = __builtin_rintf(d * 0.636619772f);
  if (__builtin_amdgcn_ballot_w64(!(k == 0.f)) == 0) {     // |d| <= pi/4 wave-wide: see the f2 form
    sincos_poly(d, s, c);
    return;
  }
  float r = vfma(-k, 1.5703125f, d);
  r = vfma(-k, 4.837512969970703125e-4f, r);
  r = vfma(-k, 7.54978995489188216e-8f, r);
  float s1, c1;
  sincos_poly(r, s1, c1);
  sincos_quadrant((int)k, s1, c1, s, c);
  if (__builtin_expect(!(fabsf(d) <= 8192.f), 0)) sincosf(d, &s, &c);
}
DEV void sincos_fast(f2 d, f2& s, f2& c) {
  const f2 k = f2{__builtin_rintf(d.x * 0.636619772f), __builtin_rintf(d.y * 0.636619772f)};
  // The usual case, |d| <= pi/4 in every lane of the wave (k = 0: the
  // reduction leaves r = d exactly and the quadrant fix-up is the identity):
  // the polynomials alone, the same values bit for bit, ~25 fewer instructions.
  if (__builtin_amdgcn_ballot_w64(!(k.x == 0.f && k.y == 0.f)) == 0) {
    sincos_poly(d, s, c);
    return;
  }
  f2 r = vfma(-k, f2(1.5703125f), d);
  r = vfma(-k, f2(4.837512969970703125e-4f), r);
  r = vfma(-k, f2(7.54978995489188216e-8f), r);
  f2 s1, c1;
  sincos_poly(r, s1, c1);
  float sa, ca, sb, cb;
  sincos_quadrant((int)k.x, s1.x, c1.x, sa, ca);
  sincos_quadrant((int)k.y, s1.y, c1.y, sb, cb);
  if (__builtin_expect(!(fabsf(d.x) <= 8192.f) || !(fabsf(d.y) <= 8192.f), 0)) {
    if (!(fabsf(d.x) <= 8192.f)) sincosf(d.x, &sa, &ca);
    if (!(fabsf(d.y) <= 8192.f)) sincosf(d.y, &sb, &cb);
  }
  s = f2{sa, sb}; c = f2{ca, cb};
}

// cos and sin of atan2(s, c) + delta without the atan2 (the angle update of the
// pendulum and cartpole dynamics, pendulum.py:88-93, cartpole.py:87-95): with
// r = |(c, s)|, cos(atan2(s, c)) = c / r and sin(atan2(s, c)) = s / r, so the
// angle-sum formulas need sin and cos of the small increment delta only.
// atan2(0, 0) = 0: a zero (c, s) acts as (1, 0).
template <class S>
DEV void angle_step(S c, S s, S delta, S& co, S& so) {
  S sd, cd;
  sincos_fast(delta, sd, cd);
  const S r2 = c * c + s * s;
  const S ir = vrsq(r2);
  S cn = c * ir, sn = s * ir;
  if constexpr (sizeof(S) == sizeof(float)) {
    if (r2 == 0.f) { cn = 1.f; sn = 0.f; }
  } else {
    if (r2.x == 0.f) { cn.x = 1.f; sn.x = 0.f; }
    if (r2.y == 0.f) { cn.y = 1.f; sn.y = 0.f; }
  }
  co = cn * cd - sn * sd;
  so = sn * cd + cn * sd;
}

// ------------------------------------------------------------------ loads/stores
// Vectorised load/store of one lane's contiguous record of K floats.  Record
// offsets are multiples of K floats and the base is 16-byte aligned (checked on
// the host), so K%4==0 -> dwordx4, K%2==0 -> dwordx2.
template <int K>
DEV void ld(float (&r)[K], const float* __restrict__ p) {
  if constexpr (K % 4 == 0) {
    const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int i = 0; i < K / 4; ++i) {
      float4 v = q[i];
      r[4 * i] = v.x; r[4 * i + 1] = v.y; r[4 * i + 2] = v.z; r[4 * i + 3] = v.w;
    }
  } else if constexpr (K % 2 == 0) {
    const float2* q = reinterpret_cast<const float2*>(p);
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
      float2 v = q[i];
      r[2 * i] = v.x; r[2 * i + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < K; ++i) r[i] = p[i];
  }
}

template <int K>
DEV void st(float* __restrict__ p, const float (&r)[K]) {
  if constexpr (K % 4 == 0) {
    float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
    for (int i = 0; i < K / 4; ++i) q[i] = make_float4(r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]);
  } else if constexpr (K % 2 == 0) {
    float2* q = reinterpret_cast<float2*>(p);
#pragma unroll
    for (int i = 0; i < K / 2; ++i) q[i] = make_float2(r[2 * i], r[2 * i + 1]);
  } else {
#pragma unroll
    for (int i = 0; i < K; ++i) p[i] = r[i];
  }
}

template <int R, int Cc>
DEV void ld2(float (&r)[R][Cc], const float* __restrict__ p) {
  ld<R * Cc>(*reinterpret_cast<float(*)[R * Cc]>(&r[0][0]), p);
}
// st with non-temporal stores (write-once outputs nothing in the kernel
// reads back: the implicit backward's dC), K a multiple of 4
typedef float f4 __attribute__((ext_vector_type(4)));
template <int K>
DEV void st_nt(float* __restrict__ p, const float (&r)[K]) {
  static_assert(K % 4 == 0, "16-byte pieces");
  f4* q = reinterpret_cast<f4*>(p);
#pragma unroll
  for (int i = 0; i < K / 4; ++i) __builtin_nontemporal_store(f4{r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]}, q + i);
}

template <int R, int Cc>
DEV void st2(float* __restrict__ p, const float (&r)[R][Cc]) {
  st<R * Cc>(p, *reinterpret_cast<const float(*)[R * Cc]>(&r[0][0]));
}

// ------------------------------------------------------------------ bounds
// records of K floats stored as column planes of the widest vector loads:
// K/4 float4 planes, then a float2 plane if K%4 >= 2, then a float plane if K
// is odd (plane q of width w: w*[(t*nq + q)*B + b] floats from its base).
// Fewer, wider load instructions than K scalar planes (measured: 27 dword
// planes ran the fused kernel 8% slower than 7 float4 planes).
template <int K>
struct SoaRec {
  static constexpr int Q4 = K / 4, R2 = (K % 4) >= 2 ? 1 : 0, R1 = K % 2;
  static DEV size_t off2(int T, int B) { return (size_t)T * B * Q4 * 4; }
  static DEV size_t off1(int T, int B) { return off2(T, B) + (size_t)T * B * 2 * R2; }
  static DEV void load(float (&r)[K], const float* __restrict__ p, int T, size_t t, int B, int b) {
    const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int j = 0; j < Q4; ++j) {
      float4 v = q[(t * Q4 + j) * B + b];
      r[4 * j] = v.x; r[4 * j + 1] = v.y; r[4 * j + 2] = v.z; r[4 * j + 3] = v.w;
    }
    if constexpr (R2) {
      float2 v = reinterpret_cast<const float2*>(p + off2(T, B))[t * B + b];
      r[4 * Q4] = v.x; r[4 * Q4 + 1] = v.y;
    }
    if constexpr (R1) r[K - 1] = (p + off1(T, B))[t * B + b];
  }
  static DEV void store(float* __restrict__ p, const float (&r)[K], int T, size_t t, int B, int b) {
    float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
    for (int j = 0; j < Q4; ++j) q[(t * Q4 + j) * B + b] = make_float4(r[4 * j], r[4 * j + 1], r[4 * j + 2], r[4 * j + 3]);
    if constexpr (R2) reinterpret_cast<float2*>(p + off2(T, B))[t * B + b] = make_float2(r[4 * Q4], r[4 * Q4 + 1]);
    if constexpr (R1) (p + off1(T, B))[t * B + b] = r[K - 1];
  }
};

struct Bounds {
  int mode;
  float lo, hi;
  const float* __restrict__ lo_t;
  const float* __restrict__ hi_t;
};

// util.eclamp (util.py:58-72): x<lo -> lo, x>hi -> hi, written exactly (the
// equality tests of pnqp.py:32 depend on it).  NaN stays NaN.
DEV float eclamp(float x, float lo, float hi) {
  x = (x < lo) ? lo : x;
  x = (x > hi) ? hi : x;
  return x;
}

// ------------------------------------------------------------------ small solves
// Gaussian elimination with partial pivoting for an MxM system with R right-hand
// sides, everything in registers (M<=4).  Used for Q_uu^{-1} (pinverse of a
// nonsingular matrix), pnqp's masked LU (pnqp.py:53-54) and lu_solve of the
// free block (lqr_step_explicit.py:150).
// RCP: each pivot's reciprocal is v_rcp_f32 (1 ulp), formed once for the
// elimination and the back substitution, instead of the IEEE division's
// ~10-instruction sequence (the 16-lane group gain solves, one per lane per
// step; results agree with the division to a few ulp).
template <int M, int R, bool RCP = false>
DEV void gauss_solve(float (&A)[M][M], float (&X)[M][R]) {
  float invs[M];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    // pivot search (compile-time indexed conditional swaps keep data in VGPRs)
    int p = k;
    float best = fabsf(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < M; ++i) {
      float a = fabsf(A[i][k]);
      if (a > best) { best = a; p = i; }
    }
#pragma unroll
    for (int i = k + 1; i < M; ++i) {
      if (p == i) {
#pragma unroll
        for (int j = 0; j < M; ++j) { float t = A[k][j]; A[k][j] = A[i][j]; A[i][j] = t; }
#pragma unroll
        for (int j = 0; j < R; ++j) { float t = X[k][j]; X[k][j] = X[i][j]; X[i][j] = t; }
      }
    }
    float inv = RCP ? __builtin_amdgcn_rcpf(A[k][k]) : 1.0f / A[k][k];
    invs[k] = inv;
#pragma unroll
    for (int i = k + 1; i < M; ++i) {
      float l = A[i][k] * inv;
#pragma unroll
      for (int j = k + 1; j < M; ++j) A[i][j] -= l * A[k][j];
#pragma unroll
      for (int j = 0; j < R; ++j) X[i][j] -= l * X[k][j];
    }
  }
#pragma unroll
  for (int k = M - 1; k >= 0; --k) {
    const float inv = invs[k];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      float s = X[k][j];
#pragma unroll
      for (int i = k + 1; i < M; ++i) s -= A[k][i] * X[i][j];
      X[k][j] = s * inv;
    }
  }
}

// Cholesky solve (A + 0 already regularised by the caller), lqr_step_backup.py:202-204.
template <int M, int R>
DEV void chol_solve(const float (&A)[M][M], float (&X)[M][R]) {
  float L[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = 0; j < M; ++j) L[i][j] = 0.f;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    float s = A[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
    float d = sqrtf(s);
    L[j][j] = d;
    float inv = 1.0f / d;
#pragma unroll
    for (int i = j + 1; i < M; ++i) {
      float t = A[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
      L[i][j] = t * inv;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float y[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      float s = X[i][r];
#pragma unroll
      for (int k = 0; k < i; ++k) s -= L[i][k] * y[k];
      y[i] = s / L[i][i];
    }
#pragma unroll
    for (int i = M - 1; i >= 0; --i) {
      float s = y[i];
#pragma unroll
      for (int k = i + 1; k < M; ++k) s -= L[k][i] * X[k][r];
      X[i][r] = s / L[i][i];
    }
  }
}

// ------------------------------------------------------------------ pnqp
// Projected-Newton box QP  min 1/2 x^T H x + q^T x, lb <= x <= ub, pnqp.py:5-82,
// evaluated for ONE problem (the reference's semantics at batch size 1).
// Returns the iteration index at exit (pnqp.py:59 / 82); writes x, the free
// mask If and the masked matrix H_ (whose inverse gives the gains).
template <int M>
DEV int pnqp(const float (&H)[M][M], const float (&q)[M], const float (&lb)[M],
             const float (&ub)[M], bool have_init, float (&x)[M], float (&If)[M],
             float (&Hf)[M][M]) {
  const float GAMMA = 0.1f;
  // m = 1: the reciprocals are v_rcp_f32 (1 ulp) instead of IEEE divisions
  // (~10 instructions each, three per Newton iteration), the stop test's
  // norm of a 1-vector is |dx| and the Armijo ratio is num * rcp(den): each
  // differs from the reference's fp32 value by rounding only, so only a
  // decision sitting on its threshold to within an ulp can go the other way
  // (the parity tests replay decisions and bound such near-ties)
  if (!have_init) {                                     // pnqp.py:14-19
    if constexpr (M == 1) {
      x[0] = -__builtin_amdgcn_rcpf(H[0][0]) * q[0];
    } else {
      float A[M][M], X[M][1];
#pragma unroll
      for (int i = 0; i < M; ++i) {
#pragma unroll
        for (int j = 0; j < M; ++j) A[i][j] = H[i][j];
        X[i][0] = q[i];
      }
      gauss_solve<M, 1>(A, X);
#pragma unroll
      for (int i = 0; i < M; ++i) x[i] = -X[i][0];
    }
  }
#pragma unroll
  for (int i = 0; i < M; ++i) x[i] = eclamp(x[i], lb[i], ub[i]);

  auto obj = [&](const float (&z)[M]) {
    // 0.5*bquad(z,H) + bdot(q,z)  (pnqp.py:11-12, util.py:50-56)
    float quad = 0.f;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      float r = 0.f;
#pragma unroll
      for (int i = 0; i < M; ++i) r += z[i] * H[i][j];
      quad += r * z[j];
    }
    float lin = 0.f;
#pragma unroll
    for (int i = 0; i < M; ++i) lin += q[i] * z[i];
    return 0.5f * quad + lin;
  };

  if constexpr (M == 1) {
    // The common case straight-line (no loop control, no divergence between
    // lanes stopping at iteration 0 or 1): iteration 0's Newton step taken at
    // alpha = 1 by the first Armijo test, iteration 1 stopping.  Exactly the
    // loop's operations in the loop's order, so the same bits; a lane that
    // leaves this path (a second Armijo pass, or no stop at iteration 1) runs
    // the loop below from the start.
    const float h = H[0][0], qq = q[0], l0 = lb[0], u0 = ub[0];
    auto grad = [&](float z) { float s_ = 0.f; s_ += h * z; return s_ + qq; };
    auto obj1 = [&](float z) {
      float r_ = 0.f; r_ += z * h;
      float quad = 0.f; quad += r_ * z;
      float lin = 0.f; lin += qq * z;
      return 0.5f * quad + lin;
    };
    auto newton = [&](float z, float g0, float& If0, float& Hf0) {
      const bool clamped = (z == l0 && g0 > 0.f) || (z == u0 && g0 < 0.f);
      If0 = clamped ? 0.f : 1.f;
      const float gf = clamped ? 0.f : g0;
      Hf0 = ((If0 * If0) != 0.f ? h : 0.f) + 1e-11f;
      return -__builtin_amdgcn_rcpf(Hf0) * gf;
    };
    const float x0 = x[0];
    const float g0 = grad(x0);
    float If0, Hf0;
    const float dx0 = newton(x0, g0, If0, Hf0);
    if (!(fabsf(dx0) >= 1e-4f)) { If[0] = If0; Hf[0][0] = Hf0; return 0; }
    const float alpha = 1.f;
    const float x1 = eclamp(x0 + alpha * dx0, l0, u0);
    const float den = 0.f + g0 * (x0 - x1);
    const float armijo = (obj1(x0) - obj1(x1)) * __builtin_amdgcn_rcpf(den);
    if (!(armijo <= GAMMA)) {
      const float g1 = grad(x1);
      float If1, Hf1;
      const float dx1 = newton(x1, g1, If1, Hf1);
      if (!(fabsf(dx1) >= 1e-4f)) { x[0] = x1; If[0] = If1; Hf[0][0] = Hf1; return 1; }
    }
  }
  int it = 0;
  for (it = 0; it < 20; ++it) {                         // pnqp.py:28-78
    float g[M], g_[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < M; ++j) s += H[i][j] * x[j];
      g[i] = s + q[i];
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
      bool clamped = (x[i] == lb[i] && g[i] > 0.f) || (x[i] == ub[i] && g[i] < 0.f);
      If[i] = clamped ? 0.f : 1.f;
      g_[i] = clamped ? 0.f : g[i];
    }
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = 0; j < M; ++j)
        Hf[i][j] = ((If[i] * If[j]) != 0.f ? H[i][j] : 0.f) + (i == j ? 1e-11f : 0.f);
    float dx[M];
    if constexpr (M == 1) {
      dx[0] = -__builtin_amdgcn_rcpf(Hf[0][0]) * g_[0];
    } else {
      float A[M][M], X[M][1];
#pragma unroll
      for (int i = 0; i < M; ++i) {
#pragma unroll
        for (int j = 0; j < M; ++j) A[i][j] = Hf[i][j];
        X[i][0] = g_[i];
      }
      gauss_solve<M, 1>(A, X);
#pragma unroll
      for (int i = 0; i < M; ++i) dx[i] = -X[i][0];
    }
    if constexpr (M == 1) {
      if (!(fabsf(dx[0]) >= 1e-4f)) return it;          // pnqp.py:56-59 (per problem)
    } else {
      float nrm = 0.f;
#pragma unroll
      for (int i = 0; i < M; ++i) nrm += dx[i] * dx[i];
      if (!(sqrtf(nrm) >= 1e-4f)) return it;
    }

    float alpha = 1.f;
    float ox = obj(x);
    float maybe[M];
    int count = 0;
    float max_armijo = GAMMA;
    while (max_armijo <= GAMMA && count < 10) {         // pnqp.py:65-76
#pragma unroll
      for (int i = 0; i < M; ++i) maybe[i] = eclamp(x[i] + alpha * dx[i], lb[i], ub[i]);
      float den = 0.f;
#pragma unroll
      for (int i = 0; i < M; ++i) den += g[i] * (x[i] - maybe[i]);
      float armijo = (M == 1) ? (ox - obj(maybe)) * __builtin_amdgcn_rcpf(den) : (ox - obj(maybe)) / den;
      if (armijo <= GAMMA) alpha *= 0.1f;
      max_armijo = armijo;
      ++count;
    }
    // The loop's only state is x: an iteration that leaves x unchanged bit for
    // bit (every Armijo pass failed and x + 1e-9 dx rounds to x: g is rounding
    // noise on a tiny Q_uu, e.g. the last step's C_uu = 0.001 of cartpole) is
    // repeated verbatim by every later one, so the loop's result is this one's:
    // x, If, Hf and i = 19 (config 4: 0.5 % of problems, a quarter of the waves,
    // used to spend ~17 more iterations of 10 Armijo passes each)
    bool same = true;
#pragma unroll
    for (int i = 0; i < M; ++i) same &= __float_as_uint(maybe[i]) == __float_as_uint(x[i]);
    if (same) return 19;
#pragma unroll
    for (int i = 0; i < M; ++i) x[i] = maybe[i];
  }
  return 19;                                            // pnqp.py:80-82 (i after the loop)
}

// ------------------------------------------------------------------ Riccati step
// One step of lqr_backward (lqr_step_explicit.py:63-160) for one problem.
//   in : C_t [D][D], cb_t [D] (= C_t tau_t + c_t), F_t [N][D] (zero for t = T-1,
//        which makes Q = C exactly), V/v of step t+1 (zero at t = T-1)
//   out: K_t [M][N], k_t [M]; V/v of step t.
enum GainMode { GAIN_UNC = 0, GAIN_CHOL = 1, GAIN_ZERO_I = 2, GAIN_BOX = 3 };

// Dense F by default; a model's Jacobian can declare its structural zeros
// (static constexpr bool nz(i, j)) so the fused kernel skips those products.
struct DenseF {
  static constexpr bool nz(int, int) { return true; }
};

// A sum of products whose first term starts it (s = a*b, then s += a*b): no
// leading "0 +" — which the compiler must keep (0 + -0 is +0) and which costs
// an instruction wherever the first factor is a literal 1 the product folds
// away (a Jacobian's identity entries).  The values equal the 0-started sum's
// except for the sign of an exact zero.  Under full unrolling `first` is a
// compile-time constant.
#ifndef DILQR_ACC0
#define DILQR_ACC0 0                        // 1: the 0-started sums (A/B builds)
#endif
struct Acc {
  float s = 0.f;
  bool first = true;
  DEV void add(float a, float b) {
    if (first && !DILQR_ACC0) s = a * b;
    else s += a * b;
    first = false;
  }
};

template <int D>
DEV bool bitwise_symmetric(const float (&C)[D][D]) {
  unsigned asym = 0u;                       // an xor/or reduction, one compare
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = i + 1; j < D; ++j) asym |= __float_as_uint(C[i][j]) ^ __float_as_uint(C[j][i]);
  return asym == 0u;
}

template <int N, int M>
struct RiccatiState {
  static constexpr int D = N + M;
  float V[N][N];
  float v[N];
  float prev_k[M];     // pnqp warm start (lqr_step_explicit.py:137-143)
  bool have_prev;
  int n_qp;

  DEV void init() {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      v[i] = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) V[i][j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < M; ++i) prev_k[i] = 0.f;
    have_prev = false;
    n_qp = 0;
  }

  // mode GAIN_ZERO_I uses zI[M] (1 = active); GAIN_BOX uses lb/ub [M] (already
  // lower-u_t / upper-u_t, lqr_step_explicit.py:132-133).
  // SYM: C_t and every later C are bitwise symmetric (so V_{t+1} is, as this
  // mode keeps it): F^T V F is formed as F^T (V F) on and above the diagonal
  // and mirrored, and V_t likewise — the products of the upper triangle only
  // (cartpole: 118 instead of 187 for Q, 15 instead of 25 entries of V).  The
  // mirrored entries are the exact-arithmetic values; in fp32 they differ from
  // the full products by rounding, as any two summation orders do.  Every
  // caller that must agree bit for bit (the fused and the unfused sweep) picks
  // SYM by the same rule: all C_t' (t' >= t) of the problem bitwise symmetric.
  template <int MODE, class FS = DenseF, bool DIAG = false, bool SYM = false>
  DEV void step(const float (&C)[D][D], const float (&cb)[D], const float (&F)[N][D],
                const float (&zI)[M], const float (&lb)[M], const float (&ub)[M],
                float (&K)[M][N], float (&k)[M]) {
    float Q[D][D], q[D];
    if constexpr (SYM) {
      // W = V F (N x D), S = F^T W on and above the diagonal
      float W[N][D];
#pragma unroll
      for (int l = 0; l < N; ++l)
#pragma unroll
        for (int j = 0; j < D; ++j) {
          Acc s;
#pragma unroll
          for (int kk = 0; kk < N; ++kk)
            if (FS::nz(kk, j)) s.add(V[l][kk], F[kk][j]);
          W[l][j] = s.s;
        }
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int j = i; j < D; ++j) {
          Acc a;
#pragma unroll
          for (int l = 0; l < N; ++l)
            if (FS::nz(l, i)) a.add(F[l][i], W[l][j]);
          const float s = a.s;
          Q[i][j] = (DIAG && i != j) ? s : C[i][j] + s;     // DIAG: C[i][j] is +0.0
          if (j != i) Q[j][i] = (DIAG) ? s : C[j][i] + s;
        }
    } else {
      // Q = C + (F^T V) F   (lqr_step_explicit.py:68-72)
      float P[D][N];
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int kk = 0; kk < N; ++kk) {
          Acc s;
#pragma unroll
          for (int l = 0; l < N; ++l)
            if (FS::nz(l, i)) s.add(F[l][i], V[l][kk]);
          P[i][kk] = s.s;
        }
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int j = 0; j < D; ++j) {
          Acc a;
#pragma unroll
          for (int kk = 0; kk < N; ++kk)
            if (FS::nz(kk, j)) a.add(P[i][kk], F[kk][j]);
          const float s = a.s;
          Q[i][j] = (DIAG && i != j) ? s : C[i][j] + s;     // DIAG: C[i][j] is +0.0
        }
    }
    // q = cb + F^T v
#pragma unroll
    for (int i = 0; i < D; ++i) {
      Acc s;
#pragma unroll
      for (int l = 0; l < N; ++l)
        if (FS::nz(l, i)) s.add(F[l][i], v[l]);
      q[i] = cb[i] + s.s;
    }
    // partitions (lqr_step_explicit.py:78-83)
    float Quu[M][M], qu[M];
#pragma unroll
    for (int a = 0; a < M; ++a) {
      qu[a] = q[N + a];
#pragma unroll
      for (int b = 0; b < M; ++b) Quu[a][b] = Q[N + a][N + b];
    }

    if constexpr (MODE == GAIN_UNC && M == 1) {          // lqr_step_explicit.py:86-88
      // v_rcp_f32 (1 ulp) instead of the correctly rounded 1/Q_uu, whose IEEE
      // division expands to ~10 instructions (div_scale/fmas/fixup) per step;
      // the reference's -Q_ux/Q_uu and this -(r*Q_ux) differ by rounding either way
      float r = __builtin_amdgcn_rcpf(Quu[0][0]);
#pragma unroll
      for (int j = 0; j < N; ++j) K[0][j] = -(r * Q[N][j]);
      k[0] = -(r * qu[0]);
    } else if constexpr (MODE == GAIN_UNC || MODE == GAIN_CHOL) {
      // pinverse (90-96) / cholesky(Q_uu + 1e-6 I) (lqr_step_backup.py:199-208)
      float A[M][M], X[M][N + 1];
#pragma unroll
      for (int a = 0; a < M; ++a) {
#pragma unroll
        for (int b = 0; b < M; ++b) A[a][b] = Quu[a][b] + ((MODE == GAIN_CHOL && a == b) ? 1e-6f : 0.f);
#pragma unroll
        for (int j = 0; j < N; ++j) X[a][j] = Q[N + a][j];
        X[a][N] = qu[a];
      }
      if constexpr (MODE == GAIN_CHOL) chol_solve<M, N + 1>(A, X);
      else gauss_solve<M, N + 1>(A, X);
#pragma unroll
      for (int a = 0; a < M; ++a) {
#pragma unroll
        for (int j = 0; j < N; ++j) K[a][j] = -X[a][j];
        k[a] = -X[a][N];
      }
    } else if constexpr (MODE == GAIN_ZERO_I) {          // lqr_step_backup.py:210-232
      float A[M][M], X[M][N + 1];
#pragma unroll
      for (int a = 0; a < M; ++a) {
        bool Ia = zI[a] != 0.f;
#pragma unroll
        for (int b = 0; b < M; ++b) {
          bool free_ab = (zI[a] == 0.f) && (zI[b] == 0.f);
          A[a][b] = (free_ab ? Quu[a][b] : 0.f) + ((a == b && Ia) ? 1e-8f : 0.f);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) X[a][j] = Ia ? 0.f : Q[N + a][j];
        X[a][N] = Ia ? 0.f : qu[a];
      }
      if constexpr (M == 1) {
        float r = 1.0f / A[0][0];
#pragma unroll
        for (int j = 0; j < N; ++j) K[0][j] = -(r * X[0][j]);
        k[0] = -((1.0f / Quu[0][0]) * X[0][N]);          // note: the UNMASKED Q_uu (124-125)
      } else {
        gauss_solve<M, N + 1>(A, X);
#pragma unroll
        for (int a = 0; a < M; ++a) {
#pragma unroll
          for (int j = 0; j < N; ++j) K[a][j] = -X[a][j];
          k[a] = -X[a][N];
        }
      }
    } else {                                             // GAIN_BOX: pnqp (130-150)
      float x[M], If[M], Hf[M][M];
#pragma unroll
      for (int a = 0; a < M; ++a) x[a] = prev_k[a];
      int it = pnqp<M>(Quu, qu, lb, ub, have_prev, x, If, Hf);
      n_qp += 1 + it;
#pragma unroll
      for (int a = 0; a < M; ++a) { k[a] = x[a]; prev_k[a] = x[a]; }
      have_prev = true;
      if constexpr (M == 1) {
        float r = __builtin_amdgcn_rcpf(Hf[0][0]);
#pragma unroll
        for (int j = 0; j < N; ++j) K[0][j] = -(r * (If[0] != 0.f ? Q[N][j] : 0.f));
      } else {
        float X[M][N];
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
          for (int j = 0; j < N; ++j) X[a][j] = If[a] != 0.f ? Q[N + a][j] : 0.f;
        gauss_solve<M, N>(Hf, X);
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
          for (int j = 0; j < N; ++j) K[a][j] = -X[a][j];
      }
    }

    // V = Qxx + Qxu K + K^T Qux + (K^T Quu) K ; v = qx + Qxu k + K^T qu + (K^T Quu) k
    // (lqr_step_explicit.py:157-160).  Unconstrained m = 1, where K = -Qux/Quu and
    // k = -qu/Quu: the last two terms cancel (K^T Qux = -(K^T Quu) K, K^T qu =
    // -(K^T Quu) k), leaving the Schur complement V = Qxx + Qxu K, v = qx + Qxu k.
    if constexpr (MODE == GAIN_UNC && M == 1) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int j = SYM ? i : 0; j < N; ++j) {
          V[i][j] = Q[i][N] * K[0][j] + Q[i][j];
          if (SYM && j != i) V[j][i] = V[i][j];
        }
        v[i] = Q[i][N] * k[0] + q[i];
      }
      return;
    }
    // Box, m = 1: K = -Q_ux / (Q_uu + 1e-11) on a free control, 0 on a clamped
    // one, so K^T Q_ux + K^T Q_uu K = K^T Q_ux (1e-11 / (Q_uu + 1e-11)) — zero to
    // 1e-11 relative, far below fp32 rounding — and V = Q_xx + Q_xu K as above;
    // the k terms keep their exact form, v = q_x + Q_xu k + K^T (q_u + Q_uu k)
    // (pnqp stops within 1e-4 of the box optimum, so q_u + Q_uu k is not ~0)
    if constexpr (MODE == GAIN_BOX && M == 1) {
      const float gk = qu[0] + Quu[0][0] * k[0];
#pragma unroll
      for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int j = SYM ? i : 0; j < N; ++j) {
          V[i][j] = Q[i][N] * K[0][j] + Q[i][j];
          if (SYM && j != i) V[j][i] = V[i][j];
        }
        v[i] = (Q[i][N] * k[0] + q[i]) + K[0][i] * gk;
      }
      return;
    }
    float KtQuu[N][M];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int b = 0; b < M; ++b) {
        float s = 0.f;
#pragma unroll
        for (int a = 0; a < M; ++a) s += K[a][i] * Quu[a][b];
        KtQuu[i][b] = s;
      }
#pragma unroll
    for (int i = 0; i < N; ++i) {
#pragma unroll
      for (int j = SYM ? i : 0; j < N; ++j) {
        float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int a = 0; a < M; ++a) {
          s1 += Q[i][N + a] * K[a][j];
          s2 += K[a][i] * Q[N + a][j];
          s3 += KtQuu[i][a] * K[a][j];
        }
        V[i][j] = ((Q[i][j] + s1) + s2) + s3;
        if (SYM && j != i) V[j][i] = V[i][j];
      }
      float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int a = 0; a < M; ++a) {
        s1 += Q[i][N + a] * k[a];
        s2 += K[a][i] * qu[a];
        s3 += KtQuu[i][a] * k[a];
      }
      v[i] = ((q[i] + s1) + s2) + s3;
    }
  }
};

// 0.5*bquad(tau, C) + bdot(tau, c)  (util.py:130-153 / lqr_step_explicit.py:234);
// also returns C tau (for c_back = C tau + c), and forms the quadratic term as
// tau . (C tau) so the product is computed once.
// DIAG: every off-diagonal C entry is +0.0 (the packed diagonal cost), so the
// row sums reduce to their one nonzero term — the same value the full sum
// rounds to (adding exact zeros changes nothing but the sign of a zero).  The
// full sum also carries the products +0 * tau_j, which are NaN when some tau_j
// is inf or NaN; nonfinite_probe() restores that term (NaN for a non-finite
// tau, a zero otherwise), so a diverged trajectory costs NaN on both paths —
// and the line search accepts a NaN cost (`cost > old` is false,
// lqr_step_explicit.py:180, 249) where it would reject +inf.
template <int D, class S>
DEV S nonfinite_probe(const S (&tau)[D]) {
  const S z = S(0.f);
  S p = z * tau[0];
#pragma unroll
  for (int j = 1; j < D; ++j) p = z * tau[j] + p;
  return p;
}

// C tau alone (the sweep's c_back term when the stage cost itself is not
// needed); the same expressions as quad_cost's, so the same bits
template <int D, bool DIAG = false>
DEV void c_tau(const float (&C)[D][D], const float (&tau)[D], float (&Ctau)[D]) {
  float nf = 0.f;
  if constexpr (DIAG) nf = nonfinite_probe<D>(tau);
#pragma unroll
  for (int i = 0; i < D; ++i) {
    if constexpr (DIAG) {
      Ctau[i] = C[i][i] * tau[i] + nf;
    } else {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < D; ++j) s += C[i][j] * tau[j];
      Ctau[i] = s;
    }
  }
}

template <int D, bool DIAG = false>
DEV float quad_cost(const float (&C)[D][D], const float (&c)[D], const float (&tau)[D],
                    float (&Ctau)[D]) {
  c_tau<D, DIAG>(C, tau, Ctau);
  float quad = 0.f, lin = 0.f;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    quad += tau[i] * Ctau[i];
    lin += tau[i] * c[i];
  }
  return 0.5f * quad + lin;
}

// The stage cost alone, as tau . (tau^T C) (columns); S = float, or f2 for two
// trajectories at once (each component rounds like the float evaluation).
template <int D, bool DIAG = false, class S = float>
DEV S quad_cost(const float (&C)[D][D], const float (&c)[D], const S (&tau)[D]) {
  S quad = S(0.f), nf = S(0.f);
  if constexpr (DIAG) nf = nonfinite_probe<D>(tau);
#pragma unroll
  for (int j = 0; j < D; ++j) {
    S r = S(0.f);
    if constexpr (DIAG) {
      r = tau[j] * C[j][j] + nf;
    } else {
#pragma unroll
      for (int i = 0; i < D; ++i) r += tau[i] * C[i][j];
    }
    quad += r * tau[j];
  }
  S lin = S(0.f);
#pragma unroll
  for (int i = 0; i < D; ++i) lin += tau[i] * c[i];
  return 0.5f * quad + lin;
}

}  // namespace dilqr
