// dilqr_common.h — what every translation unit of libdilqr.so shares: the
// launch geometry, the diagnostic stamp macro, bound accessors, the
// 16-lanes-per-problem building blocks, and the C-ABI argument helpers.
// The library is split into several .hip translation units (Makefile) so that
// the heavy template instantiations compile in parallel; each unit launches
// only the kernels it instantiates.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dilqr_device.h"
#include "dilqr_models.h"

namespace dilqr {

constexpr int kBlock = 64;   // one wave per workgroup: 64 problems, 4 workgroups per CU
                             // at B=65536, freely distributed over the 8 XCDs.
constexpr size_t kLdsPerCU = 160 * 1024;   // CDNA4 LDS per CU
#ifndef DILQR_NO_LDS_GAINS
#define DILQR_NO_LDS_GAINS 0
#endif
constexpr bool kNoLdsGains = DILQR_NO_LDS_GAINS;   // test builds: gain records in HBM always

static inline int grid_for(long long n) { return (int)((n + kBlock - 1) / kBlock); }

// Diagnostic build only (-DDILQR_STAMPS, tools/phase_stamps.py; never the
// shipped library): lane 0 of every wave of the fused MPC iteration writes
// s_memtime at its phase boundaries (kernel entry, after the stop-rule
// prologue, after the sweep, after the line search, exit) and s_memrealtime
// at entry/exit into a buffer of its own that nothing else reads.
#ifdef DILQR_STAMPS
constexpr int kStampSlots = 8, kStampWaves = 4096;
static __device__ unsigned long long g_stamps[kStampWaves * kStampSlots];
#define DILQR_STAMP(k)                                                                     \
  do {                                                                                     \
    const unsigned w_ = (blockIdx.x * blockDim.x + threadIdx.x) / 64u;                     \
    if ((threadIdx.x & 63u) == 0 && w_ < (unsigned)kStampWaves)                             \
      g_stamps[w_ * kStampSlots + (k)] = (k) >= 6 ? __builtin_amdgcn_s_memrealtime()       \
                                                  : __builtin_amdgcn_s_memtime();          \
  } while (0)
#else
#define DILQR_STAMP(k) do {} while (0)
#endif

DEV float bound_lo(const Bounds& bd, long long idx) { return bd.mode == DILQR_BOUNDS_TENSOR ? bd.lo_t[idx] : bd.lo; }
DEV float bound_hi(const Bounds& bd, long long idx) { return bd.mode == DILQR_BOUNDS_TENSOR ? bd.hi_t[idx] : bd.hi; }
}  // namespace dilqr

#include "dilqr_group.h"   // 16-lanes-per-problem kernels (rocket-sized d <= 16)

// ---------------------------------------------------------------- host side
namespace dilqr {
namespace {

inline int herr(hipError_t e) { return e == hipSuccess ? 0 : -(int)e; }
inline int launched() { return herr(hipGetLastError()); }
inline bool al16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline Bounds mkb(const dilqr_bounds& b) { return Bounds{b.mode, b.lo, b.hi, b.lo_t, b.hi_t}; }
inline bool bad_bounds(const dilqr_bounds& b) {
  if (b.mode == DILQR_BOUNDS_TENSOR) return !b.lo_t || !b.hi_t;
  return b.mode != DILQR_BOUNDS_NONE && b.mode != DILQR_BOUNDS_SCALAR;
}

// (n, m) shapes compiled for the generic (LinDx / Riccati / adjoint) kernels.
// Model kernels use their own fixed shapes.
#define DILQR_FOR_EACH_SHAPE(X) X(3, 1) X(5, 1) X(4, 3) X(4, 1) X(2, 1) X(4, 2) X(6, 2) X(6, 1)
// shapes served by the 16-lanes-per-problem kernels (dilqr_group.h)
#define DILQR_FOR_EACH_GROUP_SHAPE(X) X(13, 3)
#define DILQR_FOR_ALL_SHAPES(X) DILQR_FOR_EACH_SHAPE(X) DILQR_FOR_EACH_GROUP_SHAPE(X)

// k_mpc_norm_rows geometry: rows staged in LDS when a block's span fits 64 KiB
struct NormGeom {
  int threads, blocks;
  bool stage;
};
inline NormGeom norm_geom(int TM, int B) {
  int threads = 256;
  while (threads > 64 && (size_t)threads * TM * sizeof(float) > 65536) threads >>= 1;
  const bool stage = (size_t)threads * TM * sizeof(float) <= 65536;
  if (!stage) threads = 256;
  return {threads, (B + threads - 1) / threads, stage};
}

inline int grid_group(long long B) { return (int)((B + kGPW - 1) / kGPW); }

}  // namespace

// every model (per-problem kernels whose state fits a lane: dynamics,
// Jacobians, rollouts)
#define MODEL_SWITCH(model, CALL)                       \
  switch (model) {                                      \
    case DILQR_MODEL_PENDULUM: { using MD = Pendulum; CALL; break; } \
    case DILQR_MODEL_CARTPOLE: { using MD = Cartpole; CALL; break; } \
    case DILQR_MODEL_ROCKET: { using MD = Rocket; CALL; break; }     \
    case DILQR_MODEL_PENDULUM_COMPLEX: { using MD = PendulumComplex; CALL; break; } \
    default: return DILQR_E_SHAPE;                      \
  }
// models whose Riccati state fits one lane (thread-per-problem kernels)
#define MODEL_SWITCH_TPP(model, CALL)                   \
  switch (model) {                                      \
    case DILQR_MODEL_PENDULUM: { using MD = Pendulum; CALL; break; } \
    case DILQR_MODEL_CARTPOLE: { using MD = Cartpole; CALL; break; } \
    case DILQR_MODEL_PENDULUM_COMPLEX: { using MD = PendulumComplex; CALL; break; } \
    default: return DILQR_E_SHAPE;                      \
  }
// ... of those, the models with generated second-order terms (D2Of: the
// implicit backward, the dynamics VJP)
#define MODEL_SWITCH_TPP_D2(model, CALL)                \
  switch (model) {                                      \
    case DILQR_MODEL_PENDULUM: { using MD = Pendulum; CALL; break; } \
    case DILQR_MODEL_CARTPOLE: { using MD = Cartpole; CALL; break; } \
    default: return DILQR_E_SHAPE;                      \
  }
}  // namespace dilqr
