// How fast can iteration 0 stream the caller's cost at one wave per SIMD?
// The fused iteration-0 sweep reads, per step t (backward), each lane's own
// C_t,b (144 B) and c_t,b (24 B): [T,B,6,6] and [T,B,6], B = 65536, T = 25,
// 1024 waves of 64 lanes (one per SIMD).  Variants, each with a dependent FMA
// chain of FMAS instructions per step standing in for the sweep's arithmetic:
//   rec1 / rec2:  lane-own 144-B + 24-B records (9 + 2 dwordx4/x2 per lane),
//                 prefetched one / two steps ahead in registers (the shipped form);
//   coal1 / coal2: the wave's step block (64 x 168 B, contiguous per array)
//                 read coalesced (lane l takes float4 j*64+l), one / two steps
//                 ahead — an upper bound: the values are consumed where they
//                 land, not redistributed to the lanes that own them.
// hipcc -O3 --offload-arch=gfx950 -o c_stream c_stream.hip && ./c_stream
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int T = 25, B = 65536, D = 6;

template <int FMAS>
__device__ __forceinline__ float chain(float acc, const float* v, int nv) {
#pragma unroll
  for (int i = 0; i < FMAS; ++i) acc = __builtin_fmaf(acc, 0.999f, v[i % nv]);
  return acc;
}

template <int PF, int FMAS>
__global__ void __launch_bounds__(64) rec(const float* __restrict__ C, const float* __restrict__ c, float* out) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  float buf[PF + 1][42];
  auto load = [&](int s, int t) {
    const float4* p = reinterpret_cast<const float4*>(C + ((size_t)t * B + b) * 36);
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      float4 v = p[j];
      buf[s][4 * j] = v.x; buf[s][4 * j + 1] = v.y; buf[s][4 * j + 2] = v.z; buf[s][4 * j + 3] = v.w;
    }
    const float2* q = reinterpret_cast<const float2*>(c + ((size_t)t * B + b) * 6);
#pragma unroll
    for (int j = 0; j < 3; ++j) { float2 v = q[j]; buf[s][36 + 2 * j] = v.x; buf[s][37 + 2 * j] = v.y; }
  };
  float acc = 0.f;
#pragma unroll
  for (int s = 0; s < PF; ++s) load(s, T - 1 - s);
  for (int t = T - 1; t >= 0; t -= PF + 1) {
#pragma unroll
    for (int s = 0; s <= PF; ++s) {
      const int tt = t - s;
      if (tt < 0) break;
      const int ahead = tt - PF;
      load((s + PF) % (PF + 1), ahead >= 0 ? ahead : 0);
      acc = chain<FMAS>(acc, buf[s], 42);
    }
  }
  out[b] = acc;
}

template <int PF, int FMAS>
__global__ void __launch_bounds__(64) coal(const float* __restrict__ C, const float* __restrict__ c, float* out) {
  const int lane = threadIdx.x, b0 = blockIdx.x * 64;
  // per step: 576 float4 of C (9 per lane) + 96 float4 of c (lanes 0..31 take 2... use 2 loads, 1.5 avg)
  float4 bc[PF + 1][9], bcc[PF + 1][2];
  auto load = [&](int s, int t) {
    const float4* p = reinterpret_cast<const float4*>(C + ((size_t)t * B + b0) * 36);
#pragma unroll
    for (int j = 0; j < 9; ++j) bc[s][j] = p[j * 64 + lane];
    const float4* q = reinterpret_cast<const float4*>(c + ((size_t)t * B + b0) * 6);
    bcc[s][0] = q[lane];
    bcc[s][1] = lane < 32 ? q[64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float acc = 0.f;
#pragma unroll
  for (int s = 0; s < PF; ++s) load(s, T - 1 - s);
  for (int t = T - 1; t >= 0; t -= PF + 1) {
#pragma unroll
    for (int s = 0; s <= PF; ++s) {
      const int tt = t - s;
      if (tt < 0) break;
      const int ahead = tt - PF;
      load((s + PF) % (PF + 1), ahead >= 0 ? ahead : 0);
      // upper bound: the coalesced registers consumed as they are (no
      // redistribution to the owning lanes)
      float v[42];
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        v[4 * j] = bc[s][j].x; v[4 * j + 1] = bc[s][j].y; v[4 * j + 2] = bc[s][j].z; v[4 * j + 3] = bc[s][j].w;
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) v[36 + j] = j < 4 ? (&bcc[s][0].x)[j] : (&bcc[s][1].x)[j - 4];
      acc = chain<FMAS>(acc, v, 42);
    }
  }
  out[b0 + lane] = acc;
}

template <class K>
float time_it(K k, const float* C, const float* c, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k<<<B / 64, 64>>>(C, c, out);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) k<<<B / 64, 64>>>(C, c, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  float *C, *c, *out;
  const size_t nC = (size_t)T * B * 36, nc = (size_t)T * B * 6;
  hipMalloc(&C, nC * 4); hipMalloc(&c, nc * 4); hipMalloc(&out, B * 4);
  hipMemset(C, 0, nC * 4); hipMemset(c, 0, nc * 4);
  const double bytes = (nC + nc) * 4.0;
#define RUN(NAME, K)                                                                                  \
  {                                                                                                   \
    float ms = time_it(K, C, c, out);                                                                 \
    printf("%-14s %8.1f us  %6.2f TB/s\n", NAME, ms * 1e3, bytes / (ms * 1e-3) / 1e12);               \
  }
  RUN("rec1 f42", (rec<1, 42>)); RUN("rec2 f42", (rec<2, 42>));
  RUN("coal1 f42", (coal<1, 42>)); RUN("coal2 f42", (coal<2, 42>));
  RUN("rec1 f252", (rec<1, 252>)); RUN("rec2 f252", (rec<2, 252>));
  RUN("coal1 f252", (coal<1, 252>)); RUN("coal2 f252", (coal<2, 252>));
  RUN("rec1 f504", (rec<1, 504>)); RUN("coal1 f504", (coal<1, 504>)); RUN("rec3 f252", (rec<3, 252>));
  return 0;
}
