// Microbenchmark: per-lane strided 144-B rows (thread-per-problem layout of
// C [T,B,6,6]) vs the same bytes loaded wave-coalesced, T steps in sequence.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int D2 = 36;   // floats per (t,b) block

__global__ void __launch_bounds__(64) k_strided(int T, int B, const float4* __restrict__ C, float* out) {
  int b = blockIdx.x * 64 + threadIdx.x;
  float acc = 0.f;
  for (int t = 0; t < T; ++t) {
    const float4* p = C + ((size_t)t * B + b) * (D2 / 4);
    float4 v[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) v[j] = p[j];
#pragma unroll
    for (int j = 0; j < 9; ++j) acc += v[j].x + v[j].y + v[j].z + v[j].w;
  }
  out[b] = acc;
}

__global__ void __launch_bounds__(64) k_coalesced(int T, int B, const float4* __restrict__ C, float* out) {
  __shared__ float4 s[64 * 9];
  int b0 = blockIdx.x * 64;
  float acc = 0.f;
  for (int t = 0; t < T; ++t) {
    const float4* p = C + ((size_t)t * B + b0) * (D2 / 4);
    float4 v[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) v[j] = p[threadIdx.x + 64 * j];
#pragma unroll
    for (int j = 0; j < 9; ++j) s[threadIdx.x + 64 * j] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 9; ++j) { float4 w = s[threadIdx.x * 9 + j]; acc += w.x + w.y + w.z + w.w; }
    __syncthreads();
  }
  out[b0 + threadIdx.x] = acc;
}

int main() {
  const int T = 100, B = 65536;
  size_t nf = (size_t)T * B * D2;
  float4* C; float* out;
  hipMalloc(&C, nf * 4); hipMalloc(&out, B * 4);
  hipMemset(C, 0, nf * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int kind = 0; kind < 2; ++kind) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      for (int i = 0; i < 10; ++i) {
        if (kind == 0) k_strided<<<B / 64, 64>>>(T, B, C, out);
        else k_coalesced<<<B / 64, 64>>>(T, B, C, out);
      }
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("%s: %.1f us/launch, %.2f TB/s\n", kind ? "coalesced" : "strided", ms * 100, nf * 4 / (ms / 10 * 1e-3) / 1e12);
    }
  }
  return 0;
}
