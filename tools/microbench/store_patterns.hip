// Microbenchmark: per-lane strided 112-B records (7 x 16-B stores per lane,
// lanes 112 B apart) vs the same bytes staged through LDS and stored
// wave-coalesced; T steps of B records each.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int R4 = 7;   // float4 per record

__global__ void __launch_bounds__(64) k_strided(int T, int B, float4* __restrict__ P) {
  int b = blockIdx.x * 64 + threadIdx.x;
  for (int t = 0; t < T; ++t) {
    float4* p = P + ((size_t)t * B + b) * R4;
#pragma unroll
    for (int j = 0; j < R4; ++j) p[j] = make_float4(t, j, b, 1.f);
  }
}

__global__ void __launch_bounds__(64) k_staged(int T, int B, float4* __restrict__ P) {
  __shared__ float4 s[64 * R4];
  int b0 = blockIdx.x * 64;
  for (int t = 0; t < T; ++t) {
#pragma unroll
    for (int j = 0; j < R4; ++j) s[threadIdx.x * R4 + j] = make_float4(t, j, b0 + threadIdx.x, 1.f);
    __syncthreads();
    float4* p = P + ((size_t)t * B + b0) * R4;
#pragma unroll
    for (int j = 0; j < R4; ++j) p[threadIdx.x + 64 * j] = s[threadIdx.x + 64 * j];
    __syncthreads();
  }
}

int main() {
  const int T = 25, B = 65536;
  size_t n4 = (size_t)T * B * R4;
  float4* P;
  (void)hipMalloc(&P, n4 * 16);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int kind = 0; kind < 2; ++kind)
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(a);
      for (int i = 0; i < 10; ++i) {
        if (kind == 0) k_strided<<<B / 64, 64>>>(T, B, P);
        else k_staged<<<B / 64, 64>>>(T, B, P);
      }
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      printf("%s: %.1f us/launch, %.2f TB/s\n", kind ? "staged" : "strided", ms * 100, n4 * 16 / (ms / 10 * 1e-3) / 1e12);
    }
  return 0;
}
