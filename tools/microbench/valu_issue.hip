// VALU issue rate of plain vs packed fp32 FMA chains at one and two waves per
// SIMD (is v_pk_fma_f32 two FMAs per issue slot for a lone wave?).
// hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize -Wno-unused-result -o valu_issue valu_issue.hip && ./valu_issue
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int ACC>
__global__ void __launch_bounds__(64) k_scalar(float* out, float a, float b, int iters) {
  float acc[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_fmaf(acc[i], a, b);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int ACC>
__global__ void __launch_bounds__(64) k_packed(float* out, float a, float b, int iters) {
  f2 acc[ACC / 2];
#pragma unroll
  for (int i = 0; i < ACC / 2; ++i) acc[i] = f2{threadIdx.x * 1e-3f + 2 * i, threadIdx.x * 1e-3f + 2 * i + 1};
  const f2 av = {a, a}, bv = {b, b};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC / 2; ++i) acc[i] = __builtin_elementwise_fma(acc[i], av, bv);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < ACC / 2; ++i) s += acc[i].x + acc[i].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

// the same count of transcendental-free mixed mul/add, scalar vs packed
template <typename K>
float timeit(K kern, int blocks, float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  kern<<<blocks, 64>>>(out, 1.0000001f, 1e-7f, iters);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) kern<<<blocks, 64>>>(out, 1.0000001f, 1e-7f, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  float* out;
  hipMalloc(&out, 64 * 8192 * sizeof(float));
  const int iters = 20000;
  constexpr int ACC = 16;
  for (int waves_per_simd = 1; waves_per_simd <= 4; waves_per_simd *= 2) {
    int blocks = 1024 * waves_per_simd;
    float ts = timeit(k_scalar<ACC>, blocks, out, iters);
    float tp = timeit(k_packed<ACC>, blocks, out, iters);
    double fmas = (double)blocks * 64 * iters * ACC;
    printf("waves/SIMD=%d scalar: %.3f ms (%.1f TFLOP/s, %.2f cyc/instr/wave@2.4GHz)  packed: %.3f ms (%.1f TFLOP/s)\n",
           waves_per_simd, ts, 2 * fmas / ts / 1e9, ts * 1e-3 * 2.4e9 / (iters * ACC) / waves_per_simd, tp,
           2 * fmas / tp / 1e9);
  }
  return 0;
}
