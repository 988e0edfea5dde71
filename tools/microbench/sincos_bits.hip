// Is sincosf(x) bit-identical to (sinf(x), cosf(x))?  Counts mismatches over a
// sweep of float bit patterns (every 7th pattern, all signs/exponents).
// hipcc -O3 --offload-arch=gfx950 -Wno-unused-result -o sincos_bits sincos_bits.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long start, unsigned long long n, unsigned* bad) {
  unsigned long long i = start + (blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x) * 7ull;
  if (i >= start + n * 7ull || i > 0xffffffffull) return;
  float x = __uint_as_float((unsigned)i);
  float s1, c1;
  sincosf(x, &s1, &c1);
  float s2 = sinf(x), c2 = cosf(x);
  bool bs = __float_as_uint(s1) != __float_as_uint(s2) && !(s1 != s1 && s2 != s2);
  bool bc = __float_as_uint(c1) != __float_as_uint(c2) && !(c1 != c1 && c2 != c2);
  if (bs) atomicAdd(bad, 1u);
  if (bc) atomicAdd(bad + 1, 1u);
}
int main() {
  unsigned* bad;
  hipMalloc(&bad, 8);
  hipMemset(bad, 0, 8);
  const unsigned long long total = (1ull << 32) / 7 + 1, chunk = 1ull << 26;
  for (unsigned long long s = 0; s < total; s += chunk) {
    unsigned long long n = s + chunk < total ? chunk : total - s;
    k<<<(n + 255) / 256, 256>>>(s * 7ull, n, bad);
  }
  unsigned h[2];
  hipMemcpy(h, bad, 8, hipMemcpyDeviceToHost);
  printf("sincosf vs sinf/cosf mismatches over %llu inputs: sin %u cos %u\n", total, h[0], h[1]);
  return 0;
}
