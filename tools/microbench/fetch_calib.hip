// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE (KiB) against known byte
// counts, per access pattern, on gfx950 (MI355X_MICROARCH.md: FETCH_SIZE reads
// 1/2 of a wide coalesced stream; other widths uncalibrated).  Each kernel
// moves exactly BYTES bytes once (buffers 512 MiB, beyond the 256 MiB MALL).
//   patterns: rd_dword (4 B per lane, coalesced: the MPC slots' component
//   planes), rd_dwordx4 (16 B per lane, coalesced: the float4 planes),
//   rd_rec144 (a lane reads its own 144-B record with 9 dwordx4: the caller's
//   C [T,B,6,6]), wr_dword, wr_dwordx4.
// hipcc -O3 --offload-arch=gfx950 -Wno-unused-result -o fetch_calib fetch_calib.hip
// rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./fetch_calib ; ... --pmc WRITE_SIZE
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t BYTES = 512ull << 20;

__global__ void rd_dword(const float* __restrict__ p, float* __restrict__ sink, size_t n) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
  if (s == 12345.f) sink[0] = s;
}
__global__ void rd_dwordx4(const float4* __restrict__ p, float* __restrict__ sink, size_t n) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = p[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) sink[0] = s;
}
__global__ void rd_rec144(const float4* __restrict__ p, float* __restrict__ sink, size_t nrec) {
  float s = 0.f;
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < nrec; r += (size_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      float4 v = p[r * 9 + j];
      s += v.x + v.y + v.z + v.w;
    }
  }
  if (s == 12345.f) sink[0] = s;
}
__global__ void wr_dword(float* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (float)i;
}
__global__ void wr_dwordx4(float4* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

int main() {
  float *buf, *sink;
  hipMalloc(&buf, BYTES);
  hipMalloc(&sink, 64);
  hipMemset(buf, 0, BYTES);
  const int grid = 256 * 8, blk = 256;
  for (int rep = 0; rep < 3; ++rep) {
    rd_dword<<<grid, blk>>>(buf, sink, BYTES / 4);
    rd_dwordx4<<<grid, blk>>>((const float4*)buf, sink, BYTES / 16);
    rd_rec144<<<grid, blk>>>((const float4*)buf, sink, BYTES / 144);
    wr_dword<<<grid, blk>>>(buf, BYTES / 4);
    wr_dwordx4<<<grid, blk>>>((float4*)buf, BYTES / 16);
  }
  hipDeviceSynchronize();
  printf("bytes per kernel: %zu (rd_rec144: %zu)\n", BYTES, (BYTES / 144) * 144);
  return 0;
}
