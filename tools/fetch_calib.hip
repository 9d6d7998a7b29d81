// FETCH_SIZE / WRITE_SIZE calibration on known byte counts (test tooling, not
// product code).  MI355X_MICROARCH.md §HBM: FETCH_SIZE reports 1/2 of the bytes
// of a 16-B-per-lane coalesced streaming read on gfx950, other widths are
// uncalibrated.  Each kernel below moves an exactly known number of bytes of a
// 1 GiB buffer (4x the 256 MiB Infinity Cache, so nothing is served on-die):
//   rd16   : 16 B/lane float4 stream                         (the guide's case)
//   rd4    : 4 B/lane float stream (256 B per wave-instruction)
//   rdrows : the edge kernels' pattern (pfsgnn_mfma.hip ld_frows): each group
//            of 16 lanes reads a 64-B run of one channel row of a channel-major
//            [F][E] tensor, the 4 groups read 4 different rows
//   wr4    : 4 B/lane float stores, wr16: 16 B/lane float4 stores
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
// Run:   rocprofv3 --pmc FETCH_SIZE ... -- ./tools/fetch_calib   (one counter per pass)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ __launch_bounds__(256) void rd16(const float4* __restrict__ p, size_t n4,
                                            float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = p[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[blockIdx.x] = s;   // never true: keeps the loads alive
}

__global__ __launch_bounds__(256) void rd4(const float* __restrict__ p, size_t n,
                                           float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i];
  if (s == 12345.f) out[blockIdx.x] = s;
}

// [F][E] channel-major, F = 10 rows spread over the 4 lane groups as in the
// kernels' compact row map (group g holds rows 3g, 3g+1, 3g+2; group 3 row 9);
// a wave handles 16 consecutive edges per step.
__global__ __launch_bounds__(256) void rdrows(const float* __restrict__ p, size_t E,
                                              float* __restrict__ out) {
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const size_t nw = (size_t)gridDim.x * 4;
  float s = 0.f;
  for (size_t e0 = wave * 16; e0 < E; e0 += nw * 16) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int k = 3 * g + r;
      if (k < 10 && e0 + j < E) s += p[(size_t)k * E + e0 + j];
    }
  }
  if (s == 12345.f) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void wr4(float* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = (float)(i & 7);
}

__global__ __launch_bounds__(256) void wr16(float4* __restrict__ p, size_t n4) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    p[i] = float4{1.f, 2.f, 3.f, (float)(i & 7)};
}

int main() {
  const size_t bytes = (size_t)1 << 30;   // 1 GiB
  const size_t n = bytes / 4;
  const size_t E = (n / 10) & ~(size_t)15; // rdrows: 10 rows of E floats (E*10 <= n)
  float *buf, *out;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, 4096 * sizeof(float)));
  CHECK(hipMemset(buf, 0, bytes));
  const int grid = 4096;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(rd16, dim3(grid), dim3(256), 0, 0, (const float4*)buf, n / 4, out);
    hipLaunchKernelGGL(rd4, dim3(grid), dim3(256), 0, 0, buf, n, out);
    hipLaunchKernelGGL(rdrows, dim3(grid), dim3(256), 0, 0, buf, E, out);
    hipLaunchKernelGGL(wr4, dim3(grid), dim3(256), 0, 0, buf, n);
    hipLaunchKernelGGL(wr16, dim3(grid), dim3(256), 0, 0, (float4*)buf, n / 4);
  }
  CHECK(hipDeviceSynchronize());
  printf("fetch_calib: rd16 rd4 %zu bytes each, rdrows %zu bytes, wr4 wr16 %zu bytes each\n",
         bytes, E * 10 * 4, bytes);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
