// Cycles per MFMA instruction on one SIMD (one wave per SIMD, 8 independent
// accumulators, back-to-back issue), for the shapes the edge kernels use or
// could use: v_mfma_f32_16x16x4_f32, v_mfma_f32_16x16x16_bf16 (the K=16 "_1k"
// form), v_mfma_f32_16x16x32_bf16 (gfx950).  s_memtime ticks = shader cycles.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_cycles tools/mfma_cycles.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

#define ITERS 512
#define NACC 8

template <int KIND>
__global__ __launch_bounds__(64) void kmf(float* out, long long* cyc, float seed) {
  floatx4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = floatx4{seed * i, 0.f, 0.f, 0.f};
  const float a = seed + threadIdx.x * 1e-3f, b = seed - threadIdx.x * 1e-3f;
  const s16x4 a4 = {(short)(threadIdx.x + 1), 2, 3, 4}, b4 = {5, 6, (short)threadIdx.x, 8};
  b16x8 a8, b8;
#pragma unroll
  for (int i = 0; i < 8; ++i) { a8[i] = (__bf16)(a + i); b8[i] = (__bf16)(b - i); }
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if constexpr (KIND == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
      if constexpr (KIND == 1) acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[i], 0, 0, 0);
      if constexpr (KIND == 2) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[i], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static void run(const char* name, int blocks) {
  float* out;
  long long* cyc;
  hipMalloc(&out, blocks * 64 * sizeof(float));
  hipMalloc(&cyc, blocks * sizeof(long long));
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kmf<KIND>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0f);
  hipDeviceSynchronize();
  long long* h = new long long[blocks];
  hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < blocks; ++i) s += h[i];
  printf("%-28s blocks=%5d  %.2f cycles per MFMA (s_memtime)\n", name, blocks,
         s / blocks / (double)(ITERS * NACC));
  delete[] h;
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int blocks : {1, 1024}) {
    run<0>("v_mfma_f32_16x16x4_f32", blocks);
    run<1>("v_mfma_f32_16x16x16_bf16", blocks);
    run<2>("v_mfma_f32_16x16x32_bf16", blocks);
  }
  return 0;
}
