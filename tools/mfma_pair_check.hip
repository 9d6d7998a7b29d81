// Checks that one v_mfma_f32_16x16x32_bf16 on concatenated operands equals two
// v_mfma_f32_16x16x16_bf16 (the pairing LayerB3 relies on), on random bf16 data.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_pair_check tools/mfma_pair_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstring>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

__global__ void kcheck(const short* A, const short* B, float* out2, float* out1) {
  const int l = threadIdx.x;
  s16x4 a0, a1, b0, b1;
  for (int j = 0; j < 4; ++j) {
    a0[j] = A[l * 8 + j];
    a1[j] = A[l * 8 + 4 + j];
    b0[j] = B[l * 8 + j];
    b1[j] = B[l * 8 + 4 + j];
  }
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a0, b0, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a1, b1, c, 0, 0, 0);
  const s16x8 a8 = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
  const s16x8 b8 = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
  floatx4 d = {0.f, 0.f, 0.f, 0.f};
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b16x8, a8),
                                             __builtin_bit_cast(b16x8, b8), d, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    out2[l * 4 + r] = c[r];
    out1[l * 4 + r] = d[r];
  }
}

int main() {
  short hA[512], hB[512];
  unsigned s = 12345;
  for (int i = 0; i < 512; ++i) {
    s = s * 1103515245u + 12345u;
    float v = ((s >> 8) & 0xFFFF) / 65536.0f - 0.5f;
    unsigned u;
    memcpy(&u, &v, 4);
    hA[i] = (short)(u >> 16);
    s = s * 1103515245u + 12345u;
    v = ((s >> 8) & 0xFFFF) / 65536.0f - 0.5f;
    memcpy(&u, &v, 4);
    hB[i] = (short)(u >> 16);
  }
  short *dA, *dB;
  float *d2, *d1;
  hipMalloc(&dA, 1024);
  hipMalloc(&dB, 1024);
  hipMalloc(&d2, 1024);
  hipMalloc(&d1, 1024);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(kcheck, dim3(1), dim3(64), 0, 0, dA, dB, d2, d1);
  float h2[256], h1[256];
  hipMemcpy(h2, d2, 1024, hipMemcpyDeviceToHost);
  hipMemcpy(h1, d1, 1024, hipMemcpyDeviceToHost);
  double mx = 0, sc = 0;
  for (int i = 0; i < 256; ++i) {
    mx = fmax(mx, fabs(h2[i] - h1[i]));
    sc = fmax(sc, fabs(h2[i]));
  }
  printf("pair check: max |two 16x16x16 - one 16x16x32| = %.3e (scale %.3e)\n", mx, sc);
  for (int i = 0; i < 8; ++i) printf("  %d: %.6f %.6f\n", i, h2[i], h1[i]);
  return mx <= 1e-5 * sc ? 0 : 1;
}
