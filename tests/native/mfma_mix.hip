// Test-only kernels (tests/test_gpu_mfma_forms.py): an accumulation chain of
// v_mfma_f32_16x16x32_bf16 finished by a v_mfma_f32_16x16x16_bf16 on the SAME
// accumulator -- the MFMA "form mixing" that gave wrong sums in the round-2
// edge kernels (DESIGN.md §MFMA form mixing) -- built three ways:
//   variant 0: as hipcc schedules it (no wait states between the two forms);
//   variant 1: the same chain with s_nop 7 x2 (16 wait states) before the
//              16x16x16 that reads the 16x16x32's result as its C operand;
//   variant 2: the 16x16x16 first, then the two 16x16x32s (the other order).
// Each lane's operands come from plain arrays; the test compares every output
// with a float64 reference of the same sums.  Built by pfs-neural-net_amd/Makefile
// (target `tests`) as tests/native/libmfmamix.so; not part of libpfsgnn.so.
#include <hip/hip_runtime.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ floatx4 x32(s16x8 a, s16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b16x8, a),
                                                 __builtin_bit_cast(b16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ floatx4 x16(s16x4 a, s16x4 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

template <int V>
__global__ void kmix(const s16x8* A, const s16x8* B, const s16x4* A2, const s16x4* B2,
                     floatx4* out) {
  const int l = threadIdx.x;
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
  if (V == 2) c = x16(A2[l], B2[l], c);
  c = x32(A[l], B[l], c);
  c = x32(A[64 + l], B[64 + l], c);
  if (V == 1) asm volatile("s_nop 7\n\ts_nop 7" : "+v"(c));
  if (V != 2) c = x16(A2[l], B2[l], c);
  out[l] = c;
}

extern "C" int mfma_mix_run(const short* hA, const short* hB, const short* hA2, const short* hB2,
                            float* hout, int variant) {
  short *A, *B, *A2, *B2;
  float* out;
  if (hipMalloc(&A, 2 * 64 * 16) || hipMalloc(&B, 2 * 64 * 16) || hipMalloc(&A2, 64 * 8) ||
      hipMalloc(&B2, 64 * 8) || hipMalloc(&out, 64 * 16))
    return 1;
  hipMemcpy(A, hA, 2 * 64 * 16, hipMemcpyHostToDevice);
  hipMemcpy(B, hB, 2 * 64 * 16, hipMemcpyHostToDevice);
  hipMemcpy(A2, hA2, 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(B2, hB2, 64 * 8, hipMemcpyHostToDevice);
  auto a = (const s16x8*)A, b = (const s16x8*)B;
  auto a2 = (const s16x4*)A2, b2 = (const s16x4*)B2;
  if (variant == 0) hipLaunchKernelGGL(kmix<0>, dim3(1), dim3(64), 0, 0, a, b, a2, b2, (floatx4*)out);
  else if (variant == 1) hipLaunchKernelGGL(kmix<1>, dim3(1), dim3(64), 0, 0, a, b, a2, b2, (floatx4*)out);
  else hipLaunchKernelGGL(kmix<2>, dim3(1), dim3(64), 0, 0, a, b, a2, b2, (floatx4*)out);
  int rc = hipDeviceSynchronize() != hipSuccess;
  hipMemcpy(hout, out, 64 * 16, hipMemcpyDeviceToHost);
  hipFree(A); hipFree(B); hipFree(A2); hipFree(B2); hipFree(out);
  return rc;
}
