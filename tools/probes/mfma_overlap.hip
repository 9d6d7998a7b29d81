// Does v_mfma_f32_16x16x32_bf16 with its result register block equal to its
// own B (or A) operand compute the same as the non-overlapped instruction on
// gfx950?  Every lane runs ITERS dependent steps d = mfma(a, b, d) where b is
// refreshed from memory each step; mode 0 uses distinct result registers (the
// compiler's choice with the operand kept live), mode 1 writes the result over
// B (dst == SrcB, exact overlap), mode 2 over A.  Wide s_nop padding around the
// hand-written MFMA keeps every VALU <-> MFMA hazard out of the comparison.
// Many blocks per CU keep the matrix pipes contended.  Build:
//   hipcc -O3 --offload-arch=gfx950 -o tools/probes/mfma_overlap tools/probes/mfma_overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(256) void k(const floatx4* __restrict__ A, const floatx4* __restrict__ B,
                                         floatx4* __restrict__ out, int iters) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  __shared__ floatx4 junk[256];
  junk[threadIdx.x] = floatx4{1e3f, -1e3f, 7.f, 3.f};
  __syncthreads();
  floatx4 a = A[gid & 4095];
  floatx4 d = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
    floatx4 b = B[(gid + it * 977) & 4095];
    if constexpr (MODE == 0) {
      asm volatile("s_nop 7\n s_nop 7\n v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7"
                   : "+v"(d) : "v"(a), "v"(b));
    } else if constexpr (MODE == 1) {
      // result over B: b holds the sum afterwards; d (SrcC) is read
      asm volatile("s_nop 7\n s_nop 7\n v_mfma_f32_16x16x32_bf16 %0, %1, %0, %2\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7"
                   : "+v"(b) : "v"(a), "v"(d));
      d = b;
    } else if constexpr (MODE == 3 || MODE == 4) {
      // the compiler's sequence in km_source_fwd_ft (round 4): t = mfma(a, b, d);
      // d = mfma(a, b, t) with t as SrcC (not the same registers as the result),
      // then an LDS load into t's registers right behind the dependent MFMA.
      // MODE 4 pads the load with s_nops (the instructions finish first).
      floatx4 t, junkv;
      if constexpr (MODE == 3)
        asm volatile("s_nop 7\n s_nop 7\n"
                     "v_mfma_f32_16x16x32_bf16 %1, %3, %4, %0\n"
                     "v_mfma_f32_16x16x32_bf16 %0, %3, %4, %1\n"
                     "ds_read_b128 %1, %5\n"
                     "s_waitcnt lgkmcnt(0)\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7"
                     : "+v"(d), "=&v"(t), "=&v"(junkv) : "v"(a), "v"(b), "v"((unsigned)(size_t)&junk[threadIdx.x]));
      else
        asm volatile("s_nop 7\n s_nop 7\n"
                     "v_mfma_f32_16x16x32_bf16 %1, %3, %4, %0\n"
                     "s_nop 7\n s_nop 7\n s_nop 7\n"
                     "v_mfma_f32_16x16x32_bf16 %0, %3, %4, %1\n"
                     "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
                     "ds_read_b128 %1, %5\n"
                     "s_waitcnt lgkmcnt(0)\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7"
                     : "+v"(d), "=&v"(t), "=&v"(junkv) : "v"(a), "v"(b), "v"((unsigned)(size_t)&junk[threadIdx.x]));
      (void)junkv;
    } else {
      floatx4 a2 = a;
      asm volatile("s_nop 7\n s_nop 7\n v_mfma_f32_16x16x32_bf16 %0, %0, %1, %2\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7"
                   : "+v"(a2) : "v"(b), "v"(d));
      d = a2;
    }
    d = d * 0.5f;   // keep magnitudes bounded
  }
  out[gid] = d;
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 4096, iters = argc > 2 ? atoi(argv[2]) : 256;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;
  const size_t n = (size_t)blocks * 256;
  std::vector<unsigned> hA(4 * 4096), hB(4 * 4096);
  srand(7);
  for (int i = 0; i < 4 * 4096; ++i) {
    // bf16 pairs packed in 32-bit words: small finite values of both signs
    hA[i] = (0x3c00u + (rand() & 0x1ff)) | ((0x3c00u + (rand() & 0x1ff)) << 16);
    hB[i] = (0x3c00u + (rand() & 0x1ff)) | ((0xbc00u + (rand() & 0x1ff)) << 16);
  }
  floatx4 *A, *B, *o0, *o1;
  (void)hipMalloc(&A, 4096 * 16); (void)hipMalloc(&B, 4096 * 16);
  (void)hipMalloc(&o0, n * 16); (void)hipMalloc(&o1, n * 16);
  (void)hipMemcpy(A, hA.data(), 4096 * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(B, hB.data(), 4096 * 16, hipMemcpyHostToDevice);
  std::vector<unsigned> r0(4 * n), r1(4 * n);
  hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, A, B, o0, iters);
  (void)hipMemcpy(r0.data(), o0, n * 16, hipMemcpyDeviceToHost);
  floatx4* o4;
  (void)hipMalloc(&o4, n * 16);
  hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, A, B, o4, iters);
  std::vector<unsigned> r4(4 * n);
  (void)hipMemcpy(r4.data(), o4, n * 16, hipMemcpyDeviceToHost);
  for (int mode = 3; mode < 5; ++mode)
    for (int r = 0; r < rounds; ++r) {
      if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, A, B, o1, iters);
      if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, A, B, o1, iters);
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      (void)hipMemcpy(r1.data(), o1, n * 16, hipMemcpyDeviceToHost);
      size_t diff = 0;
      for (size_t i = 0; i < 4 * n; ++i) diff += r4[i] != r1[i];
      printf("mode %d (%s) round %d: %zu of %zu floats differ from the padded sequence's first run\n",
             mode, mode == 3 ? "LDS load into a chained SrcC right behind the MFMA" : "the same, padded",
             r, diff, n * 4);
    }
  for (int mode = 0; mode < 3; ++mode)
    for (int r = 0; r < rounds; ++r) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, A, B, o1, iters);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, A, B, o1, iters);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, A, B, o1, iters);
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      (void)hipMemcpy(r1.data(), o1, n * 16, hipMemcpyDeviceToHost);
      size_t diff = 0;
      for (size_t i = 0; i < 4 * n; ++i) diff += r0[i] != r1[i];
      printf("mode %d (%s) round %d: %zu of %zu floats differ from mode 0's first run\n", mode,
             mode == 0 ? "distinct result" : mode == 1 ? "result over B" : "result over A", r, diff,
             n * 4);
    }
  return 0;
}
