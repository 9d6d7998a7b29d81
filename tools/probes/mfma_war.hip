// Round 6: is a VALU write to a register that a just-issued
// v_mfma_f32_16x16x32_bf16 reads (SrcC, SrcA or SrcB) safe on gfx950 after the
// number of wait states hipcc (ROCm 7.2, -amdgpu-mfma-vgpr-form=1) leaves?
// km_source_fwd_ft<10, bf16x3> built without MF_SRC_KEEP issues
//     v_mfma_f32_16x16x32_bf16 v[108:111], v[34:37], v[104:107], v[90:93]
//     s_nop 2
//     v_mov_b32 v92, v106          ; SrcC[2] overwritten 4 wait states later
// (DESIGN.md §Reproducibility).  Each lane runs ITERS steps of one such MFMA
// on fixed registers (inline asm, v[100:115]) followed, after W wait states
// (s_nop), by v_mov writes of junk into two registers of the chosen source;
// the result is compared with the same sequence padded by 32 wait states.
// Many blocks per CU keep every SIMD's matrix pipe contended by other waves.
//   hipcc -O3 --offload-arch=gfx950 -o tools/probes/mfma_war tools/probes/mfma_war.hip
//   tools/probes/mfma_war [blocks] [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define NOPS_0 ""
#define NOPS_1 "s_nop 0\n"
#define NOPS_2 "s_nop 1\n"
#define NOPS_3 "s_nop 2\n"
#define NOPS_4 "s_nop 3\n"
#define NOPS_6 "s_nop 5\n"
#define NOPS_8 "s_nop 7\n"
#define NOPS_12 "s_nop 7\n s_nop 3\n"
#define NOPS_32 "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
// SRC: 0 = SrcC (v100..103), 1 = SrcA (v104..107), 2 = SrcB (v108..111); the
// MFMA itself is one wait state, so NOPS_k gives k + 1 wait states before the
// first v_mov
#define STEP(NOPS, R0, R1)                                                            \
  asm volatile(                                                                       \
      "v_mov_b32 v100, %4\n v_mov_b32 v101, %5\n v_mov_b32 v102, %6\n v_mov_b32 v103, %7\n" \
      "v_mov_b32 v104, %8\n v_mov_b32 v105, %9\n v_mov_b32 v106, %10\n v_mov_b32 v107, %11\n" \
      "v_mov_b32 v108, %12\n v_mov_b32 v109, %13\n v_mov_b32 v110, %14\n v_mov_b32 v111, %15\n" \
      "s_nop 7\n s_nop 7\n"                                                           \
      "v_mfma_f32_16x16x32_bf16 v[112:115], v[104:107], v[108:111], v[100:103]\n"     \
      NOPS                                                                            \
      "v_mov_b32 " R0 ", %16\n v_mov_b32 " R1 ", %16\n"                              \
      "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"                  \
      "v_mov_b32 %0, v112\n v_mov_b32 %1, v113\n v_mov_b32 %2, v114\n v_mov_b32 %3, v115\n" \
      : "=v"(d[0]), "=v"(d[1]), "=v"(d[2]), "=v"(d[3])                                \
      : "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(a[0]), "v"(a[1]), "v"(a[2]),  \
        "v"(a[3]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(junk)                \
      : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", \
        "v110", "v111", "v112", "v113", "v114", "v115")

template <int SRC, int W>
__global__ __launch_bounds__(256) void k(const floatx4* __restrict__ A, const floatx4* __restrict__ B,
                                         floatx4* __restrict__ out, int iters) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  floatx4 a = A[gid & 4095];
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
  const float junk = 1.0e6f;
  for (int it = 0; it < iters; ++it) {
    floatx4 b = B[(gid + it * 977) & 4095];
    floatx4 d;
#define PICK(NOPS)                                                       \
    if constexpr (SRC == 0) STEP(NOPS, "v100", "v102");                 \
    else if constexpr (SRC == 1) STEP(NOPS, "v104", "v106");            \
    else STEP(NOPS, "v108", "v110");
    if constexpr (W == 0) { PICK(NOPS_0) }
    else if constexpr (W == 1) { PICK(NOPS_1) }
    else if constexpr (W == 2) { PICK(NOPS_2) }
    else if constexpr (W == 3) { PICK(NOPS_3) }
    else if constexpr (W == 4) { PICK(NOPS_4) }
    else if constexpr (W == 6) { PICK(NOPS_6) }
    else if constexpr (W == 8) { PICK(NOPS_8) }
    else if constexpr (W == 12) { PICK(NOPS_12) }
    else { PICK(NOPS_32) }
    c = d * 0.5f;   // the next step accumulates onto this one's result
  }
  out[gid] = c;
}

template <int SRC, int W>
static size_t run(int blocks, int iters, const floatx4* dA, const floatx4* dB, floatx4* dO,
                  std::vector<float>& h) {
  hipLaunchKernelGGL((k<SRC, W>), dim3(blocks), dim3(256), 0, 0, dA, dB, dO, iters);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
  h.resize((size_t)blocks * 256 * 4);
  hipMemcpy(h.data(), dO, h.size() * 4, hipMemcpyDeviceToHost);
  return h.size();
}

template <int SRC, int W>
static void cmp(const char* name, int blocks, int iters, const floatx4* dA, const floatx4* dB,
                floatx4* dO, const std::vector<float>& ref) {
  std::vector<float> h;
  for (int r = 0; r < 3; ++r) {
    run<SRC, W>(blocks, iters, dA, dB, dO, h);
    size_t bad = 0;
    for (size_t i = 0; i < h.size(); ++i) bad += h[i] != ref[i];
    printf("%s: write after %d wait states, run %d: %zu of %zu floats differ from the padded run\n",
           name, W + 1, r, bad, h.size());
  }
}

template <int SRC>
static void sweep(const char* name, int blocks, int iters, const floatx4* dA, const floatx4* dB,
                  floatx4* dO) {
  std::vector<float> ref;
  run<SRC, 32>(blocks, iters, dA, dB, dO, ref);
  cmp<SRC, 0>(name, blocks, iters, dA, dB, dO, ref);
  cmp<SRC, 1>(name, blocks, iters, dA, dB, dO, ref);
  cmp<SRC, 2>(name, blocks, iters, dA, dB, dO, ref);
  cmp<SRC, 3>(name, blocks, iters, dA, dB, dO, ref);
  cmp<SRC, 4>(name, blocks, iters, dA, dB, dO, ref);
  cmp<SRC, 6>(name, blocks, iters, dA, dB, dO, ref);
  cmp<SRC, 8>(name, blocks, iters, dA, dB, dO, ref);
  cmp<SRC, 12>(name, blocks, iters, dA, dB, dO, ref);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 4096, iters = argc > 2 ? atoi(argv[2]) : 64;
  std::vector<unsigned> hA(4 * 4096), hB(4 * 4096);
  srand(7);
  for (int i = 0; i < 4 * 4096; ++i) {
    hA[i] = (0x3c00u + (rand() & 0x1ff)) | ((0x3c00u + (rand() & 0x1ff)) << 16);
    hB[i] = (0x3c00u + (rand() & 0x1ff)) | ((0xbc00u + (rand() & 0x1ff)) << 16);
  }
  floatx4 *dA, *dB, *dO;
  hipMalloc(&dA, 4 * 4096 * 4);
  hipMalloc(&dB, 4 * 4096 * 4);
  hipMalloc(&dO, (size_t)blocks * 256 * 16);
  hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice);
  sweep<0>("SrcC", blocks, iters, dA, dB, dO);
  sweep<1>("SrcA", blocks, iters, dA, dB, dO);
  sweep<2>("SrcB", blocks, iters, dA, dB, dO);
  hipFree(dA);
  hipFree(dB);
  hipFree(dO);
  return 0;
}
