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


// The exact 5-MFMA sequence of km_source_fwd_ft<10, bf16x3> built without
// MF_SRC_KEEP (the SModel message MLP's second layer, two output tiles, ISA of
// round 5's hipcc): chained accumulators fed back as SrcC one instruction apart,
// results written over their own B operand (M3, M5), and an LDS load into M5's
// SrcC 6 wait states behind it.  PAD = 1 spaces every MFMA by 32 wait states
// (the reference).
template <int PAD>
__global__ __launch_bounds__(256) void kseq(const floatx4* __restrict__ A, const floatx4* __restrict__ B,
                                            floatx4* __restrict__ out, int iters) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  __shared__ floatx4 junk[256];
  junk[threadIdx.x] = floatx4{1e3f, -1e3f, 7.f, 3.f};
  __syncthreads();
  const unsigned la = (unsigned)(size_t)&junk[threadIdx.x];
  floatx4 a1 = A[gid & 4095], a2 = A[(gid + 1) & 4095], a3 = A[(gid + 2) & 4095];
  floatx4 acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
    const floatx4 b90 = B[(gid + it * 977) & 4095], b96 = B[(gid + it * 613 + 5) & 4095];
    const floatx4 c22 = acc;
    floatx4 r90, r104 = acc2;
#define SEQASM(NOPSEQ) asm volatile( \
        "v_mov_b32 v22, %[c0]\n v_mov_b32 v23, %[c1]\n v_mov_b32 v24, %[c2]\n v_mov_b32 v25, %[c3]\n" \
        "v_mov_b32 v30, %[p0]\n v_mov_b32 v31, %[p1]\n v_mov_b32 v32, %[p2]\n v_mov_b32 v33, %[p3]\n" \
        "v_mov_b32 v38, %[q0]\n v_mov_b32 v39, %[q1]\n v_mov_b32 v40, %[q2]\n v_mov_b32 v41, %[q3]\n" \
        "v_mov_b32 v26, %[s0]\n v_mov_b32 v27, %[s1]\n v_mov_b32 v28, %[s2]\n v_mov_b32 v29, %[s3]\n" \
        "v_mov_b32 v90, %[x0]\n v_mov_b32 v91, %[x1]\n v_mov_b32 v92, %[x2]\n v_mov_b32 v93, %[x3]\n" \
        "v_mov_b32 v96, %[y0]\n v_mov_b32 v97, %[y1]\n v_mov_b32 v98, %[y2]\n v_mov_b32 v99, %[y3]\n" \
        "v_mov_b32 v104, %[r0]\n v_mov_b32 v105, %[r1]\n v_mov_b32 v106, %[r2]\n v_mov_b32 v107, %[r3]\n" \
        "s_nop 7\n s_nop 7\n" \
        "v_mfma_f32_16x16x32_bf16 v[108:111], v[30:33], v[90:93], v[22:25]\n" \
        NOPSEQ \
        "v_mfma_f32_16x16x32_bf16 v[104:107], v[38:41], v[96:99], v[104:107]\n" \
        NOPSEQ \
        "v_mfma_f32_16x16x32_bf16 v[96:99], v[26:29], v[96:99], v[108:111]\n" \
        NOPSEQ \
        "v_mfma_f32_16x16x32_bf16 v[104:107], v[38:41], v[90:93], v[104:107]\n" \
        NOPSEQ \
        "v_mfma_f32_16x16x32_bf16 v[90:93], v[26:29], v[90:93], v[96:99]\n" \
        "s_nop 5\n" \
        "ds_read_b128 v[96:99], %[la]\n" \
        "s_waitcnt lgkmcnt(0)\n" \
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n" \
        "v_mov_b32 %[o0], v90\n v_mov_b32 %[o1], v91\n v_mov_b32 %[o2], v92\n v_mov_b32 %[o3], v93\n" \
        "v_mov_b32 %[u0], v104\n v_mov_b32 %[u1], v105\n v_mov_b32 %[u2], v106\n v_mov_b32 %[u3], v107\n" \
        : [o0] "=v"(r90[0]), [o1] "=v"(r90[1]), [o2] "=v"(r90[2]), [o3] "=v"(r90[3]), \
          [u0] "=v"(r104[0]), [u1] "=v"(r104[1]), [u2] "=v"(r104[2]), [u3] "=v"(r104[3]) \
        : [c0] "v"(c22[0]), [c1] "v"(c22[1]), [c2] "v"(c22[2]), [c3] "v"(c22[3]), \
          [p0] "v"(a1[0]), [p1] "v"(a1[1]), [p2] "v"(a1[2]), [p3] "v"(a1[3]), \
          [q0] "v"(a2[0]), [q1] "v"(a2[1]), [q2] "v"(a2[2]), [q3] "v"(a2[3]), \
          [s0] "v"(a3[0]), [s1] "v"(a3[1]), [s2] "v"(a3[2]), [s3] "v"(a3[3]), \
          [x0] "v"(b90[0]), [x1] "v"(b90[1]), [x2] "v"(b90[2]), [x3] "v"(b90[3]), \
          [y0] "v"(b96[0]), [y1] "v"(b96[1]), [y2] "v"(b96[2]), [y3] "v"(b96[3]), \
          [r0] "v"(acc2[0]), [r1] "v"(acc2[1]), [r2] "v"(acc2[2]), [r3] "v"(acc2[3]), [la] "v"(la) \
        : "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", \
          "v38", "v39", "v40", "v41", "v90", "v91", "v92", "v93", "v96", "v97", "v98", "v99", \
          "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "memory");

    if constexpr (PAD) { SEQASM("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"); }
    else { SEQASM(""); }

    acc = r90 * 0.25f;
    acc2 = r104 * 0.25f;
  }
  out[2 * gid] = acc;
  out[2 * gid + 1] = acc2;
}

static void seq_test(int blocks, int iters, const floatx4* dA, const floatx4* dB) {
  floatx4* dO;
  const size_t n = (size_t)blocks * 256 * 8;
  if (hipMalloc(&dO, n * 4) != hipSuccess) { printf("alloc failed\n"); exit(1); }
  std::vector<float> ref(n), h(n);
  hipLaunchKernelGGL((kseq<1>), dim3(blocks), dim3(256), 0, 0, dA, dB, dO, iters);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
  if (hipMemcpy(ref.data(), dO, n * 4, hipMemcpyDeviceToHost) != hipSuccess) exit(1);
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL((kseq<0>), dim3(blocks), dim3(256), 0, 0, dA, dB, dO, iters);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
    if (hipMemcpy(h.data(), dO, n * 4, hipMemcpyDeviceToHost) != hipSuccess) exit(1);
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += h[i] != ref[i];
    printf("km_source_fwd_ft's 5-MFMA sequence (no padding) run %d: %zu of %zu floats differ "
           "from the padded sequence\n", r, bad, n);
  }
  (void)hipFree(dO);
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
  if (argc > 3 && atoi(argv[3]) == 1) {   // the kernel's 5-MFMA sequence only
    seq_test(blocks, iters, dA, dB);
    return 0;
  }
  sweep<0>("SrcC", blocks, iters, dA, dB, dO);
  sweep<1>("SrcA", blocks, iters, dA, dB, dO);
  sweep<2>("SrcB", blocks, iters, dA, dB, dO);
  hipFree(dA);
  hipFree(dB);
  hipFree(dO);
  return 0;
}
