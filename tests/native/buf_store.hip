// Test-only kernels (tests/test_gpu_buffer_store.py): the edge-row STORE forms
// the per-edge kernels could use for a lane's F rows of a channel-major [F][E]
// edge tensor, with the product's own row map and offsets
// (pfs-neural-net_amd/csrc/pfsgnn_mfma_core.h: GM, RowOff, rsrc, st_frows).
// Round 3 recorded that buffer stores of a lane's rows were miscompiled (one
// row's value stored to every row); these kernels isolate the pattern:
//   variant 0: buffer_store per row under the row's exec mask (valid fiber,
//              row < F), the form pfsgnn_mfma_core.h:414 names;
//   variant 1: buffer_store per row, unconditional, the offset of an invalid
//              row moved past the buffer's range (discarded by the bounds
//              check): the branch-free form DESIGN.md §Performance tried;
//   variant 2: global stores under per-row exec masks (the kernels' form
//              until round 4);
//   variants 3 / 4: variants 0 / 1 with the row's value first copied out of
//              the vector into a float (`const float e = v[r]`) and THAT
//              bit-cast to the builtin's unsigned data operand.
//   variant 5: the product's st_frows (pfsgnn_mfma_core.h: variant 4's form).
// Variants 0 / 1 bit-cast the vector element itself,
// __builtin_bit_cast(unsigned int, v[r]) -- the only way to hand a float
// element to __builtin_amdgcn_raw_buffer_store_b32 without a temporary.
// Each lane loads its rows with the product's buffer loads (ld_frows), stores
// 2 x + 1, and the test compares every element with the host's.
// Built by pfs-neural-net_amd/Makefile as tests/native/libbufstore.so; not part
// of libpfsgnn.so.
#include "../../pfs-neural-net_amd/csrc/pfsgnn_mfma_core.h"

namespace {

constexpr int F = 10;   // the bench's Fdim: 3 row slots per lane group, group 3 holds 1 row

template <int V>
__global__ __launch_bounds__(256) void kstore(const float* __restrict__ x, float* __restrict__ y,
                                              int NF, int NC) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int g4 = lane >> 4, j16 = lane & 15;
  const int f = blockIdx.x * 64 + wave * 16 + j16;
  const bool fvalid = f < NF;
  const uint32_t E = (uint32_t)NF * (uint32_t)NC, RB = E * 4u;
  const uint32_t eo0 = (uint32_t)(fvalid ? f : 0) * 4u, eoc = (uint32_t)NF * 4u;
  const RowOff<F> ro(eo0, RB, g4);
  const Rsrc rx = rsrc(x, RB * F), ry = rsrc(y, RB * F);
  for (int c = 0; c < NC; ++c) {
    const uint32_t co = (uint32_t)c * eoc;
    floatx4 v = ld_frows<F>(rx, co, ro);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaf(v[r], 2.f, 1.f);
    if constexpr (V == 0) {
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        const int k = GM<F>::row(g4, r);
        if (fvalid && k >= 0)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v[r]), ry,
                                                ro.o[r], co, 0);
      }
    } else if constexpr (V == 1) {
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        const int k = GM<F>::row(g4, r);
        const uint32_t off = (fvalid && k >= 0) ? ro.o[r] : RB * F;   // past the range
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v[r]), ry, off,
                                              co, 0);
      }
    } else if constexpr (V == 2) {   // global stores under per-row exec masks
      char* base = reinterpret_cast<char*>(y) + co;
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        const int k = GM<F>::row(g4, r);
        if (fvalid && k >= 0) *reinterpret_cast<float*>(base + opaque(ro.o[r])) = v[r];
      }
    } else if constexpr (V == 5) {   // the product's st_frows
      st_frows<F>(y, RB * F, co, ro, g4, fvalid, v);
    } else {
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        const int k = GM<F>::row(g4, r);
        const float e = v[r];
        const bool ok = fvalid && k >= 0;
        if (V == 4 || ok)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, e), ry,
                                                (V == 3 || ok) ? ro.o[r] : RB * F, co, 0);
      }
    }
  }
}

}  // namespace

extern "C" int buf_store_run(const float* hx, float* hy, int NF, int NC, int variant) {
  const size_t n = (size_t)F * NF * NC;
  float *x, *y;
  if (variant < 0 || variant > 5) return 2;
  if (hipMalloc(&x, n * 4) || hipMalloc(&y, n * 4)) return 1;
  int rc = 0;
  rc |= hipMemcpy(x, hx, n * 4, hipMemcpyHostToDevice) != hipSuccess;
  rc |= hipMemcpy(y, hy, n * 4, hipMemcpyHostToDevice) != hipSuccess;   // the caller's sentinel
  const dim3 grid((NF + 63) / 64), block(256);
  if (variant == 0) hipLaunchKernelGGL(kstore<0>, grid, block, 0, 0, x, y, NF, NC);
  else if (variant == 1) hipLaunchKernelGGL(kstore<1>, grid, block, 0, 0, x, y, NF, NC);
  else if (variant == 2) hipLaunchKernelGGL(kstore<2>, grid, block, 0, 0, x, y, NF, NC);
  else if (variant == 3) hipLaunchKernelGGL(kstore<3>, grid, block, 0, 0, x, y, NF, NC);
  else if (variant == 4) hipLaunchKernelGGL(kstore<4>, grid, block, 0, 0, x, y, NF, NC);
  else hipLaunchKernelGGL(kstore<5>, grid, block, 0, 0, x, y, NF, NC);
  rc |= hipDeviceSynchronize() != hipSuccess;
  rc |= hipMemcpy(hy, y, n * 4, hipMemcpyDeviceToHost) != hipSuccess;
  rc |= hipFree(x) != hipSuccess;
  rc |= hipFree(y) != hipSuccess;
  return rc;
}
