// Minimal form of the defect tests/test_bitcast_vector_element.py pins
// (DESIGN.md §Edge-row stores): __builtin_bit_cast of an ext_vector_type
// element subscript.  `k_elem` bit-casts v[r] directly, `k_temp` copies the
// element to a float first.  Compiled to LLVM IR only (never linked or run).
#include <hip/hip_runtime.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void k_elem(const floatx4* in, unsigned* out) {
  const floatx4 v = in[threadIdx.x];
#pragma unroll
  for (int r = 0; r < 4; ++r) out[4 * threadIdx.x + r] = __builtin_bit_cast(unsigned int, v[r]);
}

__global__ void k_temp(const floatx4* in, unsigned* out) {
  const floatx4 v = in[threadIdx.x];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float e = v[r];
    out[4 * threadIdx.x + r] = __builtin_bit_cast(unsigned int, e);
  }
}
