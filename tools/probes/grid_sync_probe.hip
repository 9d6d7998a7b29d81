// Cost of a device-wide barrier among one workgroup per CU (GPU box):
//   hipcc -O3 --offload-arch=gfx950 tools/probes/grid_sync_probe.hip -o /tmp/gsp && /tmp/gsp
// Form 0: one arrival counter + generation (pfsgnn_mlp.hip grid_sync).
// Form 1: per-XCD-slot counters (b % 8), the last arrival of each slot counts
//         into a top counter: 8 contenders per top atomic instead of all.
// Form 2: no read-modify-write: each workgroup stores the barrier's epoch to
//         its own flag, workgroup 0 polls all flags (one per thread) and then
//         publishes the epoch; the others poll that.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ unsigned bar0[2];
__device__ unsigned bar1[8 * 32 + 2];

__device__ void sync0(unsigned nb) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned gen = __hip_atomic_load(&bar0[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned a = __hip_atomic_fetch_add(&bar0[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (a == nb - 1) {
      __hip_atomic_store(&bar0[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&bar0[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(&bar0[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen &&
             ++spins < (1u << 24))
        __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// slot s = b % 8 holds nb / 8 (or one more) workgroups
__device__ void sync1(unsigned nb) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned b = blockIdx.x, s = b & 7;
    const unsigned ns = nb / 8 + (s < nb % 8 ? 1u : 0u);
    unsigned* top = &bar1[8 * 32];
    const unsigned gen = __hip_atomic_load(&top[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned a = __hip_atomic_fetch_add(&bar1[s * 32], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    bool last = false;
    if (a == ns - 1) {
      __hip_atomic_store(&bar1[s * 32], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned nslots = nb < 8 ? nb : 8;
      last = __hip_atomic_fetch_add(&top[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nslots - 1;
    }
    if (last) {
      __hip_atomic_store(&top[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&top[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(&top[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen &&
             ++spins < (1u << 24))
        __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__device__ unsigned flags2[1024];
__device__ unsigned gen2;
__device__ void sync2(unsigned nb) {
  __syncthreads();
  __shared__ unsigned ep;
  if (threadIdx.x == 0) {
    ep = __hip_atomic_load(&gen2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __hip_atomic_store(&flags2[blockIdx.x], ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const unsigned e = ep;
  if (blockIdx.x == 0) {
    for (unsigned i = threadIdx.x; i < nb; i += blockDim.x) {
      unsigned spins = 0;
      while (__hip_atomic_load(&flags2[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != e &&
             ++spins < (1u << 24))
        __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&gen2, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  } else if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(&gen2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != e &&
           ++spins < (1u << 24))
      __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
}

// Form 3: form 0 with relaxed atomics and no fences (pfsgnn_mlp.hip grid_sync's
//         default since round 4: the hand-off bytes go sc1 both ways instead)
__device__ unsigned bar3[2];
__device__ void sync3(unsigned nb) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned gen = __hip_atomic_load(&bar3[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned a = __hip_atomic_fetch_add(&bar3[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a == nb - 1) {
      __hip_atomic_store(&bar3[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&bar3[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(&bar3[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen &&
             ++spins < (1u << 24))
        __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// Form 4: form 3 with one word (arrivals | generation << 16): the last arrival
//         resets and bumps in one add (pfsgnn_mlp.hip grid_sync's default)
__device__ unsigned bar4;
__device__ void sync4(unsigned nb) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned a = __hip_atomic_fetch_add(&bar4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((a & 0xffffu) == nb - 1) {
      __hip_atomic_fetch_add(&bar4, 0x10000u - nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while ((__hip_atomic_load(&bar4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 16) == (a >> 16) &&
             ++spins < (1u << 24))
        __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

template <int FORM>
__global__ __launch_bounds__(256) void k_bar(int n, float* sink) {
  float v = threadIdx.x;
  for (int i = 0; i < n; ++i) {
    if (FORM == 0) sync0(gridDim.x); else if (FORM == 1) sync1(gridDim.x);
    else if (FORM == 2) sync2(gridDim.x); else if (FORM == 3) sync3(gridDim.x); else sync4(gridDim.x);
    v = v * 1.0001f + 1.f;
  }
  if (v == -1.f) sink[0] = v;
}

template <int FORM>
float run(int nb, int n) {
  float* sink;
  hipMalloc(&sink, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_bar<FORM>, dim3(nb), dim3(256), 0, 0, n, sink);
  hipEventRecord(a, 0);
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_bar<FORM>, dim3(nb), dim3(256), 0, 0, n, sink);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipFree(sink);
  return ms * 1000.f / 20.f;
}

int main() {
  for (int nb : {64, 128, 256}) {
    for (int form = 0; form < 5; ++form) {
      auto R = [&](int n) {
        return form == 0 ? run<0>(nb, n) : form == 1 ? run<1>(nb, n) : form == 2 ? run<2>(nb, n)
             : form == 3 ? run<3>(nb, n) : run<4>(nb, n);
      };
      const float t1 = R(1), t21 = R(21), t0 = R(0);
      printf("blocks %3d form %d: launch %.2f us, 1 barrier %.2f us, per barrier (21 vs 1) %.2f us\n",
             nb, form, t0, t1, (t21 - t1) / 20.f);
    }
  }
  return 0;
}
