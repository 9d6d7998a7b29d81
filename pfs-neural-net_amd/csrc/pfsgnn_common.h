// pfsgnn_common.h -- shared device/host helpers for libpfsgnn (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <string>

#define PF_LEAKY 0.1f
#define PF_BLOCK 256

// Wave-uniform read-only table (weights, per-class node rows) seen through the
// constant address space, behind an opaque copy the compiler may not hoist:
// reads inside a loop become s_load (scalar-cache hits) next to their use,
// instead of hundreds of loop-invariant values hoisted into more SGPRs than
// exist and spilled to VGPR lanes.
typedef const float __attribute__((address_space(4)))* pf_cptr;
__device__ __forceinline__ pf_cptr pf_fresh(const float* p) {
  pf_cptr q = (pf_cptr)p;
  asm volatile("" : "+s"(q));
  return q;
}

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------- bf16x3 operands
// v = hi + lo (+ ~2^-17 |v|): hi = bf16_rne(v), lo = bf16_rne(v - hi); a
// product of two split operands as Ah Bl + Al Bh + Ah Bh is ~2^-16 relative
// (the node-level gradient chains and weight gradients: pfsgnn_node.hip
// wgrad_block, pfsgnn_mlp.hip k_mlp_bwd).  In the 16x16x32 MFMA a lane's 8
// K slots are two 4-slot halves, so two hidden tiles -- or the hi and lo
// planes of one -- concatenate into one operand (pfsgnn_mfma_core.h).
typedef short pf_s16x4 __attribute__((ext_vector_type(4)));
typedef short pf_s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 pf_b16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 pf_b16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ float pf_bf(short x) {
  return __builtin_bit_cast(float, ((uint32_t)(uint16_t)x) << 16);
}
__device__ __forceinline__ void pf_split4(float a, float b, float c, float d, pf_s16x4& h,
                                          pf_s16x4& l) {
  const pf_b16x4 hb = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  h = __builtin_bit_cast(pf_s16x4, hb);
  const pf_b16x4 lb = {(__bf16)(a - pf_bf(h[0])), (__bf16)(b - pf_bf(h[1])),
                       (__bf16)(c - pf_bf(h[2])), (__bf16)(d - pf_bf(h[3]))};
  l = __builtin_bit_cast(pf_s16x4, lb);
}
__device__ __forceinline__ pf_s16x8 pf_cat8(pf_s16x4 a, pf_s16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
// (No MF_SRC_KEEP here, pfsgnn_mfma_core.h mf8: the node kernels are
// reproducible without it, tests/test_gpu_determinism.py, and the asm forced
// their results out of AGPRs: k_mlp_bwd<7> 43 -> 53 us.)
__device__ __forceinline__ floatx4 pf_mf8(pf_s16x8 a, pf_s16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(pf_b16x8, a),
                                                 __builtin_bit_cast(pf_b16x8, b), c, 0, 0, 0);
}

// ------------------------------------------------------------------ errors
namespace pf {
void set_error(const std::string& msg);
int fail(const char* where, const char* what);
// the class launch of pfsgnn_target_block_fwd (pfsgnn_mlp.hip) and its
// workspace in floats
size_t tail_ws_floats(int G, int NC, int F);
int check_launch(const char* where);
int fail_pending(const char* where, const char* what);
int take_pending(int rc);
// the node level's gradient chains / weight gradients in bf16x3 (pfsgnn_node.hip):
// env `knob` = 0 / 1 when set, else on for every edge path but the exact-fp32 ones
bool node_x3(const char* knob);
// brackets one kernel launch with HIP events when pfsgnn_timing_enable(1)
// extra back-to-back launches of a named main kernel (pfsgnn_timing_repeat;
// 0 unless bench.py measures that kernel's in-graph duration)
int repeats(const char* name);
class Timer {
 public:
  Timer(const char* name, hipStream_t st);
  void end();

 private:
  const char* name_;
  hipStream_t st_;
  hipEvent_t a_;
};
}  // namespace pf

#define PF_REQUIRE(cond, where, what) \
  do {                                \
    if (!(cond)) return pf::fail(where, what); \
  } while (0)

// ------------------------------------------------------------ activations
// torch.nn.LeakyReLU(0.1) and its backward (grad * (x > 0 ? 1 : slope)).
__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : PF_LEAKY * x; }
__device__ __forceinline__ float dlrelu(float z) { return z > 0.f ? 1.f : PF_LEAKY; }

// agent-scope relaxed atomic store / load of a float: global_store / load ... sc1
// (write-through / L1-bypassing; the in-launch hand-off below)
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------ double BatchNorm
// EdgeModel's BatchNorm applied twice (gnn.py:101) from the batch moments
// (m, v) of channel c: xe_new = sc*y + sh, and both running-stat updates.
__device__ __forceinline__ void bn2_coef(const float* gamma, const float* beta, float* rm,
                                         float* rv, int c, long long n, float momentum, float eps,
                                         float m, float v, float* sc, float* sh, float* inv1o,
                                         float* inv2o) {
  const float g = gamma[c], bt = beta[c];
  const float inv1 = 1.0f / sqrtf(v + eps);
  const float rho = v * inv1 * inv1;
  const float v2 = g * g * rho;
  const float inv2 = 1.0f / sqrtf(v2 + eps);
  const float s = g * g * inv1 * inv2;
  sc[c] = s;
  sh[c] = bt - m * s;
  inv1o[c] = inv1;
  inv2o[c] = inv2;
  if (rm) {
    const float f = n > 1 ? (float)((double)n / (double)(n - 1)) : 1.f;
    float a = (1.f - momentum) * rm[c] + momentum * m;
    float b = (1.f - momentum) * rv[c] + momentum * (v * f);
    a = (1.f - momentum) * a + momentum * bt;
    b = (1.f - momentum) * b + momentum * (v2 * f);
    rm[c] = a;
    rv[c] = b;
  }
}

// its backward as g_y = alpha*g + gam0 + gam1*y from Sg = sum g, Sgx = sum g*xhat
__device__ __forceinline__ void bn2_bwd_coef_one(int c, float Sg, float Sgx, const float* mu1,
                                                 const float* var1, const float* gamma,
                                                 long long n, float eps, float* alpha,
                                                 float* gam0, float* gam1, float* dgamma,
                                                 float* dbeta) {
  const float g = gamma[c], v = var1[c];
  const float inv1 = 1.0f / sqrtf(v + eps);
  const float rho = v * inv1 * inv1;
  const float inv2 = 1.0f / sqrtf(g * g * rho + eps);
  const float k = g * inv2;
  const float M = Sgx / (float)n;
  const float a = g * inv1 * k;
  const float g1 = -a * M * (k * k + 1.f - k * k * rho) * inv1;
  alpha[c] = a;
  gam1[c] = g1;
  gam0[c] = -a * Sg / (float)n - g1 * mu1[c];
  dgamma[c] += k * Sgx * (2.f - k * k * rho);
  dbeta[c] += Sg;
}

// ------------------------------------------------------------ edge geometry
// Canonical edge order is class-major, e = (g*NC + c)*NF + f.  A block of 4
// waves owns 64 consecutive fibers (lane = fiber) of one graph -- fiber group
// fg of NFG = ceil(NF/64) -- and a range of CPS classes (class split ks of KS);
// wave w takes classes c0 + w, c0 + w + 4, ...  KS is chosen so that the grid
// has ~512 blocks (2 per CU) when the batch is small.
struct EdgeGeo {
  int G, NF, NC, NFG, KS, CPS, nblocks;
  long long E, NS, NT;
  // XCD-aware block order of the MFMA edge kernels (pfsgnn_mfma_core.h
  // MF_GEO): 0 = blockIdx order; else the launch has 8 * xcdper blocks and
  // hardware block b (dispatched to XCD b % 8) runs logical block
  // (b % 8) * xcdper + b / 8, so each XCD works a contiguous range of logical
  // blocks -- neighbouring 64-fiber groups, whose edge rows share 128-byte
  // lines, read them through one L2
  int xcdper = 0;
};

// the launch grid of an edge kernel (EdgeGeo::xcdper: rounded to 8 blocks)
static inline unsigned edge_grid(const EdgeGeo& geo) {
  return geo.xcdper ? 8u * (unsigned)geo.xcdper : (unsigned)geo.nblocks;
}
// the logical block of this hardware block (XCD order), >= nblocks: none
#define PF_LOGICAL_BLOCK(geo)                                                          \
  ((geo).xcdper ? (int)(blockIdx.x & 7u) * (geo).xcdper + (int)(blockIdx.x >> 3)       \
                : (int)blockIdx.x)

// Blocks of 4 waves on 64 fibers; KS class splits bring the grid to about
// `target` blocks (2048 = 8 blocks of 4 waves per CU on 256 CUs: enough
// resident waves to hide the scalar-weight and HBM latencies).
static constexpr int PF_TARGET_BLOCKS = 2048;
static inline EdgeGeo make_geo(int G, int NF, int NC, int target = PF_TARGET_BLOCKS) {
  EdgeGeo g;
  g.G = G; g.NF = NF; g.NC = NC;
  g.NFG = (NF + 63) / 64;
  const int groups = G * g.NFG;
  int ks = (target + groups - 1) / groups;
  const int maxks = (NC + 3) / 4;
  if (ks > maxks) ks = maxks;
  if (ks < 1) ks = 1;
  g.CPS = (NC + ks - 1) / ks;
  g.KS = (NC + g.CPS - 1) / g.CPS;
  g.nblocks = groups * g.KS;
  g.E = (long long)G * NF * NC;
  g.NS = (long long)G * NF;
  g.NT = (long long)G * NC;
  return g;
}

// 64-lane sum via DPP row butterflies + 4 readlanes; every lane gets the total
__device__ __forceinline__ float wave_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float c = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return (a + b) + (c + d);
}

// (na, mean, M2, M3, M4) <- merge with (nb, ...)   [Pebay 2008, eq. 3.1 ff.]
template <typename T>
__device__ __forceinline__ void pebay_merge(T na, T& ma, T& M2a, T& M3a, T& M4a, T nb, T mb,
                                            T M2b, T M3b, T M4b) {
  const T n = na + nb;
  const T d = mb - ma, d2 = d * d, nanb = na * nb;
  const T in = T(1) / n, in2 = in * in;
  M4a = M4a + M4b + d2 * d2 * nanb * (na * na - nanb + nb * nb) * in2 * in +
        T(6) * d2 * (na * na * M2b + nb * nb * M2a) * in2 + T(4) * d * (na * M3b - nb * M3a) * in;
  M3a = M3a + M3b + d2 * d * nanb * (na - nb) * in2 + T(3) * d * (na * M2b - nb * M2a) * in;
  M2a = M2a + M2b + d2 * nanb * in;
  ma = ma + d * nb * in;
}

// SModel's per-fiber moments of element idx = c*NS + n from the KS class-split
// Pebay partials partS [KS][4][C][NS] (merged in k order, in double), written
// as mom [4][C][NS] = (mean, M2/n, M3/n, M4/n) and hs [4C][NS] = (mean, std,
// skew, kurt) with gnn.py:140-151's leaky variance and eps
// (SC1: the partials are read with sc1 loads -- the in-launch hand-off)
template <bool SC1 = false>
__device__ __forceinline__ void source_finalize_one(const float* __restrict__ partS, int KS,
                                                    int CPS, int C, long long NS, int NC,
                                                    long long idx, float* __restrict__ mom,
                                                    float* __restrict__ hs) {
  const long long CNS = (long long)C * NS;
  double na = 0, mean = 0, M2 = 0, M3 = 0, M4 = 0;
  for (int k = 0; k < KS; ++k) {
    const float* p = partS + (size_t)k * 4 * CNS + idx;
    const double nb = (double)(min(NC, (k + 1) * CPS) - k * CPS);
    if (nb <= 0) break;
    const float p0 = SC1 ? ld_sc1(p) : p[0], p1 = SC1 ? ld_sc1(p + CNS) : p[CNS];
    const float p2 = SC1 ? ld_sc1(p + 2 * CNS) : p[2 * CNS];
    const float p3 = SC1 ? ld_sc1(p + 3 * CNS) : p[3 * CNS];
    if (na == 0) {
      mean = p0; M2 = p1; M3 = p2; M4 = p3;
    } else {
      pebay_merge<double>(na, mean, M2, M3, M4, nb, p0, p1, p2, p3);
    }
    na += nb;
  }
  const double invn = 1.0 / (double)NC;
  const float c2 = (float)(M2 * invn), c3 = (float)(M3 * invn), c4 = (float)(M4 * invn);
  mom[idx] = (float)mean;
  mom[CNS + idx] = c2;
  mom[2 * CNS + idx] = c3;
  mom[3 * CNS + idx] = c4;
  const float var = c2 > 0.f ? c2 : 0.01f * c2;  // F.leaky_relu (slope 0.01), gnn.py:141
  const float sd = sqrtf(var + 1e-6f);
  hs[idx] = (float)mean;
  hs[CNS + idx] = sd;
  hs[2 * CNS + idx] = c3 / (sd * sd * sd);
  hs[3 * CNS + idx] = c4 / ((sd * sd) * (sd * sd));
}

// ------------------------------------------------------------ reductions
// Sum NV values over the whole 256-thread block into out[0..NV) (LDS), valid
// after the call for every thread.  `scratch` >= 4*NV floats.
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* scratch) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float x = v[i];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    v[i] = x;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) scratch[wave * NV + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i)
    v[i] = ((scratch[i] + scratch[NV + i]) + scratch[2 * NV + i]) + scratch[3 * NV + i];
}

// ------------------------------------------------------------ MFMA wgrad
// Accumulates sum over a wave's 64 lanes (one edge each) of a (x) b, with
// a in R^MA, b in R^NB, on v_mfma_f32_16x16x4_f32 (exact f32 products): the
// edge index is the MFMA K dimension, staged through LDS rows [64][LDA] and
// [64][LDB] (each lane writes its own row).  Lane l supplies A[i=l&15][k=l>>4]
// = a_{edge 4s+(l>>4)}[16mt+i] and B[k][j=l&15] = b_{edge 4s+(l>>4)}[16nt+j].
// Result D[16mt + 4*(l>>4) + r][16nt + (l&15)] = acc[mt][nt][r].
template <int MA, int NB>
struct WGrad {
  static constexpr int MT = (MA + 15) / 16;
  static constexpr int NT = (NB + 15) / 16;
  static constexpr int LDA = MA | 1;  // odd: conflict-free row writes
  static constexpr int LDB = NB | 1;
  static constexpr int LDS_FLOATS = 64 * (LDA + LDB);  // per wave
  floatx4 acc[MT][NT];

  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  // wave-private LDS region; call stage() then (after a barrier) accum().
  __device__ __forceinline__ void stage(float* region, const float* a, const float* b, int lane) {
    float* A = region;
    float* B = region + 64 * LDA;
#pragma unroll
    for (int i = 0; i < MA; ++i) A[lane * LDA + i] = a[i];
#pragma unroll
    for (int j = 0; j < NB; ++j) B[lane * LDB + j] = b[j];
  }

  __device__ __forceinline__ void accum(const float* region, int lane) {
    const float* A = region;
    const float* B = region + 64 * LDA;
    const int col = lane & 15;
    const int kq = lane >> 4;
#pragma unroll 4
    for (int s = 0; s < 16; ++s) {
      const int q = 4 * s + kq;
      float av[MT], bv[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int i = 16 * a + col;
        av[a] = (i < MA) ? A[q * LDA + i] : 0.f;
      }
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const int j = 16 * b + col;
        bv[b] = (j < NB) ? B[q * LDB + j] : 0.f;
      }
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }

  // Sum the block's 4 waves and write the block partial [MA][NB] to part.
  // `scratch` >= 4*MA*NB floats.
  __device__ __forceinline__ void block_partial(float* scratch, float* part) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    __syncthreads();
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * a + 4 * (lane >> 4) + r;
          const int j = 16 * b + (lane & 15);
          if (i < MA && j < NB) scratch[(wave * MA + i) * NB + j] = acc[a][b][r];
        }
    __syncthreads();
    for (int idx = t; idx < MA * NB; idx += PF_BLOCK)
      part[idx] = ((scratch[idx] + scratch[MA * NB + idx]) + scratch[2 * MA * NB + idx]) +
                  scratch[3 * MA * NB + idx];
  }
};

// ------------------------------------------------------------ noise
// Counter-based uniform in [0,1) (24-bit), bit-identical to tests/noise_ref.py.
__host__ __device__ __forceinline__ uint64_t pf_fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t pf_noise_key(uint64_t seed) {
  return pf_fmix64(seed ^ 0xD1B54A32D192ED03ull);
}
__device__ __forceinline__ float pf_uniform(uint64_t key, uint64_t e) {
  const uint64_t z = pf_fmix64(key + (e + 1ull) * 0x9E3779B97F4A7C15ull);
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// ------------------------------------------------------------ reduce kernels
// out[r*ldo + c] (+)= scale * sum_{b<nb} part[b*plen + r*ldp + c] -- finishes
// every per-block partial deterministically (fixed block order).
// One pending partial reduction; up to PF_MAX_RED of them share one launch.
struct RedDesc {
  const float* part;
  int nb;
  size_t plen;
  int ldp, rows, cols;
  float* out;
  int ldo, add;
  float scale;
};
#define PF_MAX_RED 96   // (packed 40-byte descriptors, pfsgnn_node.hip RedDev: 3840 B of kernel arguments)
int launch_reduce_multi(const RedDesc* d, int n, hipStream_t st);
// Deferred weight-gradient reductions (pfsgnn_defer_begin / _end): while a
// pass is open, the edge backward kernels put their weight partials in the
// caller's arena and queue the reductions; nullptr when closed or full (the
// caller then reduces at once, as outside a pass).
namespace pf {
float* defer_take(size_t nfloats);
void defer_push(const RedDesc* d, int n);
}  // namespace pf
int launch_reduce_rows(const float* part, int nb, size_t plen, int ldp, int rows, int cols,
                        float* out, int ldo, int add, float scale, hipStream_t st);
// Column partials [G][NFG][NC][C] -> channel-major node tensor out[C][G*NC].
void launch_reduce_columns(const float* part, int G, int BPG, int NC, int C, float* out,
                           hipStream_t st);

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// ------------------------------------------------------------ in-launch hand-off
// A kernel whose blocks each write a partial of a group (the KS class splits of
// a fiber group, ...) can finish the group's reduction in the block that
// arrives last, instead of a separate reduce launch.  Protocol (gfx950, the
// sc1 form of MI355X_MICROARCH.md's hand-off table, row 1): every partial byte
// is stored with an agent-scope relaxed atomic store (global_store ... sc1,
// written through to the memory side), every storing wave waits for its
// stores, a workgroup barrier, then ONE lane adds 1 to the group's counter
// (agent-scope atomic, returning); the block that draws expect-1 reads every
// partial with sc1 loads (agent-scope relaxed atomic loads) after another
// barrier, and resets the counter for the next launch.  No release fence
// (no L2 write-back) is needed: no partial is ever held in a non-coherent L2.
// The winning block's counting lane then runs ONE agent-scope acquire
// (buffer_inv sc1 + s_waitcnt vmcnt(0)) before the barrier that releases its
// other waves (round 6): the guide's table row is measured for one workgroup
// per CU, and edge_mlp_fwd runs several per CU with 84-byte partials that
// straddle lines written by other blocks, so the hand-off keeps the consumer
// acquire the guide prescribes outside a row (MI355X_MICROARCH.md, "Consumer,
// always").  It is paid once per winning block (<= 1 + 64 per launch).
// The counters live in the library's zero-initialised sync buffer
// (pfsgnn_set_sync_buffer); without one the callers keep their reduce launch.
namespace pf {
unsigned* sync_counters(size_t n);   // n counters, or nullptr
// a launch's own run of n counters (round robin over the buffer, so
// launches in flight at the same time on different streams never share one),
// or nullptr without a sync buffer
unsigned* sync_slot(size_t n);
}  // namespace pf
// true in every thread of the block that arrives last of `expect` at *cnt
// (the caller's stores of its partial must all be st_sc1); flag: an LDS word
__device__ __forceinline__ bool last_arrival(unsigned* cnt, unsigned expect, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old + 1u == expect ? 1 : 0;
    if (last) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

__device__ __forceinline__ void st_sc1d(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1d(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------ in-launch Welford finalize
// With `bn` (EdgeModel training forward): also the double BatchNorm's affine
// and running statistics of each channel, as pfsgnn_bn2_finalize computes them.
struct Bn2Args {
  const float* gamma;
  const float* beta;
  float* rm;
  float* rv;
  float momentum, eps;
  float *sc, *sh, *inv1, *inv2;
};

// The BatchNorm statistics of an edge kernel's per-block Welford partials
// ([nb][1 + 2F]: count, mean[F], M2[F], every value stored st_sc1) finished by
// the kernel's own last blocks instead of a k_moments_finalize launch (the
// hand-off protocol above): the last block of each group of MOM_GROUP partials
// merges them in double into a group partial (count, sum count*mean, M2 about
// the group mean), and the last group merges the groups and writes mu, the
// biased var (+ the double BatchNorm's coefficients and running statistics).
// Partials are assigned to threads in a fixed pattern and summed by fixed
// trees: bitwise reproducible, and within double rounding of the one-launch
// closed form.
constexpr int MOM_GROUP = 64, MOM_MAXG = 64;   // nb <= 4096
struct MomFin {
  unsigned* cnt;   // 1 + MOM_MAXG hand-off counters (pf::sync_slot); nullptr: off
  double* gp;      // [MOM_MAXG][3][16] group partials
  float* mu;
  float* var;
  long long n;     // the statistics' element count (var = M2 / n)
  Bn2Args bn;
};

template <int F>
__device__ void mom_finalize(const float* part, int nb, int b, const MomFin& f) {
  static_assert(F <= 16, "mom_finalize: 16 channels per thread slot");
  __shared__ int flag;
  __shared__ double red[4][3][16];
  const int t = threadIdx.x, k = t & 15, j = t >> 4, wv = t >> 6;
  // the 16 slots j of channel k summed in one order: lanes j, j^1.. of a wave
  // (xor 16, 32), then the 4 waves
  auto slot_sum = [&](double v, int w) -> double {
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if ((t & 63) < 16) red[wv][w][k] = v;
    __syncthreads();
    return (red[0][w][k] + red[1][w][k]) + (red[2][w][k] + red[3][w][k]);
  };
  const int grp = b / MOM_GROUP, ng = (nb + MOM_GROUP - 1) / MOM_GROUP;
  const int b0 = grp * MOM_GROUP, nin = min(MOM_GROUP, nb - b0);
  if (!last_arrival(f.cnt + 1 + grp, (unsigned)nin, &flag)) return;
  // every load unconditional (clamped index) so that all 12 are in flight at
  // once; the out-of-range ones are zeroed after
  float lc[4], lm[4], lq[4];
  const int kc = min(k, F - 1);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float* p = part + (size_t)(b0 + min(j + 16 * i, nin - 1)) * (1 + 2 * F);
    lc[i] = ld_sc1(p);
    lm[i] = ld_sc1(p + 1 + kc);
    lq[i] = ld_sc1(p + 1 + F + kc);
  }
  double c[4], m[4], q[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = j + 16 * i < nin && k < F;
    c[i] = ok ? (double)lc[i] : 0.0;
    m[i] = ok ? (double)lm[i] : 0.0;
    q[i] = ok ? (double)lq[i] : 0.0;
  }
  const double N = slot_sum((c[0] + c[1]) + (c[2] + c[3]), 0);
  const double S = slot_sum((c[0] * m[0] + c[1] * m[1]) + (c[2] * m[2] + c[3] * m[3]), 1);
  const double mg = N > 0.0 ? S / N : 0.0;
  double Q = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double d = m[i] - mg;
    Q += q[i] + c[i] * d * d;
  }
  Q = slot_sum(Q, 2);
  if (t < F) {
    double* g = f.gp + (size_t)grp * 48;
    st_sc1d(g + t, N);
    st_sc1d(g + 16 + t, S);
    st_sc1d(g + 32 + t, Q);
  }
  if (!last_arrival(f.cnt, (unsigned)ng, &flag)) return;
  // the groups, the same way (red's rows are rewritten only after the
  // barriers of last_arrival)
  double gn[4], gs[4], gq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double* g = f.gp + (size_t)min(j + 16 * i, ng - 1) * 48;
    gn[i] = ld_sc1d(g + kc);
    gs[i] = ld_sc1d(g + 16 + kc);
    gq[i] = ld_sc1d(g + 32 + kc);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = j + 16 * i < ng && k < F;
    gn[i] = ok ? gn[i] : 0.0;
    gs[i] = ok ? gs[i] : 0.0;
    gq[i] = ok ? gq[i] : 0.0;
  }
  const double NT = slot_sum((gn[0] + gn[1]) + (gn[2] + gn[3]), 0);
  const double ST = slot_sum((gs[0] + gs[1]) + (gs[2] + gs[3]), 1);
  const double M0 = NT > 0.0 ? ST / NT : 0.0;
  double QT = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double d = gn[i] > 0.0 ? gs[i] / gn[i] - M0 : 0.0;
    QT += gq[i] + gn[i] * d * d;
  }
  QT = slot_sum(QT, 2);
  if (t < F) {
    const float mu = (float)M0, v = (float)(QT / (double)f.n);
    f.mu[t] = mu;
    f.var[t] = v;
    if (f.bn.gamma)
      bn2_coef(f.bn.gamma, f.bn.beta, f.bn.rm, f.bn.rv, t, f.n, f.bn.momentum, f.bn.eps, mu, v,
               f.bn.sc, f.bn.sh, f.bn.inv1, f.bn.inv2);
  }
}
