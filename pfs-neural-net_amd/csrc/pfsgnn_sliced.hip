// pfsgnn_sliced.hip -- the per-edge kernels of GENERAL (non-complete) bipartite
// graphs, fused on the matrix cores like the complete-graph ones
// (pfsgnn_mfma.hip): the reference's scatters run on any edge_index
// (gnn.py:140-144 per fiber, gnn.py:190 per class).
//
// Layout (pfsgnn_sliced_plan / pfsgnn_sliced_fill, pfsgnn_sparse.hip).  Each
// graph's fibers are sorted by degree (descending, stable) and cut into slices
// of 16; slice s holds the k-th edge of its 16 fibers at the 16 consecutive
// positions base[s] + 16 k + lane, k < len[s] = the slice's largest degree.  A
// fiber with fewer edges leaves padding positions (class byte 0xFF; every edge
// tensor holds 0 there).  Edge tensors are channel-major [C][EP] over these
// positions.  A wave owns one slice and walks k exactly as a complete-graph wave
// walks its classes:
//   * every edge-row load / store is one 64-byte segment per lane group;
//   * the lane's fiber is fixed: its node parts (Ps, Rs, moments) stay in
//     registers and its sums over edges are thread-local; a fiber's edges are a
//     PREFIX of k, so Pebay's one-pass update runs with the count k + 1, uniform
//     over the wave (coefficient table sl.pco);
//   * the class of a lane's edge is per lane (one byte per position): the
//     class-table rows (Pt, Qt, g_hsum) of the whole graph are staged in LDS and
//     read per lane;
//   * per-class sums (TModel's scatter-sum, gnn.py:190; the class-side
//     gradients) go to a wave-private LDS accumulator [NC][D + 1] (acc_add: a
//     DPP row sum when the tile's edges share one class, else plain
//     read-add-writes in conflict-free rounds -- one wave's updates of one
//     row happen in a fixed order, so the sums are reproducible), then the
//     4 waves' accumulators are merged in fixed order into the complete path's
//     per-block column partials [G][NFG][NC][D].
// The grid is the complete path's with KS = 1 (block = 4 slices = 64 fibers of
// one graph, NFG blocks per graph), so every finishing reduction, BatchNorm
// finalize and deferred weight-gradient flush of pfsgnn_edge.hip is shared.
#include "pfsgnn_mfma_core.h"

#include <algorithm>
#include <cstdlib>

namespace {

using pfm::SlGeo;

// per-step rows of a slice: the edge rows, the position's class byte, and the
// TModel mask byte (TM kernels)
template <int NA>
struct SRows {
  floatx4 v[NA];
  uint32_t c;   // class within the graph, 0xFF: padding
  uint32_t m;
};

#define SL_GEO                                                                         \
  const int t = threadIdx.x, lane = t & 63;                                            \
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);                             \
  const int g4 = lane >> 4, j16 = lane & 15;                                           \
  const int bx = blockIdx.x;                                                           \
  const int ks = bx % geo.KS, grp = bx / geo.KS;                                       \
  const int fg = grp % geo.NFG, gg = grp / geo.NFG;                                    \
  const int slc = 4 * grp + wave;                                                      \
  const int fib = sl.fib[slc * 16 + j16];                                              \
  const bool fvalid = fib >= 0;                                                        \
  const long long n = fvalid ? fib : 0;                                                \
  const int pb = __builtin_amdgcn_readfirstlane(sl.base[slc]);                         \
  const int Ls = __builtin_amdgcn_readfirstlane(sl.len[slc]);                          \
  /* split ks of KS: steps [k0, k1) of the slice */                                    \
  const int k0 = (int)(((long long)Ls * ks) / geo.KS);                                 \
  const int k1 = (int)(((long long)Ls * (ks + 1)) / geo.KS);                           \
  const int NC = geo.NC;                                                               \
  const long long NS = geo.NS;                                                         \
  const uint32_t RB = (uint32_t)geo.E * 4u; /* channel-row bytes of an edge tensor */  \
  const uint32_t EB = RB;                                                              \
  const uint32_t eo0 = (uint32_t)(pb + j16) * 4u;                                      \
  constexpr uint32_t eoc = 64u; /* one step = 16 positions */                          \
  /* class partials [G][NFG * KS][NC][D] (columns_lin with NFG * KS blocks per graph) */ \
  const long long colbase = ((long long)grp * geo.KS + ks) * NC;                       \
  const Rsrc rcl = rsrc(sl.cls, (uint32_t)geo.E);                                      \
  (void)t; (void)n; (void)NS; (void)colbase; (void)EB; (void)fg; (void)gg; (void)k0; (void)k1;

// the class byte of step k of the lane's fiber
#define SL_CLS(k) \
  __builtin_amdgcn_raw_buffer_load_b8(rcl, (uint32_t)j16, (uint32_t)pb + 16u * (uint32_t)(k), 0)

// the step's per-lane validity: class (0 at padding), edge present, row masks
#define SL_STEP(rows)                                                                   \
  const int cls_ = (int)(rows).c;                                                       \
  const bool ev = cls_ != 0xFF;                                                         \
  const int cl = ev ? cls_ : 0;                                                         \
  bool fe[4];                                                                           \
  _Pragma("unroll") for (int r = 0; r < 4; ++r) fe[r] = fm[r] && ev;

extern __shared__ __attribute__((aligned(16))) float sl_dyn[];

// The graph's class-table rows (Pt, Qt, g_hsum) in LDS, ClassRows' slot order
// with a row stride of CP + 4 floats: the lanes of a tile read 16 different
// classes' rows, and a stride of CP = 32 / 48 words would put them all on the
// same banks.
template <int D>
struct SlRows {
  static constexpr int CP = ClassRows<D>::CP, S = CP + 4;
  __device__ __forceinline__ static void stage(float* buf, const float* P, long long NT,
                                               long long cn0, int ncl) {
    for (int i = threadIdx.x; i < ncl * CP; i += PF_BLOCK) {
      const int cl = i / CP, q = i - cl * CP;
      const int h = GM<D>::row((q >> 2) & 3, 4 * (q >> 4) + (q & 3));
      buf[cl * S + q] = h >= 0 ? P[(long long)h * NT + cn0 + cl] : 0.f;
    }
  }
  __device__ __forceinline__ static floatx4 get(const float* buf, int cl, int t, int g) {
    return *reinterpret_cast<const floatx4*>(buf + cl * S + 16 * t + 4 * g);
  }
};

// A wave's class accumulator is [NC][S]: S = D + 1 (odd: the rows of
// different classes spread over the LDS banks; a stride of 20 or 40 words maps
// every class row onto 16 / 8 bank offsets) -- or D + 2 when a lane group's
// rows come in even runs (RPG even: 4F = 32 / 40 / 64), so a lane's channel
// pairs are 8-byte aligned and its read-add-writes go as float2 (half the LDS
// instructions; S / 2 odd spreads the rows over the banks the same way).
constexpr int acc_stride(int D) { return ((D + 3) / 4) % 2 == 0 ? D + 2 : D + 1; }
template <int D>
struct Acc {
  static constexpr int S = acc_stride(D);
  static constexpr bool PAIRS = S == D + 2;
};
// The class rows of every graph in ClassRows' slot order in global memory,
// [G*NC][CP] (k_sl_rows_table): ksl_source_bwd reads its two tables from there
// (L2-resident, 16 B per lane and tile) instead of LDS, which leaves it room
// for two blocks per CU.
template <int D>
__global__ __launch_bounds__(256) void k_sl_rows_table(const float* __restrict__ P, long long NT,
                                                       float* __restrict__ out) {
  constexpr int CP = ClassRows<D>::CP;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= NT * CP) return;
  const long long c = i / CP;
  const int q = (int)(i - c * CP);
  const int h = GM<D>::row((q >> 2) & 3, 4 * (q >> 4) + (q & 3));
  out[i] = h >= 0 ? P[(long long)h * NT + c] : 0.f;
}
template <int D>
__device__ __forceinline__ floatx4 tab_get(const float* tab, long long c, int t, int g) {
  return *reinterpret_cast<const floatx4*>(tab + c * ClassRows<D>::CP + 16 * t + 4 * g);
}

// Class rows of the edge kernels: staged in LDS per block (default), or read
// from the permuted global tables (SL_GLOBAL_TABLES, the A/B variant: no
// per-block staging, but an L2 round trip per tile; measured on the 30 % /
// 99.9 % bench batches: 3 % / 9 % slower; ksl_source_bwd always reads its two
// tables from global memory, which leaves it LDS for two blocks per CU).
// CROWS_DECL(buf, P) prepares, CROW(buf, P, cl, t) reads tile t of class cl
// (within the block's graph gg).
#ifndef SL_GLOBAL_TABLES
#define CROWS_DECL(D, buf, P, base)                                  \
  float* buf = base;                                                 \
  SlRows<D>::stage(buf, P, geo.NT, (long long)gg * NC, NC);
#define CROW(D, buf, P, cl, t) SlRows<D>::get(buf, cl, t, g4)
#define CROWS_FLOATS(D) (SlRows<D>::S)
#else
#define CROWS_DECL(D, buf, P, base) const long long buf = (long long)gg * NC; (void)base;
#define CROW(D, buf, P, cl, t) tab_get<D>(P, buf + (cl), t, g4)
#define CROWS_FLOATS(D) 0
#endif

// zero the 4 waves' class accumulators [4][NC][D + 1]
__device__ __forceinline__ void acc_zero(float* acc, int len4) {
  for (int i = threadIdx.x; i < len4; i += PF_BLOCK) acc[i] = 0.f;
}
// The step's edge vectors (lane (g, j): the channels of lane group g of edge j,
// compact row map) into their classes' rows of the wave's accumulator.  When
// every valid edge of the tile has one class (complete-like slices) the 16
// edges are summed across lanes first (DPP row sums, as km_target_fwd) and one
// lane per group adds.  Otherwise the lanes add their own rows with plain LDS
// read-add-writes, in rounds: each pending lane writes its edge index to its
// class's owner slot; the lanes that read their own index back -- one edge per
// class, the hardware's fixed choice among the writers -- add, the others wait
// for the next round.  One wave's updates of a row thus happen in a fixed
// order.  (Measured on the 30 % bench batch: LDS float atomics instead,
// ~1 lane per 4 cycles on gfx950, 4-8x slower; ranks from DPP row rotations
// instead of the owner slots, +7 %.)  `own`: the wave's [NC] owner table.
template <int D>
__device__ __forceinline__ void acc_add(float* wacc, int* own, int cl, bool ev, int g, int j,
                                        const floatx4 (&v)[GM<D>::NT]) {
#ifdef SL_NO_ACC   // (timing experiment only: class sums dropped)
  return;
#endif
  const uint64_t vm = __ballot(ev);
  if (vm == 0) return;
  const int c0 = __builtin_amdgcn_readlane(cl, (int)__builtin_ctzll(vm));
  if (__ballot(ev && cl != c0) == 0) {
    float* a = wacc + c0 * Acc<D>::S;
#pragma unroll
    for (int tt = 0; tt < GM<D>::NT; ++tt)
#pragma unroll
      for (int r = 0; r < GM<D>::nreg(tt); ++r) {
        const float sum = row_sum16(ev ? v[tt][r] : 0.f);
        const int h = GM<D>::row(g, 4 * tt + r);
        if (j == 15 && h >= 0) a[h] += sum;
      }
    return;
  }
  float* a = wacc + cl * Acc<D>::S;
  bool pend = ev;
  while (__ballot(pend) != 0) {
    if (pend) own[cl] = j;
    lds_order();
    const bool win = pend && own[cl] == j;
    if (win) {
      if constexpr (Acc<D>::PAIRS) {
        // lane group g's rows g*RPG .. g*RPG + RPG - 1 (RPG even) in slot pairs
#pragma unroll
        for (int tt = 0; tt < GM<D>::NT; ++tt)
#pragma unroll
          for (int r = 0; r < GM<D>::nreg(tt); r += 2) {
            const int h = GM<D>::row(g, 4 * tt + r);
            if (h >= 0) {
              float2* q = reinterpret_cast<float2*>(a + h);
              float2 u = *q;
              u.x += v[tt][r];
              u.y += v[tt][r + 1];
              *q = u;
            }
          }
      } else {
#pragma unroll
        for (int tt = 0; tt < GM<D>::NT; ++tt)
#pragma unroll
          for (int r = 0; r < GM<D>::nreg(tt); ++r) {
            const int h = GM<D>::row(g, 4 * tt + r);
            if (h >= 0) a[h] += v[tt][r];
          }
      }
    }
    lds_order();
    pend = pend && !win;
  }
}
// the block's column partial of every class of its graph: 4-wave sums, fixed order
template <int D>
__device__ __forceinline__ void acc_flush(const float* acc, int NC, float* part, long long colbase) {
  __syncthreads();
  const int len = NC * Acc<D>::S;
  float* p = part + colbase * D;
  for (int i = threadIdx.x; i < NC * D; i += PF_BLOCK) {
    const int c = i / D, q = c * Acc<D>::S + (i - c * D);
    p[i] = ((acc[q] + acc[len + q]) + acc[2 * len + q]) + acc[3 * len + q];
  }
}

// ============================================================ EdgeModel fwd
// km_edge_mlp_fwd on slices (gnn.py:86-101): y at every position (0 at padding),
// Welford partials of y over the block's edges
template <int F, int PREC>
__global__ __launch_bounds__(256) void ksl_edge_mlp_fwd(
    EdgeGeo geo, SlGeo sl, const float* __restrict__ xe, const float* __restrict__ xsc,
    const float* __restrict__ xsh, const float* __restrict__ Ps, const float* __restrict__ PtS,
    const float* __restrict__ W1, const float* __restrict__ W2, const float* __restrict__ b2,
    float* __restrict__ y, float* __restrict__ part) {
  constexpr int H = 4 * F, NT = GM<H>::NT;
  SL_GEO
  CROWS_DECL(H, ptl, PtS, sl_dyn)   // [NC][CP]
  FwdLayer<PREC, H, F> L1;
  L1.load([&](int h, int k) { return W1[h * 4 * F + 2 * F + k]; }, lane);
  FwdLayer<PREC, F, H> L2;
  L2.load([&](int o, int h) { return W2[o * H + h]; }, lane);
  floatx4 ps[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) ps[tt] = ld_node<H>(Ps, tt, g4, NS, n, fvalid);
  const floatx4 bb = ld_fconst<F>(b2, g4, 0.f);
  const floatx4 scv = ld_fconst<F>(xsc, g4, 1.f), shv = ld_fconst<F>(xsh, g4, 0.f);
  MF_FMASK(F)
  const Rsrc rxe = rsrc(xe, EB * F);
  float cnt = 0.f;
  floatx4 mean = zero4(), m2 = zero4();
  __syncthreads();   // ptl
  auto load = [&](int k) {
    SRows<1> r;
    r.v[0] = ld_frows<F>(rxe, (uint32_t)k * eoc, ro);
    r.c = SL_CLS(k);
    return r;
  };
  class_stream<MF_DEPTH_FWD>(k0, k1, load, [&](const SRows<1>& rows, int k) {
    SL_STEP(rows)
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fe, xsc, scv, shv)};
    floatx4 z[NT], a[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) z[tt] = ps[tt] + CROW(H, ptl, PtS, cl, tt);
    L1.apply(x, z);
    lrelu_act<H>(z, a);
    floatx4 yo[1] = {bb};
    L2.apply(a, yo);
#pragma unroll
    for (int r = 0; r < 4; ++r) yo[0][r] = ev ? yo[0][r] : 0.f;
    st_frows<F>(y, EB * F, (uint32_t)k * eoc, ro, g4, true, yo[0]);
    if (ev) {
      cnt += 1.f;
      const float rc = __builtin_amdgcn_rcpf(cnt);
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        const float d = yo[0][r] - mean[r];
        mean[r] = fmaf(d, rc, mean[r]);
        m2[r] = fmaf(d, yo[0][r] - mean[r], m2[r]);
      }
    }
  });
  // Chan merge over the 16 lanes of the group, then over the 4 waves
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) {
    const float cb = __shfl_xor(cnt, off);
    const float tot = cnt + cb;
    const float wb = tot > 0.f ? cb / tot : 0.f;
    const float wab = tot > 0.f ? cnt * cb / tot : 0.f;
#pragma unroll
    for (int r = 0; r < GM<F>::RPG; ++r) {
      const float mb = __shfl_xor(mean[r], off), qb = __shfl_xor(m2[r], off);
      const float d = mb - mean[r];
      mean[r] = fmaf(d, wb, mean[r]);
      m2[r] = m2[r] + qb + d * d * wab;
    }
    cnt = tot;
  }
  __shared__ float shm[4][1 + 2 * F];
  if (j16 == 0) {
    if (g4 == 0) shm[wave][0] = cnt;
#pragma unroll
    for (int r = 0; r < GM<F>::RPG; ++r) {
      const int k = GM<F>::row(g4, r);
      if (k >= 0) { shm[wave][1 + k] = mean[r]; shm[wave][1 + F + k] = m2[r]; }
    }
  }
  __syncthreads();
  if (t < F) {
    float C0 = shm[0][0], M0 = shm[0][1 + t], Q0 = shm[0][1 + F + t];
    for (int w = 1; w < 4; ++w) {
      const float cb = shm[w][0], mb = shm[w][1 + t], qb = shm[w][1 + F + t];
      const float tot = C0 + cb;
      if (tot > 0.f) {
        const float d = mb - M0;
        M0 = M0 + d * (cb / tot);
        Q0 = Q0 + qb + d * d * (C0 * cb / tot);
      }
      C0 = tot;
    }
    float* p = part + (size_t)bx * (1 + 2 * F);
    if (t == 0) p[0] = C0;
    p[1 + t] = M0;
    p[1 + F + t] = Q0;
  }
}

// ============================================================ SModel fwd
// message m = Ws2 lrelu(Qt[c] + Ws1[:, F:2F] x) + bs2 (gnn.py:136-137) and the
// fiber's centred moments (gnn.py:140-151).  A block owns ONE slice; wave w
// walks its steps k = w, w + 4, ... with Pebay's one-pass update (the i-th step
// of a wave has count i + 1 in every lane whose fiber reaches it: a fiber's
// edges are a prefix of the steps), then the 4 waves' states are merged per
// fiber (Pebay's pairwise formula in double, fixed order 0 <- 1 <- 2 <- 3, the
// per-lane counts) and the moments and SModel's features go straight to mom /
// hs with the fiber's degree as count (an empty fiber: mean 0, var 0, as
// scatter-mean's clamped count gives).
template <int F, int PREC>
__global__ __launch_bounds__(256) void ksl_source_fwd(
    EdgeGeo geo, SlGeo sl, const float* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ QtS, const float* __restrict__ Ws1,
    const float* __restrict__ Ws2, const float* __restrict__ bs2, float* __restrict__ mom,
    float* __restrict__ hs) {
  constexpr int C = 2 * F, NT = GM<C>::NT;
  constexpr int MS = 4 * 4 * NT;   // a lane's merge state: 4 sums x NT tiles x 4 slots
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g4 = lane >> 4, j16 = lane & 15;
  const int slc = blockIdx.x;                    // one slice per block
  const int gg = slc / (4 * geo.NFG);
  const int fib = sl.fib[slc * 16 + j16];
  const bool fvalid = fib >= 0;
  const long long n = fvalid ? fib : 0;
  const int pb = __builtin_amdgcn_readfirstlane(sl.base[slc]);
  const int Ls = __builtin_amdgcn_readfirstlane(sl.len[slc]);
  const int nw = (Ls - wave + 3) >> 2;           // this wave's steps
  const int NC = geo.NC;
  const long long NS = geo.NS;
  const uint32_t RB = (uint32_t)geo.E * 4u, EB = RB;
  const uint32_t eo0 = (uint32_t)(pb + j16) * 4u;
  constexpr uint32_t eoc = 64u;
  const Rsrc rcl = rsrc(sl.cls, (uint32_t)geo.E);
  CROWS_DECL(C, qtl, QtS, sl_dyn)   // [NC][CP]
  FwdLayer<PREC, C, F> L1;
  L1.load([&](int h, int k) { return Ws1[h * 2 * F + F + k]; }, lane);
  FwdLayer<PREC, C, C> L2;
  L2.load([&](int o, int h) { return Ws2[o * C + h]; }, lane);
  floatx4 bias[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) bias[tt] = ld_vec<C>(bs2, tt, g4);
  const floatx4 scv = ld_fconst<F>(sc, g4, 1.f), shv = ld_fconst<F>(sh, g4, 0.f);
  MF_FMASK(F)
  const Rsrc ry = rsrc(y, EB * F);
  floatx4 S1[NT], S2[NT], S3[NT], S4[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) S1[tt] = S2[tt] = S3[tt] = S4[tt] = zero4();
  float cnt = 0.f;
  __syncthreads();   // qtl
  auto load = [&](int i) {
    const int k = wave + 4 * i;
    SRows<1> r;
    r.v[0] = ld_frows<F>(ry, (uint32_t)k * eoc, ro);
    r.c = SL_CLS(k);
    return r;
  };
  class_stream<MF_DEPTH_FWD>(0, nw, load, [&](const SRows<1>& rows, int i) {
    SL_STEP(rows)
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fe, sc, scv, shv)};
    floatx4 z[NT], a[NT], m[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) z[tt] = CROW(C, qtl, QtS, cl, tt);
    L1.apply(x, z);
    lrelu_act<C>(z, a);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) m[tt] = bias[tt];
    L2.apply(a, m);
    // Pebay's update (km_source_fwd), coefficients of count i + 1
    const floatx4 ca = *reinterpret_cast<const floatx4*>(sl.pco + 8 * i);
    const floatx4 cb = *reinterpret_cast<const floatx4*>(sl.pco + 8 * i + 4);
    if (ev) {
      cnt += 1.f;
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
#pragma unroll
        for (int r = 0; r < GM<C>::nreg(tt); ++r) {
          const float d = m[tt][r] - S1[tt][r], d2 = d * d;
          const float m2 = S2[tt][r], m3 = S3[tt][r];
          S4[tt][r] = fmaf(d, m3 * cb[1], fmaf(d2, fmaf(d2, ca[2], m2 * cb[0]), S4[tt][r]));
          S3[tt][r] = fmaf(d, fmaf(d2, ca[1], m2 * cb[2]), m3);
          S2[tt][r] = fmaf(d2, ca[0], m2);
          S1[tt][r] = fmaf(d, ca[3], S1[tt][r]);
        }
    }
  });
  // merge: waves 1..3 park their states and counts in LDS
  __shared__ float ms[3][MS + 1][64];
  if (wave > 0) {
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ms[wave - 1][(0 * NT + tt) * 4 + r][lane] = S1[tt][r];
        ms[wave - 1][(1 * NT + tt) * 4 + r][lane] = S2[tt][r];
        ms[wave - 1][(2 * NT + tt) * 4 + r][lane] = S3[tt][r];
        ms[wave - 1][(3 * NT + tt) * 4 + r][lane] = S4[tt][r];
      }
    ms[wave - 1][MS][lane] = cnt;
  }
  __syncthreads();
  if (wave != 0 || !fvalid) return;
  double ntot = cnt;
#pragma unroll
  for (int w = 1; w < 4; ++w) ntot += ms[w - 1][MS][lane];
  const double invn = ntot > 0 ? 1.0 / ntot : 0.0;
  const long long CNS = (long long)C * NS;
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
#pragma unroll
    for (int r = 0; r < GM<C>::nreg(tt); ++r) {
      const int o = GM<C>::row(g4, 4 * tt + r);
      if (o < 0) continue;
      double na = cnt, mean = S1[tt][r], M2 = S2[tt][r], M3 = S3[tt][r], M4 = S4[tt][r];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const double nb = ms[w - 1][MS][lane];
        if (nb <= 0) continue;
        pebay_merge<double>(na, mean, M2, M3, M4, nb, ms[w - 1][(0 * NT + tt) * 4 + r][lane],
                            ms[w - 1][(1 * NT + tt) * 4 + r][lane],
                            ms[w - 1][(2 * NT + tt) * 4 + r][lane],
                            ms[w - 1][(3 * NT + tt) * 4 + r][lane]);
        na += nb;
      }
      const long long idx = (long long)o * NS + n;
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
}

// ============================================================ TModel fwd
// a = lrelu(Rs[f] + Wt1[:, F:2F] x) per edge, summed per class (gnn.py:188-190;
// the second Linear runs after the sum, on the node side)
template <int F, int PREC>
__global__ __launch_bounds__(256) void ksl_target_fwd(
    EdgeGeo geo, SlGeo sl, const float* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ Rs, const float* __restrict__ Wt1,
    float* __restrict__ part, uint8_t* __restrict__ tmask) {
  constexpr int C = 2 * F, NT = GM<C>::NT;
  SL_GEO
  float* acc = sl_dyn;   // [4][NC][C + 1]
  acc_zero(acc, 4 * NC * Acc<C>::S);
  float* wacc = acc + wave * NC * Acc<C>::S;
  __shared__ int owners[4][pfm::SL_MAX_NC];
  int* own = owners[wave];
  FwdLayer<PREC, C, F> L1;
  L1.load([&](int h, int k) { return Wt1[h * 2 * F + F + k]; }, lane);
  floatx4 rs[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) rs[tt] = ld_node<C>(Rs, tt, g4, NS, n, fvalid);
  const floatx4 scv = ld_fconst<F>(sc, g4, 1.f), shv = ld_fconst<F>(sh, g4, 0.f);
  MF_FMASK(F)
  const Rsrc ry = rsrc(y, EB * F);
  __syncthreads();   // acc
  auto load = [&](int k) {
    SRows<1> r;
    r.v[0] = ld_frows<F>(ry, (uint32_t)k * eoc, ro);
    r.c = SL_CLS(k);
    return r;
  };
  class_stream<MF_DEPTH_FWD>(k0, k1, load, [&](const SRows<1>& rows, int k) {
    SL_STEP(rows)
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fe, sc, scv, shv)};
    floatx4 z[NT], a[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) z[tt] = rs[tt];
    L1.apply(x, z);
    if (tmask) (tmask + (uint32_t)k * eoc)[opaque(eo0 + g4)] = (uint8_t)mask_bits<C>(z);
    lrelu_act<C>(z, a);
    acc_add<C>(wacc, own, cl, ev, g4, j16, a);
  });
  acc_flush<C>(acc, NC, part, colbase);
}

// ============================================================ TModel bwd
// g_z = g_hsum[c] * lrelu'(z) per edge; the fiber's sums of g_z (-> g_Rs), the
// edge-input gradient Wt1[:, F:2F]^T g_z (optional), dWt1[:, F:2F] += g_z x^T
template <int F, int PREC, bool TM>
__global__ __launch_bounds__(256) void ksl_target_bwd(
    EdgeGeo geo, SlGeo sl, const float* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ Rs, const float* __restrict__ Wt1,
    const float* __restrict__ ghS, float* __restrict__ GzT, float* __restrict__ gxe,
    float* __restrict__ partW, const uint8_t* __restrict__ tmask) {
  constexpr int C = 2 * F, NT = GM<C>::NT;
  constexpr int NIMG = NT + 1;  // g_z tiles | x
  using WI = WgImg<PREC>;       // weight-gradient images: bf16x3, or exact fp32 at PREC 0
  SL_GEO
  __shared__ __attribute__((aligned(16))) short imgs[4 * NIMG * WI::U];
  __shared__ float scratch[4 * C * F];
  CROWS_DECL(C, ghl, ghS, sl_dyn)   // [NC][CP]
  short* img = imgs + wave * NIMG * WI::U;
  FwdLayer<FP(PREC), C, F> L1;
  if constexpr (!TM) L1.load([&](int h, int k) { return Wt1[h * 2 * F + F + k]; }, lane);
  GradLayer<PREC, F, C> LT;
  LT.load([&](int k, int h) { return gxe ? Wt1[h * 2 * F + F + k] : 0.f; }, lane);
  floatx4 rs[NT], accF[NT], accW[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    if constexpr (!TM) rs[tt] = ld_node<C>(Rs, tt, g4, NS, n, fvalid);
    accF[tt] = zero4();
    accW[tt] = zero4();
  }
  const floatx4 scv = ld_fconst<F>(sc, g4, 1.f), shv = ld_fconst<F>(sh, g4, 0.f);
  MF_FMASK(F)
  const Rsrc ry = rsrc(y, EB * F), rtm = rsrc(tmask, EB);
  __syncthreads();   // ghl
  auto load = [&](int k) {
    SRows<1> r;
    const uint32_t co = (uint32_t)k * eoc;
    r.v[0] = ld_frows<F>(ry, co, ro);
    r.c = SL_CLS(k);
    if constexpr (TM) r.m = __builtin_amdgcn_raw_buffer_load_b8(rtm, eo0 + g4, co, 0);
    return r;
  };
  class_stream<MF_DEPTH_BWD>(k0, k1, load, [&](const SRows<1>& rows, int k) {
    SL_STEP(rows)
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fe, sc, scv, shv)};
    floatx4 z[NT], gz[NT];
    if constexpr (!TM) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) z[tt] = rs[tt];
      L1.apply(x, z);
    }
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      const floatx4 gh = CROW(C, ghl, ghS, cl, tt);
      gz[tt] = zero4();
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const float slp = TM ? mask_slope(rows.m, 4 * tt + r) : dlrelu(z[tt][r]);
        gz[tt][r] = ev ? gh[r] * slp : 0.f;
      }
      accF[tt] += gz[tt];
    }
    Fr sgz[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) sgz[tt] = split(gz[tt]);
    if (gxe) {
      floatx4 gx[1] = {zero4()};
      if constexpr (PREC >= 1) LT.apply(sgz, gx); else LT.apply(gz, gx);
      st_frows<F>(gxe, EB * F, (uint32_t)k * eoc, ro, g4, true, gx[0]);
    }
    lds_order();
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) WI::put(img + tt * WI::U, lane, gz[tt], sgz[tt]);
    WI::put(img + NT * WI::U, lane, x[0], split(x[0]));
    lds_order();
    const typename WI::TB tx = WI::B(img + NT * WI::U, lane);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
      accW[tt] = WI::mma(WI::A(img + tt * WI::U, lane), tx, accW[tt]);
  });
  if (fvalid) {
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const int h = GM<C>::row(g4, 4 * tt + r);
        if (h >= 0) GzT[(size_t)ks * C * NS + (size_t)h * NS + n] = accF[tt][r];
      }
  }
  block_partial(accW, scratch, C * F, [&](int a, int s, int jj) {
    const int h = GM<C>::mrow(a, s), k = GM<F>::mrow(0, jj);
    return (h >= 0 && k >= 0) ? h * F + k : -1;
  }, partW + (size_t)bx * C * F);
}

// ============================================================ SModel bwd (+T, +BN sums)
// km_source_bwd on slices: recompute the message, g_m from the fiber's moment
// coefficients, back through the message MLP; TModel's input gradient, the
// downstream edge gradient, the edge BatchNorm's two gradient sums; dWs2, dbs2,
// dWs1[:, F:2F] partials and the per-class sums of g_zs (-> g_Qt)
template <int F, int PREC, bool TM>
__global__ __launch_bounds__(256, 2) void ksl_source_bwd(
    EdgeGeo geo, SlGeo sl, const float* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ QtS, const float* __restrict__ Ws1,
    const float* __restrict__ Ws2, const float* __restrict__ bs2, const float* __restrict__ mean,
    const float* __restrict__ coef, const float* __restrict__ Rs, const float* __restrict__ Wt1,
    const float* __restrict__ ghS, const float* __restrict__ g_next,
    const float* __restrict__ mu1, const float* __restrict__ inv1, float* __restrict__ g_tot,
    float* __restrict__ partW2, float* __restrict__ partW1, float* __restrict__ partCol,
    float* __restrict__ partBN, const uint8_t* __restrict__ tmask) {
  constexpr int C = 2 * F, NT = GM<C>::NT;
  constexpr int NIMG = 3 * NT + 1;          // g_m | a | g_zs | x
  constexpr int SCR = C * (C + 1) > C * F ? C * (C + 1) : C * F;
  using WI = WgImg<PREC>;
  SL_GEO
  __shared__ __attribute__((aligned(16))) short imgs[4 * NIMG * WI::U];
  __shared__ float scratch[4 * SCR];
  // QtS / ghS: the class tables in k_sl_rows_table's layout [G*NC][CP]
  float* acc = sl_dyn;                  // [4][NC][C + 1]
  const long long gc0 = (long long)gg * NC;
  acc_zero(acc, 4 * NC * Acc<C>::S);
  float* wacc = acc + wave * NC * Acc<C>::S;
  __shared__ int owners[4][pfm::SL_MAX_NC];
  int* own = owners[wave];
  short* img = imgs + wave * NIMG * WI::U;
  short* im_gm = img;
  short* im_a = img + NT * WI::U;
  short* im_gz = im_a + NT * WI::U;
  short* im_x = im_gz + NT * WI::U;
  const long long CNS = (long long)C * NS;
  const bool tpart = Rs != nullptr;

  RecLayer<PREC, C, F> L1s, L1t;   // the forward's arithmetic (pfsgnn_mfma_core.h RecLayer)
  RecLayer<PREC, C, C> L2;
  constexpr int R1 = RecLds<RecLayer<PREC, C, F>>::n, R2 = RecLds<RecLayer<PREC, C, C>>::n;
  __shared__ s16x8 recw[(R1 * (TM ? 1 : 2) + R2) > 0 ? R1 * (TM ? 1 : 2) + R2 : 1];
  rec_bind(L1s, recw);
  rec_bind(L2, recw + R1);
  rec_bind(L1t, recw + R1 + R2);
  L1s.load([&](int h, int k) { return Ws1[h * 2 * F + F + k]; }, lane);
  if constexpr (!TM) L1t.load([&](int h, int k) { return tpart ? Wt1[h * 2 * F + F + k] : 0.f; }, lane);
  L2.load([&](int o, int h) { return Ws2[o * C + h]; }, lane);
  GradLayer<PREC, C, C> L2T;
  L2T.load([&](int h, int o) { return Ws2[o * C + h]; }, lane);
  GradLayer<PREC, F, C> L1sT, L1tT;
  L1sT.load([&](int k, int h) { return Ws1[h * 2 * F + F + k]; }, lane);
  L1tT.load([&](int k, int h) { return tpart ? Wt1[h * 2 * F + F + k] : 0.f; }, lane);
  floatx4 rs[NT], bias[NT], mn[NT], q0[NT], q1[NT], q2[NT], q3[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    if constexpr (!TM) rs[tt] = ld_node<C>(Rs, tt, g4, NS, n, fvalid);
    bias[tt] = ld_vec<C>(bs2, tt, g4);
    mn[tt] = ld_node<C>(mean, tt, g4, NS, n, fvalid);
    q0[tt] = ld_node<C>(coef, tt, g4, NS, n, fvalid);
    q1[tt] = ld_node<C>(coef + CNS, tt, g4, NS, n, fvalid);
    q2[tt] = ld_node<C>(coef + 2 * CNS, tt, g4, NS, n, fvalid);
    q3[tt] = ld_node<C>(coef + 3 * CNS, tt, g4, NS, n, fvalid);
  }
  const floatx4 scv = ld_fconst<F>(sc, g4, 1.f), shv = ld_fconst<F>(sh, g4, 0.f);
  const floatx4 m1v = ld_fconst<F>(mu1, g4, 0.f), i1v = ld_fconst<F>(inv1, g4, 0.f);
  MF_FMASK(F)
  const Rsrc ry = rsrc(y, EB * F), rgn = rsrc(g_next, EB * F), rtm = rsrc(tmask, EB);

  floatx4 accW2[NT * NT], accW1[NT], accB[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    accW1[tt] = zero4();
    accB[tt] = zero4();
#pragma unroll
    for (int nb = 0; nb < NT; ++nb) accW2[tt * NT + nb] = zero4();
  }
  floatx4 sg = zero4(), sgx = zero4();
  __syncthreads();   // qtl, ghl, acc

  auto load = [&](int k) {
    SRows<2> r;
    const uint32_t co = (uint32_t)k * eoc;
    r.v[0] = ld_frows<F>(ry, co, ro);
    r.v[1] = g_next ? ld_frows<F>(rgn, co, ro) : zero4();
    r.c = SL_CLS(k);
    if constexpr (TM) r.m = tpart ? __builtin_amdgcn_raw_buffer_load_b8(rtm, eo0 + g4, co, 0) : 0u;
    return r;
  };
  class_stream<MF_DEPTH_BWD>(k0, k1, load, [&](const SRows<2>& rows, int k) {
    SL_STEP(rows)
    const floatx4 yr = rows.v[0], gnr = rows.v[1];
    const floatx4 x[1] = {edge_in<F>(yr, fe, sc, scv, shv)};
    floatx4 zs[NT], as[NT], m[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) zs[tt] = tab_get<C>(QtS, gc0 + cl, tt, g4);
    L1s.apply(x, zs);
    lrelu_act<C>(zs, as);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) m[tt] = bias[tt];
    L2.apply(as, m);
    floatx4 gm[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      gm[tt] = zero4();
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const float d = m[tt][r] - mn[tt][r];
        gm[tt][r] = ev ? fmaf(d, fmaf(d, fmaf(d, q3[tt][r], q2[tt][r]), q1[tt][r]), q0[tt][r]) : 0.f;
      }
      accB[tt] += gm[tt];
    }
    Fr sgm[NT], sgz[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) sgm[tt] = split(gm[tt]);
    floatx4 gz[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) gz[tt] = zero4();
    if constexpr (PREC >= 1) L2T.apply(sgm, gz); else L2T.apply(gm, gz);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) gz[tt][r] *= dlrelu(zs[tt][r]);
      sgz[tt] = split(gz[tt]);
    }
    lds_order();
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      WI::put(im_gm + tt * WI::U, lane, gm[tt], sgm[tt]);
      WI::put(im_a + tt * WI::U, lane, as[tt], split(as[tt]));
      WI::put(im_gz + tt * WI::U, lane, gz[tt], sgz[tt]);
    }
    WI::put(im_x, lane, x[0], split(x[0]));
    lds_order();
    floatx4 g[1] = {zero4()};
    if constexpr (PREC >= 1) L1sT.apply(sgz, g); else L1sT.apply(gz, g);
    if (tpart) {  // TModel's per-edge input gradient (gnn.py:188-190)
      floatx4 zt[NT];
      if constexpr (!TM) {
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) zt[tt] = rs[tt];
        L1t.apply(x, zt);
      }
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        const floatx4 gh = tab_get<C>(ghS, gc0 + cl, tt, g4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float slp = TM ? mask_slope(rows.m, 4 * tt + r) : dlrelu(zt[tt][r]);
          zt[tt][r] = (ev && r < GM<C>::nreg(tt)) ? gh[r] * slp : 0.f;
        }
      }
      if constexpr (PREC >= 1) {
        Fr szt[NT];
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) szt[tt] = split(zt[tt]);
        L1tT.apply(szt, g);
      } else {
        L1tT.apply(zt, g);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) g[0][r] = fe[r] ? g[0][r] + (g_next ? gnr[r] : 0.f) : 0.f;
    st_frows<F>(g_tot, EB * F, (uint32_t)k * eoc, ro, g4, true, g[0]);
    if (mu1) {
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        sg[r] += g[0][r];
        sgx[r] = fmaf(g[0][r], (yr[r] - m1v[r]) * i1v[r], sgx[r]);
      }
    }
    // per-class sums of g_zs (the lane's own edge)
    acc_add<C>(wacc, own, cl, ev, g4, j16, gz);
    // weight gradients (edge = K) through the transposed images
    lds_order();
    const typename WI::TB tx = WI::B(im_x, lane);
    typename WI::TB ta[NT];
#pragma unroll
    for (int nb = 0; nb < NT; ++nb) ta[nb] = WI::B(im_a + nb * WI::U, lane);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      const typename WI::TA tgm = WI::A(im_gm + tt * WI::U, lane);
#pragma unroll
      for (int nb = 0; nb < NT; ++nb) accW2[tt * NT + nb] = WI::mma(tgm, ta[nb], accW2[tt * NT + nb]);
      accW1[tt] = WI::mma(WI::A(im_gz + tt * WI::U, lane), tx, accW1[tt]);
    }
  });
  acc_flush<C>(acc, NC, partCol, colbase);
  block_partial(accW2, scratch, C * (C + 1), [&](int a, int s, int jj) {
    const int o = GM<C>::mrow(a / NT, s), h = GM<C>::mrow(a % NT, jj);
    return (o >= 0 && h >= 0) ? o * (C + 1) + h : -1;
  }, partW2 + (size_t)bx * C * (C + 1));
  {  // dbs2 (exact fp32 sums of g_m) -> column C of the same partial
    __syncthreads();
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const float v = group_sum16(accB[tt][r]);
        const int o = GM<C>::row(g4, 4 * tt + r);
        if (j16 == 0 && o >= 0) scratch[wave * C + o] = v;
      }
    __syncthreads();
    if (t < C)
      partW2[(size_t)bx * C * (C + 1) + t * (C + 1) + C] =
          ((scratch[t] + scratch[C + t]) + scratch[2 * C + t]) + scratch[3 * C + t];
  }
  block_partial(accW1, scratch, C * F, [&](int a, int s, int jj) {
    const int h = GM<C>::mrow(a, s), k = GM<F>::mrow(0, jj);
    return (h >= 0 && k >= 0) ? h * F + k : -1;
  }, partW1 + (size_t)bx * C * F);
  if (mu1) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < GM<F>::RPG; ++r) {
      const float a = group_sum16(sg[r]), b = group_sum16(sgx[r]);
      const int k = GM<F>::row(g4, r);
      if (j16 == 0 && k >= 0) { scratch[wave * 2 * F + k] = a; scratch[wave * 2 * F + F + k] = b; }
    }
    __syncthreads();
    if (t < 2 * F)
      partBN[(size_t)bx * 2 * F + t] =
          ((scratch[t] + scratch[2 * F + t]) + scratch[4 * F + t]) + scratch[6 * F + t];
  }
}

// ============================================================ EdgeModel bwd
// km_edge_mlp_bwd on slices: g_y from the double BatchNorm's coefficients, back
// through the edge MLP; dW2, db2, dW1[:, 2F:3F] partials, the fiber's sums of
// g_z (-> g_Ps), per-class sums of g_z (-> g_Pt) and the edge-input gradient
template <int F, int PREC>
__global__ __launch_bounds__(256, 2) void ksl_edge_mlp_bwd(
    EdgeGeo geo, SlGeo sl, const float* __restrict__ g_tot, const float* __restrict__ alpha,
    const float* __restrict__ gam0, const float* __restrict__ gam1, const float* __restrict__ y,
    const float* __restrict__ xe, const float* __restrict__ xsc, const float* __restrict__ xsh,
    const float* __restrict__ Ps, const float* __restrict__ PtS, const float* __restrict__ W1,
    const float* __restrict__ W2, float* __restrict__ gxe, float* __restrict__ GzEs,
    float* __restrict__ partW2, float* __restrict__ partW1, float* __restrict__ partCol) {
  constexpr int H = 4 * F, NT = GM<H>::NT;
  constexpr int NIMG = 1 + NT + NT + 1;          // g_y | a | g_z | x
  constexpr int SCR = F * (H + 1) > H * F ? F * (H + 1) : H * F;
  using WI = WgImg<PREC>;
  SL_GEO
  __shared__ __attribute__((aligned(16))) short imgs[4 * NIMG * WI::U];
  __shared__ float scratch[4 * SCR];
  CROWS_DECL(H, ptl, PtS, sl_dyn)             // [NC][CP]
  float* acc = sl_dyn + NC * CROWS_FLOATS(H);  // [4][NC][H + 1]
#ifndef SL_NO_ACC_LDS   // (timing experiment only: no accumulators, SL_NO_ACC too)
  acc_zero(acc, 4 * NC * Acc<H>::S);
#endif
  float* wacc = acc + wave * NC * Acc<H>::S;
  __shared__ int owners[4][pfm::SL_MAX_NC];
  int* own = owners[wave];
  short* img = imgs + wave * NIMG * WI::U;
  short* im_gy = img;
  short* im_a = img + WI::U;
  short* im_gz = im_a + NT * WI::U;
  short* im_x = im_gz + NT * WI::U;

  FwdLayer<FP(PREC), H, F> L1;
  L1.load([&](int h, int k) { return W1[h * 4 * F + 2 * F + k]; }, lane);
  GradLayer<PREC, H, F> L2T;
  L2T.load([&](int h, int o) { return W2[o * H + h]; }, lane);
  GradLayer<PREC, F, H> L1T;
  L1T.load([&](int k, int h) { return gxe ? W1[h * 4 * F + 2 * F + k] : 0.f; }, lane);
  floatx4 ps[NT], accF[NT], accW1[NT], accW2[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    ps[tt] = ld_node<H>(Ps, tt, g4, NS, n, fvalid);
    accF[tt] = zero4();
    accW1[tt] = zero4();
    accW2[tt] = zero4();
  }
  floatx4 accB = zero4();
  const floatx4 alv = ld_fconst<F>(alpha, g4, 0.f), g0v = ld_fconst<F>(gam0, g4, 0.f),
                g1v = ld_fconst<F>(gam1, g4, 0.f);
  const floatx4 scv = ld_fconst<F>(xsc, g4, 1.f), shv = ld_fconst<F>(xsh, g4, 0.f);
  MF_FMASK(F)
  const Rsrc rgt = rsrc(g_tot, EB * F), ry = rsrc(y, EB * F), rxe = rsrc(xe, EB * F);
  __syncthreads();   // ptl, acc

  auto load = [&](int k) {
    SRows<3> r;
    const uint32_t co = (uint32_t)k * eoc;
    r.v[0] = ld_frows<F>(rgt, co, ro);
    r.v[1] = ld_frows<F>(ry, co, ro);
    r.v[2] = ld_frows<F>(rxe, co, ro);
    r.c = SL_CLS(k);
    return r;
  };
  class_stream<MF_DEPTH_BWD>(k0, k1, load, [&](const SRows<3>& rows, int k) {
    SL_STEP(rows)
    floatx4 gy[1] = {zero4()};
#pragma unroll
    for (int r = 0; r < GM<F>::RPG; ++r)
      gy[0][r] = fe[r] ? fmaf(g1v[r], rows.v[1][r], fmaf(alv[r], rows.v[0][r], g0v[r])) : 0.f;
    accB += gy[0];
    const floatx4 x[1] = {edge_in<F>(rows.v[2], fe, xsc, scv, shv)};
    floatx4 z[NT], a[NT], gz[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      z[tt] = ps[tt] + CROW(H, ptl, PtS, cl, tt);
      gz[tt] = zero4();
    }
    L1.apply(x, z);
    lrelu_act<H>(z, a);
    const Fr sgy[1] = {split(gy[0])};
    if constexpr (PREC >= 1) L2T.apply(sgy, gz); else L2T.apply(gy, gz);
    Fr sgz[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
#pragma unroll
      for (int r = 0; r < GM<H>::nreg(tt); ++r) gz[tt][r] *= dlrelu(z[tt][r]);
      accF[tt] += gz[tt];
      sgz[tt] = split(gz[tt]);
    }
    lds_order();
    WI::put(im_gy, lane, gy[0], sgy[0]);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      WI::put(im_a + tt * WI::U, lane, a[tt], split(a[tt]));
      WI::put(im_gz + tt * WI::U, lane, gz[tt], sgz[tt]);
    }
    WI::put(im_x, lane, x[0], split(x[0]));
    lds_order();
    if (gxe) {
      floatx4 gx[1] = {zero4()};
      if constexpr (PREC >= 1) L1T.apply(sgz, gx); else L1T.apply(gz, gx);
      st_frows<F>(gxe, EB * F, (uint32_t)k * eoc, ro, g4, true, gx[0]);
    }
    acc_add<H>(wacc, own, cl, ev, g4, j16, gz);
    const typename WI::TA tgy = WI::A(im_gy, lane);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
      accW2[tt] = WI::mma(tgy, WI::B(im_a + tt * WI::U, lane), accW2[tt]);
    const typename WI::TB tx = WI::B(im_x, lane);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
      accW1[tt] = WI::mma(WI::A(im_gz + tt * WI::U, lane), tx, accW1[tt]);
  });
  if (fvalid) {
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < GM<H>::nreg(tt); ++r) {
        const int h = GM<H>::row(g4, 4 * tt + r);
        if (h >= 0) GzEs[(size_t)ks * H * NS + (size_t)h * NS + n] = accF[tt][r];
      }
  }
#ifndef SL_NO_ACC_LDS
  acc_flush<H>(acc, NC, partCol, colbase);
#endif
  block_partial(accW2, scratch, F * (H + 1), [&](int a, int s, int jj) {
    const int o = GM<F>::mrow(0, s), h = GM<H>::mrow(a, jj);
    return (o >= 0 && h >= 0) ? o * (H + 1) + h : -1;
  }, partW2 + (size_t)bx * F * (H + 1));
  {  // db2 (exact fp32 sums of g_y) -> column H of the same partial
    __syncthreads();
#pragma unroll
    for (int r = 0; r < GM<F>::RPG; ++r) {
      const float v = group_sum16(accB[r]);
      const int o = GM<F>::row(g4, r);
      if (j16 == 0 && o >= 0) scratch[wave * F + o] = v;
    }
    __syncthreads();
    if (t < F)
      partW2[(size_t)bx * F * (H + 1) + t * (H + 1) + H] =
          ((scratch[t] + scratch[F + t]) + scratch[2 * F + t]) + scratch[3 * F + t];
  }
  block_partial(accW1, scratch, H * F, [&](int a, int s, int jj) {
    const int h = GM<H>::mrow(a, s), k = GM<F>::mrow(0, jj);
    return (h >= 0 && k >= 0) ? h * F + k : -1;
  }, partW1 + (size_t)bx * H * F);
}

}  // namespace

// ============================================================ host launchers
namespace pfm {

// KS step splits per slice bring the grid near TARGET_BLOCKS (the backward
// kernels hold one or two blocks per CU: their LDS class tables)
EdgeGeo sl_geo(int G, int NF, int NC, const SlGeo& sl) {
  EdgeGeo g;
  g.G = G; g.NF = NF; g.NC = NC;
  g.NFG = (NF + 63) / 64;
  const long long groups = (long long)G * g.NFG;
  static const int ks_env = [] {   // tuning knob: PFSGNN_SL_KS (step splits)
    const char* e = getenv("PFSGNN_SL_KS");
    return e ? atoi(e) : 0;
  }();
  long long ks = ks_env > 0 ? ks_env : (TARGET_BLOCKS / 2 + groups - 1) / groups;
  ks = std::max<long long>(1, std::min<long long>(ks, std::min(8, std::max(1, sl.maxdeg / 8))));
  g.KS = (int)ks;
  g.CPS = NC;
  g.nblocks = (int)(groups * g.KS);
  g.E = sl.EP;
  g.NS = (long long)G * NF;
  g.NT = (long long)G * NC;
  return g;
}

namespace {

// static LDS of a kernel instantiation (its __shared__ arrays)
template <class K>
size_t static_lds(K kernel) {
  hipFuncAttributes a{};
  if (hipFuncGetAttributes(&a, reinterpret_cast<const void*>(kernel)) != hipSuccess) return 0;
  return a.sharedSizeBytes;
}
constexpr size_t LDS_CU = 160 * 1024;
// dynamic LDS of a kernel (class rows + accumulators), opted in above 64 KB once
// per kernel instantiation; static + dynamic must fit the CU's 160 KB
template <class K>
int dyn_lds(K kernel, size_t bytes) {
  if (bytes + static_lds(kernel) > LDS_CU)
    return pf::fail("pfsgnn sliced", "class tables exceed the LDS (NC too large)");
  if (bytes > 64 * 1024) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
      return pf::fail("pfsgnn sliced", "hipFuncSetAttribute (dynamic LDS)");
  }
  return 0;
}

template <class K, class... A>
int sl_launch(K kernel, const EdgeGeo& geo, size_t lds, hipStream_t st, A... args) {
  if (int rc = dyn_lds(kernel, lds)) return rc;
  hipLaunchKernelGGL(kernel, dim3(geo.nblocks), dim3(256), lds, st, args...);
  return 0;
}

constexpr int cp_of(int D) { return 16 * ((((D + 3) / 4) + 3) / 4) + 4; }   // SlRows<D>::S
constexpr int cpg_of(int D) { return 16 * ((((D + 3) / 4) + 3) / 4); }      // ClassRows<D>::CP

// P [D][NT] -> the permuted global table [NT][CP] (k_sl_rows_table)
int rows_table(int D, const float* P, long long NT, float* out, hipStream_t st) {
  const unsigned nb = (unsigned)((NT * cpg_of(D) + 255) / 256);
  switch (D) {
#define RT(DD) case DD: hipLaunchKernelGGL(k_sl_rows_table<DD>, dim3(nb), dim3(256), 0, st, P, NT, out); break;
    RT(16) RT(20) RT(32) RT(40) RT(64)
#undef RT
    default: return pf::fail("pfsgnn sliced", "unsupported class-table width");
  }
  return 0;
}
#ifndef SL_GLOBAL_TABLES
constexpr bool kGTab = false;
#else
constexpr bool kGTab = true;
#endif
// the lds bytes of a kernel's class table, and the table it reads (staged from
// P in LDS, or P permuted into `tabs`)
inline size_t tab_lds(const EdgeGeo& geo, int D) {
  return kGTab ? 0 : (size_t)geo.NC * cp_of(D) * sizeof(float);
}

}  // namespace

// Instantiations: the complete path's (Fdim 8 / 10 / 16 at PREC 0, 1; every
// MFMA precision at Fdim 10)
#define SL_SWITCH(F, P, CASE)                                                       \
  switch ((F) * 8 + (P)) {                                                          \
    CASE(8, 0) CASE(8, 1) CASE(10, 0) CASE(10, 1) CASE(10, 2) CASE(10, 3) CASE(10, 4) \
    CASE(16, 0) CASE(16, 1)                                                         \
    default: return pf::fail("pfsgnn sliced", "unsupported Fdim for this edge path"); \
  }

int sl_edge_mlp_fwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* xe, const float* xsc,
                    const float* xsh, const float* Ps, const float* PtS, const float* W1,
                    const float* W2, const float* b2, float* y, float* part, float* tabs,
                    int prec, hipStream_t st) {
  const size_t lds = tab_lds(geo, 4 * F);
  if (kGTab) {
    if (int rc = rows_table(4 * F, PtS, geo.NT, tabs, st)) return rc;
    PtS = tabs;
  }
#define SL_C(FF, PP)                                                                       \
  case FF * 8 + PP:                                                                        \
    return sl_launch(ksl_edge_mlp_fwd<FF, PP>, geo, lds, st, geo, sl, xe, xsc, xsh, Ps, PtS, W1, \
                     W2, b2, y, part);
  SL_SWITCH(F, FP(prec), SL_C)
#undef SL_C
}

int sl_source_fwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* y, const float* sc,
                  const float* sh, const float* QtS, const float* Ws1, const float* Ws2,
                  const float* bs2, float* mom, float* hs, float* tabs, int prec,
                  hipStream_t st) {
  const size_t lds = tab_lds(geo, 2 * F);
  if (kGTab) {
    if (int rc = rows_table(2 * F, QtS, geo.NT, tabs, st)) return rc;
    QtS = tabs;
  }
  EdgeGeo g1 = geo;   // one block per slice (its 4 waves interleave the steps)
  g1.KS = 1;
  g1.nblocks = geo.G * geo.NFG * 4;
#define SL_C(FF, PP)                                                                        \
  case FF * 8 + PP:                                                                         \
    return sl_launch(ksl_source_fwd<FF, PP>, g1, lds, st, g1, sl, y, sc, sh, QtS, Ws1, Ws2, \
                     bs2, mom, hs);
  SL_SWITCH(F, FP(prec), SL_C)
#undef SL_C
}

int sl_target_fwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* y, const float* sc,
                  const float* sh, const float* Rs, const float* Wt1, float* part, uint8_t* tmask,
                  int prec, hipStream_t st) {
  const size_t lds = (size_t)4 * geo.NC * acc_stride(2 * F) * sizeof(float);
#define SL_C(FF, PP)                                                                        \
  case FF * 8 + PP:                                                                         \
    return sl_launch(ksl_target_fwd<FF, PP>, geo, lds, st, geo, sl, y, sc, sh, Rs, Wt1, part, \
                     tmask);
  SL_SWITCH(F, FP(prec), SL_C)
#undef SL_C
}

int sl_target_bwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* y, const float* sc,
                  const float* sh, const float* Rs, const float* Wt1, const float* ghS, float* gz,
                  float* gxe, float* part, const uint8_t* tmask, float* tabs, int prec,
                  hipStream_t st) {
  const size_t lds = tab_lds(geo, 2 * F);
  if (kGTab) {
    if (int rc = rows_table(2 * F, ghS, geo.NT, tabs, st)) return rc;
    ghS = tabs;
  }
#define SL_C(FF, PP)                                                                        \
  case FF * 8 + PP:                                                                         \
    return tmask ? sl_launch(ksl_target_bwd<FF, PP, true>, geo, lds, st, geo, sl, y, sc, sh, Rs, \
                             Wt1, ghS, gz, gxe, part, tmask)                                \
                 : sl_launch(ksl_target_bwd<FF, PP, false>, geo, lds, st, geo, sl, y, sc, sh, Rs, \
                             Wt1, ghS, gz, gxe, part, tmask);
  SL_SWITCH(F, prec, SL_C)
#undef SL_C
}

int sl_source_bwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* y, const float* sc,
                  const float* sh, const float* QtS, const float* Ws1, const float* Ws2,
                  const float* bs2, const float* mean, const float* coef, const float* Rs,
                  const float* Wt1, const float* ghS, const float* g_next, const float* mu1,
                  const float* inv1, float* g_tot, float* pW2, float* pW1, float* pCol,
                  float* pBN, const uint8_t* tmask, float* tabs, int prec, hipStream_t st) {
  const size_t lds = (size_t)geo.NC * 4 * acc_stride(2 * F) * sizeof(float);
  const bool tm = tmask && Rs;
  // the two class tables in global memory (tabs: 2 * NT * CP floats of workspace)
  const long long tlen = geo.NT * cpg_of(2 * F);
  float* tq = tabs;
  float* tg = ghS ? tabs + tlen : nullptr;
  if (int rc = rows_table(2 * F, QtS, geo.NT, tq, st)) return rc;
  if (tg)
    if (int rc = rows_table(2 * F, ghS, geo.NT, tg, st)) return rc;
  QtS = tq;
  ghS = tg;
#define SL_C(FF, PP)                                                                        \
  case FF * 8 + PP:                                                                         \
    return tm ? sl_launch(ksl_source_bwd<FF, PP, true>, geo, lds, st, geo, sl, y, sc, sh, QtS, \
                          Ws1, Ws2, bs2, mean, coef, Rs, Wt1, ghS, g_next, mu1, inv1, g_tot, pW2, \
                          pW1, pCol, pBN, tmask)                                            \
              : sl_launch(ksl_source_bwd<FF, PP, false>, geo, lds, st, geo, sl, y, sc, sh, QtS, \
                          Ws1, Ws2, bs2, mean, coef, Rs, Wt1, ghS, g_next, mu1, inv1, g_tot, pW2, \
                          pW1, pCol, pBN, tmask);
  SL_SWITCH(F, prec, SL_C)
#undef SL_C
}

int sl_edge_mlp_bwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* g_tot,
                    const float* alpha, const float* gam0, const float* gam1, const float* y,
                    const float* xe, const float* xsc, const float* xsh, const float* Ps,
                    const float* PtS, const float* W1, const float* W2, float* gxe, float* gs,
                    float* pW2, float* pW1, float* pCol, float* tabs, int prec, hipStream_t st) {
#ifndef SL_NO_ACC_LDS
  const size_t lds = tab_lds(geo, 4 * F) + (size_t)geo.NC * 4 * acc_stride(4 * F) * sizeof(float);
#else
  const size_t lds = tab_lds(geo, 4 * F);
#endif
  if (kGTab) {
    if (int rc = rows_table(4 * F, PtS, geo.NT, tabs, st)) return rc;
    PtS = tabs;
  }
#define SL_C(FF, PP)                                                                         \
  case FF * 8 + PP:                                                                          \
    return sl_launch(ksl_edge_mlp_bwd<FF, PP>, geo, lds, st, geo, sl, g_tot, alpha, gam0, gam1, \
                     y, xe, xsc, xsh, Ps, PtS, W1, W2, gxe, gs, pW2, pW1, pCol);
  SL_SWITCH(F, prec, SL_C)
#undef SL_C
}

// The most classes per graph every sliced kernel of (F, prec) fits in the LDS:
// static LDS + the per-class bytes of its dynamic tables (the launchers'
// formulas above) <= 160 KB, and <= SL_MAX_NC.  0: no sliced kernels for (F, prec).
int sl_max_nc(int F, int prec) {
  auto cap = [](size_t stat, size_t per_class) {
    if (stat >= LDS_CU) return 0;
    const size_t n = per_class ? (LDS_CU - stat) / per_class : (size_t)SL_MAX_NC;
    return (int)std::min<size_t>(n, SL_MAX_NC);
  };
  const size_t tc = kGTab ? 0 : (size_t)cp_of(2 * F) * 4, th = kGTab ? 0 : (size_t)cp_of(4 * F) * 4;
  const size_t ac = (size_t)4 * acc_stride(2 * F) * 4, ah = (size_t)4 * acc_stride(4 * F) * 4;
  int m = SL_MAX_NC;
  const int fp = FP(prec);
#define SL_M(FF, PP)                                                                               \
  case FF * 8 + PP:                                                                                \
    m = std::min(m, cap(static_lds(ksl_target_bwd<FF, PP, true>), tc));                            \
    m = std::min(m, cap(static_lds(ksl_target_bwd<FF, PP, false>), tc));                           \
    m = std::min(m, cap(static_lds(ksl_source_bwd<FF, PP, true>), ac));                            \
    m = std::min(m, cap(static_lds(ksl_source_bwd<FF, PP, false>), ac));                           \
    m = std::min(m, cap(static_lds(ksl_edge_mlp_bwd<FF, PP>), th + ah));                           \
    break;
  switch (F * 8 + prec) {
    SL_M(8, 0) SL_M(8, 1) SL_M(10, 0) SL_M(10, 1) SL_M(10, 2) SL_M(10, 3) SL_M(10, 4)
    SL_M(16, 0) SL_M(16, 1)
    default: return 0;
  }
#undef SL_M
#define SL_MF(FF, PP)                                                                              \
  case FF * 8 + PP:                                                                                \
    m = std::min(m, cap(static_lds(ksl_edge_mlp_fwd<FF, PP>), th));                                \
    m = std::min(m, cap(static_lds(ksl_source_fwd<FF, PP>), tc));                                  \
    m = std::min(m, cap(static_lds(ksl_target_fwd<FF, PP>), ac));                                  \
    break;
  switch (F * 8 + fp) {
    SL_MF(8, 0) SL_MF(10, 0) SL_MF(10, 2) SL_MF(10, 3) SL_MF(10, 4) SL_MF(16, 0)
    default: return 0;
  }
#undef SL_MF
  return m;
}

}  // namespace pfm
