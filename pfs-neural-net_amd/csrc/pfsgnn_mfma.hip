// pfsgnn_mfma.hip -- the per-edge kernels of the message-passing block on the
// matrix cores (the default edge path; pfsgnn_edge.hip holds the fp32 VALU one).
//
// Arithmetic (PREC, per edge path; include/pfsgnn.h).  The layer-to-layer
// contractions of gnn.py's per-edge MLPs (EdgeModel gnn.py:86-101, SModel /
// TModel message MLPs gnn.py:136, 188) and of their backward run either on
// v_mfma_f32_16x16x4_f32 -- exact fp32 products, fp32 accumulation, the
// numerics of an fmaf chain (LayerF) -- or on v_mfma_f32_16x16x32_bf16 with
// split operands v = bf16 hi + bf16 lo and products hi*hi + hi*lo + lo*hi
// ("bf16x3", ~2^-16 relative per product, fp32 accumulation; LayerB3), at
// about 5x the fp32 form's K per cycle.  SModel's skew / kurtosis features
// divide by std^3 / std^4 of a fiber's messages and amplify message rounding,
// so the precision of every path is measured against the fp64 oracle at the
// metric shape (tests/test_gpu_precision_table.py).  The
// weight gradients -- sums over all edges of outer products -- are bf16x3 on
// every path: a product's ~2^-16 relative error has a random sign and
// averages out over the edge sum.
//
// Tile geometry.  Canonical edge order is class-major, e = (g*NC + c)*NF + f
// (channel-major [C][E] tensors), as in pfsgnn_edge.hip.  A 256-thread block
// owns 64 consecutive fibers of one graph and a range of classes; wave w owns
// fibers 16w..16w+15 and walks EVERY class of the range, one 16-edge tile
// (16 fibers x 1 class) per step.  In a tile the edge is the MFMA column
// (lane & 15) and the feature the MFMA row.  A D-wide feature vector is spread
// over the 4 lane groups g = lane >> 4 by the compact row map GM<D>: group g
// holds rows g*RPG .. g*RPG + RPG-1 (RPG = ceil(D/4)) in register slots
// s = 0..RPG-1, slot s being register s&3 of tile s>>2 (a floatx4 per tile).
// That is the C/D layout of a 16x16 MFMA, and register s of a lane group is
// exactly the B operand of the K-step that consumes input rows {g*RPG + s}:
//     Y = W X   ->   y[t] += mfma_16x16x4(A = W[out row][g*RPG + s], B = x[s]),
// so a layer's output feeds the next layer with no data movement, and an input
// of D rows costs ceil(D/4) K-steps (10 -> 3, 20 -> 5, 40 -> 10) instead of
// 4*ceil(D/16).  Consequences:
//   * F-wide edge rows are loaded / stored as 64-byte row segments per lane
//     group (16 consecutive fibers of one class), RPG_F instructions per tile;
//   * per-fiber sums over classes stay in the lane's registers;
//   * per-class sums over fibers are column sums of a tile, merged over the
//     block's 4 waves through LDS in fixed order;
//   * weight gradients sum over the tile's COLUMN index: the operand tiles go
//     through a wave-private LDS image [edge][slot] read back transposed with
//     ds_read_b64_tr_b16 (edge = MFMA K).
// Edge rows are prefetched several classes ahead through a register ring
// (class_stream).  Cross-block results go to the same per-block partials as
// the VALU kernels and are finished by the same fixed-order reductions: a step
// stays bitwise reproducible.
#include "pfsgnn_mfma_core.h"

// MF_WG_EARLY_READS (default 1): the backward kernels issue their transposed
// weight-gradient image reads right after writing the images, ahead of the
// input-gradient chains (0: at their first use, round 4's order)
#ifndef MF_WG_EARLY_READS
#define MF_WG_EARLY_READS 1
#endif
// MF_FWD_PAIRS (default 0): 1 runs edge_mlp_fwd's classes two per body
// (class_stream_pairs), their MFMA chains interleaved -- measured slower
// (profiles/r05p_*pairs_ab.txt, r05q_*pairs_ab.txt), kept for the A/B
#ifndef MF_FWD_PAIRS
#define MF_FWD_PAIRS 0
#endif
// MF_SB_PACK (default 1): source_bwd's packed weight-gradient tiles at Fdim 10
// (5 images / 5 outer-product tiles instead of 7 / 6; 0: the unpacked form)
#ifndef MF_SB_PACK
#define MF_SB_PACK 1
#endif
// MF_SB_LDSW (default 0): source_bwd's split-bf16 gradient-chain weights in
// LDS (LayerB3S) instead of registers (-32 VGPRs)
#ifndef MF_SB_LDSW
#define MF_SB_LDSW 0
#endif
// MF_WG4 (default 1): the backward kernels' split-bf16 weight gradients as the
// four products of the split operands (WgImg::mma4: B read twice, no [Bh | 0]
// operand assembled); 0: the three-product form (mma3g)
#ifndef MF_WG4
#define MF_WG4 1
#endif

namespace {

// ============================================================ EdgeModel fwd
// y = W2 lrelu(Ps[f] + Pt[c] + W1[:, 2F:3F] x) + b2 per edge (gnn.py:86-101 with
// the node parts of the first Linear precomputed per node); Welford partials of
// y per block for the (double) BatchNorm, finished in the launch by its last
// blocks when `fin` has counters (mom_finalize, pfsgnn_common.h).
#ifndef MF_EFWD_MINB
#define MF_EFWD_MINB 6   // six waves per SIMD (80 VGPRs, no spills at ring depth 3; profiles/r05aj_fwd_occupancy_ab.txt)
#endif
// MF_EFWD_B6S (default 1): at PREC 4 (bf16x6) the split weight tuples of both
// layers staged in LDS (LayerB6S) instead of registers, so that the kernel
// holds MF_EFWD_MINB6 waves per SIMD (84 VGPRs, five; the register form: 128
// VGPRs, four; six waves spill 17 VGPRs).  edge_mlp_fwd -0.02 to -0.03 ms, the
// step -0.01 / -0.02 ms with MF_SFT_B6S (profiles/r06n_ab.txt); bitwise the
// register form's results
#ifndef MF_EFWD_B6S
#define MF_EFWD_B6S 1
#endif
#ifndef MF_EFWD_MINB6
#define MF_EFWD_MINB6 5
#endif
template <int F, int PREC>
__global__ __launch_bounds__(256, (F <= 10 && PREC <= 1) ? MF_EFWD_MINB
                                  : (F <= 10 && PREC == 4 && MF_EFWD_B6S) ? MF_EFWD_MINB6 : 1)
void km_edge_mlp_fwd(EdgeGeo geo, const float* __restrict__ xe,
                                                       const float* __restrict__ xsc,
                                                       const float* __restrict__ xsh,
                                                       const float* __restrict__ Ps,
                                                       const float* __restrict__ PtS,
                                                       const float* __restrict__ W1,
                                                       const float* __restrict__ W2,
                                                       const float* __restrict__ b2,
                                                       float* __restrict__ y,
                                                       float* __restrict__ part, int bfy,
                                                       MomFin fin) {
  constexpr int H = 4 * F, NT = GM<H>::NT;
  MF_GEO
  __shared__ __attribute__((aligned(16))) float ptl[MF_MAX_CPS * ClassRows<H>::CP];
  ClassRows<H>::stage(ptl, PtS, geo.NT, (long long)gg * geo.NC + c0, c1 - c0);
  constexpr bool B6S = MF_EFWD_B6S && PREC == 4;
  std::conditional_t<B6S, LayerB6S<H, F>, FwdLayer<PREC, H, F>> L1;
  std::conditional_t<B6S, LayerB6S<F, H>, FwdLayer<PREC, F, H>> L2;
  if constexpr (B6S) {
    __shared__ s16x8 w6[(LayerB6S<H, F>::NOP + LayerB6S<F, H>::NOP) * 64];
    L1.bind(w6);
    L2.bind(w6 + LayerB6S<H, F>::NOP * 64);
  }
  L1.load([&](int h, int k) { return W1[h * 4 * F + 2 * F + k]; }, lane);
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
  auto load = [&](int c) {
    Rows<1> r;
    r.v[0] = ld_frows<F>(rxe, (uint32_t)c * eoc, ro);
    return r;
  };
#if MF_FWD_PAIRS && !defined(MF_ABL_NOL1) && !defined(MF_ABL_NOLRELU) && !defined(MF_ABL_NOL2) && \
    !defined(MF_ABL_NOSTORE) && !defined(MF_ABL_NOSTATS)
  // two classes per body: both chains interleave; the stores and the Welford
  // updates stay in class order (bitwise the single-class results)
  auto finish = [&](floatx4 yo, int c) {
    if (bfy) {
      const s16x4 h = hi4(yo);
#pragma unroll
      for (int r = 0; r < 4; ++r) yo[r] = bf_f(h[r]);
    }
    st_frows<F>(y, EB * F, (uint32_t)c * eoc, ro, g4, fvalid, yo);
    if (fvalid) {
      cnt += 1.f;
      const float rc = __builtin_amdgcn_rcpf(cnt);
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        const float d = yo[r] - mean[r];
        mean[r] = fmaf(d, rc, mean[r]);
        m2[r] = fmaf(d, yo[r] - mean[r], m2[r]);
      }
    }
  };
  auto one = [&](const Rows<1>& rows, int c) {
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fm, xsc, scv, shv)};
    floatx4 z[NT], a[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) z[tt] = ps[tt] + ClassRows<H>::get(ptl, c - c0, tt, g4);
    L1.apply(x, z);
    lrelu_act<H>(z, a);
    floatx4 yo[1] = {bb};
    L2.apply(a, yo);
    finish(yo[0], c);
  };
  auto two = [&](const Rows<1>& ra, int ca, const Rows<1>& rb, int cb) {
    const floatx4 xa[1] = {edge_in<F>(ra.v[0], fm, xsc, scv, shv)};
    const floatx4 xb[1] = {edge_in<F>(rb.v[0], fm, xsc, scv, shv)};
    floatx4 za[NT], zb[NT], aa[NT], ab[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      za[tt] = ps[tt] + ClassRows<H>::get(ptl, ca - c0, tt, g4);
      zb[tt] = ps[tt] + ClassRows<H>::get(ptl, cb - c0, tt, g4);
    }
    L1.apply(xa, za);
    L1.apply(xb, zb);
    lrelu_act<H>(za, aa);
    lrelu_act<H>(zb, ab);
    floatx4 ya[1] = {bb}, yb[1] = {bb};
    L2.apply(aa, ya);
    L2.apply(ab, yb);
    finish(ya[0], ca);
    finish(yb[0], cb);
  };
  class_stream_pairs<MF_DEPTH_FWD>(c0, c1, load, one, two);
#else
  class_stream<MF_DEPTH_FWD, true>(c0, c1, load, [&](const Rows<1>& rows, int c) {
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fm, xsc, scv, shv)};
    floatx4 z[NT], a[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) z[tt] = ps[tt] + ClassRows<H>::get(ptl, c - c0, tt, g4);
#ifndef MF_ABL_NOL1   // (MF_ABL_*: ablation builds for timing studies only, tools/variants.sh)
    L1.apply(x, z);
#else
    z[0] += x[0];
#endif
#ifndef MF_ABL_NOLRELU
    lrelu_act<H>(z, a);
#else
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) a[tt] = z[tt];
#endif
    floatx4 yo[1] = {bb};
#ifndef MF_ABL_NOL2
    L2.apply(a, yo);
#else
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) yo[0] += a[tt];
#endif
    if (bfy) {  // the edge state at bf16 (PFSGNN_EDGE_BF16Y / _BF16): every consumer
                // reads exactly what a bf16 store would hold
      const s16x4 h = hi4(yo[0]);
#pragma unroll
      for (int r = 0; r < 4; ++r) yo[0][r] = bf_f(h[r]);
    }
#ifndef MF_ABL_NOSTORE
    st_frows<F>(y, EB * F, (uint32_t)c * eoc, ro, g4, fvalid, yo[0]);
#endif
#ifdef MF_ABL_NOSTATS
    if (fvalid) { cnt += 1.f; mean += yo[0]; }
    if (false) {
#else
    if (fvalid) {
#endif
      cnt += 1.f;
      const float rc = __builtin_amdgcn_rcpf(cnt);   // v_rcp_f32 (<= 1 ulp): a Welford weight
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        const float d = yo[0][r] - mean[r];
        mean[r] = fmaf(d, rc, mean[r]);
        m2[r] = fmaf(d, yo[0][r] - mean[r], m2[r]);
      }
    }
  });
#endif
  // Chan merge over the 16 fibers of the group, then over the 4 waves
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
    float* p = part + (size_t)bx * (1 + 2 * F);   // (sc1: mom_finalize's hand-off)
    if (t == 0) st_sc1(p, C0);
    st_sc1(p + 1 + t, M0);
    st_sc1(p + 1 + F + t, Q0);
  }
  if (fin.cnt) mom_finalize<F>(part, geo.nblocks, bx, fin);
}

// ============================================================ SModel fwd
// message m = Ws2 lrelu(Qt[c] + Ws1[:, F:2F] x) + bs2 (gnn.py:136-137) and its
// per-fiber centred moments over the class range by Pebay's one-pass update
// (the wave walks every class of its 16 fibers: no cross-wave merge).
template <int F, int PREC>
__global__ __launch_bounds__(256) void km_source_fwd(EdgeGeo geo, const float* __restrict__ y,
                                                     const float* __restrict__ sc,
                                                     const float* __restrict__ sh,
                                                     const float* __restrict__ QtS,
                                                     const float* __restrict__ Ws1,
                                                     const float* __restrict__ Ws2,
                                                     const float* __restrict__ bs2,
                                                     float* __restrict__ partS) {
  constexpr int C = 2 * F, NT = GM<C>::NT;
  MF_GEO
  __shared__ __attribute__((aligned(16))) float qtl[MF_MAX_CPS * ClassRows<C>::CP];
  ClassRows<C>::stage(qtl, QtS, geo.NT, (long long)gg * geo.NC + c0, c1 - c0);
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

  floatx4 S1[NT], S2[NT], S3[NT], S4[NT];  // mean | M2 | M3 | M4
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) S1[tt] = S2[tt] = S3[tt] = S4[tt] = zero4();
  // Pebay's one-pass update of the central sums after the n-th message, with
  // its count-only coefficients per class (uniform over the wave) from a table:
  //   d = m - mean;  M4 += d^4 A4 + 6 d^2 M2 / n^2 - 4 d M3 / n;
  //   M3 += d^3 A3 - 3 d M2 / n;  M2 += d^2 A2;  mean += d / n
  // A2 = (n-1)/n, A3 = (n-1)(n-2)/n^2, A4 = (n-1)(n^2-3n+3)/n^3 (12 VALU per
  // element, the M2 / M3 of the previous count on the right-hand sides)
  static_assert(MF_MAX_CPS <= MF_PEB_ROWS, "Pebay table rows");
#if MF_PEB_CONST
  const auto& pco = c_peb.v;
#else
  __shared__ __attribute__((aligned(16))) float pco[MF_MAX_CPS][8];
  if (t < c1 - c0) {
    const double nn = t + 1, r = 1.0 / nn;
    pco[t][0] = (float)((nn - 1) * r);                            // A2
    pco[t][1] = (float)((nn - 1) * (nn - 2) * r * r);             // A3
    pco[t][2] = (float)((nn - 1) * (nn * nn - 3 * nn + 3) * r * r * r);  // A4
    pco[t][3] = (float)r;                                         // 1/n
    pco[t][4] = (float)(6 * r * r);                               // 6/n^2
    pco[t][5] = (float)(-4 * r);                                  // -4/n
    pco[t][6] = (float)(-3 * r);                                  // -3/n
    pco[t][7] = 0.f;
  }
#endif
  __syncthreads();   // qtl
  auto load = [&](int c) {
    Rows<1> r;
    r.v[0] = ld_frows<F>(ry, (uint32_t)c * eoc, ro);
    return r;
  };
  class_stream<MF_DEPTH_FWD>(c0, c1, load, [&](const Rows<1>& rows, int c) {
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fm, sc, scv, shv)};
    floatx4 z[NT], a[NT], m[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) z[tt] = ClassRows<C>::get(qtl, c - c0, tt, g4);
    L1.apply(x, z);
    lrelu_act<C>(z, a);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) m[tt] = bias[tt];
    L2.apply(a, m);
    const floatx4 ca = *reinterpret_cast<const floatx4*>(&pco[c - c0][0]);
    const floatx4 cb = *reinterpret_cast<const floatx4*>(&pco[c - c0][4]);
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
  });
  if (fvalid) {
    float* dst = partS + (size_t)ks * 4 * C * NS + n;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const int o = GM<C>::row(g4, 4 * tt + r);
        if (o >= 0) {
          dst[(size_t)o * NS] = S1[tt][r];
          dst[(size_t)(C + o) * NS] = S2[tt][r];
          dst[(size_t)(2 * C + o) * NS] = S3[tt][r];
          dst[(size_t)(3 * C + o) * NS] = S4[tt][r];
        }
      }
  }
}

// ------------------------------------------------------------ SModel fwd, fiber tiles
// The same message and Pebay update on a fiber-tile grid: a block owns 16
// fibers of one graph and ALL its classes, wave w the classes w, w+4, ...; the
// 4 waves' states are merged in the block (Pebay's pairwise formula, double,
// fixed order 0 <- 1 <- 2 <- 3) and the moments written straight to mom / hs
// (k_source_finalize's arithmetic): no class-split partials, no finalize
// launch.  Blocks are mapped XCD-aware: the 8 XCDs take blocks round-robin,
// so block b runs tile (b % 8) * ceil(nb / 8) + b / 8 -- neighbouring tiles,
// whose 64-byte rows share 128-byte lines, sit in one XCD's L2.
// WF (few classes, NC <= MF_SFT_WAVE_MAXNC): a block owns 64 fibers, wave w
// fibers 16w .. 16w + 15 over every class -- no merge, and the block's setup
// (class table, weight registers) is shared by 4x the edges.
#define MF_SFT_MAXNC 256
#define MF_SFT_WAVE_MAXNC 64
#ifndef MF_SFT_B6S
#define MF_SFT_B6S 3   // bit 0: L1's tuples in LDS, bit 1: L2's
#endif
// dynamic LDS floats of km_source_fwd_ft: the class table [NC][CP], which the
// waves' merge reuses as [3][MS][64] after the class loop
static inline size_t sft_lds_floats(int NC, int F) {
  const int C = 2 * F, NT = (((C + 3) / 4) + 3) / 4, CP = 16 * NT, MS = 16 * NT;
  return std::max((size_t)NC * CP, (size_t)3 * MS * 64);
}
#if !MF_PEB_CONST && defined(MF_PEB_DIAG)
__device__ unsigned g_peb_diag_n = 0;
#endif
template <int F, int PREC, bool WF>
__global__ __launch_bounds__(256) void km_source_fwd_ft(
    EdgeGeo geo, int ntiles, const float* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ QtS, const float* __restrict__ Ws1,
    const float* __restrict__ Ws2, const float* __restrict__ bs2, float* __restrict__ mom,
    float* __restrict__ hs, float* __restrict__ msg) {
  constexpr int C = 2 * F, NT = GM<C>::NT, CP = ClassRows<C>::CP;
  constexpr int MS = 4 * 4 * NT;   // a lane's merge state: 4 sums x NT tiles x 4 slots
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g4 = lane >> 4, j16 = lane & 15;
  const int per = (ntiles + 7) >> 3, bx = blockIdx.x;
  const int tile = (bx & 7) * per + (bx >> 3);
  constexpr int TF = WF ? 64 : 16;               // fibers per tile
  const int TPG = (geo.NF + TF - 1) / TF;        // tiles per graph
  if (tile >= ntiles) return;   // (block-uniform: the grid is rounded up to 8 * per)
  const bool tvalid = true;
  const int gg = tile / TPG, ft = tile - gg * TPG;
  const int f = ft * TF + (WF ? wave * 16 : 0) + j16;
  const bool fvalid = tvalid && f < geo.NF;
  const long long NS = geo.NS, n = (long long)gg * geo.NF + (fvalid ? f : 0);
  const int NC = geo.NC;
  const uint32_t RB = (uint32_t)geo.E * 4u;
  const uint32_t eo0 = (uint32_t)((((long long)gg * NC) * geo.NF + (fvalid ? f : 0)) * 4);
  const uint32_t eoc = (uint32_t)geo.NF * 4u, EB = (uint32_t)geo.E * 4u;
  // the class table (and, after the loop, the waves' merge scratch), sized by
  // the launch: sft_lds_floats(NC, F) floats of dynamic LDS
  extern __shared__ __attribute__((aligned(16))) float qtl[];
#if MF_PEB_CONST
  const auto& pco = c_peb.v;
  static_assert(MF_SFT_MAXNC / 4 + 1 <= MF_PEB_ROWS, "Pebay table rows");
#else
  __shared__ __attribute__((aligned(16))) float pco[MF_SFT_MAXNC / 4 + 1][8];
#endif
  ClassRows<C>::stage(qtl, QtS, geo.NT, (long long)gg * NC, NC);
  // (MF_SFT_B6S: bf16x6's split weight tuples in LDS, LayerB6S -- four waves
  // per SIMD instead of three with them in registers; source_fwd -0.01 ms)
  constexpr bool B6S1 = (MF_SFT_B6S & 1) && PREC == 4, B6S2 = (MF_SFT_B6S & 2) && PREC == 4;
  std::conditional_t<B6S1, LayerB6S<C, F>, FwdLayer<PREC, C, F>> L1;
  std::conditional_t<B6S2, LayerB6S<C, C>, FwdLayer<PREC, C, C>> L2;
  if constexpr (B6S1 || B6S2) {
    __shared__ s16x8 w6[(LayerB6S<C, F>::NOP + LayerB6S<C, C>::NOP) * 64];
    if constexpr (B6S1) L1.bind(w6);
    if constexpr (B6S2) L2.bind(w6 + LayerB6S<C, F>::NOP * 64);
  }
  L1.load([&](int h, int k) { return Ws1[h * 2 * F + F + k]; }, lane);
  L2.load([&](int o, int h) { return Ws2[o * C + h]; }, lane);
  floatx4 bias[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) bias[tt] = ld_vec<C>(bs2, tt, g4);
  const floatx4 scv = ld_fconst<F>(sc, g4, 1.f), shv = ld_fconst<F>(sh, g4, 0.f);
  MF_FMASK(F)
  const RowOff<C> roC(eo0, RB, g4);   // (the message cache's rows)
  const Rsrc ry = rsrc(y, EB * F);
  floatx4 S1[NT], S2[NT], S3[NT], S4[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) S1[tt] = S2[tt] = S3[tt] = S4[tt] = zero4();
  // Pebay coefficients of the k-th message of a wave (count k + 1), as km_source_fwd
  static_assert(MF_SFT_WAVE_MAXNC <= MF_SFT_MAXNC / 4 + 1, "pco rows");
#if !MF_PEB_CONST
  const int nk = WF ? NC : (NC + 3) >> 2;
  if (t < nk) {
    const double nn = t + 1, r = 1.0 / nn;
    pco[t][0] = (float)((nn - 1) * r);
    pco[t][1] = (float)((nn - 1) * (nn - 2) * r * r);
    pco[t][2] = (float)((nn - 1) * (nn * nn - 3 * nn + 3) * r * r * r);
    pco[t][3] = (float)r;
    pco[t][4] = (float)(6 * r * r);
    pco[t][5] = (float)(-4 * r);
    pco[t][6] = (float)(-3 * r);
    pco[t][7] = 0.f;
  }
#endif
  __syncthreads();   // qtl (and the LDS Pebay table)
  // wave w: classes w + 4k, k = 0 .. (its count) - 1, streamed as k (WF: class k)
  const int kw = WF ? NC : (NC - wave + 3) >> 2;
  auto load = [&](int k) {
    Rows<1> r;
    r.v[0] = ld_frows<F>(ry, (uint32_t)(WF ? k : wave + 4 * k) * eoc, ro);
    return r;
  };
  // the k-th message folded into the lane's moments (Pebay, count k + 1)
  auto fold = [&](const floatx4 (&m)[NT], int k) {
    const floatx4 ca = *reinterpret_cast<const floatx4*>(&pco[k][0]);
    const floatx4 cb = *reinterpret_cast<const floatx4*>(&pco[k][4]);
#if !MF_PEB_CONST && defined(MF_PEB_DIAG)
    {  // (diagnostic build, tools/race_bisect.sh: the LDS rows against c_peb)
      unsigned badm = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        badm |= ((ca[j] != c_peb.v[k][j]) ? 1u : 0u) << j | ((cb[j] != c_peb.v[k][4 + j]) ? 1u : 0u) << (4 + j);
      if (badm) {
        const unsigned nd = atomicAdd(&g_peb_diag_n, 1u);
        if (nd < 48) printf("PEBDIAG block %d wave %d lane %d k %d mask %x\n", (int)blockIdx.x, wave, lane, k, badm);
      }
    }
#endif
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
  };
  auto message = [&](const Rows<1>& rows, int k, floatx4 (&m)[NT]) {
    const int c = WF ? k : wave + 4 * k;
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fm, sc, scv, shv)};
    floatx4 z[NT], a[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) z[tt] = ClassRows<C>::get(qtl, c, tt, g4);
    L1.apply(x, z);
    lrelu_act<C>(z, a);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) m[tt] = bias[tt];
    L2.apply(a, m);
    if (msg) st_rows_nt<C>(msg, (uint32_t)c * eoc, roC, g4, fvalid, m);
  };
#if MF_FWD_PAIRS
  // two messages per body (independent chains interleaved), folded in order
  class_stream_pairs<MF_DEPTH_FWD>(
      0, kw, load,
      [&](const Rows<1>& rows, int k) {
        floatx4 m[NT];
        message(rows, k, m);
        fold(m, k);
      },
      [&](const Rows<1>& ra, int ka, const Rows<1>& rb, int kb) {
        floatx4 ma[NT], mb[NT];
        message(ra, ka, ma);
        message(rb, kb, mb);
        fold(ma, ka);
        fold(mb, kb);
      });
#else
  class_stream<MF_DEPTH_FWD>(0, kw, load, [&](const Rows<1>& rows, int k) {
    floatx4 m[NT];
    message(rows, k, m);
    fold(m, k);
  });
#endif
  const double invn = 1.0 / (double)NC;
  // the moments' finalize (k_source_finalize's arithmetic) -> mom / hs
  auto emit = [&](int o, double mean, double M2, double M3, double M4) {
    const long long idx = (long long)o * NS + n, CNS = (long long)C * NS;
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
  };
  if constexpr (WF) {
    if (!fvalid) return;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const int o = GM<C>::row(g4, 4 * tt + r);
        if (o >= 0) emit(o, S1[tt][r], S2[tt][r], S3[tt][r], S4[tt][r]);
      }
    return;
  }
  // merge: waves 1..3 park their states in LDS (qtl is free once every wave is past its loop)
  __syncthreads();
  float* ms = qtl;   // [3][MS][64]
  static_assert(3 * MS * 64 <= MF_SFT_MAXNC * CP, "merge scratch exceeds the class table");
  // (sft_lds_floats sizes the dynamic table for max(NC * CP, 3 * MS * 64))
  if (wave > 0) {
    float* p = ms + (size_t)(wave - 1) * MS * 64 + lane;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[((0 * NT + tt) * 4 + r) * 64] = S1[tt][r];
        p[((1 * NT + tt) * 4 + r) * 64] = S2[tt][r];
        p[((2 * NT + tt) * 4 + r) * 64] = S3[tt][r];
        p[((3 * NT + tt) * 4 + r) * 64] = S4[tt][r];
      }
  }
  __syncthreads();
  if (wave != 0 || !fvalid) return;
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
#pragma unroll
    for (int r = 0; r < GM<C>::nreg(tt); ++r) {
      const int o = GM<C>::row(g4, 4 * tt + r);
      if (o < 0) continue;
      double na = (double)kw, mean = S1[tt][r], M2 = S2[tt][r], M3 = S3[tt][r], M4 = S4[tt][r];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const double nb = (double)((NC - w + 3) >> 2);
        if (nb <= 0) continue;
        const float* p = ms + (size_t)(w - 1) * MS * 64 + lane;
        pebay_merge<double>(na, mean, M2, M3, M4, nb, p[((0 * NT + tt) * 4 + r) * 64],
                            p[((1 * NT + tt) * 4 + r) * 64], p[((2 * NT + tt) * 4 + r) * 64],
                            p[((3 * NT + tt) * 4 + r) * 64]);
        na += nb;
      }
      emit(o, mean, M2, M3, M4);
    }
}

// ============================================================ TModel fwd
// a = lrelu(Rs[f] + Wt1[:, F:2F] x) per edge and its per-class sum over fibers
// (gnn.py:188-190; the second Linear runs after the sum, on the node side).
template <int F, int PREC>
__global__ __launch_bounds__(256) void km_target_fwd(EdgeGeo geo, const float* __restrict__ y,
                                                     const float* __restrict__ sc,
                                                     const float* __restrict__ sh,
                                                     const float* __restrict__ Rs,
                                                     const float* __restrict__ Wt1,
                                                     float* __restrict__ part,
                                                     uint8_t* __restrict__ tmask) {
  constexpr int C = 2 * F, NT = GM<C>::NT;
  MF_GEO
  __shared__ __attribute__((aligned(16))) float colbuf[COL_CH * 4 * C];
  FwdLayer<PREC, C, F> L1;
  L1.load([&](int h, int k) { return Wt1[h * 2 * F + F + k]; }, lane);
  floatx4 rs[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) rs[tt] = ld_node<C>(Rs, tt, g4, NS, n, fvalid);
  const floatx4 scv = ld_fconst<F>(sc, g4, 1.f), shv = ld_fconst<F>(sh, g4, 0.f);
  MF_FMASK(F)
  const Rsrc ry = rsrc(y, EB * F);

  int cbase = c0;
  auto load = [&](int c) {
    Rows<1> r;
    r.v[0] = ld_frows<F>(ry, (uint32_t)c * eoc, ro);
    return r;
  };
  auto pre = [&](const Rows<1>& rows, floatx4 (&z)[NT]) {
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fm, sc, scv, shv)};
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) z[tt] = rs[tt];
    L1.apply(x, z);
  };
  auto post = [&](const floatx4 (&z)[NT], int c) {
    if (tmask && fvalid)
      (tmask + (uint32_t)c * eoc)[opaque(eo0 + g4)] = (uint8_t)mask_bits<C>(z);
    const int cl = c - cbase;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const float s = row_sum16(fvalid ? lrelu(z[tt][r]) : 0.f);
        const int h = GM<C>::row(g4, 4 * tt + r);
        if (j16 == 15 && h >= 0) colbuf[(cl * 4 + wave) * C + h] = s;
      }
    if (cl == COL_CH - 1 || c == c1 - 1) {
      __syncthreads();
      col_flush<C>(colbuf, cl + 1, cbase, part, colbase);
      __syncthreads();
      cbase = c + 1;
    }
  };
#if MF_FWD_PAIRS
  class_stream_pairs<MF_DEPTH_FWD>(
      c0, c1, load,
      [&](const Rows<1>& rows, int c) {
        floatx4 z[NT];
        pre(rows, z);
        post(z, c);
      },
      [&](const Rows<1>& ra, int ca, const Rows<1>& rb, int cb) {
        floatx4 za[NT], zb[NT];
        pre(ra, za);
        pre(rb, zb);
        post(za, ca);
        post(zb, cb);
      });
#else
  class_stream<MF_DEPTH_FWD>(c0, c1, load, [&](const Rows<1>& rows, int c) {
    floatx4 z[NT];
    pre(rows, z);
    post(z, c);
  });
#endif
}

// ============================================================ TModel bwd
// g_z = g_hsum[c] * lrelu'(z) per edge; per-fiber sums of g_z (-> g_Rs), the
// edge-input gradient Wt1[:, F:2F]^T g_z (optional) and dWt1[:, F:2F] += g_z x^T.
template <int F, int PREC, bool TM>
__global__ __launch_bounds__(256) void km_target_bwd(EdgeGeo geo, const float* __restrict__ y,
                                                     const float* __restrict__ sc,
                                                     const float* __restrict__ sh,
                                                     const float* __restrict__ Rs,
                                                     const float* __restrict__ Wt1,
                                                     const float* __restrict__ ghS,
                                                     float* __restrict__ GzT,
                                                     float* __restrict__ gxe,
                                                     float* __restrict__ partW,
                                                     const uint8_t* __restrict__ tmask) {
  constexpr int C = 2 * F, NT = GM<C>::NT;
  constexpr int NIMG = NT + 1;  // g_z tiles | x
  using WI = WgImg<PREC>;       // weight-gradient images: bf16x3, or exact fp32 at PREC 0
  MF_GEO
  __shared__ __attribute__((aligned(16))) short imgs[4 * NIMG * WI::U];
  __shared__ float scratch[4 * C * F];
  __shared__ __attribute__((aligned(16))) float ghl[MF_MAX_CPS * ClassRows<C>::CP];
  ClassRows<C>::stage(ghl, ghS, geo.NT, (long long)gg * geo.NC + c0, c1 - c0);
  short* img = imgs + wave * NIMG * WI::U;
  // the pre-activation z = Rs[f] + Wt1[:, F:2F] x is recomputed, or (TM) only
  // its LeakyReLU mask is read back from target_fwd
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

  auto load = [&](int c) {
    Rows<1> r;
    const uint32_t co = (uint32_t)c * eoc;
    r.v[0] = ld_frows<F>(ry, co, ro);
    if constexpr (TM) r.m = __builtin_amdgcn_raw_buffer_load_b8(rtm, eo0 + g4, co, 0);
    return r;
  };
  class_stream<MF_DEPTH_BWD>(c0, c1, load, [&](const Rows<1>& rows, int c) {
    const floatx4 x[1] = {edge_in<F>(rows.v[0], fm, sc, scv, shv)};
    floatx4 z[NT], gz[NT];
    if constexpr (!TM) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) z[tt] = rs[tt];
      L1.apply(x, z);
    }
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      const floatx4 gh = ClassRows<C>::get(ghl, c - c0, tt, g4);
      gz[tt] = zero4();
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const float sl = TM ? mask_slope(rows.m, 4 * tt + r) : dlrelu(z[tt][r]);
        gz[tt][r] = fvalid ? gh[r] * sl : 0.f;
      }
      accF[tt] += gz[tt];
    }
    Fr sgz[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) sgz[tt] = split(gz[tt]);
    if (gxe) {
      floatx4 gx[1] = {zero4()};
      if constexpr (PREC >= 1) LT.apply(sgz, gx); else LT.apply(gz, gx);
      st_frows<F>(gxe, EB * F, (uint32_t)c * eoc, ro, g4, fvalid, gx[0]);
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
// Per edge: recompute the message (gnn.py:136-137), g_m from the per-fiber
// moment coefficients (d loss / d m is a cubic in m - mean), back through the
// message MLP; plus TModel's recomputed input gradient, the downstream edge
// gradient and the edge BatchNorm's two gradient sums.  dWs2 += g_m a^T,
// dbs2 += g_m, dWs1[:, F:2F] += g_zs x^T, per-class sums of g_zs (-> g_Qt).
// MSG: the forward's messages m are read from the message cache (msg, written
// by km_source_fwd_ft) instead of recomputed through node_mlp_1's second Linear:
// the same values bit for bit (the cache holds what the forward computed), 10
// fewer fp32 MFMAs per class and that layer's dependent chain off the class's
// critical path, for 80 B per edge written in the forward and read here.
template <int F, int PREC, bool TM, bool MSG = false>
__global__ __launch_bounds__(256, 2) void km_source_bwd(
    EdgeGeo geo, const float* __restrict__ msg, const float* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ QtS, const float* __restrict__ Ws1,
    const float* __restrict__ Ws2, const float* __restrict__ bs2, const float* __restrict__ mean,
    const float* __restrict__ coef, const float* __restrict__ Rs, const float* __restrict__ Wt1,
    const float* __restrict__ ghS, const float* __restrict__ g_next,
    const float* __restrict__ mu1, const float* __restrict__ inv1, float* __restrict__ g_tot,
    float* __restrict__ partW2, float* __restrict__ partW1, float* __restrict__ partCol,
    float* __restrict__ partBN, const uint8_t* __restrict__ tmask) {
  constexpr int C = 2 * F, NT = GM<C>::NT;
  // PACK (Fdim 10: C = 20 messages, 2 tiles of which the second holds ONE row
  // per lane group; x has 3 rows per group): the weight-gradient operands are
  // packed into 5 images instead of 7 -- R1 = g_m tile 0, R2 = g_zs tile 0,
  // R3 = [g_m tile 1 | g_zs tile 1] (register slots 0, 1), C1 = a tile 0,
  // C2 = [a tile 1 | x] (slot 0, slots 1-3) -- and dWs2 / dWs1 come out of 5
  // outer-product tiles (R1 C1, R1 C2, R2 C2, R3 C1, R3 C2) instead of 6, the
  // padding rows of one operand carrying the other's live rows.  Every output
  // element is the same products in the same order: bitwise the unpacked sums.
  constexpr bool PACK = MF_SB_PACK && NT == 2 && GM<C>::nreg(1) == 1 && GM<F>::NT == 1 && GM<F>::RPG == 3;
  constexpr int NIMG = PACK ? 5 : 3 * NT + 1;   // g_m | a | g_zs | x (packed: R1 R2 R3 C1 C2)
  constexpr int SCR = C * (C + 1) > C * F ? C * (C + 1) : C * F;
  using WI = WgImg<PREC>;
  MF_GEO
  __shared__ __attribute__((aligned(16))) short imgs[4 * NIMG * WI::U];
  __shared__ __attribute__((aligned(16))) float colbuf[COL_CH * 4 * C];
  __shared__ float scratch[4 * SCR];
  __shared__ __attribute__((aligned(16))) float qtl[MF_MAX_CPS * ClassRows<C>::CP];
  __shared__ __attribute__((aligned(16))) float ghl[MF_MAX_CPS * ClassRows<C>::CP];
  ClassRows<C>::stage(qtl, QtS, geo.NT, (long long)gg * geo.NC + c0, c1 - c0);
  if (ghS) ClassRows<C>::stage(ghl, ghS, geo.NT, (long long)gg * geo.NC + c0, c1 - c0);
  short* img = imgs + wave * NIMG * WI::U;
  short* im_gm = img;
  short* im_a = img + NT * WI::U;
  short* im_gz = im_a + NT * WI::U;
  short* im_x = im_gz + NT * WI::U;
  // (PACK) R1 R2 R3 C1 C2
  short* im_r1 = img;
  short* im_r2 = img + WI::U;
  short* im_r3 = img + 2 * WI::U;
  short* im_c1 = img + 3 * WI::U;
  short* im_c2 = img + 4 * WI::U;
  (void)im_r1; (void)im_r2; (void)im_r3; (void)im_c1; (void)im_c2;
  const long long CNS = (long long)C * NS;
  const bool tpart = Rs != nullptr;

  RecLayer<PREC, C, F> L1s, L1t;   // L1t: TModel's layer, recomputed unless TM
  RecLayer<PREC, C, C> L2;
  constexpr int R1 = RecLds<RecLayer<PREC, C, F>>::n, R2 = RecLds<RecLayer<PREC, C, C>>::n;
  __shared__ s16x8 recw[(R1 * (TM ? 1 : 2) + R2) > 0 ? R1 * (TM ? 1 : 2) + R2 : 1];
  rec_bind(L1s, recw);
  rec_bind(L2, recw + R1);
  rec_bind(L1t, recw + R1 + R2);
  L1s.load([&](int h, int k) { return Ws1[h * 2 * F + F + k]; }, lane);
  if constexpr (!TM) L1t.load([&](int h, int k) { return tpart ? Wt1[h * 2 * F + F + k] : 0.f; }, lane);
  if constexpr (!MSG) L2.load([&](int o, int h) { return Ws2[o * C + h]; }, lane);
  // gradient chains: exact fp32, bf16x3 or bf16 by PREC (MF_SB_LDSW: the
  // split-bf16 weight operands read from LDS per use instead of registers)
  constexpr bool LW = MF_SB_LDSW && std::is_same_v<GradLayer<PREC, C, C>, LayerB3<C, C>>;
  using GL2 = std::conditional_t<LW, LayerB3S<C, C>, GradLayer<PREC, C, C>>;
  using GL1 = std::conditional_t<LW, LayerB3S<F, C>, GradLayer<PREC, F, C>>;
  GL2 L2T;
  GL1 L1sT, L1tT;
  if constexpr (LW) {
    __shared__ s16x8 gw[(LayerB3S<C, C>::NOP + 2 * LayerB3S<F, C>::NOP) * 64];
    L2T.bind(gw);
    L1sT.bind(gw + LayerB3S<C, C>::NOP * 64);
    L1tT.bind(gw + (LayerB3S<C, C>::NOP + LayerB3S<F, C>::NOP) * 64);
  }
  L2T.load([&](int h, int o) { return Ws2[o * C + h]; }, lane);
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
  [[maybe_unused]] const Rsrc rms = rsrc(msg, EB * C);
  [[maybe_unused]] const RowOff<C> roC(eo0, RB, g4);

  floatx4 accW2[NT * NT], accW1[NT], accB[NT];
  floatx4 accP[5];   // (PACK) R1 C1, R1 C2, R2 C2, R3 C1, R3 C2
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    accW1[tt] = zero4();
    accB[tt] = zero4();
#pragma unroll
    for (int nb = 0; nb < NT; ++nb) accW2[tt * NT + nb] = zero4();
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) accP[i] = zero4();
  floatx4 sg = zero4(), sgx = zero4();
  const s16x8 ones = ones_reg();
  __syncthreads();   // qtl, ghl

  int cbase = c0;
  using RowsT = Rows<MSG ? 2 + NT : 2>;
  auto load = [&](int c) {
    RowsT r;
    const uint32_t co = (uint32_t)c * eoc;
    r.v[0] = ld_frows<F>(ry, co, ro);
    r.v[1] = g_next ? ld_frows<F>(rgn, co, ro) : zero4();
    if constexpr (TM) r.m = tpart ? __builtin_amdgcn_raw_buffer_load_b8(rtm, eo0 + g4, co, 0) : 0u;
    if constexpr (MSG) {
      floatx4 mv[NT];
      ld_rows_nt<C>(rms, co, roC, mv);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) r.v[2 + tt] = mv[tt];
    }
    return r;
  };
  class_stream<MF_DEPTH_BWD>(c0, c1, load, [&](const RowsT& rows, int c) {
    const floatx4 yr = rows.v[0], gnr = rows.v[1];
    const floatx4 x[1] = {edge_in<F>(yr, fm, sc, scv, shv)};
    // ---- forward recompute: z_s, a_s, m (MSG: m from the message cache)
    floatx4 zs[NT], as[NT], m[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) zs[tt] = ClassRows<C>::get(qtl, c - c0, tt, g4);
    L1s.apply(x, zs);
    lrelu_act<C>(zs, as);
    if constexpr (MSG) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) m[tt] = rows.v[2 + tt];
    } else {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) m[tt] = bias[tt];
      L2.apply(as, m);
    }
    floatx4 gm[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      gm[tt] = zero4();
#pragma unroll
      for (int r = 0; r < GM<C>::nreg(tt); ++r) {
        const float d = m[tt][r] - mn[tt][r];
        gm[tt][r] = fvalid ? fmaf(d, fmaf(d, fmaf(d, q3[tt][r], q2[tt][r]), q1[tt][r]), q0[tt][r]) : 0.f;
      }
      accB[tt] += gm[tt];
    }
    // ---- backward through the message MLP (the operand splits also feed the
    // weight-gradient images below)
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
    // the weight-gradient images are written first: their LDS latency hides
    // behind the input-gradient chains below
    lds_order();
    [[maybe_unused]] floatx4 r3v, c2v;
    if constexpr (PACK) {
      r3v = floatx4{gm[1][0], gz[1][0], 0.f, 0.f};
      c2v = floatx4{as[1][0], x[0][0], x[0][1], x[0][2]};
      const Fr sr3 = {s16x4{sgm[1].h[0], sgz[1].h[0], 0, 0}, s16x4{sgm[1].l[0], sgz[1].l[0], 0, 0}};
      WI::put(im_r1, lane, gm[0], sgm[0]);
      WI::put(im_r2, lane, gz[0], sgz[0]);
      WI::put(im_r3, lane, r3v, sr3);
      WI::put(im_c1, lane, as[0], split(as[0]));
      WI::put(im_c2, lane, c2v, split(c2v));
    } else {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        WI::put(im_gm + tt * WI::U, lane, gm[tt], sgm[tt]);
        WI::put(im_a + tt * WI::U, lane, as[tt], split(as[tt]));
        WI::put(im_gz + tt * WI::U, lane, gz[tt], sgz[tt]);
      }
      WI::put(im_x, lane, x[0], split(x[0]));
    }
    lds_order();
#if MF_WG_EARLY_READS
    // the transposed image reads go out now, ahead of the input-gradient
    // chains (as in km_edge_mlp_bwd)
    typename WI::R rx, ra[NT], rgm[NT], rgz[NT], rp[5], rq[2];
    if constexpr (PACK) {
#pragma unroll
      for (int i = 0; i < 5; ++i) rp[i] = WI::rd(img + i * WI::U, lane);
#if MF_WG4
      lds_order();   // (the B images' second reads: mma4)
      rq[0] = WI::rd(im_c1, lane);
      rq[1] = WI::rd(im_c2, lane);
#endif
    } else {
      rx = WI::rd(im_x, lane);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        ra[tt] = WI::rd(im_a + tt * WI::U, lane);
        rgm[tt] = WI::rd(im_gm + tt * WI::U, lane);
        rgz[tt] = WI::rd(im_gz + tt * WI::U, lane);
      }
    }
    lds_order();
#endif
    floatx4 g[1] = {zero4()};
    if constexpr (PREC >= 1) L1sT.apply(sgz, g); else L1sT.apply(gz, g);
    if (tpart) {  // TModel's per-edge input gradient (gnn.py:188-190)
      floatx4 zt[NT];
      if constexpr (!TM) {   // its pre-activation recomputed
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) zt[tt] = rs[tt];
        L1t.apply(x, zt);
      }
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        const floatx4 gh = ClassRows<C>::get(ghl, c - c0, tt, g4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sl = TM ? mask_slope(rows.m, 4 * tt + r) : dlrelu(zt[tt][r]);
          zt[tt][r] = (fvalid && r < GM<C>::nreg(tt)) ? gh[r] * sl : 0.f;
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
    for (int r = 0; r < 4; ++r) g[0][r] = fm[r] ? g[0][r] + (g_next ? gnr[r] : 0.f) : 0.f;
    st_frows<F>(g_tot, EB * F, (uint32_t)c * eoc, ro, g4, fvalid, g[0]);
    if (mu1) {
#pragma unroll
      for (int r = 0; r < GM<F>::RPG; ++r) {
        sg[r] += g[0][r];
        sgx[r] = fmaf(g[0][r], (yr[r] - m1v[r]) * i1v[r], sgx[r]);
      }
    }
    // ---- weight gradients (edge = K) through the transposed images
    lds_order();
    const int cl = c - cbase;
    if constexpr (PACK) {
#if !MF_WG_EARLY_READS
#error "source_bwd's packed tiles read their images early (MF_WG_EARLY_READS)"
#endif
      const typename WI::TA t1 = WI::A(rp[0]), t2 = WI::A(rp[1]), t3 = WI::A(rp[2]);
#if MF_WG4
      const typename WI::TB4 tc1 = WI::B4(rp[3], rq[0]), tc2 = WI::B4(rp[4], rq[1]);
      accP[0] = WI::mma4(t1, tc1, accP[0]);
      accP[1] = WI::mma4(t1, tc2, accP[1]);
      accP[2] = WI::mma4(t2, tc2, accP[2]);
      accP[3] = WI::mma4(t3, tc1, accP[3]);
      accP[4] = WI::mma4(t3, tc2, accP[4]);
#else
      const typename WI::TB tc1 = WI::B(rp[3]), tc2 = WI::B(rp[4]);
      accP[0] = WI::mma(t1, tc1, accP[0]);
      accP[1] = WI::mma(t1, tc2, accP[1]);
      accP[2] = WI::mma(t2, tc2, accP[2]);
      accP[3] = WI::mma(t3, tc1, accP[3]);
      accP[4] = WI::mma(t3, tc2, accP[4]);
#endif
      // per-class sums of g_zs: R2's rows, and R3's register slot 1
      const floatx4 cs2 = WI::colsum(t2, gz[0], ones), cs3 = WI::colsum(t3, r3v, ones);
      if (j16 == WI::CS_LANE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = GM<C>::mrow(0, 4 * g4 + r);
          if (h >= 0) colbuf[(cl * 4 + wave) * C + h] = cs2[r];
        }
        const int h1 = GM<C>::row(g4, 4);
        if (h1 >= 0) colbuf[(cl * 4 + wave) * C + h1] = cs3[1];
      }
    } else {
#if MF_WG_EARLY_READS
    const typename WI::TB tx = WI::B(rx);
    typename WI::TB ta[NT];
#pragma unroll
    for (int nb = 0; nb < NT; ++nb) ta[nb] = WI::B(ra[nb]);
#else
    const typename WI::TB tx = WI::B(im_x, lane);
    typename WI::TB ta[NT];
#pragma unroll
    for (int nb = 0; nb < NT; ++nb) ta[nb] = WI::B(im_a + nb * WI::U, lane);
#endif
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
#if MF_WG_EARLY_READS
      const typename WI::TA tgm = WI::A(rgm[tt]);
#pragma unroll
      for (int nb = 0; nb < NT; ++nb) accW2[tt * NT + nb] = WI::mma(tgm, ta[nb], accW2[tt * NT + nb]);
      const typename WI::TA tgz = WI::A(rgz[tt]);
#else
      const typename WI::TA tgm = WI::A(im_gm + tt * WI::U, lane);
#pragma unroll
      for (int nb = 0; nb < NT; ++nb) accW2[tt * NT + nb] = WI::mma(tgm, ta[nb], accW2[tt * NT + nb]);
      const typename WI::TA tgz = WI::A(im_gz + tt * WI::U, lane);
#endif
      accW1[tt] = WI::mma(tgz, tx, accW1[tt]);
      const floatx4 cs = WI::colsum(tgz, gz[tt]);
      if (j16 == WI::CS_LANE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = GM<C>::mrow(tt, 4 * g4 + r);
          if (h >= 0) colbuf[(cl * 4 + wave) * C + h] = cs[r];
        }
      }
    }
    }
    if (cl == COL_CH - 1 || c == c1 - 1) {
      __syncthreads();
      col_flush<C>(colbuf, cl + 1, cbase, partCol, colbase);
      __syncthreads();
      cbase = c + 1;
    }
  });
  if constexpr (PACK) {
    // dWs2 [o][h]: R1 C1 (tile-0 rows x tile-0 columns), R1 C2 and R3 C1 (slot 0
    // of C2 / R3: the tile-1 row of each lane group), R3 C2 (both slot 0)
    block_partial(accP, scratch, C * (C + 1), [&](int a, int s, int jj) {
      int o = -1, h = -1;
      if (a == 0) { o = GM<C>::mrow(0, s); h = GM<C>::mrow(0, jj); }
      if (a == 1 && (jj & 3) == 0) { o = GM<C>::mrow(0, s); h = GM<C>::row(jj >> 2, 4); }
      if (a == 3 && (s & 3) == 0) { o = GM<C>::row(s >> 2, 4); h = GM<C>::mrow(0, jj); }
      if (a == 4 && (s & 3) == 0 && (jj & 3) == 0) { o = GM<C>::row(s >> 2, 4); h = GM<C>::row(jj >> 2, 4); }
      return (o >= 0 && h >= 0) ? o * (C + 1) + h : -1;
    }, partW2 + (size_t)bx * C * (C + 1));
  } else {
    block_partial(accW2, scratch, C * (C + 1), [&](int a, int s, int jj) {
      const int o = GM<C>::mrow(a / NT, s), h = GM<C>::mrow(a % NT, jj);
      return (o >= 0 && h >= 0) ? o * (C + 1) + h : -1;
    }, partW2 + (size_t)bx * C * (C + 1));
  }
  // dbs2 (exact fp32 sums of g_m: a bias gradient cancels to ~0 through the
  // BatchNorm that follows) -> column C of the same partial
  {
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
  if constexpr (PACK) {
    // dWs1 [h][k]: R2 C2 (tile-0 rows x C2's slots 1-3 = x) and R3 C2 (R3's
    // slot 1 = the tile-1 row of g_zs)
    block_partial(accP, scratch, C * F, [&](int a, int s, int jj) {
      int h = -1, k = -1;
      if ((jj & 3) != 0) k = GM<F>::row(jj >> 2, (jj & 3) - 1);
      if (a == 2) h = GM<C>::mrow(0, s);
      if (a == 4 && (s & 3) == 1) h = GM<C>::row(s >> 2, 4);
      return (h >= 0 && k >= 0) ? h * F + k : -1;
    }, partW1 + (size_t)bx * C * F);
  } else {
    block_partial(accW1, scratch, C * F, [&](int a, int s, int jj) {
      const int h = GM<C>::mrow(a, s), k = GM<F>::mrow(0, jj);
      return (h >= 0 && k >= 0) ? h * F + k : -1;
    }, partW1 + (size_t)bx * C * F);
  }
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
// g_y = alpha*g + gam0 + gam1*y (the double BatchNorm's backward, per channel),
// then back through the edge MLP: dW2 += g_y a^T, db2 += g_y,
// dW1[:, 2F:3F] += g_z x^T, per-fiber (-> g_Ps) and per-class (-> g_Pt) sums of
// g_z, and the edge-input gradient W1[:, 2F:3F]^T g_z when the block has an
// upstream edge input.
#ifndef MF_BWD_PIPE6
#define MF_BWD_PIPE6 0   // 1: the class pipeline on bf16x6 too: its LDS-tuple recompute then spills 16 VGPRs, edge_mlp_bwd 2.36 -> 2.42 ms (profiles/r06p_ab.txt)
#endif
template <int F, int PREC>
__global__ __launch_bounds__(256, 2) void km_edge_mlp_bwd(
    EdgeGeo geo, const float* __restrict__ g_tot, const float* __restrict__ alpha,
    const float* __restrict__ gam0, const float* __restrict__ gam1, const float* __restrict__ y,
    const float* __restrict__ xe, const float* __restrict__ xsc, const float* __restrict__ xsh,
    const float* __restrict__ Ps, const float* __restrict__ PtS, const float* __restrict__ W1,
    const float* __restrict__ W2, float* __restrict__ gxe, float* __restrict__ GzEs,
    float* __restrict__ partW2, float* __restrict__ partW1, float* __restrict__ partCol) {
  constexpr int H = 4 * F, NT = GM<H>::NT;
  constexpr int NIMG = 1 + NT + NT + 1;          // g_y | a | g_z | x
  constexpr int SCR = F * (H + 1) > H * F ? F * (H + 1) : H * F;
  using WI = WgImg<PREC>;
  MF_GEO
  __shared__ __attribute__((aligned(16))) short imgs[4 * NIMG * WI::U];
  __shared__ __attribute__((aligned(16))) float colbuf[COL_CH * 4 * H];
  __shared__ float scratch[4 * SCR];
  __shared__ __attribute__((aligned(16))) float ptl[MF_MAX_CPS * ClassRows<H>::CP];
  ClassRows<H>::stage(ptl, PtS, geo.NT, (long long)gg * geo.NC + c0, c1 - c0);
  short* img = imgs + wave * NIMG * WI::U;
  short* im_gy = img;
  short* im_a = img + WI::U;
  short* im_gz = im_a + NT * WI::U;
  short* im_x = im_gz + NT * WI::U;

#ifdef MF_EMB_REC_B6   // (A/B: the default path's recompute on bf16x6 instead of fp32 MFMA)
  std::conditional_t<PREC == 1, LayerB6<H, F>, FwdLayer<FP(PREC), H, F>> L1;
#else
  FwdLayer<FP(PREC), H, F> L1;
#endif
  L1.load([&](int h, int k) { return W1[h * 4 * F + 2 * F + k]; }, lane);
  // gradient chains: exact fp32, bf16x3 or bf16 by PREC
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
  const s16x8 ones = ones_reg();
  __syncthreads();   // ptl

  int cbase = c0;
  auto load = [&](int c) {
    Rows<3> r;
    const uint32_t co = (uint32_t)c * eoc;
    r.v[0] = ld_frows<F>(rgt, co, ro);
    r.v[1] = ld_frows<F>(ry, co, ro);
    r.v[2] = ld_frows<F>(rxe, co, ro);
    return r;
  };
  // head: g_y, the edge input and the first Linear's recompute of a class
  struct Head {
    floatx4 gy, x, z[NT];
  };
  auto head = [&](const Rows<3>& rows, int c) {
    Head hd;
#pragma unroll
    for (int r = 0; r < 4; ++r) hd.gy[r] = 0.f;
#pragma unroll
    for (int r = 0; r < GM<F>::RPG; ++r)
      hd.gy[r] = fm[r] ? fmaf(g1v[r], rows.v[1][r], fmaf(alv[r], rows.v[0][r], g0v[r])) : 0.f;
    hd.x = edge_in<F>(rows.v[2], fm, xsc, scv, shv);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) hd.z[tt] = ps[tt] + ClassRows<H>::get(ptl, c - c0, tt, g4);
    const floatx4 xx[1] = {hd.x};
    L1.apply(xx, hd.z);
    return hd;
  };
  auto tail = [&](const Head& hd, int c) {
    floatx4 gy[1] = {hd.gy};
    accB += gy[0];
    const floatx4 x[1] = {hd.x};
    floatx4 z[NT], a[NT], gz[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      z[tt] = hd.z[tt];
      gz[tt] = zero4();
    }
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
    // the weight-gradient images are written first: their LDS latency hides
    // behind the edge-input gradient chain below
    lds_order();
    WI::put(im_gy, lane, gy[0], sgy[0]);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      WI::put(im_a + tt * WI::U, lane, a[tt], split(a[tt]));
      WI::put(im_gz + tt * WI::U, lane, gz[tt], sgz[tt]);
    }
    WI::put(im_x, lane, x[0], split(x[0]));
    lds_order();
#if MF_WG_EARLY_READS
    // every transposed image read is issued before the edge-input gradient
    // chain (a wave's LDS operations run in order, so they see the writes
    // above): their latency hides behind that chain instead of stalling the
    // weight-gradient MFMAs one read group at a time
    const typename WI::R rgy = WI::rd(im_gy, lane), rx = WI::rd(im_x, lane);
    typename WI::R ra[NT], rgz[NT], ra2[NT], rx2;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      ra[tt] = WI::rd(im_a + tt * WI::U, lane);
      rgz[tt] = WI::rd(im_gz + tt * WI::U, lane);
    }
#if MF_WG4
    lds_order();   // (the B images' second reads: mma4)
    rx2 = WI::rd(im_x, lane);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) ra2[tt] = WI::rd(im_a + tt * WI::U, lane);
#endif
    lds_order();
#endif
    if (gxe) {
      floatx4 gx[1] = {zero4()};
      if constexpr (PREC >= 1) L1T.apply(sgz, gx); else L1T.apply(gz, gx);
      st_frows<F>(gxe, EB * F, (uint32_t)c * eoc, ro, g4, fvalid, gx[0]);
    }
#if MF_WG_EARLY_READS && MF_WG4
    const typename WI::TA tgy = WI::A(rgy);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) accW2[tt] = WI::mma4(tgy, WI::B4(ra[tt], ra2[tt]), accW2[tt]);
    const typename WI::TB4 tx = WI::B4(rx, rx2);
#elif MF_WG_EARLY_READS
    const typename WI::TA tgy = WI::A(rgy);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) accW2[tt] = WI::mma(tgy, WI::B(ra[tt]), accW2[tt]);
    const typename WI::TB tx = WI::B(rx);
#else
    const typename WI::TA tgy = WI::A(im_gy, lane);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
      accW2[tt] = WI::mma(tgy, WI::B(im_a + tt * WI::U, lane), accW2[tt]);
    const typename WI::TB tx = WI::B(im_x, lane);
#endif
    const int cl = c - cbase;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
#if MF_WG_EARLY_READS
      const typename WI::TA tgz = WI::A(rgz[tt]);
#else
      const typename WI::TA tgz = WI::A(im_gz + tt * WI::U, lane);
#endif
#if MF_WG_EARLY_READS && MF_WG4
      accW1[tt] = WI::mma4(tgz, tx, accW1[tt]);
#else
      accW1[tt] = WI::mma(tgz, tx, accW1[tt]);
#endif
      const floatx4 cs = WI::colsum(tgz, gz[tt], ones);
      if (j16 == WI::CS_LANE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = GM<H>::mrow(tt, 4 * g4 + r);
          if (h >= 0) colbuf[(cl * 4 + wave) * H + h] = cs[r];
        }
      }
    }
    if (cl == COL_CH - 1 || c == c1 - 1) {
      __syncthreads();
      col_flush<H>(colbuf, cl + 1, cbase, partCol, colbase);
      __syncthreads();
      cbase = c + 1;
    }
  };
  // (the pipeline's second head fits the register file at Fdim <= 10 on the
  // split-bf16 gradient paths; the fp32 and single-bf16 forms would spill or
  // lose a wave)
  if constexpr (MF_BWD_PIPE && F <= 10 && PREC != 0 && PREC != 2 && (PREC != 4 || MF_BWD_PIPE6))
    class_stream_pipe<MF_DEPTH_BWD>(c0, c1, load, head, tail);
  else
    class_stream<MF_DEPTH_BWD>(c0, c1, load, [&](const Rows<3>& rows, int c) { tail(head(rows, c), c); });
  if (fvalid) {
    float* dst = GzEs + (size_t)ks * H * NS + n;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int r = 0; r < GM<H>::nreg(tt); ++r) {
        const int h = GM<H>::row(g4, 4 * tt + r);
        if (h >= 0) dst[(size_t)h * NS] = accF[tt][r];
      }
  }
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

// Instantiations: Fdim 8, 10, 16 for the fp32 / bf16x3 precisions (PREC 0, 1);
// the single-bf16 path (PREC 2) at Fdim 10.
#define MF_CASE(FF, PP, K, ...)                                                   \
  case FF * 8 + PP: {                                                             \
    hipLaunchKernelGGL((K<FF, PP>), dim3(edge_grid(geo)), dim3(256), 0, st, geo,    \
                       __VA_ARGS__);                                              \
  } break;
#define MF_LAUNCH(F, P, K, ...)                                                   \
  switch ((F) * 8 + (P)) {                                                        \
    MF_CASE(8, 0, K, __VA_ARGS__) MF_CASE(8, 1, K, __VA_ARGS__)                  \
    MF_CASE(10, 0, K, __VA_ARGS__) MF_CASE(10, 1, K, __VA_ARGS__)                \
    MF_CASE(10, 2, K, __VA_ARGS__) MF_CASE(10, 3, K, __VA_ARGS__)                \
    MF_CASE(10, 4, K, __VA_ARGS__)                                                \
    MF_CASE(16, 0, K, __VA_ARGS__) MF_CASE(16, 1, K, __VA_ARGS__)                \
    default: return pf::fail("pfsgnn mfma", "unsupported Fdim for this edge path"); \
  }

// kernels with a third template flag (TM: the TModel mask is read, not recomputed)
#define MF_CASE3(FF, PP, TT, K, ...)                                              \
  case FF * 8 + PP: {                                                             \
    hipLaunchKernelGGL((K<FF, PP, TT>), dim3(edge_grid(geo)), dim3(256), 0, st, geo, \
                       __VA_ARGS__);                                              \
  } break;
#define MF_LAUNCH3(F, P, TT, K, ...)                                              \
  switch ((F) * 8 + (P)) {                                                        \
    MF_CASE3(8, 0, TT, K, __VA_ARGS__) MF_CASE3(8, 1, TT, K, __VA_ARGS__)        \
    MF_CASE3(10, 0, TT, K, __VA_ARGS__) MF_CASE3(10, 1, TT, K, __VA_ARGS__)      \
    MF_CASE3(10, 2, TT, K, __VA_ARGS__) MF_CASE3(10, 3, TT, K, __VA_ARGS__)      \
    MF_CASE3(10, 4, TT, K, __VA_ARGS__)                                           \
    MF_CASE3(16, 0, TT, K, __VA_ARGS__) MF_CASE3(16, 1, TT, K, __VA_ARGS__)      \
    default: return pf::fail("pfsgnn mfma", "unsupported Fdim for this edge path"); \
  }

// MF_PART: the library builds this file twice (Makefile) so that the MFMA
// helper's MF_SRC_KEEP scheduling tie can differ per kernel: part 1 = every
// launcher but edge_mlp_bwd's (MF_SRC_KEEP=0), part 2 = edge_mlp_bwd's alone
// (MF_SRC_KEEP=1: without the tie it runs 2.38 -> 2.61 ms per step, while the
// other kernels run faster without it; profiles/r06n_ab.txt, r06r_keep_ab.txt).
// A kernel is instantiated only by its launcher, so each object holds its own.
// MF_PART 0 (a plain compile) = both.
#ifndef MF_PART
#define MF_PART 0
#endif
namespace pfm {
#if MF_PART != 2

// forward kernels only distinguish fp32 (0, 1), single bf16 (2) and bf16x3 (3)
static inline int fwd_prec(int prec) { return FP(prec); }

int edge_mlp_fwd(const EdgeGeo& geo, int F, const float* xe, const float* xsc, const float* xsh,
                 const float* Ps, const float* PtS, const float* W1, const float* W2,
                 const float* b2, float* y, float* part, const MomFin& fin, int prec, int bfy,
                 hipStream_t st) {
  if (fin.cnt && (geo.nblocks > MOM_GROUP * MOM_MAXG || F > 16))
    return pf::fail("pfsgnn mfma", "edge_mlp_fwd: in-launch finalize needs <= 4096 blocks");
  MF_LAUNCH(F, fwd_prec(prec), km_edge_mlp_fwd, xe, xsc, xsh, Ps, PtS, W1, W2, b2, y, part, bfy,
            fin)
  return 0;
}

int source_fwd(const EdgeGeo& geo, int F, const float* y, const float* sc, const float* sh,
               const float* QtS, const float* Ws1, const float* Ws2, const float* bs2,
               float* partS, int prec, hipStream_t st) {
  MF_LAUNCH(F, fwd_prec(prec), km_source_fwd, y, sc, sh, QtS, Ws1, Ws2, bs2, partS)
  return 0;
}

int source_fwd_tiles(const EdgeGeo& geo, int F, const float* y, const float* sc,
                     const float* sh, const float* QtS, const float* Ws1, const float* Ws2,
                     const float* bs2, float* mom, float* hs, float* msg, int prec, int wave_nc,
                     hipStream_t st) {
  if (geo.NC > MF_SFT_MAXNC) return pf::fail("pfsgnn mfma", "source_fwd_tiles: NC > 256");
  const bool wf = geo.NC <= std::min(wave_nc, MF_SFT_WAVE_MAXNC);
  const int TF = wf ? 64 : 16;
  const int ntiles = geo.G * ((geo.NF + TF - 1) / TF);
  const int nb = 8 * ((ntiles + 7) / 8);
  const size_t lds = sft_lds_floats(geo.NC, F) * sizeof(float);
#define MF_SFT(FF, PP)                                                                     \
  case FF * 8 + PP:                                                                        \
    if (wf)                                                                                \
      hipLaunchKernelGGL((km_source_fwd_ft<FF, PP, true>), dim3(nb), dim3(256), lds, st, geo, \
                         ntiles, y, sc, sh, QtS, Ws1, Ws2, bs2, mom, hs, msg);             \
    else                                                                                   \
      hipLaunchKernelGGL((km_source_fwd_ft<FF, PP, false>), dim3(nb), dim3(256), lds, st, geo, \
                         ntiles, y, sc, sh, QtS, Ws1, Ws2, bs2, mom, hs, msg);             \
    break;
  switch (F * 8 + fwd_prec(prec)) {
    MF_SFT(8, 0) MF_SFT(8, 1) MF_SFT(10, 0) MF_SFT(10, 1) MF_SFT(10, 2) MF_SFT(10, 3)
    MF_SFT(10, 4) MF_SFT(16, 0) MF_SFT(16, 1)
    default: return pf::fail("pfsgnn mfma", "unsupported Fdim for this edge path");
  }
#undef MF_SFT
  return 0;
}

int target_fwd(const EdgeGeo& geo, int F, const float* y, const float* sc, const float* sh,
               const float* Rs, const float* Wt1, float* part, uint8_t* tmask, int prec,
               hipStream_t st) {
  MF_LAUNCH(F, fwd_prec(prec), km_target_fwd, y, sc, sh, Rs, Wt1, part, tmask)
  return 0;
}

int target_bwd(const EdgeGeo& geo, int F, const float* y, const float* sc, const float* sh,
               const float* Rs, const float* Wt1, const float* ghS, float* gz, float* gxe,
               float* part, const uint8_t* tmask, int prec, hipStream_t st) {
  if (tmask) {
    MF_LAUNCH3(F, prec, true, km_target_bwd, y, sc, sh, Rs, Wt1, ghS, gz, gxe, part, tmask)
  } else {
    MF_LAUNCH3(F, prec, false, km_target_bwd, y, sc, sh, Rs, Wt1, ghS, gz, gxe, part, tmask)
  }
  return 0;
}

int source_bwd(const EdgeGeo& geo, int F, const float* msg, const float* y, const float* sc,
               const float* sh, const float* QtS, const float* Ws1, const float* Ws2,
               const float* bs2, const float* mean, const float* coef, const float* Rs,
               const float* Wt1, const float* ghS, const float* g_next, const float* mu1,
               const float* inv1, float* g_tot, float* pW2, float* pW1, float* pCol, float* pBN,
               const uint8_t* tmask, int prec, hipStream_t st) {
  if (msg) {   // the message cache: Fdim 8 / 10 / 16 on the mfma / mfma32 paths
    if (prec != 0 && prec != 1) return pf::fail("pfsgnn mfma", "message cache: mfma paths only");
#define MF_CASE_MSG(FF, PP, TT)                                                                  \
  case FF * 8 + PP:                                                                             \
    hipLaunchKernelGGL((km_source_bwd<FF, PP, TT, true>), dim3(edge_grid(geo)), dim3(256), 0, st, \
                       geo, msg, y, sc, sh, QtS, Ws1, Ws2, bs2, mean, coef, Rs, Wt1, ghS, g_next, \
                       mu1, inv1, g_tot, pW2, pW1, pCol, pBN, tmask);                           \
    break;
    if (tmask && Rs) {
      switch (F * 8 + prec) {
        MF_CASE_MSG(8, 0, true) MF_CASE_MSG(8, 1, true) MF_CASE_MSG(10, 0, true)
        MF_CASE_MSG(10, 1, true) MF_CASE_MSG(16, 0, true) MF_CASE_MSG(16, 1, true)
        default: return pf::fail("pfsgnn mfma", "unsupported Fdim for this edge path");
      }
    } else {
      switch (F * 8 + prec) {
        MF_CASE_MSG(8, 0, false) MF_CASE_MSG(8, 1, false) MF_CASE_MSG(10, 0, false)
        MF_CASE_MSG(10, 1, false) MF_CASE_MSG(16, 0, false) MF_CASE_MSG(16, 1, false)
        default: return pf::fail("pfsgnn mfma", "unsupported Fdim for this edge path");
      }
    }
#undef MF_CASE_MSG
    return 0;
  }
  if (tmask && Rs) {
    MF_LAUNCH3(F, prec, true, km_source_bwd, nullptr, y, sc, sh, QtS, Ws1, Ws2, bs2, mean, coef, Rs, Wt1,
               ghS, g_next, mu1, inv1, g_tot, pW2, pW1, pCol, pBN, tmask)
  } else {
    MF_LAUNCH3(F, prec, false, km_source_bwd, nullptr, y, sc, sh, QtS, Ws1, Ws2, bs2, mean, coef, Rs, Wt1,
               ghS, g_next, mu1, inv1, g_tot, pW2, pW1, pCol, pBN, tmask)
  }
  return 0;
}

#endif  // MF_PART != 2
#if MF_PART != 1
int edge_mlp_bwd(const EdgeGeo& geo, int F, const float* g_tot, const float* alpha,
                 const float* gam0, const float* gam1, const float* y, const float* xe,
                 const float* xsc, const float* xsh, const float* Ps, const float* PtS,
                 const float* W1, const float* W2, float* gxe, float* gs, float* pW2, float* pW1,
                 float* pCol, int prec, hipStream_t st) {
  MF_LAUNCH(F, prec, km_edge_mlp_bwd, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, PtS, W1, W2,
            gxe, gs, pW2, pW1, pCol)
  return 0;
}
#endif  // MF_PART != 1

}  // namespace pfm
