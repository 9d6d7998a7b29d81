// pfsgnn_mfma_core.h -- the MFMA building blocks shared by the per-edge kernels
// of complete graphs (pfsgnn_mfma.hip) and of sliced general graphs
// (pfsgnn_sliced.hip): row maps, the fp32 / bf16x3 / bf16x6 / bf16 layers,
// weight-gradient images, edge-row loads and stores, class-row staging,
// column sums and the class stream.  The tile geometry they assume is
// described at the top of pfsgnn_mfma.hip.
#pragma once
#include "pfsgnn_mfma.h"

#include <type_traits>

#ifndef MF_DEPTH_FWD
#define MF_DEPTH_FWD 3   // classes of edge rows in flight per wave (forward kernels; 4 measured the same or slower with six waves of edge_mlp_fwd, r05aj)
#endif
#ifndef MF_DEPTH_BWD
#define MF_DEPTH_BWD 2   // (backward kernels: more arrays per class, more registers)
#endif
#ifndef MF_BWD_PIPE
#define MF_BWD_PIPE 1    // edge_mlp_bwd: the next class's head before this class's tail (class_stream_pipe)
#endif

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 b16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ floatx4 zero4() { return floatx4{0.f, 0.f, 0.f, 0.f}; }

// ------------------------------------------------------------ row maps
template <int D>
struct GM {
  static constexpr int RPG = (D + 3) / 4;       // rows per lane group
  static constexpr int NT = (RPG + 3) / 4;      // floatx4 tiles per lane
  // live registers of tile t
  static constexpr int nreg(int t) { return RPG - 4 * t < 4 ? RPG - 4 * t : 4; }
  // feature row of slot s in lane group g (-1: padding)
  static __device__ __forceinline__ int row(int g, int s) {
    const int h = g * RPG + s;
    return (s < RPG && h < D) ? h : -1;
  }
  // feature row of MFMA row index i (= 4g + r) of tile t
  static __device__ __forceinline__ int mrow(int t, int i) { return row(i >> 2, 4 * t + (i & 3)); }
};

// ------------------------------------------------------------ fp32 MFMA layer
// y (+)= W x for a W of M x K rows (fn(out_row, in_row) gives the weight), on
// v_mfma_f32_16x16x4_f32.  Lane (g, i) holds the A value of output row
// mrow(t, i) and input row g*RPG_K + s of K-step s.  Long chains are split over
// two accumulators (even / odd K-steps) to hide the 40-cycle MFMA latency.
template <int M, int K>
struct LayerF {
  static constexpr int MT = GM<M>::NT, KS = GM<K>::RPG;
  float a[MT][KS];
  template <class Fn>
  __device__ __forceinline__ void load(Fn fn, int lane) {
    const int g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int ro = GM<M>::mrow(t, i), ri = GM<K>::row(g, s);
        a[t][s] = (ro >= 0 && ri >= 0) ? fn(ro, ri) : 0.f;
      }
  }
  __device__ __forceinline__ void apply(const floatx4 (&x)[GM<K>::NT], floatx4 (&y)[MT]) const {
    // one output tile: a lone dependent chain unless split; several tiles
    // interleave their chains already
    if constexpr (KS >= 6 || (MT == 1 && KS >= 4)) {
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        floatx4 e = y[t], o = zero4();
#pragma unroll
        for (int s = 0; s < KS; s += 2) {
          e = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][s], x[s >> 2][s & 3], e, 0, 0, 0);
          if (s + 1 < KS)
            o = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][s + 1], x[(s + 1) >> 2][(s + 1) & 3], o,
                                                     0, 0, 0);
        }
        y[t] = e + o;
      }
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int t = 0; t < MT; ++t)
          y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][s], x[s >> 2][s & 3], y[t], 0, 0, 0);
    }
  }
};

// ------------------------------------------------------------ bf16x3 (wgrad)
struct Fr {
  s16x4 h, l;
};
__device__ __forceinline__ float bf_f(short s) {
  return __builtin_bit_cast(float, ((uint32_t)(uint16_t)s) << 16);
}
// bf16_rne of four values (v_cvt_pk_bf16_f32)
__device__ __forceinline__ s16x4 hi4(const floatx4& v) {
  const b16x4 h = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  return __builtin_bit_cast(s16x4, h);
}
// v = hi + lo (+ ~2^-17 |v|): hi = bf16_rne(v), lo = bf16_rne(v - hi)
__device__ __forceinline__ Fr split(const floatx4& v) {
  const b16x4 h = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  const s16x4 hs = __builtin_bit_cast(s16x4, h);
  const b16x4 l = {(__bf16)(v[0] - bf_f(hs[0])), (__bf16)(v[1] - bf_f(hs[1])),
                   (__bf16)(v[2] - bf_f(hs[2])), (__bf16)(v[3] - bf_f(hs[3]))};
  return {hs, __builtin_bit_cast(s16x4, l)};
}
// the 16x16x32 form: lane (g, i) holds A[i][k = 8g + q], B[k = 8g + q][i], q = 0..7;
// element q of an 8-wide operand is slot q & 3 of half q >> 2, and a product
// sums over every (lane group, element) position, so two 4-slot halves (two
// K-tiles, or the hi and lo planes of one) concatenate into one operand as
// long as A and B put matching halves in the same place
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));
struct Fr8 {
  s16x8 h, l;
};
__device__ __forceinline__ s16x8 cat8(s16x4 a, s16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ Fr8 cat(const Fr& a, const Fr& b) { return {cat8(a.h, b.h), cat8(a.l, b.l)}; }
// MF_SRC_KEEP: an empty asm after every split-bf16 MFMA reads its result and its
// A / B operands -- a scheduling choice: without it edge_mlp_bwd runs 2.38 ->
// 2.61 ms per step, the other kernels slightly faster (profiles/r06n_ab.txt),
// so the library builds edge_mlp_bwd with it and the rest of pfsgnn_mfma.hip
// without (MF_PART there, the Makefile).  Rounds 5-6 kept it for
// reproducibility: the SModel forward (km_source_fwd_ft) gave run-to-run
// different M3 / M4 without it.  That race followed the per-block LDS table of
// Pebay coefficients, not the MFMAs: only M3 / M4 of two channels (lane group 3,
// the low halves of packed-fp32 pairs) moved, S1 / S2 stayed bitwise; wait
// states behind every MFMA made it worse, while the table's coefficients from
// VALU, from scalar loads (c_peb below), or no packed-fp32 FMAs at all
// (-fno-slp-vectorize) each made every probe exact, MF_SRC_KEEP on or off
// (profiles/r06m_race_bisect.txt, r06n_opdet.txt).  The table is now c_peb.
// MF_SRC_PIN (A/B): also pass B (1) / A (2) through an opaque asm before the
// MFMA so that no result is allocated over an operand at all: 1.7 % slower
// step (profiles/r05d_pin_ab.txt).
#ifndef MF_SRC_KEEP
#define MF_SRC_KEEP 1
#endif
#ifndef MF_SRC_PIN
#define MF_SRC_PIN 0
#endif
__device__ __forceinline__ floatx4 mf8(s16x8 a, s16x8 b, floatx4 c) {
#if MF_SRC_KEEP && (MF_SRC_PIN & 1)
  asm volatile("" : "+v"(b));   // B as an opaque value: not rebuilt from its halves for the keep
#endif
#if MF_SRC_KEEP && (MF_SRC_PIN & 2)
  asm volatile("" : "+v"(a));
#endif
  floatx4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b16x8, a),
                                                      __builtin_bit_cast(b16x8, b), c, 0, 0, 0);
#if MF_SRC_KEEP
  asm volatile("" : "+v"(d) : "v"(a), "v"(b));
#endif
  return d;
}
__device__ __forceinline__ floatx4 mma3w(const Fr8& a, const Fr8& b, floatx4 c) {
  c = mf8(a.l, b.h, c);
  c = mf8(a.h, b.l, c);
  return mf8(a.h, b.h, c);
}
// ------------------------------------------------------------ bf16x3 layer
// y (+)= W x with split operands (W = Wh + Wl, x = xh + xl, products
// Wh xh + Wh xl + Wl xh, ~2^-16 relative each, fp32 accumulation) on
// v_mfma_f32_16x16x32_bf16: the backward's gradient chains (PREC 1), and every
// per-edge contraction, forward and recompute included (PREC 3).  K-step u of
// a 16-deep bf16 operand takes the 4 slots 4u..4u+3 of every lane group, so a
// D-row input is GM<D>::NT K-tiles (10 -> 1, 20 -> 2, 40 -> 3) where the fp32
// form takes GM<D>::RPG steps (3, 5, 10).  The 3 partial products of a K-tile
// are 3 halves of a 16x16x32 MFMA (twice the K of 16x16x16 in the same cycles:
// tools/mfma_cycles.hip); they are packed so that KT K-tiles cost
// ceil(3 KT / 2) MFMAs:
//   * a pair of K-tiles (2p, 2p+1): A = [Wh_2p | Wh_2p+1] and [Wl_2p | Wl_2p+1]
//     against B = [xh | xh] and [xl | xl]: 3 MFMAs for 6 halves;
//   * an odd last K-tile u: A = [Wh_u | Wl_u] against B = [xl_u | xh_u]
//     (Wh xl + Wl xh) and against [xh_u | 0] (Wh xh): 2 MFMAs for 3 halves.
// Every MFMA of a chain is the one 16x16x32 form (DESIGN.md §MFMA form mixing).
template <int M, int K>
struct LayerB3 {
  static constexpr int MT = GM<M>::NT, KT = GM<K>::NT, KP = KT / 2;
  static constexpr bool ODD = (KT & 1) != 0;
  Fr8 ap[MT][KP > 0 ? KP : 1];   // K-tile pairs
  s16x8 ao[MT];                  // odd last K-tile: [Wh | Wl]
  template <class Fn>
  __device__ __forceinline__ void load(Fn fn, int lane) {
    const int g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      Fr a[KT];
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        floatx4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ro = GM<M>::mrow(t, i), ri = GM<K>::row(g, 4 * u + j);
          v[j] = (ro >= 0 && ri >= 0) ? fn(ro, ri) : 0.f;
        }
        a[u] = split(v);
      }
#pragma unroll
      for (int p = 0; p < KP; ++p) ap[t][p] = cat(a[2 * p], a[2 * p + 1]);
      if constexpr (ODD) ao[t] = cat8(a[KT - 1].h, a[KT - 1].l);
    }
  }
  __device__ __forceinline__ void apply(const Fr (&x)[KT], floatx4 (&y)[MT]) const {
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      const Fr8 xp = cat(x[2 * p], x[2 * p + 1]);
#pragma unroll
      for (int t = 0; t < MT; ++t) y[t] = mma3w(ap[t][p], xp, y[t]);
    }
    if constexpr (ODD) {
      const s16x8 xlh = cat8(x[KT - 1].l, x[KT - 1].h), xh0 = cat8(x[KT - 1].h, s16x4{});
#pragma unroll
      for (int t = 0; t < MT; ++t) y[t] = mf8(ao[t], xh0, mf8(ao[t], xlh, y[t]));
    }
  }
  // fp32 input tiles, split here (PREC 3 forward / recompute)
  __device__ __forceinline__ void apply(const floatx4 (&x)[KT], floatx4 (&y)[MT]) const {
    Fr s[KT];
#pragma unroll
    for (int u = 0; u < KT; ++u) s[u] = split(x[u]);
    apply(s, y);
  }
};

// The same bf16x3 layer with its split weight operands staged in LDS instead
// of held in registers (per lane, in the register form's order: the pairs'
// [Wh | Wh'] and [Wl | Wl'], then an odd last K-tile's [Wh | Wl]; one
// ds_read_b128 per MFMA operand): frees 4 VGPRs per operand for a kernel
// whose registers are the limit.  bind() gives the LDS block; load() is
// executed by every wave, wave 0 writes (the kernel's __syncthreads after its
// staging publishes them).
template <int M, int K>
struct LayerB3S {
  static constexpr int MT = GM<M>::NT, KT = GM<K>::NT, KP = KT / 2;
  static constexpr bool ODD = (KT & 1) != 0;
  static constexpr int NOP = MT * (2 * KP + (ODD ? 1 : 0));   // s16x8 operands per lane
  const s16x8* w = nullptr;
  s16x8* base = nullptr;
  __device__ __forceinline__ void bind(s16x8* lds) { base = lds; }
  static __device__ __forceinline__ int op(int t, int k) { return t * (2 * KP + (ODD ? 1 : 0)) + k; }
  template <class Fn>
  __device__ __forceinline__ void load(Fn fn, int lane) {
    w = base + lane;
    if ((threadIdx.x >> 6) != 0) return;
    LayerB3<M, K> r;
    r.load(fn, lane);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
#pragma unroll
      for (int p = 0; p < KP; ++p) {
        base[op(t, 2 * p) * 64 + lane] = r.ap[t][p].h;
        base[op(t, 2 * p + 1) * 64 + lane] = r.ap[t][p].l;
      }
      if constexpr (ODD) base[op(t, 2 * KP) * 64 + lane] = r.ao[t];
    }
  }
  __device__ __forceinline__ void apply(const Fr (&x)[KT], floatx4 (&y)[MT]) const {
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      const Fr8 xp = cat(x[2 * p], x[2 * p + 1]);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const Fr8 a = {w[op(t, 2 * p) * 64], w[op(t, 2 * p + 1) * 64]};
        y[t] = mma3w(a, xp, y[t]);
      }
    }
    if constexpr (ODD) {
      const s16x8 xlh = cat8(x[KT - 1].l, x[KT - 1].h), xh0 = cat8(x[KT - 1].h, s16x4{});
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const s16x8 a = w[op(t, 2 * KP) * 64];
        y[t] = mf8(a, xh0, mf8(a, xlh, y[t]));
      }
    }
  }
};

// ------------------------------------------------------------ bf16x6 layer
// y (+)= W x with three-way split operands v = vh + vm + vl (each bf16 RNE,
// |v - vh - vm - vl| <= ~2^-27 |v|) and the six products whose order is at most
// 2^-18: Wh xh, Wh xm, Wm xh, Wh xl, Wl xh, Wm xm -- the dropped ones are
// <= ~2^-26 relative, so a product is as exact as fp32's own rounding and the
// contraction has the numerics of an fp32 one (PREC 4: the forward
// contractions and their recompute).  Per K-tile three v_mfma_f32_16x16x32_bf16,
// small terms first: [Wh | Wm].[xl | xm] (hl + mm), [Wh | Wl].[xm | xh]
// (hm + lh), [Wh | Wm].[xh | xh] (hh + mh): 48 cycles per 16 K-slots where
// v_mfma_f32_16x16x4_f32 takes 128.
struct Fr3 {
  s16x4 h, m, l;
};
__device__ __forceinline__ Fr3 split3(const floatx4& v) {
  const s16x4 h = hi4(v);
  floatx4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = v[j] - bf_f(h[j]);
  const s16x4 m = hi4(r);
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = r[j] - bf_f(m[j]);
  return {h, m, hi4(r)};
}
template <int M, int K>
struct LayerB6 {
  static constexpr int MT = GM<M>::NT, KT = GM<K>::NT;
  s16x8 ahm[MT][KT], ahl[MT][KT];   // [Wh | Wm], [Wh | Wl]
  template <class Fn>
  __device__ __forceinline__ void load(Fn fn, int lane) {
    const int g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        floatx4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ro = GM<M>::mrow(t, i), ri = GM<K>::row(g, 4 * u + j);
          v[j] = (ro >= 0 && ri >= 0) ? fn(ro, ri) : 0.f;
        }
        const Fr3 a = split3(v);
        ahm[t][u] = cat8(a.h, a.m);
        ahl[t][u] = cat8(a.h, a.l);
      }
  }
  __device__ __forceinline__ void apply(const Fr3 (&x)[KT], floatx4 (&y)[MT]) const {
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const s16x8 b1 = cat8(x[u].l, x[u].m), b2 = cat8(x[u].m, x[u].h), b3 = cat8(x[u].h, x[u].h);
#pragma unroll
      for (int t = 0; t < MT; ++t) y[t] = mf8(ahm[t][u], b3, mf8(ahl[t][u], b2, mf8(ahm[t][u], b1, y[t])));
    }
  }
  __device__ __forceinline__ void apply(const floatx4 (&x)[KT], floatx4 (&y)[MT]) const {
    Fr3 s[KT];
#pragma unroll
    for (int u = 0; u < KT; ++u) s[u] = split3(x[u]);
    apply(s, y);
  }
};

// The same bf16x6 layer with its weight tuples staged in LDS instead of held
// in registers: [2 (t * KT + u) + {0: Wh|Wm, 1: Wh|Wl}][64 lanes] x 16 bytes, one
// conflict-free ds_read_b128 per MFMA operand.  For a backward kernel's
// recompute whose registers are already full (km_source_bwd at PREC 4: the
// register-resident tuples cost 32 more VGPRs and spill), so that the recompute
// runs exactly the forward kernel's arithmetic -- same operands, same MFMA
// order, bitwise the same messages.  bind() gives the LDS block; load() is
// executed by every wave, wave 0 writes (the kernel's __syncthreads after its
// staging publishes the tuples).  The reads sit behind the loop's lds_order()
// points, so the compiler cannot hoist them back into registers.
template <int M, int K>
struct LayerB6S {
  static constexpr int MT = GM<M>::NT, KT = GM<K>::NT, NOP = 2 * MT * KT;
  const s16x8* w = nullptr;   // this lane's operand 0; operand o at w[64 o]
  s16x8* base = nullptr;
  __device__ __forceinline__ void bind(s16x8* lds) { base = lds; }
  template <class Fn>
  __device__ __forceinline__ void load(Fn fn, int lane) {
    w = base + lane;
    if ((threadIdx.x >> 6) != 0) return;
    const int g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        floatx4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ro = GM<M>::mrow(t, i), ri = GM<K>::row(g, 4 * u + j);
          v[j] = (ro >= 0 && ri >= 0) ? fn(ro, ri) : 0.f;
        }
        const Fr3 a = split3(v);
        base[(2 * (t * KT + u)) * 64 + lane] = cat8(a.h, a.m);
        base[(2 * (t * KT + u) + 1) * 64 + lane] = cat8(a.h, a.l);
      }
  }
  __device__ __forceinline__ void apply(const Fr3 (&x)[KT], floatx4 (&y)[MT]) const {
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const s16x8 b1 = cat8(x[u].l, x[u].m), b2 = cat8(x[u].m, x[u].h), b3 = cat8(x[u].h, x[u].h);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const s16x8 ahm = w[(2 * (t * KT + u)) * 64], ahl = w[(2 * (t * KT + u) + 1) * 64];
        y[t] = mf8(ahm, b3, mf8(ahl, b2, mf8(ahm, b1, y[t])));
      }
    }
  }
  __device__ __forceinline__ void apply(const floatx4 (&x)[KT], floatx4 (&y)[MT]) const {
    Fr3 s[KT];
#pragma unroll
    for (int u = 0; u < KT; ++u) s[u] = split3(x[u]);
    apply(s, y);
  }
};

// ------------------------------------------------------------ weight gradients
// acc += A B^T summed over a tile's 16 edges (edge = MFMA K), A and B read from
// wave-private bf16 images (hi and lo planes), as 2 v_mfma_f32_16x16x32_bf16:
// [Ah | Al] . [Bl | Bh] (Ah Bl + Al Bh) and [Ah | Al] . [Bh | 0] (Ah Bh).
// The A tuple [Ah | Al] against ones gives A's sums over the 16 edges (hi + lo).
__device__ __forceinline__ s16x8 ones8() {
  const short o = (short)0x3F80;
  return s16x8{o, o, o, o, o, o, o, o};
}
// ones8() as an opaque register value: made once, kept in its 4 VGPRs
__device__ __forceinline__ s16x8 ones_reg() {
  s16x8 o = ones8();
  asm volatile("" : "+v"(o));
  return o;
}
struct WgB {
  s16x8 lh, h0;   // [Bl | Bh], [Bh | 0]
};
__device__ __forceinline__ floatx4 mma3g(s16x8 a_hl, const WgB& b, floatx4 c) {
  return mf8(a_hl, b.h0, mf8(a_hl, b.lh, c));
}

// ------------------------------------------------------------ bf16 layer
// y (+)= W x with every product a single v_mfma_f32_16x16x16_bf16 on bf16
// operands (RNE), fp32 accumulation: the "bf16" edge path
// (PFSGNN_EDGE_BF16) -- one MFMA per K-tile where LayerF issues GM<K>::RPG.
template <int M, int K>
struct LayerB1 {
  static constexpr int MT = GM<M>::NT, KT = GM<K>::NT, KP = (KT + 1) / 2;
  // K-tile pairs on v_mfma_f32_16x16x32_bf16, an odd last K-tile paired with zeros
  s16x8 ap[MT][KP];
  template <class Fn>
  __device__ __forceinline__ void load(Fn fn, int lane) {
    const int g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      s16x4 a[KT];
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        floatx4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ro = GM<M>::mrow(t, i), ri = GM<K>::row(g, 4 * u + j);
          v[j] = (ro >= 0 && ri >= 0) ? fn(ro, ri) : 0.f;
        }
        a[u] = hi4(v);
      }
#pragma unroll
      for (int p = 0; p < KP; ++p) ap[t][p] = cat8(a[2 * p], 2 * p + 1 < KT ? a[2 * p + 1] : s16x4{});
    }
  }
  __device__ __forceinline__ void apply(const Fr (&x)[KT], floatx4 (&y)[MT]) const {
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      const s16x8 xp = cat8(x[2 * p].h, 2 * p + 1 < KT ? x[2 * p + 1].h : s16x4{});
#pragma unroll
      for (int t = 0; t < MT; ++t) y[t] = mf8(ap[t][p], xp, y[t]);
    }
  }
  __device__ __forceinline__ void apply(const floatx4 (&x)[KT], floatx4 (&y)[MT]) const {
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      const s16x8 xp = cat8(hi4(x[2 * p]), 2 * p + 1 < KT ? hi4(x[2 * p + 1]) : s16x4{});
#pragma unroll
      for (int t = 0; t < MT; ++t) y[t] = mf8(ap[t][p], xp, y[t]);
    }
  }
};

// Precision of the per-edge contractions (PREC, per edge path):
//   0 exact fp32 everywhere (PFSGNN_EDGE_MFMA_F32, _BF16Y);
//   1 forward fp32, backward gradient chains bf16x3 (PFSGNN_EDGE_MFMA);
//   2 every contraction single bf16 (PFSGNN_EDGE_BF16);
//   3 every contraction bf16x3, forward and recompute included (PFSGNN_EDGE_BF16X3);
//   4 forward contractions and recompute bf16x6 (fp32-class), backward gradient
//     chains bf16x3 (PFSGNN_EDGE_BF16X6).
// The forward layers of a backward kernel (its recompute) use FwdLayer<FP(PREC)>,
// exactly the arithmetic of the forward kernel, so the recomputed activations
// and LeakyReLU masks are bitwise those of the forward pass.
__host__ __device__ constexpr int FP(int prec) { return prec >= 2 ? prec : 0; }
template <int PREC, int M, int K>
using FwdLayer = std::conditional_t<
    PREC == 2, LayerB1<M, K>,
    std::conditional_t<PREC == 3, LayerB3<M, K>,
                       std::conditional_t<PREC == 4, LayerB6<M, K>, LayerF<M, K>>>>;
// The recompute layers of source_bwd: the forward's arithmetic (FwdLayer<FP>),
// with the bf16x6 tuples staged in LDS (LayerB6S) -- held in registers they
// push that kernel past 256 VGPRs.  Round 3 ran this recompute in exact fp32
// instead; the moments' backward then combined forward statistics with
// messages of another rounding, which 1/std^3 and 1/std^4 amplify on fibers
// of nearly constant messages (22x the parity bar on a 24x16 graph).
template <int PREC, int M, int K>
using RecLayer = std::conditional_t<FP(PREC) == 4, LayerB6S<M, K>, FwdLayer<FP(PREC), M, K>>;
template <class L>
struct RecLds {   // s16x8 operands of L's LDS image (0: a register layer)
  static constexpr int n = 0;
};
template <int M, int K>
struct RecLds<LayerB6S<M, K>> {
  static constexpr int n = LayerB6S<M, K>::NOP * 64;
};
template <class L>
__device__ __forceinline__ void rec_bind(L&, s16x8*) {}
template <int M, int K>
__device__ __forceinline__ void rec_bind(LayerB6S<M, K>& l, s16x8* p) { l.bind(p); }
template <int PREC, int M, int K>
using GradLayer = std::conditional_t<
    PREC == 0, LayerF<M, K>, std::conditional_t<PREC == 2, LayerB1<M, K>, LayerB3<M, K>>>;

// Wave-private image of one 16x16 bf16 block, [16 edges][16 slots] (32-byte
// rows, the four 8-byte chunks of row e XOR-swizzled by e>>2: conflict-free b64
// writes and tr reads).  Lane (g, j) writes its slots 4g..4g+3 of edge j; a
// ds_read_b64_tr_b16 hands lane (g, i) the slot-i column of edges 4g..4g+3:
// an A operand A[slot][edge] or a B operand B[edge][slot], edge = MFMA K.
#define IMG_SHORTS 256
__device__ __forceinline__ void img_put(short* img, int lane, s16x4 v) {
  const int g = lane >> 4, j = lane & 15;
  *reinterpret_cast<s16x4*>(img + j * 16 + ((g ^ (j >> 2)) & 3) * 4) = v;
}
__device__ __forceinline__ s16x4 img_tr(const short* img, int lane) {
  const int ii = lane & 15, gq = lane >> 4;
  const int row = 4 * gq + (ii >> 2);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(img + row * 16 + (((ii & 3) ^ gq) & 3) * 4));
}
__device__ __forceinline__ void img_put2(short* img, int lane, const Fr& v) {
  img_put(img, lane, v.h);
  img_put(img + IMG_SHORTS, lane, v.l);
}
__device__ __forceinline__ Fr img_tr2(const short* img, int lane) {
  return {img_tr(img, lane), img_tr(img + IMG_SHORTS, lane)};
}
// weight-gradient operands from an image (mma3g): A side [hi | lo]; B side
// [lo | hi] and [hi | 0]
__device__ __forceinline__ s16x8 img_trA(const short* img, int lane) {
  return cat8(img_tr(img, lane), img_tr(img + IMG_SHORTS, lane));
}
__device__ __forceinline__ WgB img_trB(const short* img, int lane) {
  const s16x4 h = img_tr(img, lane);
  return {cat8(img_tr(img + IMG_SHORTS, lane), h), cat8(h, s16x4{})};
}
// compiler-only ordering point between a wave's image writes and its reads
// (one wave's LDS operations execute in order)
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

// ------------------------------------------------------------ fp32 weight gradients
// The exact-fp32 form of the weight-gradient outer products (PREC 0: the
// "mfma32" edge path): a wave-private fp32 image [16 slots][IMGF_STRIDE] of a
// tile, edge e of slot i at i * IMGF_STRIDE + 4 (e & 3) + (e >> 2), so that one
// ds_read_b128 hands lane (g, i) slot i of edges g, g + 4, g + 8, g + 12 --
// the A[i][k = g] / B[k = g][j = i] operands of the four
// v_mfma_f32_16x16x4_f32 K-steps over the tile's 16 edges (exact fp32
// products, fp32 accumulation).  Stride 20: conflict-free b128 reads, 2-way
// b32 writes.
#define IMGF_STRIDE 20
#define IMGF_FLOATS (16 * IMGF_STRIDE)
__device__ __forceinline__ void imgf_put(float* img, int lane, const floatx4& v) {
  const int g = lane >> 4, j = lane & 15;
  const int c = 4 * (j & 3) + (j >> 2);
#pragma unroll
  for (int r = 0; r < 4; ++r) img[(4 * g + r) * IMGF_STRIDE + c] = v[r];
}
__device__ __forceinline__ floatx4 imgf_tr(const float* img, int lane) {
  const int g = lane >> 4, i = lane & 15;
  return *reinterpret_cast<const floatx4*>(img + i * IMGF_STRIDE + 4 * g);
}
__device__ __forceinline__ floatx4 mmaf(const floatx4& a, const floatx4& b, floatx4 c) {
#pragma unroll
  for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], c, 0, 0, 0);
  return c;
}

// The weight-gradient images of a backward kernel by precision: bf16x3 (the
// hi / lo planes, mma3g; every path but PREC 0) or exact fp32 (PREC 0).
// U: shorts per image; put() takes the tile both as fp32 and as its split;
// A() / B(): the operands of mma(); colsum(): per-slot sums of a tile over its
// 16 edges (bf16x3: the A tuple against ones; fp32: DPP row sums in fp32),
// valid in lane CS_LANE of each lane group.
template <int PREC>
struct WgImg {
  static constexpr int U = 2 * IMG_SHORTS;
  static constexpr int CS_LANE = 0;
  using TA = s16x8;
  using TB = WgB;
  // rd(): the raw transposed read of an image (issued early, its LDS latency
  // hidden behind other work); A() / B() assemble the MFMA operands from it
  using R = Fr;
  static __device__ __forceinline__ R rd(const short* im, int lane) { return img_tr2(im, lane); }
  static __device__ __forceinline__ TA A(const R& r) { return cat8(r.h, r.l); }
  static __device__ __forceinline__ TB B(const R& r) { return {cat8(r.l, r.h), cat8(r.h, s16x4{})}; }
  static __device__ __forceinline__ void put(short* im, int lane, const floatx4&, const Fr& s) {
    img_put2(im, lane, s);
  }
  static __device__ __forceinline__ TA A(const short* im, int lane) { return img_trA(im, lane); }
  static __device__ __forceinline__ TB B(const short* im, int lane) { return img_trB(im, lane); }
  static __device__ __forceinline__ floatx4 mma(const TA& a, const TB& b, floatx4 c) {
    return mma3g(a, b, c);
  }
  // The four-product form (MF_WG4): B as [Bh | Bl] and [Bl | Bh], read from the
  // image twice (r, r2: the second pass behind an lds_order(), so that hipcc
  // keeps two loads instead of one load and register copies), against
  // A = [Ah | Al]: Ah Bh + Al Bl, then Ah Bl + Al Bh -- the exact product of the
  // split operands, with no [Bh | 0] operand to assemble (3 v_mov per B
  // operand and use in the three-product form).
  using TB4 = WgB;   // {lh = [Bl | Bh], h0 = [Bh | Bl]}
  static __device__ __forceinline__ TB4 B4(const R& r, const R& r2) {
    return {cat8(r2.l, r2.h), cat8(r.h, r.l)};
  }
  static __device__ __forceinline__ floatx4 mma4(const TA& a, const TB4& b, floatx4 c) {
    return mf8(a, b.h0, mf8(a, b.lh, c));
  }
  static __device__ __forceinline__ floatx4 colsum(const TA& a, const floatx4&) {
    return mf8(a, ones8(), zero4());
  }
  // the same with the ones operand held by the caller (ones_reg(), made once
  // before the class loop: hipcc otherwise rebuilds it with 3 v_mov per use)
  static __device__ __forceinline__ floatx4 colsum(const TA& a, const floatx4&, const s16x8& ones) {
    return mf8(a, ones, zero4());
  }
};
template <>
struct WgImg<0> {
  static constexpr int U = 2 * IMGF_FLOATS;
  static constexpr int CS_LANE = 15;
  using TA = floatx4;
  using TB = floatx4;
  using R = floatx4;
  static __device__ __forceinline__ R rd(const short* im, int lane) {
    return imgf_tr(reinterpret_cast<const float*>(im), lane);
  }
  static __device__ __forceinline__ TA A(const R& r) { return r; }
  static __device__ __forceinline__ TB B(const R& r) { return r; }
  static __device__ __forceinline__ void put(short* im, int lane, const floatx4& v, const Fr&) {
    imgf_put(reinterpret_cast<float*>(im), lane, v);
  }
  static __device__ __forceinline__ TA A(const short* im, int lane) {
    return imgf_tr(reinterpret_cast<const float*>(im), lane);
  }
  static __device__ __forceinline__ TB B(const short* im, int lane) { return A(im, lane); }
  static __device__ __forceinline__ floatx4 mma(const TA& a, const TB& b, floatx4 c) {
    return mmaf(a, b, c);
  }
  using TB4 = floatx4;
  static __device__ __forceinline__ TB4 B4(const R& r, const R&) { return r; }
  static __device__ __forceinline__ floatx4 mma4(const TA& a, const TB4& b, floatx4 c) {
    return mmaf(a, b, c);
  }
  static __device__ __forceinline__ floatx4 colsum(const TA&, const floatx4& v);
  static __device__ __forceinline__ floatx4 colsum(const TA& a, const floatx4& v, const s16x8&) {
    return colsum(a, v);
  }
};

// ------------------------------------------------------------ memory
__device__ __forceinline__ float ldE(const float* p, uint32_t off) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(p) + off);
}
__device__ __forceinline__ void stE(float* p, uint32_t off, float v) {
  *reinterpret_cast<float*>(reinterpret_cast<char*>(p) + off) = v;
}

// Per-lane byte offsets of the lane's F rows of a channel-major edge tensor
// at class 0 of its wave (slots with no feature point at row 0 again -- same
// 64-B segment -- and are masked later).  Every edge tensor of a kernel has
// the same geometry, so one set serves them all: a class's rows are then
// `(char*)p + c*eoc` (wave-uniform, scalar registers) + these offsets, a
// global_load with an SGPR base and no per-load address arithmetic.
template <int F>
struct RowOff {
  uint32_t o[GM<F>::RPG];
  __device__ __forceinline__ RowOff(uint32_t eo0, uint32_t RB, int g) {
#pragma unroll
    for (int r = 0; r < GM<F>::RPG; ++r) {
      const int k = GM<F>::row(g, r);
      o[r] = eo0 + (uint32_t)(k < 0 ? 0 : k) * RB;
    }
  }
};

// An edge tensor's rows of class c.  Loads: the tensor as a buffer resource,
// the lane's byte offset (RowOff) in the VGPR offset and the wave-uniform
// class offset c*eoc in the SGPR soffset -- buffer_load ... offen, no address
// arithmetic per row (an access past `bytes` reads 0).  Stores: the SGPR-base
// global form, (char*)p + c*eoc plus the 32-bit lane offset, which goes
// through an empty asm so that hipcc keeps it 32-bit at the access rather than
// hoisting a 64-bit copy.  (Round 3's buffer-store form stored one row's value
// to all of a lane's rows.  The cause is a hipcc defect in
// __builtin_bit_cast(unsigned int, v[r]) of a vector ELEMENT -- it reads
// element 0 for every r -- not the buffer stores: bit-cast a float copy of
// the element instead.  tests/test_bitcast_vector_element.py,
// tests/test_gpu_buffer_store.py; DESIGN.md §Edge-row stores.)
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                           0x00020000);
}
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}

// the lane's rows of an F-wide edge tensor at class byte offset co = c*eoc
template <int F>
__device__ __forceinline__ floatx4 ld_frows(Rsrc p, uint32_t co, const RowOff<F>& ro) {
  floatx4 v = zero4();
#pragma unroll
  for (int r = 0; r < GM<F>::RPG; ++r)
    v[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(p, ro.o[r], co, 0));
  return v;
}

// The lane's rows of an F-wide edge tensor of `bytes` bytes at class offset co:
// global stores under per-row exec masks (default), or (MF_BUF_STORE=1)
// branch-free buffer stores, a row the lane does not own (invalid fiber,
// padding slot) given a voffset past the buffer's range and dropped by the
// range check -- measured equal on the bench step (profiles/r04k_ab.txt;
// target_bwd 4 % slower), so not the default.  The buffer form passes the
// row's value through a float temporary before its bit-cast: hipcc's
// __builtin_bit_cast of a vector ELEMENT reads element 0 (DESIGN.md
// §Edge-row stores; tests/test_bitcast_vector_element.py).
#ifndef MF_BUF_STORE
#define MF_BUF_STORE 0
#endif
template <int F>
__device__ __forceinline__ void st_frows(float* p, uint32_t bytes, uint32_t co, const RowOff<F>& ro,
                                         int g, bool valid, const floatx4& v) {
#if MF_BUF_STORE
  const Rsrc rp = rsrc(p, bytes);
#pragma unroll
  for (int r = 0; r < GM<F>::RPG; ++r) {
    const int k = GM<F>::row(g, r);
    const float e = v[r];
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, e), rp,
                                          (valid && k >= 0) ? ro.o[r] : bytes, co, 0);
  }
#else
  (void)bytes;
  char* base = reinterpret_cast<char*>(p) + co;
#pragma unroll
  for (int r = 0; r < GM<F>::RPG; ++r) {
    const int k = GM<F>::row(g, r);
    if (valid && k >= 0) *reinterpret_cast<float*>(base + opaque(ro.o[r])) = v[r];
  }
#endif
}

// The lane's rows of a D-wide edge tensor (D > 16 allowed: GM<D>::NT tiles),
// loaded / stored at class byte offset co (the SModel message cache, msg:
// source_fwd stores the message, source_bwd loads it in place of recomputing
// the message MLP's second layer)
template <int D>
__device__ __forceinline__ void ld_rows_nt(Rsrc p, uint32_t co, const RowOff<D>& ro,
                                           floatx4 (&v)[GM<D>::NT]) {
#pragma unroll
  for (int t = 0; t < GM<D>::NT; ++t) {
    v[t] = zero4();
#pragma unroll
    for (int r = 0; r < GM<D>::nreg(t); ++r)
      v[t][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(p, ro.o[4 * t + r], co, 0));
  }
}
template <int D>
__device__ __forceinline__ void st_rows_nt(float* p, uint32_t co, const RowOff<D>& ro, int g,
                                           bool valid, const floatx4 (&v)[GM<D>::NT]) {
  char* base = reinterpret_cast<char*>(p) + co;
#pragma unroll
  for (int t = 0; t < GM<D>::NT; ++t)
#pragma unroll
    for (int r = 0; r < GM<D>::nreg(t); ++r) {
      const int k = GM<D>::row(g, 4 * t + r);
      if (valid && k >= 0) *reinterpret_cast<float*>(base + opaque(ro.o[4 * t + r])) = v[t][r];
    }
}

// per-feature constants of an F-wide block in the lane's slot order
template <int F>
__device__ __forceinline__ floatx4 ld_fconst(const float* p, int g, float dflt) {
  floatx4 v = zero4();
#pragma unroll
  for (int r = 0; r < GM<F>::RPG; ++r) {
    const int k = GM<F>::row(g, r);
    v[r] = (p && k >= 0) ? p[k] : dflt;
  }
  return v;
}

// per-fiber rows of tile t of a channel-major node tensor [D][NS]
template <int D>
__device__ __forceinline__ floatx4 ld_node(const float* p, int t, int g, long long NS,
                                           long long n, bool valid) {
  floatx4 v = zero4();
#pragma unroll
  for (int r = 0; r < GM<D>::nreg(t); ++r) {
    const int h = GM<D>::row(g, 4 * t + r);
    v[r] = (p && valid && h >= 0) ? p[(long long)h * NS + n] : 0.f;
  }
  return v;
}

// Pebay's count-only coefficients of the n-th folded message (n = k + 1), one
// 32-byte row per count -- A2 A3 A4 1/n | 6/n^2 -4/n -3/n 0 -- evaluated in
// double at compile time and rounded once (the values the SModel forward
// kernels used to build in LDS per block, bitwise).  The row index is
// wave-uniform, so a fold reads its row with one scalar load into SGPRs.
// MF_PEB_CONST=0 restores the per-block LDS table: read back with ds_read_b128
// into VGPRs that packed-fp32 FMAs then broadcast (op_sel_hi), that form gave
// run-to-run different M3 / M4 on gfx950 ("the source_fwd race").
#ifndef MF_PEB_CONST
#define MF_PEB_CONST 1
#endif
#define MF_PEB_ROWS 65
struct PebayTable {
  float v[MF_PEB_ROWS][8];
  constexpr PebayTable() : v{} {
    for (int t = 0; t < MF_PEB_ROWS; ++t) {
      const double nn = t + 1, r = 1.0 / nn;
      v[t][0] = (float)((nn - 1) * r);
      v[t][1] = (float)((nn - 1) * (nn - 2) * r * r);
      v[t][2] = (float)((nn - 1) * (nn * nn - 3 * nn + 3) * r * r * r);
      v[t][3] = (float)r;
      v[t][4] = (float)(6 * r * r);
      v[t][5] = (float)(-4 * r);
      v[t][6] = (float)(-3 * r);
      v[t][7] = 0.f;
    }
  }
};
__constant__ __attribute__((aligned(32))) static const PebayTable c_peb = PebayTable();

// The block's class rows [c0, c1) of a channel-major per-class node table
// [D][NT], staged once in LDS in the kernels' slot order (they are re-read for
// every tile of every wave): buf[cl][16t + 4g + r] = P[row(g, 4t + r)][cn0 + cl].
// MF_MAX_CPS bounds the class range of an MFMA block (pfm::MAX_CPS, geo_mfma).
#define MF_MAX_CPS 64
template <int D>
struct ClassRows {
  static constexpr int CP = 16 * GM<D>::NT;
  __device__ __forceinline__ static void stage(float* buf, const float* P, long long NT,
                                               long long cn0, int ncl) {
    for (int i = threadIdx.x; i < ncl * CP; i += PF_BLOCK) {
      const int cl = i / CP, q = i - cl * CP;
      const int h = GM<D>::row((q >> 2) & 3, 4 * (q >> 4) + (q & 3));
      buf[i] = h >= 0 ? P[(long long)h * NT + cn0 + cl] : 0.f;
    }
  }
  __device__ __forceinline__ static floatx4 get(const float* buf, int cl, int t, int g) {
    return *reinterpret_cast<const floatx4*>(buf + cl * CP + 16 * t + 4 * g);
  }
};

// constants of a D-wide vector (bias) in slot order
template <int D>
__device__ __forceinline__ floatx4 ld_vec(const float* p, int t, int g) {
  floatx4 v = zero4();
#pragma unroll
  for (int r = 0; r < GM<D>::nreg(t); ++r) {
    const int h = GM<D>::row(g, 4 * t + r);
    v[r] = (p && h >= 0) ? p[h] : 0.f;
  }
  return v;
}

// (the max(x, 0.1 x) form is no cheaper here: hipcc canonicalizes an MFMA
// result before a v_max_f32 in IEEE mode, 3 VALU either way)
__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : PF_LEAKY * x; }
__device__ __forceinline__ float dlrelu(float z) { return z > 0.f ? 1.f : PF_LEAKY; }
template <int D>
__device__ __forceinline__ void lrelu_act(const floatx4 (&z)[GM<D>::NT], floatx4 (&a)[GM<D>::NT]) {
#pragma unroll
  for (int t = 0; t < GM<D>::NT; ++t) {
    a[t] = zero4();
#pragma unroll
    for (int r = 0; r < GM<D>::nreg(t); ++r) a[t][r] = lrelu(z[t][r]);
  }
}

// ------------------------------------------------------------ column sums
template <int CTRL>
__device__ __forceinline__ float dpp0(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// sum over the 16 lanes of each DPP row (= lane group); the total lands in the
// row's lane 15 (row_shr 1, 2, 4, 8 with zero fill)
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp0<0x111>(v);
  v += dpp0<0x112>(v);
  v += dpp0<0x114>(v);
  v += dpp0<0x118>(v);
  return v;
}
// exact fp32 per-slot sums of a tile over its 16 edges (lane 15 of each group)
__device__ __forceinline__ floatx4 WgImg<0>::colsum(const TA&, const floatx4& v) {
  floatx4 s;
#pragma unroll
  for (int r = 0; r < 4; ++r) s[r] = row_sum16(v[r]);
  return s;
}

// Per-class column partials of the block, chunked: each wave parks its 16-fiber
// sums of COL_CH classes in buf[COL_CH][4][CW]; the block then writes the 4-wave
// sums (fixed order) to part[(rowbase + c) * CW + h] ([G][NFG][NC][CW] layout),
// four channels per thread (CW % 4 == 0: 16-byte LDS reads and global stores).
#ifndef COL_CH
#define COL_CH 16
#endif
template <int CW>
__device__ __forceinline__ void col_flush(const float* buf, int nch, int cbase, float* part,
                                          long long rowbase) {
  static_assert(CW % 4 == 0, "column width");
  constexpr int Q = CW / 4;
  for (int i = threadIdx.x; i < nch * Q; i += PF_BLOCK) {
    const int cc = i / Q, q = i - cc * Q;
    const floatx4* b = reinterpret_cast<const floatx4*>(buf + cc * 4 * CW) + q;
    const floatx4 v = ((b[0] + b[Q]) + b[2 * Q]) + b[3 * Q];
    *reinterpret_cast<floatx4*>(part + (rowbase + cbase + cc) * CW + 4 * q) = v;
  }
}

// Sum a per-wave accumulator tile set over the block's 4 waves and write the
// block partial.  acc[a] holds D[4g+r][j] of output tile a; rc(a, 4g + r, j)
// gives the partial index of each element (negative = not an output).
template <int NA, class RC>
__device__ __forceinline__ void block_partial(const floatx4 (&acc)[NA], float* scratch, int len,
                                              RC rc, float* part) {
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, g = lane >> 4, j = lane & 15;
  __syncthreads();
  for (int idx = t; idx < 4 * len; idx += PF_BLOCK) scratch[idx] = 0.f;
  __syncthreads();
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = rc(a, 4 * g + r, j);
      if (idx >= 0) scratch[wave * len + idx] = acc[a][r];
    }
  __syncthreads();
  for (int idx = t; idx < len; idx += PF_BLOCK)
    part[idx] = ((scratch[idx] + scratch[len + idx]) + scratch[2 * len + idx]) + scratch[3 * len + idx];
}

// sum of v over the 16 lanes of each group (xor butterfly, identical in all 16)
__device__ __forceinline__ float group_sum16(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

// ------------------------------------------------------------ class stream
// The edge rows of a wave's tiles are prefetched through a register ring of D
// slots (slot d holds the rows of class c + d); load(c) returns the rows of
// class c, body(rows, c) consumes them; the loop is unrolled by D so the slot
// index is static.  Two refill orders:
//   LATE = false: a slot is refilled with class c + d + D BEFORE the body of
//     class c + d runs (conditionally, at the range's end).  The new rows and
//     the ones being consumed are live together, so hipcc parks each new load
//     in staging registers and copies it into the ring at the back edge, behind
//     an s_waitcnt on a load issued one tile earlier;
//   LATE = true: the slot is refilled AFTER the body (unconditionally, the class
//     clamped to the range: a few re-reads of the last class at the end), so
//     the slot keeps its registers across the back edge and D - 1 tiles of row
//     loads are in flight while a tile computes.
// Measured per kernel on the bench step (profiles/r05a_ring_ab.txt): LATE is
// faster for edge_mlp_fwd (4 %), slower for source_bwd (10 %: at D = 2 its
// refills start a whole body later), within noise elsewhere.
template <int D, bool LATE = false, class Load, class Body>
__device__ __forceinline__ void class_stream(int c0, int c1, Load load, Body body) {
  using R = decltype(load(c0));
  R ring[D];
  if constexpr (!LATE) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (c0 + d < c1) ring[d] = load(c0 + d);
    for (int c = c0; c < c1; c += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int cc = c + d;
        if (cc < c1) {
          const R cur = ring[d];
          if (cc + D < c1) ring[d] = load(cc + D);
          body(cur, cc);
        }
      }
    }
  } else {
    if (c1 <= c0) return;
    const int last = c1 - 1;
#pragma unroll
    for (int d = 0; d < D; ++d) ring[d] = load(min(c0 + d, last));
    int c = c0;
    for (; c + D <= c1; c += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        body(ring[d], c + d);
        // the refill stays behind the body's last read of the slot
        __builtin_amdgcn_sched_barrier(0);
        ring[d] = load(min(c + d + D, last));
      }
    }
#pragma unroll
    for (int d = 0; d < D - 1; ++d)
      if (c + d < c1) body(ring[d], c + d);
  }
}

// A two-stage software pipeline over the class stream: head(rows, c) (the
// class's independent first stage: loads consumed, its recompute MFMAs
// issued) runs for class c + 1 before tail(h, c) finishes class c, so the
// head's MFMA chains execute under the tail's vector work instead of at the
// start of the next class's dependency chain.  Loads stay D classes ahead;
// past the last class the head and the refills repeat the last class
// (clamped, side-effect free; their results are unused).
template <int D, class Load, class Head, class Tail>
__device__ __forceinline__ void class_stream_pipe(int c0, int c1, Load load, Head head, Tail tail) {
  using R = decltype(load(c0));
  if (c1 <= c0) return;
  const int last = c1 - 1;
  R ring[D];
#pragma unroll
  for (int d = 0; d < D; ++d) ring[d] = load(min(c0 + d, last));
  auto h = head(ring[0], c0);
  ring[0] = load(min(c0 + D, last));
  for (int c = c0; c < c1; c += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int cc = c + d;
      if (cc < c1) {
        const int s = (d + 1) % D;   // ring slot of class cc + 1 (constant once unrolled)
        const auto hn = head(ring[s], min(cc + 1, last));
        ring[s] = load(min(cc + 1 + D, last));
        tail(h, cc);
        h = hn;
      }
    }
  }
}

// The LATE ring with the body applied to class PAIRS: body2(rows_a, ca,
// rows_b, cb) gets two consecutive classes, so that their independent MFMA
// chains interleave in one instruction stream (a forward kernel's single-class
// body is one dependent chain per layer); body1 takes an odd last class.
template <int D, class Load, class Body1, class Body2>
__device__ __forceinline__ void class_stream_pairs(int c0, int c1, Load load, Body1 body1,
                                                   Body2 body2) {
  static_assert(D % 2 == 0, "class pairs need an even ring");
  using R = decltype(load(c0));
  R ring[D];
  if (c1 <= c0) return;
  const int last = c1 - 1;
#pragma unroll
  for (int d = 0; d < D; ++d) ring[d] = load(min(c0 + d, last));
  int c = c0;
  for (; c + D <= c1; c += D) {
#pragma unroll
    for (int d = 0; d < D; d += 2) {
      body2(ring[d], c + d, ring[d + 1], c + d + 1);
      __builtin_amdgcn_sched_barrier(0);
      ring[d] = load(min(c + d + D, last));
      ring[d + 1] = load(min(c + d + 1 + D, last));
    }
  }
#pragma unroll
  for (int d = 0; d < D; d += 2) {
    if (c + d + 1 < c1) body2(ring[d], c + d, ring[d + 1], c + d + 1);
    else if (c + d < c1) body1(ring[d], c + d);
  }
}

template <int NA>
struct Rows {
  floatx4 v[NA];
  uint32_t m;   // the edge's TModel LeakyReLU mask byte (RowsM loads only)
};

// TModel's LeakyReLU mask of a message MLP pre-activation, one byte per
// (edge, lane group): bit s set iff slot s of the lane's rows is > 0.
// target_fwd writes it at byte eo + g (eo: the edge's byte offset in a
// channel-major [C][E] fp32 tensor, i.e. 4 bytes per edge, one per lane
// group), so a wave's tile is one coalesced 64-byte store; target_bwd and
// source_bwd read it instead of recomputing the layer (tmask_bytes()).
template <int C>
__device__ __forceinline__ uint32_t mask_bits(const floatx4 (&z)[GM<C>::NT]) {
  uint32_t m = 0;
#pragma unroll
  for (int tt = 0; tt < GM<C>::NT; ++tt)
#pragma unroll
    for (int r = 0; r < GM<C>::nreg(tt); ++r) m |= (z[tt][r] > 0.f ? 1u : 0u) << (4 * tt + r);
  return m;
}
__device__ __forceinline__ float mask_slope(uint32_t m, int s) {
  return (m >> s) & 1u ? 1.f : PF_LEAKY;
}

#define MF_GEO                                                                        \
  const int t = threadIdx.x, lane = t & 63;                                           \
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);                            \
  const int g4 = lane >> 4, j16 = lane & 15;                                          \
  const int bx = PF_LOGICAL_BLOCK(geo);                                               \
  if (bx >= geo.nblocks) return; /* (block-uniform: the XCD grid is rounded to 8) */  \
  const int ks = bx % geo.KS, grp = bx / geo.KS;                                      \
  const int fg = grp % geo.NFG, gg = grp / geo.NFG;                                   \
  const int f = fg * 64 + wave * 16 + j16;                                            \
  const bool fvalid = f < geo.NF;                                                     \
  const long long n = (long long)gg * geo.NF + (fvalid ? f : 0);                      \
  const int c0 = ks * geo.CPS, c1 = min(geo.NC, c0 + geo.CPS);                        \
  const long long NS = geo.NS;                                                        \
  const uint32_t RB = (uint32_t)geo.E * 4u;                                           \
  const uint32_t eo0 =                                                                \
      (uint32_t)((((long long)gg * geo.NC) * geo.NF + (fvalid ? f : 0)) * 4);         \
  const uint32_t eoc = (uint32_t)geo.NF * 4u;                                         \
  const uint32_t EB = (uint32_t)geo.E * 4u; /* bytes per channel row and of the mask */ \
  const long long colbase = ((long long)gg * geo.NFG + fg) * geo.NC;                  \
  (void)t; (void)n; (void)NS; (void)RB; (void)colbase; (void)j16; (void)EB;

// x = valid ? (sc*raw + sh) : 0 on the lane's F slots
template <int F>
__device__ __forceinline__ floatx4 edge_in(const floatx4& raw, const bool (&fm)[4],
                                           const float* sc, const floatx4& scv,
                                           const floatx4& shv) {
  floatx4 x = zero4();
#pragma unroll
  for (int r = 0; r < GM<F>::RPG; ++r) x[r] = fm[r] ? (sc ? fmaf(raw[r], scv[r], shv[r]) : raw[r]) : 0.f;
  return x;
}

#define MF_FMASK(F)                                                                   \
  bool fm[4];                                                                         \
  _Pragma("unroll") for (int r = 0; r < 4; ++r) fm[r] = fvalid && GM<F>::row(g4, r) >= 0; \
  const RowOff<F> ro(eo0, RB, g4);

}  // namespace
