// pfsgnn_mlp.hip -- fused node-level MLPs (gnn.py:65-71, Linear -> LeakyReLU(0.1)
// -> Linear) with the BatchNorm1d that follows them in SModel / TModel
// (gnn.py:154, 192), on v_mfma_f32_16x16x4_f32 (exact fp32 products).
//
// Forward  (pfsgnn_mlp_fwd): Z = W1 cat(X) + b1, Yp = W2 lrelu(Z) + b2, Welford
//   partials of Yp per block; then one launch finishes the BatchNorm statistics
//   (every block merges the partials in the same fixed order) and writes
//   Y = BN(Yp).  Two launches for what was lin_cat + lin + stats + finalize + apply.
// Backward (pfsgnn_mlp_bwd): BatchNorm sums (one launch), then per node
//   dYp = BN'(dY), dZ = (W2^T dYp) * lrelu'(Z), dX = W1^T dZ written (or added)
//   straight into the caller's gradient blocks.  The weight gradients stay
//   pfsgnn_wgrad(_cat) calls on (dYp, lrelu Z) and (dZ, X).
//
// Geometry.  Node n is the MFMA column; a wave owns 16 nodes, a block 64 per
// chunk and walks chunks grid-stride (persistent), so the weights are staged
// in LDS once per block.  All widths are padded to M tiles of 16 (K, H <= 16M,
// O <= 16).  Layer chaining needs no data movement: the D layout of a tile
// (lane group q holds rows 16t + 4q + r in register r) is the B operand of the
// next layer's K-step (t, r), whose A operand is the permuted weight image.
#include "pfsgnn_common.h"
#include "../../include/pfsgnn.h"

#include <algorithm>
#include <climits>
#include <map>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int NM_SEG = 4;

// concatenated input rows (gnn.py:153 [x, mean, std, skew, kurt, u[batch]] etc.)
struct InSegs {
  const float* p[NM_SEG];
  int k0[NM_SEG + 1];  // first row of each block; INT_MAX past the last
  int pg[NM_SEG];      // 1: per-graph block [rows][Gc], node n reads column n / npg
  int npg, Gc;
  // the same blocks in a K index padded to whole K-steps of 4 (k_mlp_fwd RS):
  // block s at [kp0[s], kp0[s] + rows[s]), kp0 a multiple of 4, Kp the padded K
  int kp0[NM_SEG + 1], rows[NM_SEG], Kp;
};

// gradient output rows: block s covers rows [k0[s], k0[s+1]); p == nullptr drops them
struct OutSegs {
  float* p[NM_SEG];
  int k0[NM_SEG + 1];
  int add[NM_SEG];
};

// async global -> LDS copy of one float per lane: LDS row base (wave-uniform)
// + 4*lane, no VGPR destination (global_load_lds_dword)
__device__ __forceinline__ void glds4(const float* src, float* lds_row) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_row, 4, 0, 0);
}

// Row descriptors of a concatenated input (RowIn: row k's base at node 0 --
// column 0 for a per-graph block -- and the per-graph flag) or of the gradient
// outputs (RowOut: row k's base, null when dropped, and the add flag), built
// once per block in LDS by threads k < K.  The row loops then read a ready
// base pointer: selecting the block from the kernel arguments per row cost a
// dependent scalar load and wait per row (25 rows per wave and chunk of the
// 100-wide SModel MLP), in series with the copies and the stores.
struct RowIn {
  const float* p;
  int pg, pad;
};
struct RowOut {
  float* p;
  int add, pad;
};
__device__ __forceinline__ void build_in_rows(const InSegs& S, int K, int N, RowIn* tab) {
  const int k = threadIdx.x;
  if (k >= K) return;
  const float* p = S.p[0];
  int kb = 0, pg = S.pg[0];
  if (k >= S.k0[1]) { p = S.p[1]; kb = S.k0[1]; pg = S.pg[1]; }
  if (k >= S.k0[2]) { p = S.p[2]; kb = S.k0[2]; pg = S.pg[2]; }
  if (k >= S.k0[3]) { p = S.p[3]; kb = S.k0[3]; pg = S.pg[3]; }
  tab[k] = RowIn{p + (size_t)(k - kb) * (pg ? S.Gc : N), pg, 0};
}
// SModel's moment-gradient coefficients (k_moment_coef's arithmetic,
// pfsgnn_node.hip) made in k_mlp_bwd's input-gradient epilogue (coef !=
// nullptr): the dX rows [k0, k0 + 4 C2) -- d loss / d [mean; std; skew; kurt]
// of C2 = 2F message channels (gnn.py:140-153) -- are then never written;
// the epilogue turns them into coef [4][C2][N] straight from LDS.  To put a
// channel's four rows into one 64-row store group, dX row r' of the kernel
// holds input row mom_row(r'): r' = 4c + m (c < C2, m = moment) first, the
// other input rows after them in order.  (16 <= C2 <= 20: channels 0..15 fill
// the first 64-row group, 16.. open the second.)
struct MomCoef {
  const float* mom;   // [4][C2][N]: mean, c2, c3, c4 (pfsgnn_source_fwd's mom)
  float* coef;        // [4][C2][N]
  int C2, k0;
  float invn;         // 1 / messages per fiber
};
__device__ __host__ __forceinline__ int mom_row(int r, const MomCoef& mc) {
  if (!mc.coef) return r;
  const int nm = 4 * mc.C2;
  if (r < nm) return mc.k0 + (r & 3) * mc.C2 + (r >> 2);
  const int q = r - nm;
  return q < mc.k0 ? q : q + nm;
}
__device__ __forceinline__ void build_out_rows(const OutSegs& S, int K, int N, RowOut* tab,
                                               const MomCoef& mc) {
  const int r = threadIdx.x;
  if (r >= K) return;
  const int k = mom_row(r, mc);
  if (mc.coef && k >= mc.k0 && k < mc.k0 + 4 * mc.C2) {   // (made into coef, not stored)
    tab[r] = RowOut{nullptr, 0, 0};
    return;
  }
  float* p = S.p[0];
  int kb = 0, add = S.add[0];
  if (k >= S.k0[1]) { p = S.p[1]; kb = S.k0[1]; add = S.add[1]; }
  if (k >= S.k0[2]) { p = S.p[2]; kb = S.k0[2]; add = S.add[2]; }
  if (k >= S.k0[3]) { p = S.p[3]; kb = S.k0[3]; add = S.add[3]; }
  tab[r] = RowOut{p ? p + (size_t)(k - kb) * N : nullptr, add, 0};
}
// the coefficients of channels c0 .. c0 + 256 / (64 / NPT) - 1 for the chunk's
// 64 nodes from their gradient rows 4 (c - c0) + m staged in X ([row][ld]);
// thread (channel, j) takes nodes NPT j .. NPT j + NPT - 1 (NPT = 4: 16
// channels; NPT = 1: 4 channels, fewer registers for the mid-loop group)
template <int NPT>
__device__ __forceinline__ void mom_coef_epi(const MomCoef& mc, const float* X, int ld, int c0,
                                             int n0, int N) {
  constexpr int TPC = 64 / NPT;   // threads per channel
  const int t = threadIdx.x, cl = t / TPC, j = t % TPC, c = c0 + cl;
  if (c >= mc.C2) return;
  // (the bases as VGPR values: the kernel's scalar registers are spent, and
  // uniform address math here spilled them)
  const float* mom = mc.mom;
  float* coef = mc.coef;
  int C2 = mc.C2;
  float invn = mc.invn;
  asm volatile("" : "+v"(mom), "+v"(coef), "+v"(C2), "+v"(invn), "+v"(N));
  const size_t CN = (size_t)C2 * N;
  float m2[NPT], m3[NPT], m4[NPT];
#pragma unroll
  for (int e = 0; e < NPT; ++e) {   // every load in flight (clamped node)
    const int n = min(n0 + NPT * j + e, N - 1);
    const size_t i = (size_t)c * N + n;
    m2[e] = mom[CN + i];
    m3[e] = mom[2 * CN + i];
    m4[e] = mom[3 * CN + i];
  }
#pragma unroll
  for (int e = 0; e < NPT; ++e) {
    const int n = n0 + NPT * j + e;
    if (n >= N) continue;
    const float c2 = m2[e], c3 = m3[e], c4 = m4[e];
    const float* xr = X + 4 * cl * ld + NPT * j + e;
    const float gmean = xr[0], gstd = xr[ld], gskew = xr[2 * ld], gkurt = xr[3 * ld];
    const float var = c2 > 0.f ? c2 : 0.01f * c2;
    const float sd = sqrtf(var + 1e-6f);
    const float sd2 = sd * sd, sd3 = sd2 * sd, sd4 = sd2 * sd2;
    const float A3 = gskew / sd3;
    const float A4 = gkurt / sd4;
    const float gstd_tot = gstd - 3.f * gskew * c3 / sd4 - 4.f * gkurt * c4 / (sd4 * sd);
    const float gvr = gstd_tot / (2.f * sd) * (c2 > 0.f ? 1.f : 0.01f);
    const size_t i = (size_t)c * N + n;
    coef[i] = (gmean - 3.f * c2 * A3 - 4.f * c3 * A4) * invn;
    coef[CN + i] = 2.f * gvr * invn;
    coef[2 * CN + i] = 3.f * A3 * invn;
    coef[3 * CN + i] = 4.f * A4 * invn;
  }
}

// node tables of a chunk staged in LDS as [row][XS_LD]: a wave's 16-node
// column block for rows k = 4s + q puts lane groups q = 0..3 on disjoint
// 16-bank ranges (stride 80 = 16 mod 32)
constexpr int XS_LD = 80;

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int PART_LEN = 33;  // BN forward partial: count, mean[16], M2[16]

// ============================================================ forward
// RS (the wide MLPs, M >= 5): the chunk's inputs go straight to registers
// (each lane loads its 4M rows, prefetched one chunk ahead) instead of through
// the double-buffered LDS copy, so the LDS holds only the weight images
// (57 KB at M = 7) and two blocks fit a CU: two waves per SIMD to hide the
// loads and the MFMA dependency latency (one block per CU ran the 100x100
// SModel MLP at 28 % MFMA utilisation).
template <int M, bool RS>
__global__ __launch_bounds__(256, ((M <= 3 || RS) ? 2 : 1)) void k_mlp_fwd(InSegs S, int K, int N,
                                                    const float* __restrict__ W1, int ldw1, int H,
                                                    const float* __restrict__ b1,
                                                    const float* __restrict__ W2, int O,
                                                    const float* __restrict__ b2,
                                                    float* __restrict__ Z, float* __restrict__ Yp,
                                                    float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  floatx4* A1 = reinterpret_cast<floatx4*>(sm);  // [M][M][64]: W1 per (tile, 4 K-steps)
  floatx4* A2 = A1 + M * M * 64;                 // [M][64]: W2 per hidden tile
  float* B1 = reinterpret_cast<float*>(A2 + M * 64);
  float* B2 = B1 + 16 * M;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, col = lane & 15, kq = lane >> 4;
  // chunk input rows [16M][XS_LD], double-buffered: chunk c+1 streams in with
  // global_load_lds while chunk c is multiplied.  The first chunk's copy is
  // issued before the weight images are staged (its latency overlaps theirs);
  // only the padding rows >= K, which no copy writes, are zeroed.
  float* Xs0 = B2 + 16;
  constexpr int XSZ = 16 * M * XS_LD;
  const int nch = (N + 63) / 64;
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  // this wave's input rows k = wu + 4 i (LDS-staged form): bases in registers
  __shared__ RowIn rin[RS ? 1 : 16 * M];
  const float* rp[RS ? 1 : 4 * M];
  uint32_t pgm = 0;
  if (!RS) {
    build_in_rows(S, K, N, rin);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < (RS ? 0 : 4 * M); ++i) {
      const int k = wu + 4 * i;
      const RowIn r = rin[k < K ? k : 0];
      rp[i] = r.p;
      pgm |= (uint32_t)(r.pg != 0) << i;
    }
  }
  auto issue = [&](int ch, int buf) {
    const int n = ch * 64 + lane;
    const int nc = n < N ? n : N - 1;
    const int ng = S.npg ? nc / S.npg : 0;
    float* dst = Xs0 + buf * XSZ;
#pragma unroll
    for (int i = 0; i < (RS ? 0 : 4 * M); ++i) {
      const int k = wu + 4 * i;
      if (k < K) glds4(rp[i] + (((pgm >> i) & 1u) ? ng : nc), dst + k * XS_LD);
    }
  };
  // RS: lane (col, kq) holds rows 4s + kq of its node (the B operand of K-step s)
  float xq[RS ? 4 * M : 1];
  // (RS uses the padded K index: every K-step's 4 rows lie in one block, so
  // the block and its base pointer are wave-uniform scalars per step)
  auto fetch = [&](int ch) {
    const int n = ch * 64 + wave * 16 + col;
    const int nc = n < N ? n : N - 1;
    const int ng = S.npg ? nc / S.npg : 0;
#pragma unroll
    for (int s = 0; s < (RS ? 4 * M : 0); ++s) {
      int kk = 4 * s;
      asm volatile("" : "+s"(kk));   // (per fetch: 28 hoisted scalar bases spill)
      const int sg = (kk >= S.kp0[1]) + (kk >= S.kp0[2]) + (kk >= S.kp0[3]);
      const int r = kk - S.kp0[sg] + kq;
      const bool pgs = S.pg[sg] != 0;
      const float* src = S.p[sg] + (size_t)r * (pgs ? S.Gc : N) + (pgs ? ng : nc);
      xq[s] = (kk < S.Kp && r < S.rows[sg]) ? *src : 0.f;
    }
  };
  if (RS) {
    if ((int)blockIdx.x < nch) fetch(blockIdx.x);
  } else {
    if ((int)blockIdx.x < nch) issue(blockIdx.x, 0);
    for (int i = K * XS_LD + t; i < XSZ; i += 256) Xs0[i] = Xs0[XSZ + i] = 0.f;
  }
  {  // weight images: every load of the thread in flight at once (a load ->
     // store loop would pay one L2 round trip per element)
    float v[M * M], w[M];
#pragma unroll
    for (int i = 0; i < M * M; ++i) {
      const int idx = t + 256 * i;
      const int j = idx & 3, l = (idx >> 2) & 63, q = (idx >> 8) % M, mt = (idx >> 8) / M;
      const int row = 16 * mt + (l & 15);
      int k = 4 * (4 * q + j) + (l >> 4);
      bool kv = k < K;
      if (RS) {   // padded K index -> weight column (pad rows: 0)
        const int sg = (k >= S.kp0[1]) + (k >= S.kp0[2]) + (k >= S.kp0[3]);
        const int r = k - S.kp0[sg];
        kv = k < S.Kp && r < S.rows[sg];
        k = S.k0[sg] + r;
      }
      v[i] = (row < H && kv) ? W1[(size_t)row * ldw1 + k] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int idx = t + 256 * i;
      const int r = idx & 3, l = (idx >> 2) & 63, mt = idx >> 8;
      const int o = l & 15, h = 16 * mt + 4 * (l >> 4) + r;
      w[i] = (o < O && h < H) ? W2[(size_t)o * H + h] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < M * M; ++i) sm[t + 256 * i] = v[i];
#pragma unroll
    for (int i = 0; i < M; ++i) reinterpret_cast<float*>(A2)[t + 256 * i] = w[i];
  }
  for (int i = t; i < 16 * M; i += 256) B1[i] = i < H ? b1[i] : 0.f;
  if (t < 16) B2[t] = t < O ? b2[t] : 0.f;

  float cnt = 0.f, mean[4] = {0.f, 0.f, 0.f, 0.f}, m2[4] = {0.f, 0.f, 0.f, 0.f};
  int it = 0;
  if (RS) __syncthreads();   // weight images
  for (int ch = blockIdx.x; ch < nch; ch += gridDim.x, ++it) {
    const int buf = it & 1;
    if (!RS) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of chunk ch landed
      __syncthreads();                                    // ... and every other wave's
      if (ch + (int)gridDim.x < nch) issue(ch + gridDim.x, buf ^ 1);
    }
    const float* Xs = Xs0 + buf * XSZ;
    const int n = ch * 64 + wave * 16 + col;
    const bool nv = n < N;
    // the weight images are re-read from LDS every chunk: an opaque offset keeps
    // the compiler from hoisting M*M float4 loop invariants into registers
    int lo = 0;
    asm volatile("" : "+v"(lo));
    const floatx4* A1c = A1 + lo;
    const floatx4* A2c = A2 + lo;
    const float* xr = Xs + lo + kq * XS_LD + wave * 16 + col;
    // the hidden tiles in groups of MG (RS: fewer live accumulators), each
    // group's layer 1 over all K-steps, then its share of layer 2: the same
    // per-accumulator order as one group of M
    constexpr int MG = RS ? 4 : M;
    floatx4 ye = floatx4{0.f, 0.f, 0.f, 0.f}, yo = ye;
#pragma unroll
    for (int g0 = 0; g0 < M; g0 += MG) {
      constexpr int dummy = 0;
      (void)dummy;
      const int GN = (M - g0) < MG ? (M - g0) : MG;   // (compile-time after unrolling)
      floatx4 acc[MG];
#pragma unroll
      for (int i = 0; i < MG; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      // K-step group q: its weight float4s and 4 input values are read first
      // (the next group's reads are issued before this group's MFMAs), and the
      // MFMAs run across the independent accumulators (no dependent back-to-back)
      floatx4 an[MG];
      float xn[4];
#pragma unroll
      for (int i = 0; i < MG; ++i)
        if (i < GN) an[i] = A1c[(g0 + i) * M * 64 + lane];
#pragma unroll
      for (int j = 0; j < 4; ++j) xn[j] = RS ? xq[j] : xr[(4 * j) * XS_LD];
#pragma unroll
      for (int q = 0; q < M; ++q) {
        floatx4 av[MG];
        float x[4];
#pragma unroll
        for (int i = 0; i < MG; ++i) av[i] = an[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = xn[j];
        if (q + 1 < M) {
#pragma unroll
          for (int i = 0; i < MG; ++i)
            if (i < GN) an[i] = A1c[((g0 + i) * M + q + 1) * 64 + lane];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            xn[j] = RS ? xq[4 * (q + 1) + j] : xr[(4 * (4 * (q + 1) + j)) * XS_LD];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < MG; ++i)
            if (i < GN) acc[i] = mfma4(av[i][j], x[j], acc[i]);
      }
      // RS: the next chunk's rows load while this one finishes (its layer 2 and
      // epilogue, and the other block's waves on the SIMD)
      if (RS && g0 + MG >= M && ch + (int)gridDim.x < nch) fetch(ch + gridDim.x);
      floatx4 act[MG], w2[MG];
#pragma unroll
      for (int i = 0; i < MG; ++i) {
        if (i >= GN) continue;
        const int mt = g0 + i;
        w2[i] = A2c[mt * 64 + lane];
        const floatx4 bb = *reinterpret_cast<const floatx4*>(B1 + 16 * mt + 4 * kq);
        const floatx4 z = acc[i] + bb;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = 16 * mt + 4 * kq + r;
          if (Z && nv && h < H) Z[(size_t)h * N + n] = z[r];
          act[i][r] = lrelu(z[r]);
        }
      }
      // two accumulators (even / odd hidden tiles), each in K order
#pragma unroll
      for (int i = 0; i < MG; ++i) {
        if (i >= GN) continue;
        const int mt = g0 + i;
        if ((mt & 1) == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ye = mfma4(w2[i][r], act[i][r], ye);
            if (i + 1 < GN) yo = mfma4(w2[i + 1][r], act[i + 1][r], yo);
          }
        }
      }
    }
    const floatx4 bo = *reinterpret_cast<const floatx4*>(B2 + 4 * kq);
    const floatx4 y = ye + yo + bo;
    if (nv) {
      cnt += 1.f;
      const float rc = 1.f / cnt;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = 4 * kq + r;
        if (o < O) {
          Yp[(size_t)o * N + n] = y[r];
          const float d = y[r] - mean[r];
          mean[r] = fmaf(d, rc, mean[r]);
          m2[r] = fmaf(d, y[r] - mean[r], m2[r]);
        }
      }
    }
  }
  if (!part) return;
  // Chan merge over the 16 nodes of each lane group, then over the 4 waves
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) {
    const float cb = __shfl_xor(cnt, off);
    const float tot = cnt + cb;
    const float wb = tot > 0.f ? cb / tot : 0.f;
    const float wab = tot > 0.f ? cnt * cb / tot : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mb = __shfl_xor(mean[r], off), qb = __shfl_xor(m2[r], off);
      const float d = mb - mean[r];
      mean[r] = fmaf(d, wb, mean[r]);
      m2[r] = m2[r] + qb + d * d * wab;
    }
    cnt = tot;
  }
  __shared__ float shm[4][PART_LEN];
  __syncthreads();
  if (col == 0) {
    if (kq == 0) shm[wave][0] = cnt;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      shm[wave][1 + 4 * kq + r] = mean[r];
      shm[wave][17 + 4 * kq + r] = m2[r];
    }
  }
  __syncthreads();
  if (t < 16) {
    float C0 = shm[0][0], M0 = shm[0][1 + t], Q0 = shm[0][17 + t];
    for (int w = 1; w < 4; ++w) {
      const float cb = shm[w][0], mb = shm[w][1 + t], qb = shm[w][17 + t];
      const float tot = C0 + cb;
      if (tot > 0.f) {
        const float d = mb - M0;
        M0 = M0 + d * (cb / tot);
        Q0 = Q0 + qb + d * d * (C0 * cb / tot);
      }
      C0 = tot;
    }
    float* p = part + (size_t)blockIdx.x * PART_LEN;
    if (t == 0) p[0] = C0;
    p[1 + t] = M0;
    p[17 + t] = Q0;
  }
}

// BatchNorm1d training statistics from the MLP's per-block partials, in every
// block of the calling kernel: the partials merged in the same fixed order
// (double); `write` (one block) stores mu / var and updates the running
// statistics (unbiased variance).  -> cf[0][o] = mean, cf[1][o] = 1/sqrt(var +
// eps), cf[2] = gamma, cf[3] = beta (256 threads; nb <= 512).
template <bool SC1 = false>   // SC1: the partials were handed over in-launch (grid_sync)
__device__ void bn_stats_part(const float* __restrict__ part, int nb, int O, int N,
                              const float* __restrict__ gamma, const float* __restrict__ beta,
                              float eps, float* __restrict__ rm, float* __restrict__ rv,
                              float momentum, float* __restrict__ mu, float* __restrict__ var,
                              bool write, float (*cf)[16]) {
  __shared__ double acc[16][16][2];
  __shared__ double mean_s[16];
  const int t = threadIdx.x, c = t & 15, u = (t >> 4) & 15;
  const bool act = t < 256;   // (blocks wider than 256 threads: the first 256 merge)
  // partials per thread per round: 16 (one round for nb <= 256, the MLP grids
  // of <= 256 blocks; two for <= 512, re-read for the second pass)
  constexpr int PB = 16;
  const int rounds = (nb + 255) >> 8;
  float pc[PB], pm[PB], pq[PB];
  auto fetch = [&](int r) {
#pragma unroll
    for (int i = 0; i < PB; ++i) {  // every load of the round in flight before the sums
      const int b = act ? r * 256 + u + 16 * i : nb;
      const float* p = part + (size_t)(b < nb ? b : 0) * PART_LEN;
      if constexpr (SC1) {
        pc[i] = b < nb ? ld_sc1(p) : 0.f;
        pm[i] = b < nb ? ld_sc1(p + 1 + c) : 0.f;
        pq[i] = b < nb ? ld_sc1(p + 17 + c) : 0.f;
      } else {
        pc[i] = b < nb ? p[0] : 0.f;
        pm[i] = b < nb ? p[1 + c] : 0.f;
        pq[i] = b < nb ? p[17 + c] : 0.f;
      }
    }
  };
  // the partials combined in closed form (fixed order, no serial chain of
  // divisions): mean = sum c_b m_b / N, M2 = sum (q_b + c_b (m_b - mean)^2)
  double S = 0.0;
  for (int r = 0; r < rounds; ++r) {
    fetch(r);
#pragma unroll
    for (int i = 0; i < PB; ++i) S += (double)pc[i] * (double)pm[i];
  }
  if (act) acc[u][c][0] = S;
  __syncthreads();
  if (t < 16) {
    double St = 0.0;
    for (int s = 0; s < 16; ++s) St += acc[s][t][0];
    mean_s[t] = St / (double)N;
  }
  __syncthreads();
  const double mean = mean_s[c];
  double Q = 0.0;
  for (int r = 0; r < rounds; ++r) {
    if (rounds > 1) fetch(r);
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const double d = (double)pm[i] - mean;
      Q += (double)pq[i] + (double)pc[i] * d * d;
    }
  }
  if (act) acc[u][c][1] = Q;
  __syncthreads();
  if (t < 16) {
    double Qc = 0.0;
    for (int s = 0; s < 16; ++s) Qc += acc[s][t][1];
    const double Mc = mean_s[t];
    const double v = Qc / (double)N;
    const float muf = (float)Mc, vf = (float)v;
    const bool live = t < O;
    cf[0][t] = muf;
    cf[1][t] = 1.0f / sqrtf(vf + eps);
    cf[2][t] = live ? gamma[t] : 0.f;
    cf[3][t] = live ? beta[t] : 0.f;
    if (write && live) {
      mu[t] = muf;
      var[t] = vf;
      if (rm) {
        const double unb = N > 1 ? Qc / (double)(N - 1) : v;
        rm[t] = (float)((1.0 - momentum) * rm[t] + momentum * Mc);
        rv[t] = (float)((1.0 - momentum) * rv[t] + momentum * unb);
      }
    }
  }
  __syncthreads();
}

// Linear maps of the normalised output, done where it is written (the node
// parts the next consumers need: TModel's Rs = Wt1[:, :F] x_s' + bt1 and the
// next block's EdgeModel Ps = W1[:, :F] x_s', gnn.py:100/188):
// out_e[k][n] = sum_o W_e[k][col0_e + o] Y[o][n] + b_e[k]
constexpr int EPI_MAXK = 64;
struct BnEpi {
  const float* W[2];
  int ldw[2], col0[2], nk[2];
  const float* b[2];
  float* out[2];
};

// BatchNorm1d training forward from the MLP's per-block partials: every block
// merges them (bn_stats_part), block 0 writes mu / var and the running
// statistics, all apply the norm (+ the epilogues, thread per node).
// (OT: the output width when known at compile time -- the epilogue's FMA
// loops then run over the O live channels instead of 16; 0: any O <= 16)
template <int OT>
__global__ __launch_bounds__(256) void k_bn_apply_part(const float* __restrict__ part, int nb,
                                                       int O, int N, const float* __restrict__ Yp,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps,
                                                       float* __restrict__ rm,
                                                       float* __restrict__ rv, float momentum,
                                                       float* __restrict__ Y,
                                                       float* __restrict__ mu,
                                                       float* __restrict__ var, BnEpi E) {
  __shared__ float cf[4][16];
  __shared__ __attribute__((aligned(16))) float ew[2][EPI_MAXK * 16];
  __shared__ float eb[2][EPI_MAXK];
  const int t = threadIdx.x;
  const bool epi = E.W[0] || E.W[1];
  if (epi) {  // weight blocks staged before the statistics (latency overlapped)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (!E.W[e]) continue;
      const int nk4 = (E.nk[e] + 3) & ~3;   // rows past nk are zero (4-row groups below)
      for (int i = t; i < nk4 * 16; i += 256) {
        const int k = i >> 4, o = i & 15;
        ew[e][i] = (o < O && k < E.nk[e]) ? E.W[e][(size_t)k * E.ldw[e] + E.col0[e] + o] : 0.f;
      }
      for (int k = t; k < nk4; k += 256) eb[e][k] = (E.b[e] && k < E.nk[e]) ? E.b[e][k] : 0.f;
    }
  }
  bn_stats_part(part, nb, O, N, gamma, beta, eps, rm, rv, momentum, mu, var, blockIdx.x == 0, cf);
  if (!epi) {
    for (int o = 0; o < O; ++o) {
      const float m = cf[0][o], a = cf[1][o] * cf[2][o], b = cf[3][o];
      const float* yp = Yp + (size_t)o * N;
      float* y = Y + (size_t)o * N;
      for (int n = blockIdx.x * 256 + t; n < N; n += gridDim.x * 256) y[n] = (yp[n] - m) * a + b;
    }
    return;
  }
  constexpr int OW = OT ? (OT + 3) / 4 * 4 : 16;   // channels the epilogue multiplies
  // two nodes per thread and step (8 independent FMA chains: one wave per SIMD
  // at this grid, so the chains are the latency hiding)
  const int stride = gridDim.x * 256;
  for (int n = blockIdx.x * 256 + t; n < N; n += 2 * stride) {
    const int n2 = n + stride;
    const bool v2 = n2 < N;
    float y[2][16];
#pragma unroll
    for (int o = 0; o < 16; ++o) {
      y[0][o] = y[1][o] = 0.f;
      if (o < O) {
        const float sc = cf[1][o] * cf[2][o];
        y[0][o] = (Yp[(size_t)o * N + n] - cf[0][o]) * sc + cf[3][o];
        Y[(size_t)o * N + n] = y[0][o];
        if (v2) {
          y[1][o] = (Yp[(size_t)o * N + n2] - cf[0][o]) * sc + cf[3][o];
          Y[(size_t)o * N + n2] = y[1][o];
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (!E.W[e]) continue;
      for (int k0 = 0; k0 < E.nk[e]; k0 += 4) {   // 4 rows x 2 nodes per step
        float a[2][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[0][j] = a[1][j] = eb[e][k0 + j];
#pragma unroll
        for (int o4 = 0; o4 < OW; o4 += 4)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const floatx4 w = *reinterpret_cast<const floatx4*>(&ew[e][(k0 + j) * 16 + o4]);
#pragma unroll
            for (int u = 0; u < 2; ++u)
              a[u][j] = fmaf(w[0], y[u][o4], fmaf(w[1], y[u][o4 + 1], fmaf(w[2], y[u][o4 + 2],
                             fmaf(w[3], y[u][o4 + 3], a[u][j]))));
          }
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (k0 + j < E.nk[e]) {
            E.out[e][(size_t)(k0 + j) * N + n] = a[0][j];
            if (v2) E.out[e][(size_t)(k0 + j) * N + n2] = a[1][j];
          }
      }
    }
  }
}

// ---------------------------------------------------------------- class side + GlobalModel
// The block's tail after TModel's node_mlp_2 (k_mlp_fwd: Yp and BatchNorm
// partials), one workgroup per graph: TModel's BatchNorm1d (gnn.py:192; the
// statistics merged in every workgroup in the same order, workgroup 0 writes
// mu / var / running stats) applied to the graph's classes; GlobalModel
// (gnn.py:218-223: the x_s / x_t means, MLP(3F -> H -> F), RMSNorm twice, the
// arithmetic of k_global_fwd); then the next block's class parts from the new
// x_t and u: Pt = We[:, F:2F] x_t + We[:, 3F:4F] u[g] + be (EdgeModel,
// gnn.py:100) and Qt = Ws[:, :F] x_t + bs (SModel, gnn.py:136).  One launch for
// what was bn_apply + graph_mean2 + global_fwd + the next block's class GEMMs.
constexpr int CG_MAXF = 16, CG_MAXH = 192, CG_GW1 = 4096;
struct ClassGlobalArgs {
  const float* part;  // TModel node_mlp_2's BatchNorm partials (k_mlp_fwd), nb of them
  int nb, F, NC, G, NF;
  const float* Yp;    // [F][G*NC] pre-norm node_mlp_2 output
  const float *gamma, *beta;
  float eps, momentum;
  float *rm, *rv, *xt, *mu, *var;    // xt [F][G*NC]: the new x_t
  const float* xs;    // [F][G*NF] the new x_s
  const float* u;     // [F][G]
  const float *W1, *b1, *W2, *b2, *w;  // GlobalModel MLP (W1 [H][3F]) and RMSNorm weight (or null)
  int H;
  float reps;
  float *means, *Z, *V, *Y, *y1, *r1, *r2;  // as k_global_fwd
  const float *We, *be, *Ws, *bs;           // next block (We null: none)
  float *Pt, *Qt;                           // [4F][G*NC], [2F][G*NC]
};

constexpr int CG_THREADS = 512;
// (templated on F: every per-channel loop has an exact trip count -- with 16
// guarded iterations the straight-line code of this 16-block kernel grew past
// 5000 instructions and it ran at 43 us)
template <int F>
__global__ __launch_bounds__(CG_THREADS) void k_class_global_fwd(ClassGlobalArgs A) {
  __shared__ float cf[4][16];
  __shared__ float h[CG_MAXH], z[CG_MAXH], vv[CG_MAXH];
  __shared__ float scratch[CG_THREADS / 64][2 * F];
  __shared__ float wt[4 * F * F], ws2[2 * F * F], cu[4 * F], bq[2 * F], rw[F], rs[2];
  __shared__ float gw1[CG_GW1], gw2[F * CG_MAXH];
  const int g = blockIdx.x, t = threadIdx.x, NC = A.NC, K = 3 * F;
  const long long NT = (long long)A.G * NC, NS = (long long)A.G * A.NF;
  const bool gws = A.H * K <= CG_GW1;   // GlobalModel weights staged in LDS (F = 10: 900 + 300)
  if (gws) {
    for (int i = t; i < A.H * K; i += CG_THREADS) gw1[i] = A.W1[i];
    for (int i = t; i < F * A.H; i += CG_THREADS) gw2[i] = A.W2[i];
  }
  if (t < F) rw[t] = A.w ? A.w[t] : 1.f;
  if (A.We) {  // next block's weight blocks
    for (int i = t; i < 4 * F * F; i += CG_THREADS) wt[i] = A.We[(size_t)(i / F) * 4 * F + F + i % F];
    for (int i = t; i < 2 * F * F; i += CG_THREADS) ws2[i] = A.Ws[(size_t)(i / F) * 2 * F + i % F];
  }
  bn_stats_part(A.part, A.nb, F, (int)NT, A.gamma, A.beta, A.eps, A.rm, A.rv, A.momentum, A.mu,
                A.var, g == 0, cf);
  float sm[2 * F];
#pragma unroll
  for (int o = 0; o < 2 * F; ++o) sm[o] = 0.f;
  // the graph's classes: x_t = BN(Yp), and their sum for the x_t mean
  for (int c = t; c < NC; c += CG_THREADS) {
    const long long n = (long long)g * NC + c;
    float v[F];
#pragma unroll
    for (int o = 0; o < F; ++o) v[o] = A.Yp[(size_t)o * NT + n];
#pragma unroll
    for (int o = 0; o < F; ++o) {
      v[o] = (v[o] - cf[0][o]) * (cf[1][o] * cf[2][o]) + cf[3][o];
      A.xt[(size_t)o * NT + n] = v[o];
      sm[F + o] += v[o];
    }
  }
  // the graph's x_s: U fibers x F channels of loads in flight per thread
  constexpr int U = 4;
  for (int f0 = 0; f0 < A.NF; f0 += CG_THREADS * U) {
    float v[U][F];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int f = f0 + q * CG_THREADS + t;
      const long long n = (long long)g * A.NF + (f < A.NF ? f : 0);
#pragma unroll
      for (int o = 0; o < F; ++o) v[q][o] = f < A.NF ? A.xs[(size_t)o * NS + n] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < U; ++q)
#pragma unroll
      for (int o = 0; o < F; ++o) sm[o] += v[q][o];
  }
  {  // block sums, fixed order: DPP within each wave, then the waves in order
    const int wv = t >> 6, ln = t & 63;
#pragma unroll
    for (int i = 0; i < 2 * F; ++i) {
      const float x = wave_sum(sm[i]);
      if (ln == 0) scratch[wv][i] = x;
    }
    __syncthreads();
    if (t < 2 * F) {
      float x = 0.f;
      for (int w = 0; w < CG_THREADS / 64; ++w) x += scratch[w][t];
      const float m = x / (float)(t < F ? A.NF : NC);
      h[F + t] = m;   // [u, mean x_s, mean x_t] (gnn.py:220-222)
      A.means[(size_t)t * A.G + g] = m;
    } else if (t >= 64 && t < 64 + F) {
      h[t - 64] = A.u[(size_t)(t - 64) * A.G + g];
    }
  }
  __syncthreads();
  for (int j = t; j < A.H; j += CG_THREADS) {
    float acc = A.b1[j];
    for (int k = 0; k < K; ++k) acc = fmaf(gws ? gw1[j * K + k] : A.W1[(size_t)j * K + k], h[k], acc);
    z[j] = acc;
    A.Z[(size_t)j * A.G + g] = acc;
  }
  __syncthreads();
  if (t < F) {
    float acc = A.b2[t];
    for (int j = 0; j < A.H; ++j)
      acc = fmaf(gws ? gw2[t * A.H + j] : A.W2[(size_t)t * A.H + j], lrelu(z[j]), acc);
    vv[t] = acc;
    A.V[(size_t)t * A.G + g] = acc;
  }
  __syncthreads();
  if (t == 0) {   // RMSNorm twice (k_rms2_fwd's arithmetic), LDS operands only
    if (!A.w) {
#pragma unroll
      for (int c = 0; c < F; ++c) h[c] = vv[c];
    } else {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < F; ++c) s += vv[c] * vv[c];
      const float a = rsqrtf(s / F + A.reps);
      float s2 = 0.f;
#pragma unroll
      for (int c = 0; c < F; ++c) {
        const float q = vv[c] * a * rw[c];
        z[c] = q;
        s2 += q * q;
      }
      const float b = rsqrtf(s2 / F + A.reps);
#pragma unroll
      for (int c = 0; c < F; ++c) h[c] = z[c] * b * rw[c];
      rs[0] = a;
      rs[1] = b;
    }
  }
  __syncthreads();
  if (t < F) {
    A.Y[(size_t)t * A.G + g] = h[t];   // u_new
    if (A.w) A.y1[(size_t)t * A.G + g] = z[t];
  }
  if (A.w && t == 0) {
    A.r1[g] = rs[0];
    A.r2[g] = rs[1];
  }
  if (!A.We) return;
  // next block: per-graph constant of Pt (u term + bias), then per class
  if (t < 4 * F) {
    float acc = A.be[t];
#pragma unroll
    for (int o = 0; o < F; ++o) acc = fmaf(A.We[(size_t)t * 4 * F + 3 * F + o], h[o], acc);
    cu[t] = acc;
  } else if (t >= 128 && t - 128 < 2 * F) {
    bq[t - 128] = A.bs[t - 128];
  }
  __syncthreads();
  for (int c = t; c < NC; c += CG_THREADS) {
    const long long n = (long long)g * NC + c;
    float x[F];
#pragma unroll
    for (int o = 0; o < F; ++o) x[o] = A.Yp[(size_t)o * NT + n];
#pragma unroll
    for (int o = 0; o < F; ++o) x[o] = (x[o] - cf[0][o]) * (cf[1][o] * cf[2][o]) + cf[3][o];
    for (int k = 0; k < 4 * F; ++k) {
      float acc = cu[k];
#pragma unroll
      for (int o = 0; o < F; ++o) acc = fmaf(wt[k * F + o], x[o], acc);
      A.Pt[(size_t)k * NT + n] = acc;
    }
    for (int k = 0; k < 2 * F; ++k) {
      float acc = bq[k];
#pragma unroll
      for (int o = 0; o < F; ++o) acc = fmaf(ws2[k * F + o], x[o], acc);
      A.Qt[(size_t)k * NT + n] = acc;
    }
  }
}

// ---------------------------------------------------------------- fused block tail
// A block's whole class side on a complete batch in ONE launch
// (pfsgnn_target_block_fwd): units of 32 classes of one graph, one workgroup
// per CU at most (persistent over the units), in two phases around one
// device-wide barrier:
//   1. TModel's per-class sum of the edge kernel's column partials (hsum, its
//      second Linear agg = Wt2 hsum + bscale bt2, gnn.py:188-190), node_mlp_2
//      over [x_t, agg, u[g]] (gnn.py:191; fp32 FMA chains in k order), its
//      Welford partials, and the unit's share of the graph sums of x_s and of
//      the pre-norm output;
//   2. every workgroup merges the partials in one fixed order (bn_stats_part;
//      workgroup 0 writes mu / var / running statistics), normalises its
//      classes (gnn.py:192), runs the GlobalModel of its graph (gnn.py:218-223;
//      the mean of x_t from the pre-norm sums -- the norm is affine per
//      channel) and the next block's Pt / Qt (gnn.py:100, 136) of its classes.
// One launch for what were reduce_columns_lin + mlp_fwd + class_global_fwd.
constexpr int CT_QBMAX = 64;                // most units per graph (NC <= 64 * CT)
constexpr int CT_CLS = 32;                  // most classes per unit (8, 16 or 32: the
                                            // smallest that keeps the units <= 512)
// Device-wide barrier state: a pool of slots, one 128-byte line each; every
// launch of a barrier kernel takes the next slot (pf::bar_slot(), round robin
// on the host), so two such launches share no word as long as fewer than
// PF_BAR_SLOTS of them are in flight at once (a captured step holds 7).  The
// round-robin counter is plain host state: launches come from ONE host thread
// (the library's contract, include/pfsgnn.h).  Word 0: arrivals | generation << 16
// (default form); words 1, 2: arrivals, generation (fenced form).  A slot is
// clean between launches: the last arrival of every barrier resets the count.
constexpr int PF_BAR_SLOTS = 64;
__device__ unsigned pf_bar_pool[PF_BAR_SLOTS][32];
__device__ unsigned pf_sync_fault_count;    // barrier time-outs (sticky)

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "grid_sync's sc1 hand-off is measured for gfx950 only (MI355X_MICROARCH.md)"
#endif

// Every workgroup of the grid waits here.  The launchers check that the grid
// is co-resident (pf::check_coresident: at most the occupancy API's blocks per
// CU times the CUs); a wait that still outlives ~2^24 sleeps (~1.5 s) means a
// workgroup was never scheduled -- another process holding the CUs -- and
// the kernel stops: the sticky fault count is raised and the wave traps, so
// the launch fails (hipErrorLaunchFailure) instead of going on with partials
// that were never handed over.
// Default (fenced = 0): no cache maintenance.  Every byte handed across the
// barrier is stored and loaded with agent-scope relaxed atomics (global_store /
// load sc1: st_sc1 / ld_sc1), every wave waits for its stores (vmcnt(0)) before
// the workgroup barrier, one lane counts the workgroup in with a relaxed
// agent-scope add, and the last arrival -- told by the value its add returned
// -- resets the count and bumps the generation in one add on the same word
// (arrivals in the low 16 bits), which the others poll with sc1 loads (MI355X_MICROARCH.md,
// the sc1 hand-off table's first row).
// fenced = 1 (pfsgnn_set_grid_sync_fenced / PFSGNN_GRID_SYNC_FENCED=1): the
// arrival is an agent-scope acq_rel add and the poll an acquire -- an L2
// write-back and an L1 invalidate per workgroup and barrier (grid_sync_probe:
// 4.6 us at 64 workgroups, 15.6 at 256).  Both forms give bitwise the same
// results (tests/test_gpu_grid_sync.py).
__device__ __forceinline__ void grid_sync_fault() {
  __hip_atomic_fetch_add(&pf_sync_fault_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_trap();
}
__device__ void grid_sync(unsigned* bar, unsigned nb, int fenced) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (fenced) {
      const unsigned gen = __hip_atomic_load(&bar[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned a = __hip_atomic_fetch_add(&bar[1], 1u, __ATOMIC_ACQ_REL,
                                                __HIP_MEMORY_SCOPE_AGENT);
      if (a == nb - 1) {
        __hip_atomic_store(&bar[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&bar[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        unsigned spins = 0;
        while (__hip_atomic_load(&bar[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) {
          __builtin_amdgcn_s_sleep(4);
          if (++spins > (1u << 24)) grid_sync_fault();
        }
      }
    } else {
      // one word: arrivals in the low 16 bits, the generation above; the last
      // arrival resets the count and bumps the generation in ONE add
      unsigned* w = &bar[0];
      const unsigned a = __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned gen = a >> 16;
      if ((a & 0xffffu) == nb - 1) {
        __hip_atomic_fetch_add(w, 0x10000u - nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        unsigned spins = 0;
        while ((__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 16) == gen) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > (1u << 24)) grid_sync_fault();
        }
      }
    }
  }
  __syncthreads();
}

#ifdef PF_TAIL_STAMPS   // (diagnostic build: per-workgroup phase clocks, tools/tail_stamps.py)
__device__ unsigned long long pf_tail_stamps[512][8];
__device__ unsigned long long pf_cb_stamps[512][8];
#define TAIL_STAMP(i) \
  if (threadIdx.x == 0) pf_tail_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime();
#define CB_STAMP(i) \
  if (threadIdx.x == 0) pf_cb_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime();
#else
#define TAIL_STAMP(i)
#define CB_STAMP(i)
#endif

struct TailArgs {
  pfsgnn_block_tail a;
  const float* cpart;   // [G][BPG][NC][2F] the edge kernel's column partials
  int BPG, CT, QB, nunits;   // CT classes per unit, QB units per graph
  float bscale;
  float *part, *xss, *yps;   // [nunits][PART_LEN], [nunits][F], [nunits][F] (sc1 hand-off)
  int fenced;                // grid_sync form
  unsigned* bar;             // grid_sync slot (pf_bar_pool)
};

template <int F>
__global__ __launch_bounds__(256) void k_class_tail_fwd(TailArgs T) {
  constexpr int C2 = 2 * F, K = 4 * F, H = 4 * F, K3 = 3 * F;
  const pfsgnn_block_tail& A = T.a;
  const int t = threadIdx.x, G = A.G, NC = A.NC, NF = A.NF;
  const long long NT = (long long)G * NC, NS = (long long)G * NF;
  TAIL_STAMP(0)
  __shared__ float w1[H * K], w2[F * H], wt2[C2 * C2], bb1[H], bb2[F], bt[C2];
  __shared__ float xin[CT_CLS][K + 1], act[CT_CLS][H + 1], ypl[CT_CLS][F + 1];
  __shared__ float hs[CT_CLS][C2 + 1];
  __shared__ float red[4][F];
  // every weight load of the thread in flight before the first LDS store (a
  // load -> store loop pays one round trip per element)
  const bool gws = A.gH * K3 <= CG_GW1;
  __shared__ float gw1[CG_GW1], gw2[F * CG_MAXH];
  constexpr int N1 = (H * K + 255) / 256, N2 = (F * H + 255) / 256, N3 = (C2 * C2 + 255) / 256;
  constexpr int NG1 = (CG_GW1 + 255) / 256, NG2 = (F * CG_MAXH + 255) / 256;
  float v1[N1], v2[N2], v3[N3], g1[NG1], g2[NG2];
  float b1v, b2v, btv;
  {
    const int ng1 = gws ? A.gH * K3 : 0, ng2 = gws ? F * A.gH : 0;
#pragma unroll
    for (int i = 0; i < N1; ++i) v1[i] = t + 256 * i < H * K ? A.W1[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < N2; ++i) v2[i] = t + 256 * i < F * H ? A.W2[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < N3; ++i) v3[i] = t + 256 * i < C2 * C2 ? A.Wt2[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < NG1; ++i) g1[i] = t + 256 * i < ng1 ? A.gW1[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < NG2; ++i) g2[i] = t + 256 * i < ng2 ? A.gW2[t + 256 * i] : 0.f;
    b1v = t < H ? A.b1[t] : 0.f;
    b2v = t < F ? A.b2[t] : 0.f;
    btv = t < C2 ? A.bt2[t] : 0.f;
  }
  {
    const int ng1 = gws ? A.gH * K3 : 0, ng2 = gws ? F * A.gH : 0;
#pragma unroll
    for (int i = 0; i < N1; ++i) if (t + 256 * i < H * K) w1[t + 256 * i] = v1[i];
#pragma unroll
    for (int i = 0; i < N2; ++i) if (t + 256 * i < F * H) w2[t + 256 * i] = v2[i];
#pragma unroll
    for (int i = 0; i < N3; ++i) if (t + 256 * i < C2 * C2) wt2[t + 256 * i] = v3[i];
#pragma unroll
    for (int i = 0; i < NG1; ++i) if (t + 256 * i < ng1) gw1[t + 256 * i] = g1[i];
#pragma unroll
    for (int i = 0; i < NG2; ++i) if (t + 256 * i < ng2) gw2[t + 256 * i] = g2[i];
    if (t < H) bb1[t] = b1v;
    if (t < F) bb2[t] = b2v;
    if (t < C2) bt[t] = btv;
  }
  __syncthreads();
  // the next block's weight blocks: We[:, F:2F], We[:, 3F:4F], be, Ws[:, 0:F], bs
  __shared__ float wet[4 * F * F], weu[4 * F * F], wbe[4 * F], wst[2 * F * F], wbs[2 * F];
  if (A.We) {
    constexpr int NE = (4 * F * F + 255) / 256, NS2 = (2 * F * F + 255) / 256;
    float e1[NE], e2[NE], e3[NS2];
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int x = t + 256 * i, k = x / F, o = x - k * F;
      e1[i] = x < 4 * F * F ? A.We[(size_t)k * 4 * F + F + o] : 0.f;
      e2[i] = x < 4 * F * F ? A.We[(size_t)k * 4 * F + 3 * F + o] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NS2; ++i) {
      const int x = t + 256 * i, k = x / F, o = x - k * F;
      e3[i] = x < 2 * F * F ? A.Ws[(size_t)k * 2 * F + o] : 0.f;
    }
    const float bev = t < 4 * F ? A.be[t] : 0.f, bsv = t < 2 * F ? A.bs[t] : 0.f;
#pragma unroll
    for (int i = 0; i < NE; ++i)
      if (t + 256 * i < 4 * F * F) { wet[t + 256 * i] = e1[i]; weu[t + 256 * i] = e2[i]; }
#pragma unroll
    for (int i = 0; i < NS2; ++i)
      if (t + 256 * i < 2 * F * F) wst[t + 256 * i] = e3[i];
    if (t < 4 * F) wbe[t] = bev;
    if (t < 2 * F) wbs[t] = bsv;
  }
  TAIL_STAMP(1)
  // ---------------------------------------------------------------- phase 1
  for (int un = blockIdx.x; un < T.nunits; un += gridDim.x) {
    const int g = un / T.QB, q = un - g * T.QB;
    const int c0 = q * T.CT, ncl = min(T.CT, NC - c0);
    const long long nb = (long long)g * NC + c0;
    // per-class sums of the column partials, in partial order (32 loads of a
    // thread in flight at once: this is the phase's latency)
    for (int i = t; i < ncl * C2; i += 256) {
      const int cl = i / C2, j = i - cl * C2;
      const float* p = T.cpart + ((size_t)g * T.BPG * NC + c0 + cl) * C2 + j;
      const size_t bs = (size_t)NC * C2;
      float s = 0.f;
      for (int b = 0; b < T.BPG; b += 32) {
        float v[32];
#pragma unroll
        for (int e = 0; e < 32; ++e) v[e] = b + e < T.BPG ? p[(size_t)(b + e) * bs] : 0.f;
#pragma unroll
        for (int e = 0; e < 32; ++e) s += v[e];
      }
      hs[cl][j] = s;
      A.hsum[(size_t)j * NT + nb + cl] = s;
    }
    TAIL_STAMP(2)
    for (int i = t; i < ncl * F; i += 256) {
      const int o = i / ncl, cl = i - o * ncl;
      xin[cl][o] = A.xt[(size_t)o * NT + nb + cl];
      xin[cl][3 * F + o] = A.u[(size_t)o * G + g];
    }
    // the unit's share of graph g's x_s sums (fibers [f0, f1))
    {
      const int f0 = (int)(((long long)NF * q) / T.QB), f1 = (int)(((long long)NF * (q + 1)) / T.QB);
      float sx[F];
#pragma unroll
      for (int o = 0; o < F; ++o) sx[o] = 0.f;
      for (int f = f0 + t; f < f1; f += 256) {
#pragma unroll
        for (int o = 0; o < F; ++o) sx[o] += A.xs[(size_t)o * NS + (size_t)g * NF + f];
      }
      const int wv = t >> 6, ln = t & 63;
#pragma unroll
      for (int o = 0; o < F; ++o) {
        const float v = wave_sum(sx[o]);
        if (ln == 0) red[wv][o] = v;
      }
    }
    __syncthreads();
    if (t < F) st_sc1(T.xss + (size_t)un * F + t, ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t]);
    // agg = Wt2 hsum + bscale bt2 (the MLP input's middle block)
    for (int i = t; i < ncl * C2; i += 256) {
      const int k = i / ncl, cl = i - k * ncl;
      float acc = T.bscale * bt[k];
#pragma unroll
      for (int j = 0; j < C2; ++j) acc = fmaf(wt2[k * C2 + j], hs[cl][j], acc);
      xin[cl][F + k] = acc;
      A.agg[(size_t)k * NT + nb + cl] = acc;
    }
    __syncthreads();
    // node_mlp_2: Z = W1 x + b1, a = lrelu(Z)
    for (int i = t; i < ncl * H; i += 256) {
      const int h = i / ncl, cl = i - h * ncl;
      float z = bb1[h];
#pragma unroll
      for (int k = 0; k < K; ++k) z = fmaf(w1[h * K + k], xin[cl][k], z);
      A.Z[(size_t)h * NT + nb + cl] = z;
      act[cl][h] = lrelu(z);
    }
    __syncthreads();
    // Yp = W2 a + b2
    for (int i = t; i < ncl * F; i += 256) {
      const int o = i / ncl, cl = i - o * ncl;
      float y = bb2[o];
#pragma unroll
      for (int h = 0; h < H; ++h) y = fmaf(w2[o * H + h], act[cl][h], y);
      A.Yp[(size_t)o * NT + nb + cl] = y;
      ypl[cl][o] = y;
    }
    __syncthreads();
    // Welford partial of the unit's classes (bn_stats_part's layout) and the
    // pre-norm sums for the x_t mean
    if (t < 16) {
      float* pp = T.part + (size_t)un * PART_LEN;
      if (t < F) {
        float mean = 0.f, m2 = 0.f, sum = 0.f;
        for (int cl = 0; cl < ncl; ++cl) {
          const float v = ypl[cl][t];
          const float d = v - mean;
          mean = fmaf(d, 1.f / (float)(cl + 1), mean);
          m2 = fmaf(d, v - mean, m2);
          sum += v;
        }
        st_sc1(pp + 1 + t, mean);
        st_sc1(pp + 17 + t, m2);
        st_sc1(T.yps + (size_t)un * F + t, sum);
      } else {
        st_sc1(pp + 1 + t, 0.f);
        st_sc1(pp + 17 + t, 0.f);
      }
      if (t == 0) st_sc1(pp, (float)ncl);
    }
    __syncthreads();   // (LDS reuse by the next unit)
  }
  TAIL_STAMP(3)
  grid_sync(T.bar, gridDim.x, T.fenced);
  TAIL_STAMP(4)
  // ---------------------------------------------------------------- phase 2
  __shared__ float cf[4][16];
  __shared__ float qs[2][CT_QBMAX * F];   // a graph's xss / yps unit sums
  // the graph's unit sums: every load in flight at once (one memory round
  // trip, not QB serial ones), then summed in unit order; for the block's
  // first unit issued before the statistics merge, with its Yp
  auto stage_qs = [&](int g) {
    for (int i = t; i < 2 * F * T.QB; i += 256) {
      const int w = i / (F * T.QB), r = i - w * F * T.QB;
      qs[w][r] = ld_sc1((w ? T.yps : T.xss) + (size_t)g * T.QB * F + r);
    }
  };
  float yp0 = 0.f;
  if ((int)blockIdx.x < T.nunits) {
    const int un = blockIdx.x, g = un / T.QB, q = un - g * T.QB;
    const int c0 = q * T.CT, ncl = min(T.CT, NC - c0);
    if (t < ncl * F) {
      const int o = t / ncl, cl = t - o * ncl;
      yp0 = A.Yp[(size_t)o * NT + (long long)g * NC + c0 + cl];
    }
    stage_qs(g);
  }
  bn_stats_part<true>(T.part, T.nunits, F, (int)NT, A.gamma, A.beta, A.eps, A.rm, A.rv, A.momentum,
                A.mu, A.var, blockIdx.x == 0, cf);   // (its barriers publish qs)
  TAIL_STAMP(5)
  __shared__ float h3[K3], gz[CG_MAXH], vv[F], un3[F], cu[4 * F], zz[F], rs2[2];
  float* xn = &ypl[0][0];   // [CT_CLS][F + 1]: the normalised x_t of the unit
  for (int un = blockIdx.x; un < T.nunits; un += gridDim.x) {
    const int g = un / T.QB, q = un - g * T.QB;
    const int c0 = q * T.CT, ncl = min(T.CT, NC - c0);
    const long long nb = (long long)g * NC + c0;
    const bool first = un == (int)blockIdx.x;
    for (int i = t; i < ncl * F; i += 256) {
      const int o = i / ncl, cl = i - o * ncl;
      const float y = (first && i == t) ? yp0 : A.Yp[(size_t)o * NT + nb + cl];
      const float v = (y - cf[0][o]) * (cf[1][o] * cf[2][o]) + cf[3][o];
      A.xt_new[(size_t)o * NT + nb + cl] = v;
      xn[cl * (F + 1) + o] = v;
    }
    if (!first) stage_qs(g);
    __syncthreads();
    if (t < F) {
      float sx = 0.f, sy = 0.f;
      for (int qq = 0; qq < T.QB; ++qq) {
        sx += qs[0][qq * F + t];
        sy += qs[1][qq * F + t];
      }
      const float mx = sx / (float)NF;
      const float mt = (sy / (float)NC - cf[0][t]) * (cf[1][t] * cf[2][t]) + cf[3][t];
      h3[t] = A.u[(size_t)t * G + g];
      h3[F + t] = mx;
      h3[2 * F + t] = mt;
      if (q == 0) {
        A.means[(size_t)t * G + g] = mx;
        A.means[(size_t)(F + t) * G + g] = mt;
      }
    }
    __syncthreads();
    // GlobalModel MLP(3F -> gH -> F) of graph g
    for (int j = t; j < A.gH; j += 256) {
      float acc = A.gb1[j];
      for (int k = 0; k < K3; ++k)
        acc = fmaf(gws ? gw1[j * K3 + k] : A.gW1[(size_t)j * K3 + k], h3[k], acc);
      gz[j] = acc;
      if (q == 0) A.gZ[(size_t)j * G + g] = acc;
    }
    __syncthreads();
    if (t < F) {
      float acc = A.gb2[t];
      for (int j = 0; j < A.gH; ++j)
        acc = fmaf(gws ? gw2[t * A.gH + j] : A.gW2[(size_t)t * A.gH + j], lrelu(gz[j]), acc);
      vv[t] = acc;
      if (q == 0) A.gV[(size_t)t * G + g] = acc;
    }
    __syncthreads();
    if (t == 0) {   // RMSNorm twice (k_rms2_fwd's arithmetic)
      if (!A.gw) {
        for (int c = 0; c < F; ++c) un3[c] = vv[c];
      } else {
        float s = 0.f;
        for (int c = 0; c < F; ++c) s += vv[c] * vv[c];
        const float a = rsqrtf(s / F + A.reps);
        float s2 = 0.f;
        for (int c = 0; c < F; ++c) {
          const float qv = vv[c] * a * A.gw[c];
          zz[c] = qv;
          s2 += qv * qv;
        }
        const float b = rsqrtf(s2 / F + A.reps);
        for (int c = 0; c < F; ++c) un3[c] = zz[c] * b * A.gw[c];
        rs2[0] = a;
        rs2[1] = b;
      }
    }
    __syncthreads();
    if (q == 0) {
      if (t < F) {
        A.unew[(size_t)t * G + g] = un3[t];
        if (A.gw) A.y1[(size_t)t * G + g] = zz[t];
      }
      if (A.gw && t == 0) {
        A.r1[g] = rs2[0];
        A.r2[g] = rs2[1];
      }
    }
    if (A.We) {
      if (t < 4 * F) {
        float acc = wbe[t];
#pragma unroll
        for (int o = 0; o < F; ++o) acc = fmaf(weu[t * F + o], un3[o], acc);
        cu[t] = acc;
      }
      __syncthreads();
      for (int i = t; i < ncl * 4 * F; i += 256) {
        const int k = i / ncl, cl = i - k * ncl;
        float acc = cu[k];
#pragma unroll
        for (int o = 0; o < F; ++o) acc = fmaf(wet[k * F + o], xn[cl * (F + 1) + o], acc);
        A.Pt[(size_t)k * NT + nb + cl] = acc;
      }
      for (int i = t; i < ncl * 2 * F; i += 256) {
        const int k = i / ncl, cl = i - k * ncl;
        float acc = wbs[k];
#pragma unroll
        for (int o = 0; o < F; ++o) acc = fmaf(wst[k * F + o], xn[cl * (F + 1) + o], acc);
        A.Qt[(size_t)k * NT + nb + cl] = acc;
      }
    }
    __syncthreads();   // (LDS reuse by the next unit)
  }
  TAIL_STAMP(6)
}

// ---------------------------------------------------------------- fused class backward
// pfsgnn_target_class_bwd: the class side of a block's backward in one launch
// (include/pfsgnn.h), units of CB_CLS classes of one graph, three phases
// around two device-wide barriers (the per-graph u-gradient sums feed the
// GlobalModel backward; TModel's BatchNorm sums need every class).
constexpr int CB_CLS = 16;
constexpr int CB_QBMAX = 64;   // most units per graph (NC <= 1024)
constexpr int CB_PLEN = 32;   // BatchNorm-sum partial: sg[16], sx[16]

struct CbArgs {
  pfsgnn_class_bwd a;
  int QB, nunits;
  float *p1, *p2;   // [nunits][F] u-gradient partials, [nunits][CB_PLEN] BatchNorm sums (sc1)
  int fenced;       // grid_sync form
  unsigned* bar;    // grid_sync slot (pf_bar_pool)
};

template <int F>
__global__ __launch_bounds__(256) void k_class_bwd(CbArgs T) {
  constexpr int C2 = 2 * F, K = 4 * F, H = 4 * F, K3 = 3 * F;
  const pfsgnn_class_bwd& A = T.a;
  const int t = threadIdx.x, G = A.G, NC = A.NC, NF = A.NF;
  const long long NT = (long long)G * NC, NS = (long long)G * NF;
  CB_STAMP(0)
  __shared__ float w1[H * K], w2[F * H], wt2[C2 * C2];
  __shared__ float gw1[CG_GW1], gw2[F * CG_MAXH];
  const bool gws = A.gH * K3 <= CG_GW1;
  {  // every weight load in flight before the LDS stores
    constexpr int N1 = (H * K + 255) / 256, N2 = (F * H + 255) / 256, N3 = (C2 * C2 + 255) / 256;
    constexpr int NG1 = (CG_GW1 + 255) / 256, NG2 = (F * CG_MAXH + 255) / 256;
    float v1[N1], v2[N2], v3[N3], g1[NG1], g2[NG2];
    const int ng1 = gws ? A.gH * K3 : 0, ng2 = gws ? F * A.gH : 0;
#pragma unroll
    for (int i = 0; i < N1; ++i) v1[i] = t + 256 * i < H * K ? A.W1[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < N2; ++i) v2[i] = t + 256 * i < F * H ? A.W2[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < N3; ++i) v3[i] = t + 256 * i < C2 * C2 ? A.Wt2[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < NG1; ++i) g1[i] = t + 256 * i < ng1 ? A.gW1[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < NG2; ++i) g2[i] = t + 256 * i < ng2 ? A.gW2[t + 256 * i] : 0.f;
#pragma unroll
    for (int i = 0; i < N1; ++i) if (t + 256 * i < H * K) w1[t + 256 * i] = v1[i];
#pragma unroll
    for (int i = 0; i < N2; ++i) if (t + 256 * i < F * H) w2[t + 256 * i] = v2[i];
#pragma unroll
    for (int i = 0; i < N3; ++i) if (t + 256 * i < C2 * C2) wt2[t + 256 * i] = v3[i];
#pragma unroll
    for (int i = 0; i < NG1; ++i) if (t + 256 * i < ng1) gw1[t + 256 * i] = g1[i];
#pragma unroll
    for (int i = 0; i < NG2; ++i) if (t + 256 * i < ng2) gw2[t + 256 * i] = g2[i];
  }
  __shared__ float red[4][F];
  CB_STAMP(1)
  // ---------------------------------------------------------------- phase 1
  // the unit's share of its graph's sums of the pending u[batch] gradients
  for (int un = blockIdx.x; un < T.nunits; un += gridDim.x) {
    const int g = un / T.QB, q = un - g * T.QB;
    float s[F];
#pragma unroll
    for (int o = 0; o < F; ++o) s[o] = 0.f;
    for (int i = 0; i < A.npend; ++i) {
      const int n = A.pend_n[i];
      const int b0 = (int)(((long long)n * q) / T.QB), b1 = (int)(((long long)n * (q + 1)) / T.QB);
      const float* X = A.pend[i];
      const long long ld = (long long)G * n;
      for (int j = b0 + t; j < b1; j += 256) {
#pragma unroll
        for (int o = 0; o < F; ++o) s[o] += X[(size_t)o * ld + (size_t)g * n + j];
      }
    }
    const int wv = t >> 6, ln = t & 63;
#pragma unroll
    for (int o = 0; o < F; ++o) {
      const float v = wave_sum(s[o]);
      if (ln == 0) red[wv][o] = v;
    }
    __syncthreads();
    if (t < F) st_sc1(T.p1 + (size_t)un * F + t, ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t]);
    __syncthreads();
  }
  CB_STAMP(2)
  grid_sync(T.bar, gridDim.x, T.fenced);
  CB_STAMP(3)
  // ---------------------------------------------------------------- phase 2
  __shared__ float sdy[F], sy1[F], sv[F], sw[F], sdw[F], gv[F], d1[F];
  __shared__ float dzg[CG_MAXH], dh[CG_MAXH];
  __shared__ float ps1[CB_QBMAX * F];
  for (int un = blockIdx.x; un < T.nunits; un += gridDim.x) {
    const int g = un / T.QB, q = un - g * T.QB;
    const int c0 = q * CB_CLS, ncl = min(CB_CLS, NC - c0);
    const long long nb = (long long)g * NC + c0;
    // the unit's later operands loaded up front (their latency behind the
    // GlobalModel backward): gZ, and the x_t gradient / Yp / statistics of
    // the BatchNorm sums below
    const float gzv = t < A.gH ? A.gZ[(size_t)t * G + g] : 0.f;
    const int xo = t / CB_CLS, xcl = t - xo * CB_CLS;
    const bool xlive = t < F * CB_CLS && xcl < ncl;
    float* const xp = A.g_xt + (size_t)xo * NT + nb + xcl;
    const float xtv = xlive ? *xp : 0.f;
    const float ypv = xlive ? A.Yp[(size_t)xo * NT + nb + xcl] : 0.f;
    const float vrv = xlive ? A.var[xo] : 0.f, muv = xlive ? A.mu[xo] : 0.f;
    // the graph's unit partials: every load in flight at once, summed in unit order
    for (int i = t; i < F * T.QB; i += 256) ps1[i] = ld_sc1(T.p1 + (size_t)g * T.QB * F + i);
    __syncthreads();
    if (t < F) {
      float sacc = A.gu_up[(size_t)t * G + g];
      for (int qq = 0; qq < T.QB; ++qq) sacc += ps1[qq * F + t];
      sdy[t] = sacc;
      if (A.w) {
        sy1[t] = A.y1[(size_t)t * G + g];
        sv[t] = A.V[(size_t)t * G + g];
        sw[t] = A.w[t];
      }
    }
    __syncthreads();
    // GlobalModel backward (k_global_bwd's arithmetic): RMSNorm twice, then the MLP
    if (!A.w) {
      if (t < F) gv[t] = sdy[t];
    } else if (t == 0) {
      const float a = A.r1[g], b = A.r2[g];
      float dot = 0.f;
      for (int c = 0; c < F; ++c) {
        const float dy = sdy[c], x = sy1[c];
        sdw[c] = dy * x * b;
        dot += dy * sw[c] * x;
      }
      float dot2 = 0.f;
      for (int c = 0; c < F; ++c) {
        const float dy = sdy[c], x1 = sy1[c];
        const float qv = b * dy * sw[c] - x1 * b * b * b * dot / F;
        d1[c] = qv;
        const float x0 = sv[c];
        sdw[c] += qv * x0 * a;
        dot2 += qv * sw[c] * x0;
      }
      for (int c = 0; c < F; ++c) {
        const float x0 = sv[c];
        gv[c] = a * d1[c] * sw[c] - x0 * a * a * a * dot2 / F;
      }
    }
    __syncthreads();
    if (q == 0 && t < F) {
      if (A.w) A.dwp[(size_t)t * G + g] = sdw[t];
      A.gV[(size_t)t * G + g] = gv[t];
    }
    for (int j = t; j < A.gH; j += 256) {
      float acc = 0.f;
      for (int o = 0; o < F; ++o) acc = fmaf(gws ? gw2[o * A.gH + j] : A.gW2[(size_t)o * A.gH + j], gv[o], acc);
      const float qv = acc * dlrelu(j == t ? gzv : A.gZ[(size_t)j * G + g]);
      dzg[j] = qv;
      if (q == 0) A.gdZ[(size_t)j * G + g] = qv;
    }
    __syncthreads();
    for (int k = t; k < K3; k += 256) {
      float acc = 0.f;
      for (int j = 0; j < A.gH; ++j)
        acc = fmaf(gws ? gw1[j * K3 + k] : A.gW1[(size_t)j * K3 + k], dzg[j], acc);
      dh[k] = acc;
    }
    __syncthreads();
    if (q == 0 && t < F) A.gu[(size_t)t * G + g] += dh[t];
    // the means' gradients broadcast: x_s over the unit's fiber share, x_t over its classes
    // (the read-modify-writes 8 per thread at a time: their loads in flight together)
    {
      const int f0 = (int)(((long long)NF * q) / T.QB), f1 = (int)(((long long)NF * (q + 1)) / T.QB);
      const int nf = f1 - f0, n = nf * F;
      auto at = [&](int i) {
        const int o = i / nf, f = f0 + (i - o * nf);
        return A.g_xs + (size_t)o * NS + (size_t)g * NF + f;
      };
      for (int i0 = t; i0 < n; i0 += 256 * 8) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = i0 + 256 * e;
          v[e] = i < n ? *at(i) : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = i0 + 256 * e;
          if (i < n) *at(i) = v[e] + dh[F + i / nf] * (1.0f / (float)NF);
        }
      }
    }
    // TModel's BatchNorm sums on the updated g_xt (k_bn_sums_part's arithmetic)
    float sg = 0.f, sx = 0.f;
    if (xlive) {
      const float v = xtv + dh[2 * F + xo] * (1.0f / (float)NC);
      *xp = v;
      const float ic = 1.0f / sqrtf(vrv + A.eps);
      sg = v;
      sx = v * ((ypv - muv) * ic);
    }
    // per channel over the unit's classes: 16 consecutive lanes hold one channel
#pragma unroll
    for (int off = 1; off < CB_CLS; off <<= 1) {
      sg += __shfl_xor(sg, off);
      sx += __shfl_xor(sx, off);
    }
    if (t < F * CB_CLS && (t % CB_CLS) == 0) {
      const int o = t / CB_CLS;
      st_sc1(T.p2 + (size_t)un * CB_PLEN + o, sg);
      st_sc1(T.p2 + (size_t)un * CB_PLEN + 16 + o, sx);
    }
    __syncthreads();   // (LDS reuse by the next unit)
  }
  CB_STAMP(4)
  grid_sync(T.bar, gridDim.x, T.fenced);
  CB_STAMP(5)
  // ---------------------------------------------------------------- phase 3
  __shared__ float BC[5][16];
  __shared__ float mg[16][16], mx[16][16];
  {  // the units' sums merged in one fixed order: 16 subsets of units (loads
     // of a subset in flight together), then the subsets in order
    const int o = t & 15, u0 = t >> 4;
    float sg = 0.f, sx = 0.f;
    for (int u = u0; u < T.nunits; u += 64) {
      float a[4], b[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int uu = u + 16 * e;
        a[e] = uu < T.nunits ? ld_sc1(T.p2 + (size_t)uu * CB_PLEN + o) : 0.f;
        b[e] = uu < T.nunits ? ld_sc1(T.p2 + (size_t)uu * CB_PLEN + 16 + o) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sg += a[e];
        sx += b[e];
      }
    }
    mg[u0][o] = sg;
    mx[u0][o] = sx;
  }
  __syncthreads();
  if (t < F) {
    float sg = 0.f, sx = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      sg += mg[k][t];
      sx += mx[k][t];
    }
    const float inv = 1.0f / sqrtf(A.var[t] + A.eps);
    BC[0][t] = A.gamma[t] * inv;
    BC[1][t] = sg / (float)NT;
    BC[2][t] = sx / (float)NT;
    BC[3][t] = A.mu[t];
    BC[4][t] = inv;
    if (blockIdx.x == 0) {
      A.dgamma[t] += sx;
      A.dbeta[t] += sg;
    }
  }
  __shared__ float gp[CB_CLS][F + 1], dzl[CB_CLS][H + 1], gag[CB_CLS][C2 + 1];
  __syncthreads();
  for (int un = blockIdx.x; un < T.nunits; un += gridDim.x) {
    const int g = un / T.QB, q = un - g * T.QB;
    const int c0 = q * CB_CLS, ncl = min(CB_CLS, NC - c0);
    const long long nb = (long long)g * NC + c0;
    for (int i = t; i < ncl * F; i += 256) {
      const int o = i / ncl, cl = i - o * ncl;
      const size_t e = (size_t)o * NT + nb + cl;
      const float v = BC[0][o] * (A.g_xt[e] - BC[1][o] - (A.Yp[e] - BC[3][o]) * BC[4][o] * BC[2][o]);
      A.dYp[e] = v;
      gp[cl][o] = v;
    }
    __syncthreads();
    {  // (every Z load of the thread issued before the first store)
      constexpr int NZ = (CB_CLS * H + 255) / 256;
      float zv[NZ];
#pragma unroll
      for (int e = 0; e < NZ; ++e) {
        const int i = t + 256 * e, h = i / max(ncl, 1), cl = i - h * ncl;
        zv[e] = i < ncl * H ? A.Z[(size_t)h * NT + nb + cl] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < NZ; ++e) {
        const int i = t + 256 * e;
        if (i >= ncl * H) continue;
        const int h = i / ncl, cl = i - h * ncl;
        float acc = 0.f;
#pragma unroll
        for (int o = 0; o < F; ++o) acc = fmaf(w2[o * H + h], gp[cl][o], acc);
        const float v = acc * dlrelu(zv[e]);
        A.dZ[(size_t)h * NT + nb + cl] = v;
        dzl[cl][h] = v;
      }
    }
    __syncthreads();
    for (int i = t; i < ncl * K; i += 256) {
      const int k = i / ncl, cl = i - k * ncl;
      float acc = 0.f;
#pragma unroll
      for (int h = 0; h < H; ++h) acc = fmaf(w1[h * K + k], dzl[cl][h], acc);
      if (k < F) {
        float* p = A.gxt_in + (size_t)k * NT + nb + cl;
        *p = *p + acc;
      } else if (k < 3 * F) {
        A.g_agg[(size_t)(k - F) * NT + nb + cl] = acc;
        gag[cl][k - F] = acc;
      } else {
        A.gu_t[(size_t)(k - 3 * F) * NT + nb + cl] = acc;
      }
    }
    __syncthreads();
    for (int i = t; i < ncl * C2; i += 256) {
      const int j = i / ncl, cl = i - j * ncl;
      float acc = 0.f;
#pragma unroll
      for (int m = 0; m < C2; ++m) acc = fmaf(wt2[m * C2 + j], gag[cl][m], acc);
      A.g_hsum[(size_t)j * NT + nb + cl] = acc;
    }
    __syncthreads();   // (LDS reuse by the next unit)
  }
  CB_STAMP(6)
}

// ============================================================ backward
// BatchNorm backward sums per block: Sg[c] = sum dY, Sgx[c] = sum dY * xhat.
constexpr int SUM_LEN = 32;
__global__ __launch_bounds__(256) void k_bn_sums_part(const float* __restrict__ dY,
                                                      const float* __restrict__ Yp, int O, int N,
                                                      const float* __restrict__ mu,
                                                      const float* __restrict__ var, float eps,
                                                      float* __restrict__ part) {
  const int t = threadIdx.x;
  float sg[16], sx[16], mc[16], ic[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    sg[c] = sx[c] = 0.f;
    mc[c] = c < O ? mu[c] : 0.f;
    ic[c] = c < O ? 1.0f / sqrtf(var[c] + eps) : 0.f;
  }
  for (int n = blockIdx.x * 256 + t; n < N; n += gridDim.x * 256) {
    float g[16], y[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      g[c] = c < O ? dY[(size_t)c * N + n] : 0.f;
      y[c] = c < O ? Yp[(size_t)c * N + n] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      sg[c] += g[c];
      sx[c] += g[c] * ((y[c] - mc[c]) * ic[c]);
    }
  }
  __shared__ float scratch[4 * 32];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    sg[c] = wave_sum(sg[c]);
    sx[c] = wave_sum(sx[c]);
  }
  const int wave = t >> 6, lane = t & 63;
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      scratch[wave * 32 + c] = sg[c];
      scratch[wave * 32 + 16 + c] = sx[c];
    }
  }
  __syncthreads();
  if (t < 32)
    part[(size_t)blockIdx.x * SUM_LEN + t] =
        ((scratch[t] + scratch[32 + t]) + scratch[64 + t]) + scratch[96 + t];
}

// Rows [kb, ke) of a chunk's input gradient, staged in LDS (row k at
// X + (k - kx) * XS_LD, the chunk's 64 nodes), to their output blocks: lane
// (q, j) takes rows kb + 16 i + 4 wu + q, nodes n0 + 4 j .. + 3 (R >= the
// rows' 16-row rounds).  Every add block's old values are loaded before the
// first store, so a wave waits once per call, not once per row.
template <int R>
__device__ __forceinline__ void store_rows(const RowOut* tab, const float* X, int kx, int kb,
                                           int ke, int n0, int N, int wu, int lane) {
  const int q = lane >> 4, j = lane & 15, nb = n0 + 4 * j;
  float* p[R];
  bool ad[R];
  float o[R][4];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = kb + 16 * i + 4 * wu + q;
    const RowOut d = r < ke ? tab[r] : RowOut{nullptr, 0, 0};
    p[i] = d.p;
    ad[i] = d.p && d.add;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[i][e] = (ad[i] && nb + e < N) ? d.p[nb + e] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    if (!p[i]) continue;
    const int r = kb + 16 * i + 4 * wu + q;
    const floatx4 v = *reinterpret_cast<const floatx4*>(X + (r - kx) * XS_LD + 4 * j);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (nb + e < N) p[i][nb + e] = ad[i] ? o[i][e] + v[e] : v[e];
  }
}

// RS (the wide MLPs, M >= 5): no LDS staging of the input gradient -- each
// lane writes its rows straight from the MFMA output layout (64-byte row
// segments) -- the output tiles in groups of 4 and no prefetch of Z, so the
// kernel fits 256 registers and 2 blocks per CU (LDS: the weight images only).
// X3 (RS only): both gradient chains, dZ = W2^T dYp and dX = W1^T dZ, on
// split-bf16 16x16x32 MFMAs (pfsgnn_common.h): the weight images hold
// [hi | lo] of one K-tile (W2^T; W1^T's odd last hidden tile) or the hi and
// the lo planes of two hidden tiles (W1^T pairs) in the fp32 images' bytes.
// Per wave and 16 nodes at M = 7: 18 + 77 bf16 MFMAs (16 cycles) instead of
// 28 + 196 fp32 ones (32 cycles).
template <int M, bool RS, bool X3 = false>
__global__ __launch_bounds__(256, ((M <= 3 || RS) ? 2 : 1)) void k_mlp_bwd(
    int K, int N, int H, int O, const float* __restrict__ dY, const float* __restrict__ Yp,
    const float* __restrict__ spart, int nsp, const float* __restrict__ mu,
    const float* __restrict__ var, const float* __restrict__ gamma, float eps,
    float* __restrict__ dgamma, float* __restrict__ dbeta, const float* __restrict__ Z,
    const float* __restrict__ W1, int ldw1, const float* __restrict__ W2,
    float* __restrict__ dYp, float* __restrict__ dZ, OutSegs outs, int want_dx, MomCoef mc) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  floatx4* T2 = reinterpret_cast<floatx4*>(sm);  // [M][64]: W2^T per hidden tile
  floatx4* T1 = T2 + M * 64;                     // [M][M][64]: W1^T per (input tile, hidden tile)
  float* BC = reinterpret_cast<float*>(T1 + M * M * 64);  // [5][16] BN backward coefficients
  float* DXs = BC + 80;                                     // [16M][XS_LD] chunk input gradient
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, col = lane & 15, kq = lane >> 4;
  {  // weight images, all loads in flight at once (see k_mlp_fwd)
    float w[M], v[M * M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int idx = t + 256 * i;
      const int r = idx & 3, l = (idx >> 2) & 63, mt = idx >> 8;
      const int o = 4 * (l >> 4) + r, h = 16 * mt + (l & 15);
      w[i] = (o < O && h < H) ? W2[(size_t)o * H + h] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < M * M; ++i) {
      const int idx = t + 256 * i;
      const int r = idx & 3, l = (idx >> 2) & 63, mt = (idx >> 8) % M, mk = (idx >> 8) / M;
      const int h = 16 * mt + 4 * (l >> 4) + r, k = 16 * mk + (l & 15);
      v[i] = (want_dx && h < H && k < K) ? W1[(size_t)h * ldw1 + mom_row(k, mc)] : 0.f;
    }
    if constexpr (X3) {
      static_assert(!X3 || RS, "X3: the RS form only");
      short* s2 = reinterpret_cast<short*>(T2);
      short* s1 = reinterpret_cast<short*>(T1);
#pragma unroll
      for (int i = 0; i < M; ++i) {   // T2x[mt][l] = [hi(r) | lo(r)]
        const int idx = t + 256 * i;
        const int r = idx & 3, l = (idx >> 2) & 63, mt = idx >> 8;
        const short h = __builtin_bit_cast(short, (__bf16)w[i]);
        s2[(mt * 64 + l) * 8 + r] = h;
        s2[(mt * 64 + l) * 8 + 4 + r] = __builtin_bit_cast(short, (__bf16)(w[i] - pf_bf(h)));
      }
#pragma unroll
      for (int i = 0; i < M * M; ++i) {   // T1x[mk][slot][l]: pairs [hi | hi'], [lo | lo']; odd last [hi | lo]
        const int idx = t + 256 * i;
        const int r = idx & 3, l = (idx >> 2) & 63, mt = (idx >> 8) % M, mk = (idx >> 8) / M;
        const short h = __builtin_bit_cast(short, (__bf16)v[i]);
        const short lo = __builtin_bit_cast(short, (__bf16)(v[i] - pf_bf(h)));
        const bool pair = mt < 2 * (M / 2);
        const int sh = pair ? (mt & ~1) : mt, sl = pair ? sh + 1 : mt;
        const int ph = pair ? 4 * (mt & 1) + r : r, pl = pair ? ph : 4 + r;
        s1[((mk * M + sh) * 64 + l) * 8 + ph] = h;
        s1[((mk * M + sl) * 64 + l) * 8 + pl] = lo;
      }
    } else {
#pragma unroll
      for (int i = 0; i < M; ++i) sm[t + 256 * i] = w[i];
      float* t1 = reinterpret_cast<float*>(T1);
#pragma unroll
      for (int i = 0; i < M * M; ++i) t1[t + 256 * i] = v[i];
    }
  }
  __shared__ RowOut rout[16 * M];   // the input-gradient rows' outputs
  if (want_dx) build_out_rows(outs, K, N, rout, mc);
  const bool bn = spart != nullptr;
  if (bn) {
    // (the merge's scratch is the chunk buffer DXs, free until the chunk loop:
    // a static array would push the RS form's LDS past the 80 KB of two
    // blocks per CU)
    float (*ss)[SUM_LEN] = reinterpret_cast<float (*)[SUM_LEN]>(DXs);
    const int c = t & 31, u = t >> 5;  // 8 subsets of the partial list per sum
    float s = 0.f;
    for (int r0 = 0; r0 < nsp; r0 += 256) {   // (one round for nsp <= 256)
      float v[32];  // every load of the round in flight, then a fixed-order sum
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const int b = r0 + u + 8 * i;
        v[i] = b < nsp ? spart[(size_t)b * SUM_LEN + c] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 32; ++i) s += v[i];
    }
    ss[u][c] = s;
    __syncthreads();
    if (t < 16) {
      float sg = 0.f, sx = 0.f;
      for (int i = 0; i < 8; ++i) {
        sg += ss[i][t];
        sx += ss[i][16 + t];
      }
      const bool live = t < O;
      const float inv = live ? 1.0f / sqrtf(var[t] + eps) : 0.f;
      BC[t] = live ? gamma[t] * inv : 0.f;       // gi
      BC[16 + t] = sg / (float)N;                // k0
      BC[32 + t] = sx / (float)N;                // k1
      BC[48 + t] = live ? mu[t] : 0.f;
      BC[64 + t] = inv;
      if (blockIdx.x == 0 && live) {
        dgamma[t] += sx;
        dbeta[t] += sg;
      }
    }
  }
  __syncthreads();
  float gi[4], k0[4], k1[4], mm[4], iv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int o = 4 * kq + r;
    gi[r] = bn ? BC[o] : 1.f;
    k0[r] = bn ? BC[16 + o] : 0.f;
    k1[r] = bn ? BC[32 + o] : 0.f;
    mm[r] = bn ? BC[48 + o] : 0.f;
    iv[r] = bn ? BC[64 + o] : 0.f;
  }

  const int nch = (N + 63) / 64;
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  float gv[4], yv[4], zv[4 * M];
  auto load = [&](int ch) {
    const int n = ch * 64 + wave * 16 + col;
    const bool nv = n < N;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 4 * kq + r;
      gv[r] = (nv && o < O) ? dY[(size_t)o * N + n] : 0.f;
      yv[r] = (bn && nv && o < O) ? Yp[(size_t)o * N + n] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < M; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * mt + 4 * kq + r;
        zv[4 * mt + r] = (nv && h < H) ? Z[(size_t)h * N + n] : 0.f;
      }
  };
  int ch = blockIdx.x;
  if (ch < nch) load(ch);
  for (; ch < nch; ch += gridDim.x) {
    float g[4], y[4], z[4 * M];
    if (RS && ch != (int)blockIdx.x) load(ch);   // (RS: no prefetch, one set of z registers)
#pragma unroll
    for (int r = 0; r < 4; ++r) { g[r] = gv[r]; y[r] = yv[r]; }
#pragma unroll
    for (int s = 0; s < 4 * M; ++s) z[s] = zv[s];
    if (!RS && ch + (int)gridDim.x < nch) load(ch + gridDim.x);
    const int n = ch * 64 + wave * 16 + col;
    const bool nv = n < N;
    int lo = 0;  // opaque: weight images re-read from LDS per chunk (see k_mlp_fwd)
    asm volatile("" : "+v"(lo));
    const floatx4* T1c = T1 + lo;
    const floatx4* T2c = T2 + lo;
    float gp[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 4 * kq + r;
      if (RS) {   // (the coefficients re-read from LDS: registers are the limit here)
        gp[r] = bn ? BC[o] * (g[r] - BC[16 + o] - (y[r] - BC[48 + o]) * BC[64 + o] * BC[32 + o])
                   : g[r];
      } else {
        gp[r] = bn ? gi[r] * (g[r] - k0[r] - (y[r] - mm[r]) * iv[r] * k1[r]) : g[r];
      }
      if (o >= O) gp[r] = 0.f;
      if (bn && dYp && nv && o < O) dYp[(size_t)o * N + n] = gp[r];
    }
    floatx4 dz[M];
    if constexpr (X3) {
      const pf_s16x8* T2x = reinterpret_cast<const pf_s16x8*>(T2c);
      pf_s16x4 gh, gl;
      pf_split4(gp[0], gp[1], gp[2], gp[3], gh, gl);
      const pf_s16x8 b1 = pf_cat8(gl, gh), b2 = pf_cat8(gh, pf_s16x4{0, 0, 0, 0});
#pragma unroll
      for (int mt = 0; mt < M; ++mt) {
        const pf_s16x8 a = T2x[mt * 64 + lane];
        dz[mt] = pf_mf8(a, b1, floatx4{0.f, 0.f, 0.f, 0.f});
        dz[mt] = pf_mf8(a, b2, dz[mt]);
      }
    } else {
      floatx4 w[M];
#pragma unroll
      for (int mt = 0; mt < M; ++mt) {
        w[mt] = T2c[mt * 64 + lane];
        dz[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int mt = 0; mt < M; ++mt) dz[mt] = mfma4(w[mt][r], gp[r], dz[mt]);
    }
#pragma unroll
    for (int mt = 0; mt < M; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * mt + 4 * kq + r;
        dz[mt][r] *= dlrelu(z[4 * mt + r]);
        if (nv && h < H) dZ[(size_t)h * N + n] = dz[mt][r];
      }
    if (RS && want_dx) {
      // dX = W1^T dZ by output-tile groups of 4: each group's 64 rows staged in
      // a 64-row LDS buffer, then written as coalesced 256-byte rows (the
      // block and add flag wave-uniform per row), as below
      constexpr int MG = 4;
      pf_s16x4 zh[M], zl[M];
      if constexpr (X3) {
#pragma unroll
        for (int mt = 0; mt < M; ++mt) pf_split4(dz[mt][0], dz[mt][1], dz[mt][2], dz[mt][3], zh[mt], zl[mt]);
      }
      // (groups last to first: with the moment epilogue, group 0's 16 channels
      // are turned into coefficients after the loop, when the split dZ
      // registers are dead)
      constexpr int NG = (M + MG - 1) / MG;
#pragma unroll
      for (int gi = NG - 1; gi >= 0; --gi) {
        const int g0 = gi * MG;
        const int GN = (M - g0) < MG ? (M - g0) : MG;
        floatx4 dx[MG];
#pragma unroll
        for (int i = 0; i < MG; ++i) dx[i] = floatx4{0.f, 0.f, 0.f, 0.f};
        if constexpr (X3) {
          const pf_s16x8* T1x = reinterpret_cast<const pf_s16x8*>(T1c);
#pragma unroll
          for (int p = 0; p < M / 2; ++p) {
            const pf_s16x8 bl = pf_cat8(zl[2 * p], zl[2 * p + 1]), bh = pf_cat8(zh[2 * p], zh[2 * p + 1]);
#pragma unroll
            for (int i = 0; i < MG; ++i)
              if (i < GN) {
                const pf_s16x8 ah = T1x[((g0 + i) * M + 2 * p) * 64 + lane];
                const pf_s16x8 al = T1x[((g0 + i) * M + 2 * p + 1) * 64 + lane];
                dx[i] = pf_mf8(ah, bl, dx[i]);
                dx[i] = pf_mf8(al, bh, dx[i]);
                dx[i] = pf_mf8(ah, bh, dx[i]);
              }
          }
          if constexpr (M & 1) {
            const pf_s16x8 b1 = pf_cat8(zl[M - 1], zh[M - 1]), b2 = pf_cat8(zh[M - 1], pf_s16x4{0, 0, 0, 0});
#pragma unroll
            for (int i = 0; i < MG; ++i)
              if (i < GN) {
                const pf_s16x8 a = T1x[((g0 + i) * M + M - 1) * 64 + lane];
                dx[i] = pf_mf8(a, b1, dx[i]);
                dx[i] = pf_mf8(a, b2, dx[i]);
              }
          }
        }
#pragma unroll
        for (int mt = 0; mt < (X3 ? 0 : M); ++mt) {
          floatx4 w[MG];   // (no read-ahead: the other block's waves cover the LDS latency)
#pragma unroll
          for (int i = 0; i < MG; ++i)
            if (i < GN) w[i] = T1c[((g0 + i) * M + mt) * 64 + lane];
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < MG; ++i)
              if (i < GN) dx[i] = mfma4(w[i][r], dz[mt][r], dx[i]);
        }
        __syncthreads();                           // the previous group's rows are stored
#pragma unroll
        for (int i = 0; i < MG; ++i) {
          if (i >= GN) continue;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            DXs[(16 * i + 4 * kq + r) * XS_LD + wave * 16 + col] = dx[i][r];
        }
        __syncthreads();
        store_rows<4>(rout, DXs, 16 * g0, 16 * g0, min(K, 16 * (g0 + GN)), ch * 64, N, wu, lane);
#if !defined(MLP_NO_MOMEPI) && !defined(MLP_NO_MOMEPI1)
        if (gi == 1 && mc.coef && 16 < mc.C2) {
          __builtin_amdgcn_sched_barrier(0);
          mom_coef_epi<1>(mc, DXs, XS_LD, 16, ch * 64, N);
          __builtin_amdgcn_sched_barrier(0);
        }
#endif
      }
#ifndef MLP_NO_MOMEPI
      if (mc.coef) {   // (group 0 is in DXs)
        __builtin_amdgcn_sched_barrier(0);
        mom_coef_epi<4>(mc, DXs, XS_LD, 0, ch * 64, N);
      }
#endif
    } else if (want_dx) {
      __syncthreads();                             // previous chunk's stores from DXs done
      // dX = W1^T dZ: K-step group mt (hidden tile) over the M output tiles, its
      // weight float4s read one group ahead, independent accumulators back to back
      floatx4 dx[M], wn[M];
#pragma unroll
      for (int mk = 0; mk < M; ++mk) {
        dx[mk] = floatx4{0.f, 0.f, 0.f, 0.f};
        wn[mk] = T1c[(mk * M) * 64 + lane];
      }
#pragma unroll
      for (int mt = 0; mt < M; ++mt) {
        floatx4 w[M];
#pragma unroll
        for (int mk = 0; mk < M; ++mk) w[mk] = wn[mk];
        if (mt + 1 < M) {
#pragma unroll
          for (int mk = 0; mk < M; ++mk) wn[mk] = T1c[(mk * M + mt + 1) * 64 + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int mk = 0; mk < M; ++mk) dx[mk] = mfma4(w[mk][r], dz[mt][r], dx[mk]);
      }
#pragma unroll
      for (int mk = 0; mk < M; ++mk) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = 16 * mk + 4 * kq + r;
          if (k < K) DXs[k * XS_LD + wave * 16 + col] = dx[mk][r];
        }
      }
      __syncthreads();
      store_rows<M>(rout, DXs, 0, 0, K, ch * 64, N, wu, lane);
    }
  }
}

// ------------------------------------------------------------ host side
int tiles_for(int K, int H) {
  const int m = (std::max(K, H) + 15) / 16;
  for (int v : {1, 2, 3, 4, 5, 7})
    if (m <= v) return v;
  return -1;
}

template <class Fn>
int with_tiles(int m, Fn fn) {
  switch (m) {
    case 1: return fn(std::integral_constant<int, 1>{});
    case 2: return fn(std::integral_constant<int, 2>{});
    case 3: return fn(std::integral_constant<int, 3>{});
    case 4: return fn(std::integral_constant<int, 4>{});
    case 5: return fn(std::integral_constant<int, 5>{});
    case 7: return fn(std::integral_constant<int, 7>{});
  }
  return -1;
}

// the wide MLPs (M >= 5) stage their inputs in registers (k_mlp_fwd RS) and
// run their backward with a 64-row input-gradient buffer (k_mlp_bwd RS);
// A/B knobs PFSGNN_MLP_FWD_RS / PFSGNN_MLP_BWD_RS = 0: the LDS-staged forms
static bool env_on(const char* name) {
  const char* e = getenv(name);
  return !(e && atoi(e) == 0);
}
bool fwd_rs(int m) {   // (default off: the LDS-staged forward is 0.38 ms/step faster at the bench shape)
  static const bool on = [] {
    const char* e = getenv("PFSGNN_MLP_FWD_RS");
    return e && atoi(e) != 0;
  }();
  return m >= 5 && on;
}
bool bwd_rs(int m) {
  static const bool on = env_on("PFSGNN_MLP_BWD_RS");
  return m >= 5 && on;
}
size_t fwd_lds(int m) {
  return ((size_t)m * m * 256 + (size_t)m * 256 + 16 * m + 16 +
          (fwd_rs(m) ? 0 : (size_t)2 * 16 * m * XS_LD)) * 4;
}
size_t bwd_lds(int m) {   // (RS: a 64-row input-gradient buffer, one output-tile group)
  return ((size_t)m * 256 + (size_t)m * m * 256 + 80 + (size_t)16 * (bwd_rs(m) ? 4 : m) * XS_LD) * 4;
}

// blocks per CU: the M <= 3 kernels fit 2 (registers, LDS), the wider ones
// run one 4-wave block per CU with up to 512 registers per lane; one block per
// slot of the device's CUs (persistent grid-stride over the 64-node chunks).
// (Balancing the grid over the chunk rounds -- 300 blocks of 2 chunks instead
// of 512 with 87 running a second one -- measured no different at either
// bench shape, profiles/r04l_ab.txt, and was removed.)
int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      return 256;
    return v;
  }();
  return n;
}
// lds: the block's whole LDS, dynamic + the kernel's static arrays
int grid_for(int N, int m, size_t lds) {
  (void)m;
  const int nch = (N + 63) / 64;
  const int per_cu = (lds <= 80 * 1024) ? 2 : 1;   // (160 KB of LDS per CU)
  return std::max(1, std::min(nch, cu_count() * per_cu));
}
// static LDS of a kernel (its __shared__ arrays), read once per instantiation
template <class K>
size_t static_lds(K* kernel) {
  hipFuncAttributes a{};
  if (hipFuncGetAttributes(&a, reinterpret_cast<const void*>(kernel)) != hipSuccess) return 0;
  return a.sharedSizeBytes;
}

// pfsgnn_seg list -> InSegs (blocks must be contiguous in the weight columns)
int make_in(const pfsgnn_seg* segs, int nseg, int N, InSegs& S) {
  if (!segs || nseg < 1 || nseg > NM_SEG) return -1;
  S = InSegs{};
  int k = 0, npg = 0;
  for (int i = 0; i < nseg; ++i) {
    const pfsgnn_seg& g = segs[i];
    if (!g.x || g.rows <= 0 || g.col != k || g.per_graph < 0) return -1;
    if (g.per_graph) {
      if (N % g.per_graph || (npg && npg != g.per_graph)) return -1;
      npg = g.per_graph;
    }
    S.p[i] = g.x;
    S.k0[i] = k;
    S.pg[i] = g.per_graph ? 1 : 0;
    S.rows[i] = g.rows;
    S.kp0[i] = i == 0 ? 0 : S.kp0[i - 1] + ((S.rows[i - 1] + 3) & ~3);
    k += g.rows;
  }
  S.Kp = S.kp0[nseg - 1] + ((S.rows[nseg - 1] + 3) & ~3);
  for (int i = nseg; i <= NM_SEG; ++i) S.kp0[i] = INT_MAX;
  for (int i = nseg; i < NM_SEG; ++i) S.rows[i] = 0;
  for (int i = nseg; i <= NM_SEG; ++i) S.k0[i] = INT_MAX;
  for (int i = nseg; i < NM_SEG; ++i) S.p[i] = S.p[0];
  S.npg = npg;
  S.Gc = npg ? N / npg : 1;
  return k;
}

}  // namespace

extern "C" size_t pfsgnn_mlp_ws_bytes(int N) {
  return align256((size_t)512 * PART_LEN * sizeof(float)) +
         align256((size_t)256 * SUM_LEN * sizeof(float)) + (N > 0 ? 0 : 0);
}

namespace {
// the MLP launch of pfsgnn_mlp_fwd (BatchNorm partials into `part` when given)
int mlp_fwd_launch(const InSegs& S, int K, int N, const float* W1, int ldw1, int H,
                   const float* b1, const float* W2, int O, const float* b2, float* Z, float* Yp,
                   float* part, int* grid_out, hipStream_t st) {
  int m = tiles_for(K, H);
  if (m > 0 && fwd_rs(m)) m = tiles_for(S.Kp, H);   // (RS: the padded K must fit the tiles)
  if (m <= 0 || (fwd_rs(m) && 16 * m < S.Kp)) return -2;
  const size_t lds = fwd_lds(m);
  const bool rs = fwd_rs(m);
  return with_tiles(m, [&](auto mc) {
    constexpr int MM = decltype(mc)::value;
    auto launch = [&](auto rsc) {
      constexpr bool RS = decltype(rsc)::value && MM >= 5;
      static const size_t stat = static_lds(&k_mlp_fwd<MM, RS>);
      const int grid = grid_for(N, m, lds + stat);
      *grid_out = grid;
      static size_t attr = 0;  // dynamic LDS above the 64 KB default must be opted into
      if (lds > 65536 && attr < lds) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mlp_fwd<MM, RS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
          return -3;
        attr = lds;
      }
      hipLaunchKernelGGL((k_mlp_fwd<MM, RS>), dim3(grid), dim3(256), lds, st, S, K, N, W1, ldw1, H,
                         b1, W2, O, b2, Z, Yp, part);
      return 0;
    };
    return rs ? launch(std::true_type{}) : launch(std::false_type{});
  });
}
}  // namespace

namespace pf {
// the class launch of pfsgnn_target_block_fwd (k_class_tail_fwd): scratch =
// tail_ws_floats(...) floats of workspace
// classes per unit: the smallest of 8, 16, 32 with at most 512 units (one
// workgroup per CU or fewer, each over its units); 0: too many graphs
static int tail_ct(int G, int NC) {
  static const int ct0 = [] {   // tuning knob PFSGNN_TAIL_CT: the smallest unit tried
    const char* e = getenv("PFSGNN_TAIL_CT");
    const int v = e ? atoi(e) : 16;   // (measured: 16 -- r04u_tail_ct.txt)
    return v == 8 || v == 16 || v == 32 ? v : 16;
  }();
  for (int ct = ct0; ct <= CT_CLS; ct *= 2) {
    const int qb = (NC + ct - 1) / ct;
    if ((long long)G * qb <= 512 && qb <= CT_QBMAX) return ct;
  }
  return 0;
}
size_t tail_ws_floats(int G, int NC, int F) {
  const int ct = tail_ct(G, NC);
  const size_t nu = (size_t)G * ((NC + (ct ? ct : CT_CLS) - 1) / (ct ? ct : CT_CLS));
  return nu * PART_LEN + 2 * nu * F + 64;
}
// grid_sync's form: 0 the sc1 hand-off (default), 1 the acq_rel form
// (PFSGNN_GRID_SYNC_FENCED=1 at load, or pfsgnn_set_grid_sync_fenced)
static int g_grid_sync_fenced = [] {
  const char* e = getenv("PFSGNN_GRID_SYNC_FENCED");
  return e && atoi(e) != 0 ? 1 : 0;
}();
static int grid_sync_fenced() { return g_grid_sync_fenced; }
// the barrier slot of the next launch (round robin over pf_bar_pool)
static unsigned* bar_slot() {
  static unsigned* pool[64] = {};
  static int next = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!pool[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(pf_bar_pool)) != hipSuccess) return nullptr;
    pool[dev] = static_cast<unsigned*>(p);
  }
  const int slot = next;
  next = (next + 1) % PF_BAR_SLOTS;
  return pool[dev] + (size_t)slot * 32;
}
// every workgroup of a grid_sync launch must be resident at once: the grid is
// at most one per CU, so the occupancy API must admit >= 1 block per CU (LDS,
// registers) -- checked once per kernel
static bool check_coresident(const void* kernel, int grid) {
  static std::map<const void*, int> per_cu;
  auto it = per_cu.find(kernel);
  if (it == per_cu.end()) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, 256, 0) != hipSuccess) n = 0;
    it = per_cu.emplace(kernel, n).first;
  }
  return it->second >= 1 && grid <= it->second * cu_count();
}
int class_tail_fwd(const pfsgnn_block_tail& a, const float* cpart, int BPG, float bscale,
                   float* scratch, hipStream_t st) {
  const char* where = "pfsgnn_target_block_fwd";
  TailArgs T{};
  T.a = a;
  T.cpart = cpart;
  T.BPG = BPG;
  T.CT = tail_ct(a.G, a.NC);
  PF_REQUIRE(T.CT > 0, where, "more than 512 class units (G * ceil(NC / 32)) or NC > 2048");
  T.QB = (a.NC + T.CT - 1) / T.CT;
  PF_REQUIRE(T.QB <= CT_QBMAX, where, "more than 64 class units per graph");
  T.nunits = a.G * T.QB;
  T.bscale = bscale;
  T.part = scratch;
  T.xss = T.part + (size_t)T.nunits * PART_LEN;
  T.yps = T.xss + (size_t)T.nunits * a.F;
  T.fenced = grid_sync_fenced();
  T.bar = bar_slot();
  PF_REQUIRE(T.bar, where, "barrier slot");
  const int grid = std::min(T.nunits, cu_count());
  const void* kern = a.F == 8 ? (const void*)k_class_tail_fwd<8>
                   : a.F == 10 ? (const void*)k_class_tail_fwd<10>
                   : a.F == 16 ? (const void*)k_class_tail_fwd<16> : nullptr;
  PF_REQUIRE(kern, where, "Fdim must be 8, 10 or 16");
  PF_REQUIRE(check_coresident(kern, grid), where, "the barrier grid is not co-resident");
  switch (a.F) {
    case 8: hipLaunchKernelGGL(k_class_tail_fwd<8>, dim3(grid), dim3(256), 0, st, T); break;
    case 10: hipLaunchKernelGGL(k_class_tail_fwd<10>, dim3(grid), dim3(256), 0, st, T); break;
    default: hipLaunchKernelGGL(k_class_tail_fwd<16>, dim3(grid), dim3(256), 0, st, T); break;
  }
  return 0;
}
}  // namespace pf

#ifdef PF_TAIL_STAMPS
extern "C" int pfsgnn_debug_cb_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_cb_stamps), sizeof(unsigned long long) * 512 * 8) ==
                 hipSuccess ? 0 : -1;
}
extern "C" int pfsgnn_debug_tail_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_tail_stamps), sizeof(unsigned long long) * 512 * 8) ==
                 hipSuccess ? 0 : -1;
}
#endif

extern "C" size_t pfsgnn_class_bwd_bytes(void) { return sizeof(pfsgnn_class_bwd); }

extern "C" int pfsgnn_target_class_bwd(const pfsgnn_class_bwd* a, void* ws, size_t ws_bytes,
                                       void* stream) {
  const char* where = "pfsgnn_target_class_bwd";
  PF_REQUIRE(a && a->G > 0 && a->NF > 0 && a->NC > 0, where, "bad arguments");
  PF_REQUIRE(a->npend >= 0 && a->npend <= 4, where, "at most 4 pending tables");
  for (int i = 0; i < a->npend; ++i)
    PF_REQUIRE(a->pend[i] && (a->pend_n[i] == a->NF || a->pend_n[i] == a->NC), where,
               "pending tables are per fiber or per class");
  PF_REQUIRE(a->V && a->gZ && a->gW1 && a->gW2 && a->gu_up && a->gV && a->gdZ && a->gu &&
                 a->g_xs && a->g_xt && a->Yp && a->mu && a->var && a->gamma && a->Z && a->W1 &&
                 a->W2 && a->Wt2 && a->dgamma && a->dbeta && a->dYp && a->dZ && a->gxt_in &&
                 a->g_agg && a->gu_t && a->g_hsum,
             where, "null");
  PF_REQUIRE(a->gH > 0 && a->gH <= CG_MAXH && 3 * a->F <= CG_MAXH, where, "GlobalModel width <= 192");
  PF_REQUIRE(!a->w || (a->y1 && a->r1 && a->r2 && a->dwp), where, "RMSNorm needs y1, r1, r2, dwp");
  CbArgs T{};
  T.a = *a;
  T.QB = (a->NC + CB_CLS - 1) / CB_CLS;
  PF_REQUIRE(T.QB <= CB_QBMAX, where, "more than 1024 classes per graph");
  T.nunits = a->G * T.QB;
  PF_REQUIRE(T.nunits <= 4096, where, "too many class units");
  const size_t need = ((size_t)T.nunits * a->F + (size_t)T.nunits * CB_PLEN) * sizeof(float);
  PF_REQUIRE(ws && ws_bytes >= need, where, "workspace too small");
  T.p1 = static_cast<float*>(ws);
  T.p2 = T.p1 + (size_t)T.nunits * a->F;
  T.fenced = pf::grid_sync_fenced();
  T.bar = pf::bar_slot();
  PF_REQUIRE(T.bar, where, "barrier slot");
  const int grid = std::min(T.nunits, cu_count());
  const void* kern = a->F == 8 ? (const void*)k_class_bwd<8>
                   : a->F == 10 ? (const void*)k_class_bwd<10>
                   : a->F == 16 ? (const void*)k_class_bwd<16> : nullptr;
  PF_REQUIRE(kern, where, "Fdim must be 8, 10 or 16");
  PF_REQUIRE(pf::check_coresident(kern, grid), where, "the barrier grid is not co-resident");
  hipStream_t st = as_stream(stream);
  switch (a->F) {
    case 8: hipLaunchKernelGGL(k_class_bwd<8>, dim3(grid), dim3(256), 0, st, T); break;
    case 10: hipLaunchKernelGGL(k_class_bwd<10>, dim3(grid), dim3(256), 0, st, T); break;
    default: hipLaunchKernelGGL(k_class_bwd<16>, dim3(grid), dim3(256), 0, st, T); break;
  }
  return pf::check_launch(where);
}

extern "C" int pfsgnn_set_grid_sync_fenced(int fenced) {
  PF_REQUIRE(fenced == 0 || fenced == 1, "pfsgnn_set_grid_sync_fenced", "0 or 1");
  pf::g_grid_sync_fenced = fenced;
  return 0;
}

extern "C" int pfsgnn_sync_faults(unsigned* n) {
  PF_REQUIRE(n, "pfsgnn_sync_faults", "null");
  if (hipMemcpyFromSymbol(n, HIP_SYMBOL(pf_sync_fault_count), sizeof(unsigned)) != hipSuccess)
    return pf::fail("pfsgnn_sync_faults", "hipMemcpyFromSymbol");
  return 0;
}

extern "C" int pfsgnn_mlp_fwd(const pfsgnn_seg* segs, int nseg, int N, const float* W1, int ldw1,
                              int H, const float* b1, const float* W2, int O, const float* b2,
                              float* Z, float* Yp, const float* gamma, const float* beta,
                              float* rm, float* rv, float momentum, float eps, float* Y,
                              float* mu, float* var, void* ws, size_t ws_bytes, void* stream) {
  return pfsgnn_mlp_fwd_epi(segs, nseg, N, W1, ldw1, H, b1, W2, O, b2, Z, Yp, gamma, beta, rm, rv,
                            momentum, eps, Y, mu, var, nullptr, 0, ws, ws_bytes, stream);
}

extern "C" int pfsgnn_mlp_fwd_epi(const pfsgnn_seg* segs, int nseg, int N, const float* W1,
                                  int ldw1, int H, const float* b1, const float* W2, int O,
                                  const float* b2, float* Z, float* Yp, const float* gamma,
                                  const float* beta, float* rm, float* rv, float momentum,
                                  float eps, float* Y, float* mu, float* var,
                                  const pfsgnn_linmap* epi, int nepi, void* ws, size_t ws_bytes,
                                  void* stream) {
  const char* where = "pfsgnn_mlp_fwd";
  PF_REQUIRE(W1 && b1 && W2 && b2 && Yp && N > 0 && H > 0 && O > 0 && O <= 16, where,
             "bad arguments");
  InSegs S;
  const int K = make_in(segs, nseg, N, S);
  PF_REQUIRE(K > 0, where, "bad segment list (blocks must cover weight columns 0..K in order)");
  PF_REQUIRE(tiles_for(K, H) > 0, where, "K, H > 112 not supported");
  const bool bn = gamma != nullptr;
  PF_REQUIRE(!bn || (beta && Y && mu && var && N > 1), where,
             "BatchNorm needs beta, Y, mu, var and more than one node");
  PF_REQUIRE(ws && ws_bytes >= pfsgnn_mlp_ws_bytes(N), where, "workspace too small");
  PF_REQUIRE(nepi >= 0 && nepi <= 2 && (nepi == 0 || (epi && bn)), where,
             "epilogues (at most 2) need the BatchNorm");
  BnEpi E{};
  for (int e = 0; e < nepi; ++e) {
    PF_REQUIRE(epi[e].W && epi[e].out && epi[e].nk > 0 && epi[e].nk <= EPI_MAXK &&
                   epi[e].col0 >= 0 && epi[e].col0 + O <= epi[e].ldw,
               where, "bad epilogue (nk <= 64, columns col0..col0+O inside ldw)");
    E.W[e] = epi[e].W;
    E.ldw[e] = epi[e].ldw;
    E.col0[e] = epi[e].col0;
    E.nk[e] = epi[e].nk;
    E.b[e] = epi[e].b;
    E.out[e] = epi[e].out;
  }
  hipStream_t st = as_stream(stream);
  float* part = bn ? reinterpret_cast<float*>(ws) : nullptr;
  int grid = 0;
  const int rc = mlp_fwd_launch(S, K, N, W1, ldw1, H, b1, W2, O, b2, Z, Yp, part, &grid, st);
  PF_REQUIRE(rc != -3, where, "hipFuncSetAttribute (dynamic LDS) failed");
  PF_REQUIRE(rc == 0, where, "no kernel for this width");
  if (bn) {
    // most blocks (A/B knob PFSGNN_BN_APPLY_BLOCKS): 1024 -- one wave per SIMD at
    // 256 left the epilogue's FMA chains exposed (configs[2] 26.11 -> 25.90 ms,
    // the bench batch unchanged at 374 blocks: profiles/r04aj_*)
    static const int agmax = [] {
      const char* e = getenv("PFSGNN_BN_APPLY_BLOCKS");
      return e && atoi(e) > 0 ? atoi(e) : 1024;
    }();
    const int ag = std::max(1, std::min(agmax, (int)(((size_t)O * N + 1023) / 1024)));
    // (zero weights pad the channels past O within a 4-channel group: ew rows are
    // 16 wide with o >= O zero, so OW = round-up(O, 4) is exact)
    if (O == 10)
      hipLaunchKernelGGL(k_bn_apply_part<10>, dim3(ag), dim3(256), 0, st, part, grid, O, N, Yp,
                         gamma, beta, eps, rm, rv, momentum, Y, mu, var, E);
    else if (O == 8)
      hipLaunchKernelGGL(k_bn_apply_part<8>, dim3(ag), dim3(256), 0, st, part, grid, O, N, Yp,
                         gamma, beta, eps, rm, rv, momentum, Y, mu, var, E);
    else
      hipLaunchKernelGGL(k_bn_apply_part<0>, dim3(ag), dim3(256), 0, st, part, grid, O, N, Yp,
                         gamma, beta, eps, rm, rv, momentum, Y, mu, var, E);
  }
  return pf::check_launch(where);
}

extern "C" int pfsgnn_target_global_fwd(
    const pfsgnn_seg* segs, int nseg, int G, int NC, const float* W1, int ldw1, int H,
    const float* b1, const float* W2, int F, const float* b2, float* Z, float* Yp,
    const float* gamma, const float* beta, float* rm, float* rv, float momentum, float eps,
    float* xt, float* mu, float* var, const float* xs, int NF, const float* u, const float* gW1,
    int gH, const float* gb1, const float* gW2, const float* gb2, const float* gw, float reps,
    float* means, float* gZ, float* gV, float* unew, float* y1, float* r1, float* r2,
    const float* We, const float* be, const float* Ws, const float* bs, float* Pt, float* Qt,
    void* ws, size_t ws_bytes, void* stream) {
  const char* where = "pfsgnn_target_global_fwd";
  PF_REQUIRE(G > 0 && NC > 0 && NF > 0 && F > 0 && F <= CG_MAXF && W1 && b1 && W2 && b2 && Z &&
                 Yp && gamma && beta && xt && mu && var && xs && u && gW1 && gb1 && gW2 && gb2 &&
                 means && gZ && gV && unew && gH > 0 && gH <= CG_MAXH && 3 * F <= CG_MAXH,
             where, "bad arguments (F <= 16, GlobalModel widths <= 192)");
  PF_REQUIRE(!gw || (y1 && r1 && r2), where, "RMSNorm needs y1, r1, r2");
  PF_REQUIRE(!We || (be && Ws && bs && Pt && Qt), where, "next-block parts need be, Ws, bs, Pt, Qt");
  const int N = G * NC;
  PF_REQUIRE(N > 1, where, "BatchNorm needs more than one node");
  InSegs S;
  const int K = make_in(segs, nseg, N, S);
  PF_REQUIRE(K > 0, where, "bad segment list (blocks must cover weight columns 0..K in order)");
  PF_REQUIRE(ws && ws_bytes >= pfsgnn_mlp_ws_bytes(N), where, "workspace too small");
  hipStream_t st = as_stream(stream);
  float* part = reinterpret_cast<float*>(ws);
  int grid = 0;
  const int rc = mlp_fwd_launch(S, K, N, W1, ldw1, H, b1, W2, F, b2, Z, Yp, part, &grid, st);
  PF_REQUIRE(rc != -3, where, "hipFuncSetAttribute (dynamic LDS) failed");
  PF_REQUIRE(rc == 0, where, "no kernel for this width (K, H <= 112)");
  ClassGlobalArgs A{};
  A.part = part; A.nb = grid; A.F = F; A.NC = NC; A.G = G; A.NF = NF;
  A.Yp = Yp; A.gamma = gamma; A.beta = beta; A.eps = eps; A.momentum = momentum;
  A.rm = rm; A.rv = rv; A.xt = xt; A.mu = mu; A.var = var;
  A.xs = xs; A.u = u; A.W1 = gW1; A.b1 = gb1; A.W2 = gW2; A.b2 = gb2; A.w = gw; A.H = gH;
  A.reps = reps; A.means = means; A.Z = gZ; A.V = gV; A.Y = unew; A.y1 = y1; A.r1 = r1; A.r2 = r2;
  A.We = We; A.be = be; A.Ws = Ws; A.bs = bs; A.Pt = Pt; A.Qt = Qt;
  switch (F) {
    case 8: hipLaunchKernelGGL(k_class_global_fwd<8>, dim3(G), dim3(CG_THREADS), 0, st, A); break;
    case 10: hipLaunchKernelGGL(k_class_global_fwd<10>, dim3(G), dim3(CG_THREADS), 0, st, A); break;
    case 16: hipLaunchKernelGGL(k_class_global_fwd<16>, dim3(G), dim3(CG_THREADS), 0, st, A); break;
    default: return pf::fail(where, "Fdim must be 8, 10 or 16");
  }
  return pf::check_launch(where);
}

// pre_part / pre_n: the BatchNorm sums' per-block partials ([pre_n][32]) made
// by the producer of dY (pfsgnn_target_bwd_bn); nullptr: k_bn_sums_part here
static int mlp_bwd_impl(const char* where, const float* dY, int N, const float* Yp,
                        const float* mu, const float* var, const float* gamma, float eps,
                        float* dgamma, float* dbeta, const float* Z, const float* W1, int ldw1,
                        int H, int K, const float* W2, int O, float* dYp, float* dZ,
                        const pfsgnn_oseg* outs, int nout, void* ws, size_t ws_bytes,
                        void* stream, const float* pre_part, int pre_n,
                        const MomCoef& mco = MomCoef{}) {
  PF_REQUIRE(dY && Z && W1 && W2 && dZ && N > 0 && H > 0 && K > 0 && O > 0 && O <= 16, where,
             "bad arguments");
  const bool bn = gamma != nullptr;
  PF_REQUIRE(!bn || (Yp && mu && var && dgamma && dbeta && dYp), where,
             "BatchNorm backward needs Yp, mu, var, dgamma, dbeta and dYp");
  PF_REQUIRE(nout >= 0 && nout <= NM_SEG && (nout == 0 || outs), where, "bad output list");
  OutSegs OS{};
  int k = 0;
  for (int i = 0; i < nout; ++i) {
    PF_REQUIRE(outs[i].rows > 0, where, "bad output block");
    OS.p[i] = outs[i].x;
    OS.k0[i] = k;
    OS.add[i] = outs[i].add;
    k += outs[i].rows;
  }
  PF_REQUIRE(nout == 0 || k == K, where, "output blocks must cover the K input rows");
  for (int i = nout; i <= NM_SEG; ++i) OS.k0[i] = INT_MAX;
  const int m = tiles_for(K, H);
  PF_REQUIRE(m > 0, where, "K, H > 112 not supported");
  PF_REQUIRE(ws && ws_bytes >= pfsgnn_mlp_ws_bytes(N), where, "workspace too small");
  hipStream_t st = as_stream(stream);
  const float* spart = nullptr;
  int nsp = 0;
  if (bn && pre_part) {
    spart = pre_part;
    nsp = pre_n;
  } else if (bn) {
    float* sp = reinterpret_cast<float*>(static_cast<char*>(ws) +
                                         align256((size_t)512 * PART_LEN * sizeof(float)));
    nsp = std::max(1, std::min(256, (N + 255) / 256));
    hipLaunchKernelGGL(k_bn_sums_part, dim3(nsp), dim3(256), 0, st, dY, Yp, O, N, mu, var, eps,
                       sp);
    spart = sp;
  }
  const size_t lds = bwd_lds(m);
  const int want_dx = nout > 0 ? 1 : 0;
  const bool rs = bwd_rs(m);
  PF_REQUIRE(!mco.coef || (rs && want_dx && mco.mom && mco.C2 >= 16 && mco.C2 <= 20 &&
                           mco.k0 >= 0 && mco.k0 + 4 * mco.C2 <= K),
             where, "the moment epilogue needs the RS form, dX and 16..20 channels inside K");
  // the gradient chains in bf16x3 (RS form): PFSGNN_NODE_DX_X3, pf::node_x3's policy
  const bool x3 = rs && pf::node_x3("PFSGNN_NODE_DX_X3");
  const int rc = with_tiles(m, [&](auto mc) {
    constexpr int MM = decltype(mc)::value;
    auto launch = [&](auto rsc, auto x3c) {
      constexpr bool RS = decltype(rsc)::value && MM >= 5;
      constexpr bool X3 = decltype(x3c)::value && RS;
      static const size_t stat = static_lds(&k_mlp_bwd<MM, RS, X3>);
      const int grid = grid_for(N, m, lds + stat);
      static size_t attr = 0;  // dynamic LDS above the 64 KB default must be opted into
      if (lds > 65536 && attr < lds) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mlp_bwd<MM, RS, X3>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
          return -3;
        attr = lds;
      }
      hipLaunchKernelGGL((k_mlp_bwd<MM, RS, X3>), dim3(grid), dim3(256), lds, st, K, N, H, O, dY,
                         Yp, spart, nsp, mu, var, gamma, eps, dgamma, dbeta, Z, W1, ldw1, W2, dYp,
                         dZ, OS, want_dx, mco);
      return 0;
    };
    if (!rs) return launch(std::false_type{}, std::false_type{});
    return x3 ? launch(std::true_type{}, std::true_type{})
              : launch(std::true_type{}, std::false_type{});
  });
  PF_REQUIRE(rc != -3, where, "hipFuncSetAttribute (dynamic LDS) failed");
  PF_REQUIRE(rc == 0, where, "no kernel for this width");
  return pf::check_launch(where);
}

extern "C" int pfsgnn_mlp_bwd(const float* dY, int N, const float* Yp, const float* mu,
                              const float* var, const float* gamma, float eps, float* dgamma,
                              float* dbeta, const float* Z, const float* W1, int ldw1, int H,
                              int K, const float* W2, int O, float* dYp, float* dZ,
                              const pfsgnn_oseg* outs, int nout, void* ws, size_t ws_bytes,
                              void* stream) {
  return mlp_bwd_impl("pfsgnn_mlp_bwd", dY, N, Yp, mu, var, gamma, eps, dgamma, dbeta, Z, W1,
                      ldw1, H, K, W2, O, dYp, dZ, outs, nout, ws, ws_bytes, stream, nullptr, 0);
}

extern "C" int pfsgnn_mlp_bwd_pre(const float* dY, int N, const float* Yp, const float* mu,
                                  const float* var, const float* gamma, float eps, float* dgamma,
                                  float* dbeta, const float* Z, const float* W1, int ldw1, int H,
                                  int K, const float* W2, int O, float* dYp, float* dZ,
                                  const pfsgnn_oseg* outs, int nout, const float* bn_part,
                                  int bn_nparts, const float* mom, float* coef, int mom_k0,
                                  int mom_c, int mom_n, void* ws, size_t ws_bytes, void* stream) {
  PF_REQUIRE(!bn_part || (gamma && bn_nparts > 0 && bn_nparts <= 65536), "pfsgnn_mlp_bwd_pre",
             "BatchNorm sum partials need gamma and 1..65536 partials");
  PF_REQUIRE(!coef || (mom && mom_n > 0), "pfsgnn_mlp_bwd_pre", "coef needs mom and mom_n > 0");
  const MomCoef mc{coef ? mom : nullptr, coef, mom_c, mom_k0, coef ? 1.0f / (float)mom_n : 0.f};
  return mlp_bwd_impl("pfsgnn_mlp_bwd_pre", dY, N, Yp, mu, var, gamma, eps, dgamma, dbeta, Z, W1,
                      ldw1, H, K, W2, O, dYp, dZ, outs, nout, ws, ws_bytes, stream, bn_part,
                      bn_part ? bn_nparts : 0, mc);
}
