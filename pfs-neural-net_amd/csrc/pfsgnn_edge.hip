// pfsgnn_edge.hip -- per-edge kernels of the bipartite message-passing block.
//
// Every kernel streams the channel-major edge tensors once (one coalesced
// dword load per channel per edge), runs the small per-edge MLP in fp32 on
// the VALU with the weights as wave-uniform (scalar) operands, and does all of
// its reductions on chip:
//   * per-fiber sums  -> butterflies inside the fiber's SW-lane segment
//                        (reference: scatter(..., src, reduce='mean'), gnn.py:140-144);
//   * per-class sums  -> per-thread registers across the fiber tiles a block
//                        visits, then one block-level pass (gnn.py:190);
//   * weight grads    -> sum over edges of an outer product, on
//                        v_mfma_f32_16x16x4_f32 with the edge as the K index;
//   * batch moments   -> per-thread Welford / sums, merged per block.
// Per-block partials are finished by deterministic reduce kernels, so a
// training step is bitwise reproducible.
#include "pfsgnn_common.h"
#include "../../include/pfsgnn.h"

#include <algorithm>

#define EDGE_PROLOGUE                                                  \
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;             \
  const int bx = blockIdx.x;                                           \
  const int gg = bx / geo.BPG, jj = bx - gg * geo.BPG;                 \
  const int slot = t / geo.SW, cl = t - slot * geo.SW;                 \
  const bool cvalid = cl < geo.NC;                                     \
  const int tile0 = jj * geo.TPB;                                      \
  const int tile1 = min(geo.TPG, tile0 + geo.TPB);                     \
  const long long E = geo.E, NS = geo.NS, NT = geo.NT;                 \
  const long long cn = (long long)gg * geo.NC + cl;                    \
  (void)lane; (void)wave; (void)E; (void)NS; (void)NT; (void)cn;

#define EDGE_TILE                                                      \
  const int f = tile * geo.FPI + slot;                                 \
  const bool fvalid = f < geo.NF;                                      \
  const bool valid = cvalid && fvalid;                                 \
  const long long n = (long long)gg * geo.NF + (fvalid ? f : 0);       \
  const long long e = n * geo.NC + cl;                                 \
  (void)e;

template <int F>
__device__ __forceinline__ void load_edge(float (&x)[F], const float* __restrict__ src,
                                          const float* __restrict__ sc,
                                          const float* __restrict__ sh, long long e, long long E,
                                          bool valid) {
#pragma unroll
  for (int k = 0; k < F; ++k) {
    float v = valid ? src[(long long)k * E + e] : 0.f;
    if (sc) v = valid ? fmaf(v, sc[k], sh[k]) : 0.f;
    x[k] = v;
  }
}

// ============================================================ EdgeModel fwd
template <int F>
__global__ __launch_bounds__(256) void k_edge_mlp_fwd(EdgeGeo geo, const float* __restrict__ xe,
                                                      const float* __restrict__ xsc,
                                                      const float* __restrict__ xsh,
                                                      const float* __restrict__ Ps,
                                                      const float* __restrict__ Pt,
                                                      const float* __restrict__ W1,
                                                      const float* __restrict__ W2,
                                                      const float* __restrict__ b2,
                                                      float* __restrict__ y,
                                                      float* __restrict__ part) {
  constexpr int H = 4 * F;
  EDGE_PROLOGUE
  float cnt = 0.f, mean[F], m2[F];
#pragma unroll
  for (int k = 0; k < F; ++k) { mean[k] = 0.f; m2[k] = 0.f; }
  for (int tile = tile0; tile < tile1; ++tile) {
    EDGE_TILE
    if (valid) {
      float x[F];
      load_edge<F>(x, xe, xsc, xsh, e, E, true);
      float a[H];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        float z = Ps[(long long)h * NS + n] + Pt[(long long)h * NT + cn];
#pragma unroll
        for (int k = 0; k < F; ++k) z = fmaf(W1[h * H + 2 * F + k], x[k], z);
        a[h] = lrelu(z);
      }
      cnt += 1.f;
      const float rc = 1.0f / cnt;
#pragma unroll
      for (int o = 0; o < F; ++o) {
        float s = b2[o];
#pragma unroll
        for (int h = 0; h < H; ++h) s = fmaf(W2[o * H + h], a[h], s);
        y[(long long)o * E + e] = s;
        const float d = s - mean[o];
        mean[o] = fmaf(d, rc, mean[o]);
        m2[o] = fmaf(d, s - mean[o], m2[o]);
      }
    }
  }
  // Chan merge over the block: lanes (butterfly) then waves (LDS)
  for (int off = 32; off > 0; off >>= 1) {
    const float cb = __shfl_xor(cnt, off);
    const float tot = cnt + cb;
    const float wb = tot > 0.f ? cb / tot : 0.f;
    const float wab = tot > 0.f ? cnt * cb / tot : 0.f;
#pragma unroll
    for (int k = 0; k < F; ++k) {
      const float mb = __shfl_xor(mean[k], off), qb = __shfl_xor(m2[k], off);
      const float d = mb - mean[k];
      mean[k] = fmaf(d, wb, mean[k]);
      m2[k] = m2[k] + qb + d * d * wab;
    }
    cnt = tot;
  }
  __shared__ float sh[4][1 + 2 * F];
  if (lane == 0) {
    sh[wave][0] = cnt;
#pragma unroll
    for (int k = 0; k < F; ++k) { sh[wave][1 + k] = mean[k]; sh[wave][1 + F + k] = m2[k]; }
  }
  __syncthreads();
  if (t < F) {
    float C0 = sh[0][0], M0 = sh[0][1 + t], Q0 = sh[0][1 + F + t];
    for (int w = 1; w < 4; ++w) {
      const float cb = sh[w][0], mb = sh[w][1 + t], qb = sh[w][1 + F + t];
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

// merge per-block Welford partials (double) -> mu, biased var
__global__ void k_moments_finalize(const float* __restrict__ part, int nb, int F, long long n,
                                   float* __restrict__ mu, float* __restrict__ var) {
  const int k = threadIdx.x;
  if (k >= F) return;
  double cnt = 0, mean = 0, m2 = 0;
  for (int b = 0; b < nb; ++b) {
    const float* p = part + (size_t)b * (1 + 2 * F);
    const double cb = p[0], mb = p[1 + k], qb = p[1 + F + k];
    const double tot = cnt + cb;
    if (tot > 0) {
      const double d = mb - mean;
      mean += d * (cb / tot);
      m2 += qb + d * d * (cnt * cb / tot);
    }
    cnt = tot;
  }
  mu[k] = (float)mean;
  var[k] = (float)(m2 / (double)n);
}

// ============================================================ SModel fwd
template <int F>
__global__ __launch_bounds__(256) void k_source_fwd(EdgeGeo geo, const float* __restrict__ y,
                                                    const float* __restrict__ sc,
                                                    const float* __restrict__ sh,
                                                    const float* __restrict__ Qt,
                                                    const float* __restrict__ Ws1,
                                                    const float* __restrict__ Ws2,
                                                    const float* __restrict__ bs2,
                                                    float* __restrict__ mom,
                                                    float* __restrict__ hs) {
  constexpr int C = 2 * F;
  EDGE_PROLOGUE
  __shared__ float scratch[4 * 3 * C];
  const float invn = 1.0f / (float)geo.NC;
  for (int tile = tile0; tile < tile1; ++tile) {
    EDGE_TILE
    float x[F];
    load_edge<F>(x, y, sc, sh, e, E, valid);
    float a[C];
#pragma unroll
    for (int h = 0; h < C; ++h) {
      float z = valid ? Qt[(long long)h * NT + cn] : 0.f;
#pragma unroll
      for (int k = 0; k < F; ++k) z = fmaf(Ws1[h * C + F + k], x[k], z);
      a[h] = lrelu(z);
    }
    float m[C], s1[C];
#pragma unroll
    for (int o = 0; o < C; ++o) {
      float s = bs2[o];
#pragma unroll
      for (int h = 0; h < C; ++h) s = fmaf(Ws2[o * C + h], a[h], s);
      m[o] = valid ? s : 0.f;
      s1[o] = m[o];
    }
    seg_sum<C>(s1, geo.SW, scratch);
    float p[3 * C];
#pragma unroll
    for (int o = 0; o < C; ++o) {
      const float mean = s1[o] * invn;
      const float d = valid ? m[o] - mean : 0.f;
      const float d2 = d * d;
      p[o] = d2;
      p[C + o] = d2 * d;
      p[2 * C + o] = d2 * d2;
    }
    seg_sum<3 * C>(p, geo.SW, scratch);
    if (cl == 0 && fvalid) {
      const long long CN = (long long)C * NS;
#pragma unroll
      for (int o = 0; o < C; ++o) {
        const float mean = s1[o] * invn;
        const float c2 = p[o] * invn, c3 = p[C + o] * invn, c4 = p[2 * C + o] * invn;
        mom[(long long)o * NS + n] = mean;
        mom[CN + (long long)o * NS + n] = c2;
        mom[2 * CN + (long long)o * NS + n] = c3;
        mom[3 * CN + (long long)o * NS + n] = c4;
        const float var = c2 > 0.f ? c2 : 0.01f * c2;        // F.leaky_relu (slope 0.01)
        const float sd = sqrtf(var + 1e-6f);
        hs[(long long)o * NS + n] = mean;
        hs[(long long)(C + o) * NS + n] = sd;
        hs[(long long)(2 * C + o) * NS + n] = c3 / (sd * sd * sd);
        hs[(long long)(3 * C + o) * NS + n] = c4 / ((sd * sd) * (sd * sd));
      }
    }
  }
}

// ============================================================ TModel fwd
template <int F>
__global__ __launch_bounds__(256) void k_target_fwd(EdgeGeo geo, const float* __restrict__ y,
                                                    const float* __restrict__ sc,
                                                    const float* __restrict__ sh,
                                                    const float* __restrict__ Rs,
                                                    const float* __restrict__ Wt1,
                                                    float* __restrict__ part) {
  constexpr int C = 2 * F;
  EDGE_PROLOGUE
  __shared__ float scratch[256 * C];
  float acc[C];
#pragma unroll
  for (int h = 0; h < C; ++h) acc[h] = 0.f;
  for (int tile = tile0; tile < tile1; ++tile) {
    EDGE_TILE
    if (valid) {
      float x[F];
      load_edge<F>(x, y, sc, sh, e, E, true);
#pragma unroll
      for (int h = 0; h < C; ++h) {
        float z = Rs[(long long)h * NS + n];
#pragma unroll
        for (int k = 0; k < F; ++k) z = fmaf(Wt1[h * C + F + k], x[k], z);
        acc[h] += lrelu(z);
      }
    }
  }
  column_partial<C>(acc, geo.SW, geo.FPI, geo.NC, scratch, part + (size_t)bx * geo.NC * C);
}

// ============================================================ TModel bwd
template <int F>
__global__ __launch_bounds__(256) void k_target_bwd(EdgeGeo geo, const float* __restrict__ y,
                                                    const float* __restrict__ sc,
                                                    const float* __restrict__ sh,
                                                    const float* __restrict__ Rs,
                                                    const float* __restrict__ Wt1,
                                                    const float* __restrict__ g_hsum,
                                                    float* __restrict__ GzT,
                                                    float* __restrict__ gxe,
                                                    float* __restrict__ part) {
  constexpr int C = 2 * F;
  using WG = WGrad<C, F>;
  EDGE_PROLOGUE
  constexpr int LDS_N = 4 * WG::LDS_FLOATS + 4 * C;
  static_assert(LDS_N >= 4 * C * F, "lds");
  __shared__ float lds[LDS_N];
  float* region = lds + wave * WG::LDS_FLOATS;
  float* scratch = lds + 4 * WG::LDS_FLOATS;
  WG wg;
  wg.zero();
  for (int tile = tile0; tile < tile1; ++tile) {
    EDGE_TILE
    float x[F];
    load_edge<F>(x, y, sc, sh, e, E, valid);
    float gz[C];
#pragma unroll
    for (int h = 0; h < C; ++h) {
      float z = valid ? Rs[(long long)h * NS + n] : 0.f;
#pragma unroll
      for (int k = 0; k < F; ++k) z = fmaf(Wt1[h * C + F + k], x[k], z);
      gz[h] = valid ? g_hsum[(long long)h * NT + cn] * dlrelu(z) : 0.f;
    }
    if (gxe && valid) {
#pragma unroll
      for (int k = 0; k < F; ++k) {
        float s = 0.f;
#pragma unroll
        for (int h = 0; h < C; ++h) s = fmaf(Wt1[h * C + F + k], gz[h], s);
        gxe[(long long)k * E + e] = s;
      }
    }
    wg.stage(region, gz, x, lane);
    __syncthreads();
    wg.accum(region, lane);
    __syncthreads();
    seg_sum<C>(gz, geo.SW, scratch);
    if (cl == 0 && fvalid) {
#pragma unroll
      for (int h = 0; h < C; ++h) GzT[(long long)h * NS + n] = gz[h];
    }
  }
  wg.block_partial(lds, part + (size_t)bx * C * F);
}

// ============================================================ SModel bwd (+T, +BN sums)
template <int F>
__global__ __launch_bounds__(256) void k_source_bwd(
    EdgeGeo geo, const float* __restrict__ y, const float* __restrict__ sc,
    const float* __restrict__ sh, const float* __restrict__ Qt, const float* __restrict__ Ws1,
    const float* __restrict__ Ws2, const float* __restrict__ bs2, const float* __restrict__ mean,
    const float* __restrict__ coef, const float* __restrict__ Rs, const float* __restrict__ Wt1,
    const float* __restrict__ g_hsum, const float* __restrict__ g_next,
    const float* __restrict__ mu1, const float* __restrict__ inv1, float* __restrict__ g_tot,
    float* __restrict__ partW2, float* __restrict__ partW1, float* __restrict__ partCol,
    float* __restrict__ partBN) {
  constexpr int C = 2 * F;
  using WG2 = WGrad<C, C + 1>;  // g_m (x) [a, 1]  -> dWs2 | dbs2
  using WG1 = WGrad<C, F>;      // g_zs (x) x      -> dWs1[:, F:2F]
  constexpr int STAGE = WG2::LDS_FLOATS > WG1::LDS_FLOATS ? WG2::LDS_FLOATS : WG1::LDS_FLOATS;
  constexpr int LOOP_N = 4 * STAGE;
  constexpr int TAIL_N0 = (4 * C * (C + 1) > 256 * C) ? 4 * C * (C + 1) : 256 * C;
  constexpr int LDS_N = LOOP_N > TAIL_N0 ? LOOP_N : TAIL_N0;
  EDGE_PROLOGUE
  __shared__ float lds[LDS_N];
  float* region = lds + wave * STAGE;
  float* scratch = lds;
  WG2 wg2;
  WG1 wg1;
  wg2.zero();
  wg1.zero();
  float colS[C];
#pragma unroll
  for (int h = 0; h < C; ++h) colS[h] = 0.f;
  float sg[F], sgx[F];
#pragma unroll
  for (int k = 0; k < F; ++k) { sg[k] = 0.f; sgx[k] = 0.f; }
  const long long CN = (long long)C * NS;
  for (int tile = tile0; tile < tile1; ++tile) {
    EDGE_TILE
    float yv[F], x[F];
#pragma unroll
    for (int k = 0; k < F; ++k) {
      yv[k] = valid ? y[(long long)k * E + e] : 0.f;
      x[k] = valid ? (sc ? fmaf(yv[k], sc[k], sh[k]) : yv[k]) : 0.f;
    }
    // forward recompute of the SModel message
    float zs[C], a[C + 1];
#pragma unroll
    for (int h = 0; h < C; ++h) {
      float z = valid ? Qt[(long long)h * NT + cn] : 0.f;
#pragma unroll
      for (int k = 0; k < F; ++k) z = fmaf(Ws1[h * C + F + k], x[k], z);
      zs[h] = z;
      a[h] = lrelu(z);
    }
    a[C] = 1.f;
    float gm[C];
#pragma unroll
    for (int o = 0; o < C; ++o) {
      float s = bs2[o];
#pragma unroll
      for (int h = 0; h < C; ++h) s = fmaf(Ws2[o * C + h], a[h], s);
      const long long idx = (long long)o * NS + n;
      const float d = s - mean[idx];
      const float c0 = coef[idx], c1 = coef[CN + idx], c2 = coef[2 * CN + idx],
                  c3 = coef[3 * CN + idx];
      gm[o] = valid ? fmaf(d, fmaf(d, fmaf(d, c3, c2), c1), c0) : 0.f;
    }
    wg2.stage(region, gm, a, lane);
    __syncthreads();
    wg2.accum(region, lane);
    __syncthreads();
    float gz[C];
#pragma unroll
    for (int h = 0; h < C; ++h) {
      float s = 0.f;
#pragma unroll
      for (int o = 0; o < C; ++o) s = fmaf(Ws2[o * C + h], gm[o], s);
      gz[h] = s * dlrelu(zs[h]);
      colS[h] += gz[h];
    }
    wg1.stage(region, gz, x, lane);
    __syncthreads();
    wg1.accum(region, lane);
    __syncthreads();
    float g[F];
#pragma unroll
    for (int k = 0; k < F; ++k) {
      float s = 0.f;
#pragma unroll
      for (int h = 0; h < C; ++h) s = fmaf(Ws1[h * C + F + k], gz[h], s);
      g[k] = s;
    }
    if (Rs) {  // TModel's per-edge input gradient, recomputed
      float gzt[C];
#pragma unroll
      for (int h = 0; h < C; ++h) {
        float z = valid ? Rs[(long long)h * NS + n] : 0.f;
#pragma unroll
        for (int k = 0; k < F; ++k) z = fmaf(Wt1[h * C + F + k], x[k], z);
        gzt[h] = valid ? g_hsum[(long long)h * NT + cn] * dlrelu(z) : 0.f;
      }
#pragma unroll
      for (int k = 0; k < F; ++k) {
        float s = g[k];
#pragma unroll
        for (int h = 0; h < C; ++h) s = fmaf(Wt1[h * C + F + k], gzt[h], s);
        g[k] = s;
      }
    }
    if (g_next) {
#pragma unroll
      for (int k = 0; k < F; ++k) g[k] += valid ? g_next[(long long)k * E + e] : 0.f;
    }
    if (valid) {
#pragma unroll
      for (int k = 0; k < F; ++k) g_tot[(long long)k * E + e] = g[k];
    }
    if (mu1) {
#pragma unroll
      for (int k = 0; k < F; ++k) {
        const float gk = valid ? g[k] : 0.f;
        sg[k] += gk;
        sgx[k] = fmaf(gk, (yv[k] - mu1[k]) * inv1[k], sgx[k]);
      }
    }
  }
  wg2.block_partial(scratch, partW2 + (size_t)bx * C * (C + 1));
  wg1.block_partial(scratch, partW1 + (size_t)bx * C * F);
  column_partial<C>(colS, geo.SW, geo.FPI, geo.NC, scratch, partCol + (size_t)bx * geo.NC * C);
  if (mu1) {
    float v[2 * F];
#pragma unroll
    for (int k = 0; k < F; ++k) { v[k] = sg[k]; v[F + k] = sgx[k]; }
    block_sum<2 * F>(v, scratch);
    if (t < 2 * F) {
      float val = 0.f;
#pragma unroll
      for (int i = 0; i < 2 * F; ++i) val = (i == t) ? v[i] : val;
      partBN[(size_t)bx * 2 * F + t] = val;
    }
  }
}

// ============================================================ edge BN grad sums
template <int F>
__global__ __launch_bounds__(256) void k_edge_bn_sums(EdgeGeo geo, const float* __restrict__ g,
                                                      const float* __restrict__ y,
                                                      const float* __restrict__ mu1,
                                                      const float* __restrict__ inv1,
                                                      float* __restrict__ partBN) {
  EDGE_PROLOGUE
  __shared__ float scratch[4 * 2 * F];
  float v[2 * F];
#pragma unroll
  for (int k = 0; k < 2 * F; ++k) v[k] = 0.f;
  for (int tile = tile0; tile < tile1; ++tile) {
    EDGE_TILE
    if (valid) {
#pragma unroll
      for (int k = 0; k < F; ++k) {
        const float gk = g[(long long)k * E + e];
        v[k] += gk;
        v[F + k] = fmaf(gk, (y[(long long)k * E + e] - mu1[k]) * inv1[k], v[F + k]);
      }
    }
  }
  block_sum<2 * F>(v, scratch);
  if (t < 2 * F) {
    float val = 0.f;
#pragma unroll
    for (int i = 0; i < 2 * F; ++i) val = (i == t) ? v[i] : val;
    partBN[(size_t)bx * 2 * F + t] = val;
  }
}

// ============================================================ EdgeModel bwd
template <int F>
__global__ __launch_bounds__(256) void k_edge_mlp_bwd(
    EdgeGeo geo, const float* __restrict__ g_tot, const float* __restrict__ alpha,
    const float* __restrict__ gam0, const float* __restrict__ gam1, const float* __restrict__ y,
    const float* __restrict__ xe, const float* __restrict__ xsc, const float* __restrict__ xsh,
    const float* __restrict__ Ps, const float* __restrict__ Pt, const float* __restrict__ W1,
    const float* __restrict__ W2, float* __restrict__ gxe, float* __restrict__ GzEs,
    float* __restrict__ partW2, float* __restrict__ partW1, float* __restrict__ partCol) {
  constexpr int H = 4 * F;
  using WG2 = WGrad<F, H + 1>;  // g_y (x) [a1, 1] -> dW2 | db2
  using WG1 = WGrad<H, F>;      // g_z1 (x) x      -> dW1[:, 2F:3F]
  constexpr int STAGE = WG2::LDS_FLOATS > WG1::LDS_FLOATS ? WG2::LDS_FLOATS : WG1::LDS_FLOATS;
  constexpr int LOOP_N = 4 * STAGE + 4 * H;
  constexpr int TAIL_N0 = (4 * H * (F + 1) > 256 * H) ? 4 * H * (F + 1) : 256 * H;
  constexpr int LDS_N = LOOP_N > TAIL_N0 ? LOOP_N : TAIL_N0;
  EDGE_PROLOGUE
  __shared__ float lds[LDS_N];
  float* region = lds + wave * STAGE;
  float* scratch = lds + 4 * STAGE;  // seg_sum scratch during the loop
  WG2 wg2;
  WG1 wg1;
  wg2.zero();
  wg1.zero();
  float colT[H];
#pragma unroll
  for (int h = 0; h < H; ++h) colT[h] = 0.f;
  for (int tile = tile0; tile < tile1; ++tile) {
    EDGE_TILE
    float gy[F], x[F];
#pragma unroll
    for (int k = 0; k < F; ++k) {
      const float gt = valid ? g_tot[(long long)k * E + e] : 0.f;
      const float yk = valid ? y[(long long)k * E + e] : 0.f;
      gy[k] = valid ? fmaf(gam1[k], yk, fmaf(alpha[k], gt, gam0[k])) : 0.f;
    }
    load_edge<F>(x, xe, xsc, xsh, e, E, valid);
    float z[H], a[H + 1];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float s = valid ? Ps[(long long)h * NS + n] + Pt[(long long)h * NT + cn] : 0.f;
#pragma unroll
      for (int k = 0; k < F; ++k) s = fmaf(W1[h * H + 2 * F + k], x[k], s);
      z[h] = s;
      a[h] = lrelu(s);
    }
    a[H] = 1.f;
    wg2.stage(region, gy, a, lane);
    __syncthreads();
    wg2.accum(region, lane);
    __syncthreads();
    float gz[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float s = 0.f;
#pragma unroll
      for (int o = 0; o < F; ++o) s = fmaf(W2[o * H + h], gy[o], s);
      gz[h] = s * dlrelu(z[h]);
      colT[h] += gz[h];
    }
    if (gxe && valid) {
#pragma unroll
      for (int k = 0; k < F; ++k) {
        float s = 0.f;
#pragma unroll
        for (int h = 0; h < H; ++h) s = fmaf(W1[h * H + 2 * F + k], gz[h], s);
        gxe[(long long)k * E + e] = s;
      }
    }
    wg1.stage(region, gz, x, lane);
    __syncthreads();
    wg1.accum(region, lane);
    __syncthreads();
    seg_sum<H>(gz, geo.SW, scratch);
    if (cl == 0 && fvalid) {
#pragma unroll
      for (int h = 0; h < H; ++h) GzEs[(long long)h * NS + n] = gz[h];
    }
  }
  wg2.block_partial(lds, partW2 + (size_t)bx * F * (H + 1));
  wg1.block_partial(lds, partW1 + (size_t)bx * H * F);
  column_partial<H>(colT, geo.SW, geo.FPI, geo.NC, lds, partCol + (size_t)bx * geo.NC * H);
}

// ============================================================ host side
namespace {

struct Ws {
  char* p;
  size_t left;
  float* take(size_t nfloats) {
    const size_t b = align256(nfloats * sizeof(float));
    if (b > left) return nullptr;
    float* r = reinterpret_cast<float*>(p);
    p += b;
    left -= b;
    return r;
  }
};

int check_dims(const char* where, int G, int NF, int NC, int F) {
  if (G <= 0 || NF <= 0 || NC <= 0) return pf::fail(where, "G, NF, NC must be positive");
  if (NC > 256) return pf::fail(where, "NC > 256 is not supported by the dense edge kernels");
  if (F != 8 && F != 10 && F != 16) return pf::fail(where, "unsupported Fdim (8, 10, 16)");
  if ((long long)G * NF * NC * 16 >= (1ll << 31) * 16ll) return pf::fail(where, "too many edges");
  return 0;
}

#define DISPATCH_F(F, ...)                                   \
  switch (F) {                                               \
    case 8: { constexpr int FF = 8; __VA_ARGS__; } break;    \
    case 10: { constexpr int FF = 10; __VA_ARGS__; } break;  \
    case 16: { constexpr int FF = 16; __VA_ARGS__; } break;  \
    default: return pf::fail("dispatch", "unsupported F");   \
  }

}  // namespace

extern "C" size_t pfsgnn_workspace_bytes(int G, int NF, int NC, int F) {
  const EdgeGeo geo = make_geo(G, NF, NC);
  const size_t nb = geo.nblocks;
  const size_t H = 4 * F, C = 2 * F;
  size_t edge = 0;
  edge = std::max(edge, nb * (1 + 2 * F));                                   // mlp fwd
  edge = std::max(edge, nb * NC * C);                                        // target fwd
  edge = std::max(edge, nb * C * F);                                         // target bwd
  edge = std::max(edge, nb * (C * (C + 1) + C * F + NC * C + 2 * F) + 1024); // source bwd
  edge = std::max(edge, nb * (F * (H + 1) + H * F + NC * H) + 1024);         // edge bwd
  edge = std::max(edge, nb * (NC * 4 + F * (F + 1) + F + 1) + 1024);         // loss
  size_t node = (size_t)64 * 128 * 128 + 4096;                               // wgrad splits
  size_t lay = (size_t)geo.E + 1024;                                         // layout counts
  return (std::max(std::max(edge, node), lay) + 64 * 8) * sizeof(float) + 8 * 256;
}

extern "C" int pfsgnn_edge_mlp_fwd(int G, int NF, int NC, int F, const float* xe,
                                   const float* xsc, const float* xsh, const float* Ps,
                                   const float* Pt, const float* W1, const float* W2,
                                   const float* b2, float* y, float* mu, float* var, void* ws,
                                   size_t ws_bytes, void* stream) {
  if (int rc = check_dims("pfsgnn_edge_mlp_fwd", G, NF, NC, F)) return rc;
  PF_REQUIRE(xe && Ps && Pt && W1 && W2 && b2 && y && mu && var, "pfsgnn_edge_mlp_fwd", "null");
  const EdgeGeo geo = make_geo(G, NF, NC);
  Ws w{reinterpret_cast<char*>(ws), ws_bytes};
  float* part = w.take((size_t)geo.nblocks * (1 + 2 * F));
  PF_REQUIRE(part, "pfsgnn_edge_mlp_fwd", "workspace too small");
  hipStream_t st = as_stream(stream);
  { pf::Timer tm_("edge_mlp_fwd", st);
  DISPATCH_F(F, hipLaunchKernelGGL(k_edge_mlp_fwd<FF>, dim3(geo.nblocks), dim3(256), 0, st, geo,
                                   xe, xsc, xsh, Ps, Pt, W1, W2, b2, y, part));
  tm_.end(); }
  hipLaunchKernelGGL(k_moments_finalize, dim3(1), dim3(64), 0, st, part, geo.nblocks, F, geo.E,
                     mu, var);
  return pf::check_launch("pfsgnn_edge_mlp_fwd");
}

extern "C" int pfsgnn_source_fwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                                 const float* sh, const float* Qt, const float* Ws1,
                                 const float* Ws2, const float* bs2, float* mom, float* hs,
                                 void* stream) {
  if (int rc = check_dims("pfsgnn_source_fwd", G, NF, NC, F)) return rc;
  PF_REQUIRE(y && Qt && Ws1 && Ws2 && bs2 && mom && hs, "pfsgnn_source_fwd", "null");
  const EdgeGeo geo = make_geo(G, NF, NC);
  hipStream_t st = as_stream(stream);
  { pf::Timer tm_("source_fwd", st);
  DISPATCH_F(F, hipLaunchKernelGGL(k_source_fwd<FF>, dim3(geo.nblocks), dim3(256), 0, st, geo, y,
                                   sc, sh, Qt, Ws1, Ws2, bs2, mom, hs));
  tm_.end(); }
  return pf::check_launch("pfsgnn_source_fwd");
}

extern "C" int pfsgnn_target_fwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                                 const float* sh, const float* Rs, const float* Wt1, float* hsum,
                                 void* ws, size_t ws_bytes, void* stream) {
  if (int rc = check_dims("pfsgnn_target_fwd", G, NF, NC, F)) return rc;
  PF_REQUIRE(y && Rs && Wt1 && hsum, "pfsgnn_target_fwd", "null");
  const EdgeGeo geo = make_geo(G, NF, NC);
  Ws w{reinterpret_cast<char*>(ws), ws_bytes};
  float* part = w.take((size_t)geo.nblocks * NC * 2 * F);
  PF_REQUIRE(part, "pfsgnn_target_fwd", "workspace too small");
  hipStream_t st = as_stream(stream);
  { pf::Timer tm_("target_fwd", st);
  DISPATCH_F(F, hipLaunchKernelGGL(k_target_fwd<FF>, dim3(geo.nblocks), dim3(256), 0, st, geo, y,
                                   sc, sh, Rs, Wt1, part));
  tm_.end(); }
  launch_reduce_columns(part, G, geo.BPG, NC, 2 * F, hsum, st);
  return pf::check_launch("pfsgnn_target_fwd");
}

extern "C" int pfsgnn_target_bwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                                 const float* sh, const float* Rs, const float* Wt1,
                                 const float* g_hsum, float* GzT, float* dWt1, float* gxe,
                                 void* ws, size_t ws_bytes, void* stream) {
  if (int rc = check_dims("pfsgnn_target_bwd", G, NF, NC, F)) return rc;
  PF_REQUIRE(y && Rs && Wt1 && g_hsum && GzT && dWt1, "pfsgnn_target_bwd", "null");
  const EdgeGeo geo = make_geo(G, NF, NC);
  const int C = 2 * F;
  Ws w{reinterpret_cast<char*>(ws), ws_bytes};
  float* part = w.take((size_t)geo.nblocks * C * F);
  PF_REQUIRE(part, "pfsgnn_target_bwd", "workspace too small");
  hipStream_t st = as_stream(stream);
  { pf::Timer tm_("target_bwd", st);
  DISPATCH_F(F, hipLaunchKernelGGL(k_target_bwd<FF>, dim3(geo.nblocks), dim3(256), 0, st, geo, y,
                                   sc, sh, Rs, Wt1, g_hsum, GzT, gxe, part));
  tm_.end(); }
  launch_reduce_rows(part, geo.nblocks, (size_t)C * F, F, C, F, dWt1 + F, C, 1, 1.f, st);
  return pf::check_launch("pfsgnn_target_bwd");
}

extern "C" int pfsgnn_source_bwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                                 const float* sh, const float* Qt, const float* Ws1,
                                 const float* Ws2, const float* bs2, const float* mean,
                                 const float* coef, const float* Rs, const float* Wt1,
                                 const float* g_hsum, const float* g_next, const float* mu1,
                                 const float* inv1, float* g_tot, float* GzS, float* dWs1,
                                 float* dWs2, float* dbs2, float* Sg, float* Sgx, void* ws,
                                 size_t ws_bytes, void* stream) {
  if (int rc = check_dims("pfsgnn_source_bwd", G, NF, NC, F)) return rc;
  PF_REQUIRE(y && Qt && Ws1 && Ws2 && bs2 && mean && coef && g_tot && GzS && dWs1 && dWs2 && dbs2,
             "pfsgnn_source_bwd", "null");
  PF_REQUIRE((Rs == nullptr) == (Wt1 == nullptr) && (Rs == nullptr) == (g_hsum == nullptr),
             "pfsgnn_source_bwd", "Rs, Wt1, g_hsum must be given together");
  PF_REQUIRE(!mu1 || (inv1 && Sg && Sgx), "pfsgnn_source_bwd", "mu1 needs inv1, Sg, Sgx");
  const EdgeGeo geo = make_geo(G, NF, NC);
  const int C = 2 * F;
  const size_t nb = geo.nblocks;
  Ws w{reinterpret_cast<char*>(ws), ws_bytes};
  float* pW2 = w.take(nb * C * (C + 1));
  float* pW1 = w.take(nb * C * F);
  float* pCol = w.take(nb * NC * C);
  float* pBN = w.take(nb * 2 * F);
  PF_REQUIRE(pW2 && pW1 && pCol && pBN, "pfsgnn_source_bwd", "workspace too small");
  hipStream_t st = as_stream(stream);
  { pf::Timer tm_("source_bwd", st);
  DISPATCH_F(F, hipLaunchKernelGGL(k_source_bwd<FF>, dim3(geo.nblocks), dim3(256), 0, st, geo, y,
                                   sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, Rs, Wt1, g_hsum, g_next,
                                   mu1, inv1, g_tot, pW2, pW1, pCol, pBN));
  tm_.end(); }
  launch_reduce_rows(pW2, nb, (size_t)C * (C + 1), C + 1, C, C, dWs2, C, 1, 1.f, st);
  launch_reduce_rows(pW2 + C, nb, (size_t)C * (C + 1), C + 1, C, 1, dbs2, 1, 1, 1.f, st);
  launch_reduce_rows(pW1, nb, (size_t)C * F, F, C, F, dWs1 + F, C, 1, 1.f, st);
  launch_reduce_columns(pCol, G, geo.BPG, NC, C, GzS, st);
  if (mu1) {
    launch_reduce_rows(pBN, nb, (size_t)2 * F, F, 1, F, Sg, F, 0, 1.f, st);
    launch_reduce_rows(pBN + F, nb, (size_t)2 * F, F, 1, F, Sgx, F, 0, 1.f, st);
  }
  return pf::check_launch("pfsgnn_source_bwd");
}

extern "C" int pfsgnn_edge_bn_grad_sums(int G, int NF, int NC, int F, const float* g,
                                        const float* y, const float* mu1, const float* inv1,
                                        float* Sg, float* Sgx, void* ws, size_t ws_bytes,
                                        void* stream) {
  if (int rc = check_dims("pfsgnn_edge_bn_grad_sums", G, NF, NC, F)) return rc;
  PF_REQUIRE(g && y && mu1 && inv1 && Sg && Sgx, "pfsgnn_edge_bn_grad_sums", "null");
  const EdgeGeo geo = make_geo(G, NF, NC);
  Ws w{reinterpret_cast<char*>(ws), ws_bytes};
  float* pBN = w.take((size_t)geo.nblocks * 2 * F);
  PF_REQUIRE(pBN, "pfsgnn_edge_bn_grad_sums", "workspace too small");
  hipStream_t st = as_stream(stream);
  { pf::Timer tm_("edge_bn_sums", st);
  DISPATCH_F(F, hipLaunchKernelGGL(k_edge_bn_sums<FF>, dim3(geo.nblocks), dim3(256), 0, st, geo, g,
                                   y, mu1, inv1, pBN));
  tm_.end(); }
  launch_reduce_rows(pBN, geo.nblocks, (size_t)2 * F, F, 1, F, Sg, F, 0, 1.f, st);
  launch_reduce_rows(pBN + F, geo.nblocks, (size_t)2 * F, F, 1, F, Sgx, F, 0, 1.f, st);
  return pf::check_launch("pfsgnn_edge_bn_grad_sums");
}

extern "C" int pfsgnn_edge_mlp_bwd(int G, int NF, int NC, int F, const float* g_tot,
                                   const float* alpha, const float* gam0, const float* gam1,
                                   const float* y, const float* xe, const float* xsc,
                                   const float* xsh, const float* Ps, const float* Pt,
                                   const float* W1, const float* W2, float* dW1, float* dW2,
                                   float* db2, float* gxe, float* GzEs, float* GzEt, void* ws,
                                   size_t ws_bytes, void* stream) {
  if (int rc = check_dims("pfsgnn_edge_mlp_bwd", G, NF, NC, F)) return rc;
  PF_REQUIRE(g_tot && alpha && gam0 && gam1 && y && xe && Ps && Pt && W1 && W2 && dW1 && dW2 &&
                 db2 && GzEs && GzEt,
             "pfsgnn_edge_mlp_bwd", "null");
  const EdgeGeo geo = make_geo(G, NF, NC);
  const int H = 4 * F;
  const size_t nb = geo.nblocks;
  Ws w{reinterpret_cast<char*>(ws), ws_bytes};
  float* pW2 = w.take(nb * F * (H + 1));
  float* pW1 = w.take(nb * H * F);
  float* pCol = w.take(nb * NC * H);
  PF_REQUIRE(pW2 && pW1 && pCol, "pfsgnn_edge_mlp_bwd", "workspace too small");
  hipStream_t st = as_stream(stream);
  { pf::Timer tm_("edge_mlp_bwd", st);
  DISPATCH_F(F, hipLaunchKernelGGL(k_edge_mlp_bwd<FF>, dim3(geo.nblocks), dim3(256), 0, st, geo,
                                   g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2, gxe,
                                   GzEs, pW2, pW1, pCol));
  tm_.end(); }
  launch_reduce_rows(pW2, nb, (size_t)F * (H + 1), H + 1, F, H, dW2, H, 1, 1.f, st);
  launch_reduce_rows(pW2 + H, nb, (size_t)F * (H + 1), H + 1, F, 1, db2, 1, 1, 1.f, st);
  launch_reduce_rows(pW1, nb, (size_t)H * F, F, H, F, dW1 + 2 * F, H, 1, 1.f, st);
  launch_reduce_columns(pCol, G, geo.BPG, NC, H, GzEt, st);
  return pf::check_launch("pfsgnn_edge_mlp_bwd");
}
