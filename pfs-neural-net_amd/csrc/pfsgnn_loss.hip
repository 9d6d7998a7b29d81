// pfsgnn_loss.hip -- the training objective (train.py:21-80) fused over edges,
// and the edge-layout helpers (canonical order <-> the caller's edge_index).
#include "pfsgnn_common.h"
#include "../../include/pfsgnn.h"

#include <algorithm>
#include <cmath>

#define EDGE_PROLOGUE                                                       \
  const int t = threadIdx.x, lane = t & 63;                                 \
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);                  \
  const int bx = PF_LOGICAL_BLOCK(geo);                                     \
  if (bx >= geo.nblocks) return;                                            \
  const int ks = bx % geo.KS, grp = bx / geo.KS;                            \
  const int fg = grp % geo.NFG, gg = grp / geo.NFG;                         \
  const int f = fg * 64 + lane;                                             \
  const bool fvalid = f < geo.NF;                                           \
  const long long n = (long long)gg * geo.NF + (fvalid ? f : 0);            \
  const long long nbase = (long long)gg * geo.NF + (long long)fg * 64;      \
  const int nvalid = min(64, geo.NF - fg * 64);                             \
  const int c0 = ks * geo.CPS, c1 = min(geo.NC, c0 + geo.CPS);              \
  const long long E = geo.E, NS = geo.NS, NT = geo.NT;                      \
  (void)E; (void)NS; (void)NT; (void)n; (void)nbase; (void)nvalid; (void)t;

#define CLASS_LOOP_BEGIN                                                    \
  for (int c = c0 + wave; c < c1; c += 4) {                                 \
    const long long cn = (long long)gg * geo.NC + c;                        \
    const long long e = cn * geo.NF + (fvalid ? f : 0);                     \
    const long long eu = n * geo.NC + c; /* train.py's fiber-major position */

#define CLASS_LOOP_END }

// the next class's edge rows of this wave prefetched one iteration ahead
// (register ring; the loop body is one long dependent chain per class)
#define Y_PREFETCH_DECL(F)                                                    \
  float yq[F];                                                              \
  auto yload = [&](int cc) {                                                \
    const long long ee = ((long long)gg * geo.NC + cc) * geo.NF + (fvalid ? f : 0); \
    _Pragma("unroll") for (int k = 0; k < F; ++k)                           \
      yq[k] = (fvalid && cc < c1) ? y[(long long)k * E + ee] : 0.f;         \
  };                                                                        \
  yload(c0 + wave);
#define Y_TAKE(F, x)                                                          \
  _Pragma("unroll") for (int k = 0; k < F; ++k)                             \
    x[k] = sc ? fmaf(yq[k], sc[k], sh[k]) : yq[k];                          \
  yload(c + 4);

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

struct SoftFloor {
  float r, corr, two_pi, inv_pi;  // r = exp(-1/sharpness) (0 if sharpness == 0)
};

static SoftFloor make_softfloor(float sharpness) {
  SoftFloor s;
  const float pi = (float)M_PI;                           // x.new_tensor(np.pi)
  s.r = sharpness == 0.f ? 0.f : expf(-1.0f / sharpness); // train.py:26
  s.corr = atanf(s.r / (1.0f - s.r));
  s.two_pi = 2.0f * pi;
  s.inv_pi = 1.0f / pi;
  return s;
}

// decoder_e + softplus*scale + softfloor + clamp (train.py:42-49, gnn.py:307-312).
// LOSS_FAST: sin / cos of 2 pi x as one sincospi of 2x (the reduction is exact
// in revolutions, no large-argument path) and one reciprocal of T_i per edge
// for the two divisions by it
#ifndef LOSS_FAST
#define LOSS_FAST 1
#endif
template <int F>
struct EdgeLoss {
  float zd[F], ad[F], pred, time, Ti, xx, th, graw, gal, tt, cth, invTi;
  __device__ __forceinline__ void run(const float (&x)[F], const float* __restrict__ Wd1,
                                      const float* __restrict__ bd1, const float* __restrict__ Wd2,
                                      const float* __restrict__ bd2, float scale, float Ti_,
                                      float noise, const SoftFloor& sf) {
    pred = bd2[0];
#pragma unroll
    for (int j = 0; j < F; ++j) {
      float s = bd1[j];
#pragma unroll
      for (int k = 0; k < F; ++k) s = fmaf(Wd1[j * F + k], x[k], s);
      zd[j] = s;
      ad[j] = lrelu(s);
      pred = fmaf(Wd2[j], ad[j], pred);
    }
    const float sp = pred > 20.f ? pred : log1pf(expf(pred));  // F.softplus (threshold 20)
    time = sp * scale;
    Ti = Ti_;
#if LOSS_FAST
    invTi = 1.0f / Ti;
    xx = fmaf(time, invTi, noise);
    float sth;
    sincospif(2.0f * xx, &sth, &cth);
    graw = xx + sf.inv_pi * (atanf(sf.r * sth / (1.0f - sf.r * cth)) - sf.corr);
#else
    xx = time / Ti + noise;
    th = sf.two_pi * xx;
    cth = cosf(th);
    graw = xx + sf.inv_pi * (atanf(sf.r * sinf(th) / (1.0f - sf.r * cth)) - sf.corr);
#endif
    gal = graw < 0.f ? 0.f : graw;  // torch.maximum(0, g) (NaN propagates)
    tt = gal * Ti;
  }
};

// decoder_e's weights staged in LDS (read as broadcasts inside the edge loop):
// held in SGPRs they overflowed the scalar file (119 / 139 SGPR spills, each
// use a v_readlane in the loop)
template <int F>
struct DecW {
  static constexpr int N = F * F + 2 * F + 1;
  float w[N];   // Wd1 [F][F] | bd1 [F] | Wd2 [F] | bd2
  __device__ __forceinline__ void load(const float* __restrict__ Wd1, const float* __restrict__ bd1,
                                       const float* __restrict__ Wd2, const float* __restrict__ bd2) {
    for (int i = threadIdx.x; i < N; i += blockDim.x)
      w[i] = i < F * F ? Wd1[i] : i < F * F + F ? bd1[i - F * F]
                                : i < F * F + 2 * F ? Wd2[i - F * F - F] : bd2[0];
  }
};
// the weights' base as an opaque value per loop iteration: the compiler would
// otherwise hoist all F*F + 2F + 1 loop-invariant reads into VGPRs (occupancy 7 -> 3)
template <int F>
__device__ __forceinline__ const float* dec_base(const DecW<F>& d) {
  int lo = 0;
  asm volatile("" : "+v"(lo));
  return d.w + lo;
}

template <int F>
__global__ __launch_bounds__(256) void k_loss_fwd(EdgeGeo geo, const float* __restrict__ y,
                                                  const float* __restrict__ sc,
                                                  const float* __restrict__ sh,
                                                  const float* __restrict__ Wd1,
                                                  const float* __restrict__ bd1,
                                                  const float* __restrict__ Wd2,
                                                  const float* __restrict__ bd2,
                                                  const float* __restrict__ ci, float scale,
                                                  SoftFloor sf, float noiselevel, uint64_t key0,
                                                  const unsigned long long* __restrict__ seed_dev,
                                                  float* __restrict__ fiber_time,
                                                  float* __restrict__ tt_out,
                                                  float* __restrict__ part) {
  EDGE_PROLOGUE
  const uint64_t key = seed_dev ? pf_noise_key(*seed_dev) : key0;
  __shared__ float scratch[4 * 64];
  __shared__ __attribute__((aligned(16))) DecW<F> dw;
  dw.load(Wd1, bd1, Wd2, bd2);
  __syncthreads();
  float ft = 0.f;
  const float nw = (float)nvalid;
  Y_PREFETCH_DECL(F)
  CLASS_LOOP_BEGIN
    (void)e;
    float x[F];
    Y_TAKE(F, x)
    const float noise = noiselevel * (pf_uniform(key, (uint64_t)eu) - 0.5f);
    EdgeLoss<F> L;
    const float* dwp = dec_base(dw);
    L.run(x, dwp, dwp + F * F, dwp + F * F + F, dwp + F * F + 2 * F, scale, ci[cn], noise, sf);
    const float tt = fvalid ? L.tt : 0.f;
    ft += tt;
    if (tt_out && fvalid) tt_out[eu] = L.tt;
    const float np = wave_sum(fvalid ? L.gal : 0.f);
    const float mw = wave_sum(tt) / nw;
    const float dv = fvalid ? tt - mw : 0.f;
    const float qw = wave_sum(dv * dv);
    if (lane == 0) {
      float* o = part + (((size_t)gg * geo.NFG + fg) * geo.NC + c) * 4;
      o[0] = np; o[1] = nw; o[2] = mw; o[3] = qw;
    }
  CLASS_LOOP_END
  // fiber time: merge the 4 waves, KS-partial per fiber
  __syncthreads();
  scratch[wave * 64 + lane] = ft;
  __syncthreads();
  if (t < 64 && t < nvalid)
    fiber_time[(size_t)ks * NS + nbase + t] =
        ((scratch[t] + scratch[64 + t]) + scratch[128 + t]) + scratch[192 + t];
}

__device__ __forceinline__ double wave_dsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one wave per class: lane l takes the fiber groups l, l + 64, ... and the
// moments merge in closed form (mean = sum c_b m_b / sum c_b, M2 = sum (q_b +
// c_b (m_b - mean)^2), in double; fixed lane and butterfly order): the loads
// are independent, where a per-thread Chan chain ran NFG dependent divisions
__global__ __launch_bounds__(256) void k_loss_class_reduce(const float* __restrict__ part, int G,
                                                           int NFG, int NC, int NF,
                                                           float* __restrict__ n_prime,
                                                           float* __restrict__ tmean,
                                                           float* __restrict__ tvar) {
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;  // over G*NC
  if (idx >= G * NC) return;
  const int g = idx / NC, c = idx - g * NC;
  const float* q0 = part + ((size_t)g * NFG * NC + c) * 4;
  const size_t stride = (size_t)NC * 4;
  double P = 0, C = 0, S = 0;
  for (int b = lane; b < NFG; b += 64) {
    const float* q = q0 + (size_t)b * stride;
    P += q[0];
    C += q[1];
    S += (double)q[1] * (double)q[2];
  }
  P = wave_dsum(P);
  C = wave_dsum(C);
  S = wave_dsum(S);
  const double M = C > 0 ? S / C : 0.0;
  double Q = 0;
  for (int b = lane; b < NFG; b += 64) {
    const float* q = q0 + (size_t)b * stride;
    const double d = (double)q[2] - M;
    Q += (double)q[3] + (double)q[1] * d * d;
  }
  Q = wave_dsum(Q);
  if (lane == 0) {
    n_prime[idx] = (float)P;
    tmean[idx] = (float)M;
    tvar[idx] = NF > 1 ? (float)(Q / (double)(NF - 1)) : NAN;  // torch.var, correction=1
  }
}

// torch.min propagates NaN (train.py:53: a class with N_i = 0 gives 0/0);
// fminf would drop it
__device__ __forceinline__ float nan_min(float a, float b) {
  return (a != a) ? a : ((b != b) ? b : (b < a ? b : a));
}

// one block per graph: train.py:53-71 and the per-node gradient coefficients
__global__ __launch_bounds__(256) void k_loss_finalize(
    int NF, int NC, int NT, const float* __restrict__ n_prime, const float* __restrict__ fiber_time,
    const float* __restrict__ tvar, const float* __restrict__ ci, float pclass, float pfiber,
    float total_time, float nfields, float wutils, float wvar, float* __restrict__ loss,
    float* __restrict__ utils, float* __restrict__ variance, float* __restrict__ Gn,
    float* __restrict__ Gf, float* __restrict__ Gv) {
  const int g = blockIdx.x, t = threadIdx.x;
  __shared__ float scratch[4 * 4];
  __shared__ float smin[256];
  // completeness min
  float mn = INFINITY;
  for (int c = t; c < NC; c += 256) {
    const long long cn = (long long)g * NC + c;
    const float Ni = ci[NT + cn] / nfields;
    const float comp = n_prime[cn] / Ni;
    mn = nan_min(mn, comp);
  }
  smin[t] = mn;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) smin[t] = nan_min(smin[t], smin[t + s]);
    __syncthreads();
  }
  const float umin = smin[0];
  float v[4] = {0.f, 0.f, 0.f, 0.f};  // ties, class penalty, fiber penalty, variance
  for (int c = t; c < NC; c += 256) {
    const long long cn = (long long)g * NC + c;
    const float Ni = ci[NT + cn] / nfields;
    const float comp = n_prime[cn] / Ni;
    v[0] += comp == umin ? 1.f : 0.f;
    const float over = fmaxf(n_prime[cn] - Ni, 0.f);
    v[1] += over * over;
    v[3] += tvar[cn];
  }
  for (int f = t; f < NF; f += 256) {
    const long long n = (long long)g * NF + f;
    const float ot = fiber_time[n] - total_time;
    const float lk = lrelu(ot);
    v[2] += lk * lk;
    Gf[n] = pfiber * 2.f * lk * dlrelu(ot);
  }
  block_sum<4>(v, scratch);
  const float ties = v[0];
  for (int c = t; c < NC; c += 256) {
    const long long cn = (long long)g * NC + c;
    const float Ni = ci[NT + cn] / nfields;
    const float comp = n_prime[cn] / Ni;
    const float over = fmaxf(n_prime[cn] - Ni, 0.f);
    Gn[cn] = (comp == umin ? -wutils / ties : 0.f) / Ni + 2.f * pclass * over;
    Gv[cn] = -wvar * 2.f / (float)(NF - 1);
  }
  if (t == 0) {
    utils[g] = umin;
    variance[g] = v[3];
    loss[g] = -wutils * umin + pfiber * v[2] + pclass * v[1] - wvar * v[3];
  }
}

template <int F, bool BN>
__global__ __launch_bounds__(256) void k_loss_bwd(EdgeGeo geo, const float* __restrict__ y,
                                                  const float* __restrict__ sc,
                                                  const float* __restrict__ sh,
                                                  const float* __restrict__ Wd1,
                                                  const float* __restrict__ bd1,
                                                  const float* __restrict__ Wd2,
                                                  const float* __restrict__ bd2,
                                                  const float* __restrict__ ci, float scale,
                                                  SoftFloor sf, float noiselevel, uint64_t key0,
                                                  const unsigned long long* __restrict__ seed_dev,
                                                  const float* __restrict__ Gn,
                                                  const float* __restrict__ Gf,
                                                  const float* __restrict__ Gv,
                                                  const float* __restrict__ tmean,
                                                  const float* __restrict__ gscale,
                                                  float* __restrict__ gxe,
                                                  float* __restrict__ partW,
                                                  float* __restrict__ partV,
                                                  const float* __restrict__ bn_mu1,
                                                  const float* __restrict__ bn_inv1,
                                                  float* __restrict__ partBN) {
  using WG = WGrad<F, F + 1>;  // g_zd (x) [x, 1] -> dWd1 | dbd1
  EDGE_PROLOGUE
  const uint64_t key = seed_dev ? pf_noise_key(*seed_dev) : key0;
  constexpr int LDS_N = (4 * WG::LDS_FLOATS > 4 * F * (F + 1)) ? 4 * WG::LDS_FLOATS
                                                                : 4 * F * (F + 1);
  __shared__ float lds[LDS_N + 4 * (F + 1)];
  __shared__ __attribute__((aligned(16))) DecW<F> dw;
  dw.load(Wd1, bd1, Wd2, bd2);
  __syncthreads();
  float* region = lds + wave * WG::LDS_FLOATS;
  WG wg;
  wg.zero();
  float acc[F + 1];
#pragma unroll
  for (int j = 0; j <= F; ++j) acc[j] = 0.f;
  const float gs = gscale ? gscale[0] : 1.f;
  const float Gf_f = fvalid ? Gf[n] : 0.f;
  // (partBN) the final edge BatchNorm's backward sums of the gradient this
  // kernel writes: sum g and sum g * (y - mu1) * inv1 per channel
  // (1/scale applied once, after the loop)
  float bsg[F], bsx[F];
#pragma unroll
  for (int k = 0; k < F; ++k) bsg[k] = bsx[k] = 0.f;
  Y_PREFETCH_DECL(F)
  CLASS_LOOP_BEGIN
    const float Ti = ci[cn], Gn_c = Gn[cn], Gv_c = Gv[cn], tm_c = tmean[cn];
    float x[F + 1], yr[F];   // (BN: y - mu1, kept for the sums)
#pragma unroll
    for (int k = 0; k < F; ++k) yr[k] = BN ? yq[k] - bn_mu1[k] : 0.f;
    Y_TAKE(F, x)
    x[F] = 1.f;
    const float noise = noiselevel * (pf_uniform(key, (uint64_t)eu) - 0.5f);
    EdgeLoss<F> L;
    float xf[F];
#pragma unroll
    for (int k = 0; k < F; ++k) xf[k] = x[k];
    const float* dwp = dec_base(dw);
    L.run(xf, dwp, dwp + F * F, dwp + F * F + F, dwp + F * F + 2 * F, scale, Ti, noise, sf);
    const float g_tt = Gf_f + Gv_c * (L.tt - tm_c);
    const float g_gal = Gn_c + Ti * g_tt;
    const float mask = L.graw > 0.f ? 1.f : (L.graw == 0.f ? 0.5f : 0.f);
    const float cth = L.cth;
    const float dsf = 1.f + 2.f * (sf.r * cth - sf.r * sf.r) / (1.f - 2.f * sf.r * cth + sf.r * sf.r);
#if LOSS_FAST
    const float g_time = g_gal * mask * dsf * L.invTi;
#else
    const float g_time = g_gal * mask * dsf / Ti;
#endif
    const float sig = L.pred > 20.f ? 1.f : 1.f / (1.f + expf(-L.pred));
    const float g_pred = fvalid ? gs * g_time * scale * sig : 0.f;
    float gz[F];
#pragma unroll
    for (int j = 0; j < F; ++j) {
      acc[j] = fmaf(g_pred, L.ad[j], acc[j]);
      gz[j] = dwp[F * F + F + j] * g_pred * dlrelu(L.zd[j]);
    }
    acc[F] += g_pred;
    if (fvalid) {
#pragma unroll
      for (int k = 0; k < F; ++k) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < F; ++j) s = fmaf(dwp[j * F + k], gz[j], s);
        gxe[(long long)k * E + e] = s;
        if (BN) {
          bsg[k] += s;
          bsx[k] = fmaf(s, yr[k], bsx[k]);
        }
      }
    }
    wg.stage(region, gz, x, lane);
    wave_lds_sync();
    wg.accum(region, lane);
    wave_lds_sync();
  CLASS_LOOP_END
  wg.block_partial(lds, partW + (size_t)bx * F * (F + 1));
  block_sum<F + 1>(acc, lds + LDS_N);
  if (t <= F) {
    float val = 0.f;
#pragma unroll
    for (int i = 0; i <= F; ++i) val = (i == t) ? acc[i] : val;
    partV[(size_t)bx * (F + 1) + t] = val;
  }
  if (BN) {   // [nb][2F]: sum g | sum g xhat, the layout k_bn2_coef_part reads
    __shared__ float bred[4 * 2 * F];
    float v[2 * F];
#pragma unroll
    for (int k = 0; k < F; ++k) {
      v[k] = bsg[k];
      v[F + k] = bsx[k] * bn_inv1[k];
    }
    block_sum<2 * F>(v, bred);
    if (t < 2 * F) {
      float val = 0.f;
#pragma unroll
      for (int i = 0; i < 2 * F; ++i) val = (i == t) ? v[i] : val;
      partBN[(size_t)bx * 2 * F + t] = val;
    }
  }
}

// ------------------------------------------------------------ layout
// Canonical index k = (g*NC + c)*NF + f.  mode 0: user edge id = perm[k];
// mode 1: user order is train.py's fiber-major (g*NF + f)*NC + c (graph.py /
// cartesian_prod, train.py:94); mode 2: user order is already canonical.
__device__ __forceinline__ long long user_index(long long k, int NF, int NC, int mode,
                                                const int32_t* __restrict__ perm) {
  if (mode == 2) return k;
  if (mode == 0) return perm[k];
  const long long gc = k / NF, f = k - gc * NF;
  const long long g = gc / NC, c = gc - g * NC;
  return (g * NF + f) * NC + c;
}

__global__ void k_layout_init(int32_t* status) {
  if (threadIdx.x == 0) { status[0] = 1; status[1] = 1; status[2] = 1; }
}

__global__ void k_layout_scatter(const int64_t* __restrict__ ei, long long E, int G, int NF, int NC,
                                 int32_t* __restrict__ perm, int32_t* __restrict__ cnt,
                                 int32_t* __restrict__ status) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const long long NS = (long long)G * NF, NT = (long long)G * NC;
  const long long s = ei[e], tg = ei[E + e];
  if (s < 0 || s >= NS || tg < 0 || tg >= NT) {
    atomicAnd(&status[0], 0); atomicAnd(&status[1], 0); atomicAnd(&status[2], 0);
    return;
  }
  const long long g = s / NF, gt = tg / NC;
  if (g != gt) {
    atomicAnd(&status[0], 0); atomicAnd(&status[1], 0); atomicAnd(&status[2], 0);
    return;
  }
  const long long f = s - g * NF, c = tg - gt * NC;
  const long long k = (g * NC + c) * NF + f;
  atomicAdd(&cnt[k], 1);
  perm[k] = (int32_t)e;
  if (e != s * NC + c) atomicAnd(&status[1], 0);
  if (e != k) atomicAnd(&status[2], 0);
}

__global__ void k_layout_check(const int32_t* __restrict__ cnt, long long E,
                               int32_t* __restrict__ status) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= E) return;
  if (cnt[k] != 1) { atomicAnd(&status[0], 0); atomicAnd(&status[1], 0); atomicAnd(&status[2], 0); }
}

__global__ void k_to_canonical(const float* __restrict__ src, long long E, int NF, int NC, int F,
                               int mode, const int32_t* __restrict__ perm,
                               float* __restrict__ dst) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= E) return;
  const long long eu = user_index(k, NF, NC, mode, perm);
  for (int j = 0; j < F; ++j) dst[(long long)j * E + k] = src[eu * F + j];
}

__global__ void k_from_canonical(const float* __restrict__ y, const float* __restrict__ sc,
                                 const float* __restrict__ sh, long long E, int NF, int NC, int F,
                                 int mode, const int32_t* __restrict__ perm, int rowmajor,
                                 float* __restrict__ dst) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= E) return;
  const long long eu = user_index(k, NF, NC, mode, perm);
  for (int j = 0; j < F; ++j) {
    float v = y[(long long)j * E + k];
    if (sc) v = fmaf(v, sc[j], sh[j]);
    if (rowmajor) dst[eu * F + j] = v;
    else dst[(long long)j * E + eu] = v;
  }
}

// Fiber-major row-major output (train.py's order) through an LDS tile: a block
// takes 64 fibers x 16 classes of one graph, reads the canonical rows
// coalesced along the fibers, and writes each fiber's 16 classes x F values as
// one contiguous run (dst row (g*NF + f)*NC + c).
#define FC_CT 16
template <int F>
__global__ __launch_bounds__(256) void k_from_canonical_fm(const float* __restrict__ y,
                                                           const float* __restrict__ sc,
                                                           const float* __restrict__ sh, int G,
                                                           int NF, int NC,
                                                           float* __restrict__ dst) {
  __shared__ float tile[64 * FC_CT * F + 64];
  const int t = threadIdx.x;
  const int nfg = (NF + 63) / 64, ncg = (NC + FC_CT - 1) / FC_CT;
  const int b = blockIdx.x;
  const int cg = b % ncg, fg = (b / ncg) % nfg, g = b / (ncg * nfg);
  const int f0 = fg * 64, cb = cg * FC_CT;
  const int nf = min(64, NF - f0), nc = min(FC_CT, NC - cb);
  const long long E = (long long)G * NF * NC;
  // tile[(fl * FC_CT + cl) * F + j]  (fiber-major, then class, then feature)
  for (int idx = t; idx < F * FC_CT * 64; idx += 256) {
    const int fl = idx & 63, rest = idx >> 6;
    const int cl = rest % FC_CT, j = rest / FC_CT;
    if (fl < nf && cl < nc) {
      float v = y[(long long)j * E + ((long long)g * NC + cb + cl) * NF + f0 + fl];
      if (sc) v = fmaf(v, sc[j], sh[j]);
      tile[(fl * FC_CT + cl) * F + j] = v;
    }
  }
  __syncthreads();
  const int run = nc * F;  // contiguous floats per fiber
  for (int idx = t; idx < nf * run; idx += 256) {
    const int fl = idx / run, r = idx - fl * run;
    dst[(((long long)g * NF + f0 + fl) * NC + cb) * F + r] = tile[fl * FC_CT * F + r];
  }
}

__global__ void k_fiber_partial_sum(const float* __restrict__ part, int KS, long long len,
                                    float* __restrict__ out) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= len) return;
  float s = 0.f;
  for (int k = 0; k < KS; ++k) s += part[(size_t)k * len + idx];
  out[idx] = s;
}

// ------------------------------------------------------------ host side
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
  if (G <= 0 || NF <= 1 || NC <= 0) return pf::fail(where, "need G > 0, NF > 1, NC > 0");
  if (NC > 256) return pf::fail(where, "NC > 256 is not supported by the dense edge kernels");
  if (F != 8 && F != 10 && F != 16) return pf::fail(where, "unsupported Fdim (8, 10, 16)");
  return 0;
}
#define DISPATCH_F(F, ...)                                   \
  switch (F) {                                               \
    case 8: { constexpr int FF = 8; __VA_ARGS__; } break;    \
    case 10: { constexpr int FF = 10; __VA_ARGS__; } break;  \
    case 16: { constexpr int FF = 16; __VA_ARGS__; } break;  \
    default: return pf::fail("dispatch", "unsupported F");   \
  }
// the loss kernels' grid: class splits to about PFSGNN_LOSS_BLOCKS blocks
// (A/B knob; default PF_TARGET_BLOCKS)
EdgeGeo loss_geo(int G, int NF, int NC) {
  static const int tb = [] {
    const char* e = getenv("PFSGNN_LOSS_BLOCKS");
    return e && atoi(e) > 0 ? atoi(e) : PF_TARGET_BLOCKS;
  }();
  return make_geo(G, NF, NC, tb);
}
}  // namespace


extern "C" int pfsgnn_loss_fwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                               const float* sh, const float* Wd1, const float* bd1,
                               const float* Wd2, const float* bd2, const float* ci, float scale,
                               float sharpness, float noiselevel, unsigned long long seed,
                               const unsigned long long* seed_dev, float* n_prime, float* fiber_time, float* tmean, float* tvar,
                               float* tt, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = check_dims("pfsgnn_loss_fwd", G, NF, NC, F)) return rc;
  PF_REQUIRE(y && Wd1 && bd1 && Wd2 && bd2 && ci && n_prime && fiber_time && tmean && tvar,
             "pfsgnn_loss_fwd", "null");
  const EdgeGeo geo = loss_geo(G, NF, NC);
  Ws w{reinterpret_cast<char*>(ws), ws_bytes};
  float* part = w.take((size_t)G * geo.NFG * NC * 4);
  float* ftp = geo.KS == 1 ? fiber_time : w.take((size_t)geo.KS * geo.NS);
  PF_REQUIRE(part && ftp, "pfsgnn_loss_fwd", "workspace too small");
  hipStream_t st = as_stream(stream);
  const SoftFloor sf = make_softfloor(sharpness);
  const uint64_t key = pf_noise_key((uint64_t)seed);
  { pf::Timer tm_("loss_fwd", st);
  DISPATCH_F(F, hipLaunchKernelGGL(k_loss_fwd<FF>, dim3(edge_grid(geo)), dim3(256), 0, st, geo, y,
                                   sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sf, noiselevel, key, seed_dev,
                                   ftp, tt, part));
  tm_.end(); }
  if (geo.KS > 1)
    hipLaunchKernelGGL(k_fiber_partial_sum, dim3((unsigned)((geo.NS + 255) / 256)), dim3(256), 0,
                       st, ftp, geo.KS, geo.NS, fiber_time);
  hipLaunchKernelGGL(k_loss_class_reduce, dim3((G * NC + 3) / 4), dim3(256), 0, st, part, G,
                     geo.NFG, NC, NF, n_prime, tmean, tvar);
  return pf::check_launch("pfsgnn_loss_fwd");
}

extern "C" int pfsgnn_loss_finalize(int G, int NF, int NC, const float* n_prime,
                                    const float* fiber_time, const float* tvar, const float* ci,
                                    float pclass, float pfiber, float total_time, float nfields,
                                    float wutils, float wvar, float* loss, float* utils,
                                    float* variance, float* Gn, float* Gf, float* Gv,
                                    void* stream) {
  PF_REQUIRE(G > 0 && NF > 1 && NC > 0, "pfsgnn_loss_finalize", "bad dims");
  PF_REQUIRE(n_prime && fiber_time && tvar && ci && loss && utils && variance && Gn && Gf && Gv,
             "pfsgnn_loss_finalize", "null");
  hipLaunchKernelGGL(k_loss_finalize, dim3(G), dim3(256), 0, as_stream(stream), NF, NC, G * NC,
                     n_prime, fiber_time, tvar, ci, pclass, pfiber, total_time, nfields, wutils,
                     wvar, loss, utils, variance, Gn, Gf, Gv);
  return pf::check_launch("pfsgnn_loss_finalize");
}

static int loss_bwd_impl(int G, int NF, int NC, int F, const float* y, const float* sc,
                         const float* sh, const float* Wd1, const float* bd1, const float* Wd2,
                         const float* bd2, const float* ci, float scale, float sharpness,
                         float noiselevel, unsigned long long seed,
                         const unsigned long long* seed_dev, const float* Gn, const float* Gf,
                         const float* Gv, const float* tmean, const float* gscale, float* dWd1,
                         float* dbd1, float* dWd2, float* dbd2, float* gxe, const float* bn_mu1,
                         const float* bn_inv1, float* bn_part, void* ws, size_t ws_bytes,
                         void* stream) {
  if (int rc = check_dims("pfsgnn_loss_bwd", G, NF, NC, F)) return rc;
  PF_REQUIRE(y && Wd1 && bd1 && Wd2 && bd2 && ci && Gn && Gf && Gv && tmean && dWd1 && dbd1 &&
                 dWd2 && dbd2 && gxe,
             "pfsgnn_loss_bwd", "null");
  const EdgeGeo geo = loss_geo(G, NF, NC);
  const size_t nb = geo.nblocks;
  Ws w{reinterpret_cast<char*>(ws), ws_bytes};
  float* pW = w.take(nb * F * (F + 1));
  float* pV = w.take(nb * (F + 1));
  PF_REQUIRE(pW && pV, "pfsgnn_loss_bwd", "workspace too small");
  hipStream_t st = as_stream(stream);
  const SoftFloor sf = make_softfloor(sharpness);
  const uint64_t key = pf_noise_key((uint64_t)seed);
  { pf::Timer tm_("loss_bwd", st);
  if (bn_part) {
    DISPATCH_F(F, hipLaunchKernelGGL((k_loss_bwd<FF, true>), dim3(edge_grid(geo)), dim3(256), 0, st,
                                     geo, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sf, noiselevel,
                                     key, seed_dev, Gn, Gf, Gv, tmean, gscale, gxe, pW, pV, bn_mu1,
                                     bn_inv1, bn_part));
  } else {
    DISPATCH_F(F, hipLaunchKernelGGL((k_loss_bwd<FF, false>), dim3(edge_grid(geo)), dim3(256), 0, st,
                                     geo, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sf, noiselevel,
                                     key, seed_dev, Gn, Gf, Gv, tmean, gscale, gxe, pW, pV, nullptr,
                                     nullptr, nullptr));
  }
  tm_.end(); }
  {
    RedDesc rd[4] = {{pW, (int)nb, (size_t)F * (F + 1), F + 1, F, F, dWd1, F, 1, 1.f},
                     {pW + F, (int)nb, (size_t)F * (F + 1), F + 1, F, 1, dbd1, 1, 1, 1.f},
                     {pV, (int)nb, (size_t)(F + 1), F, 1, F, dWd2, F, 1, 1.f},
                     {pV + F, (int)nb, (size_t)(F + 1), 1, 1, 1, dbd2, 1, 1, 1.f}};
    launch_reduce_multi(rd, 4, st);
  }
  return pf::check_launch("pfsgnn_loss_bwd");
}

extern "C" int pfsgnn_loss_bwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                               const float* sh, const float* Wd1, const float* bd1,
                               const float* Wd2, const float* bd2, const float* ci, float scale,
                               float sharpness, float noiselevel, unsigned long long seed,
                               const unsigned long long* seed_dev, const float* Gn,
                               const float* Gf, const float* Gv,
                               const float* tmean, const float* gscale, float* dWd1, float* dbd1,
                               float* dWd2, float* dbd2, float* gxe, void* ws, size_t ws_bytes,
                               void* stream) {
  return loss_bwd_impl(G, NF, NC, F, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sharpness,
                       noiselevel, seed, seed_dev, Gn, Gf, Gv, tmean, gscale, dWd1, dbd1, dWd2,
                       dbd2, gxe, nullptr, nullptr, nullptr, ws, ws_bytes, stream);
}

extern "C" int pfsgnn_loss_bn_parts(int G, int NF, int NC) {
  return loss_geo(G, NF, NC).nblocks;
}

extern "C" int pfsgnn_loss_bwd_bn(int G, int NF, int NC, int F, const float* y, const float* sc,
                                  const float* sh, const float* Wd1, const float* bd1,
                                  const float* Wd2, const float* bd2, const float* ci,
                                  float scale, float sharpness, float noiselevel,
                                  unsigned long long seed, const unsigned long long* seed_dev,
                                  const float* Gn, const float* Gf, const float* Gv,
                                  const float* tmean, const float* gscale, float* dWd1,
                                  float* dbd1, float* dWd2, float* dbd2, float* gxe,
                                  const float* bn_mu1, const float* bn_inv1, float* bn_part,
                                  void* ws, size_t ws_bytes, void* stream) {
  PF_REQUIRE(bn_mu1 && bn_inv1 && bn_part, "pfsgnn_loss_bwd_bn", "null");
  return loss_bwd_impl(G, NF, NC, F, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sharpness,
                       noiselevel, seed, seed_dev, Gn, Gf, Gv, tmean, gscale, dWd1, dbd1, dWd2,
                       dbd2, gxe, bn_mu1, bn_inv1, bn_part, ws, ws_bytes, stream);
}

extern "C" int pfsgnn_layout_analyze(const int64_t* edge_index, long long E, int G, int NF, int NC,
                                     int32_t* perm, int32_t* status, void* ws, size_t ws_bytes,
                                     void* stream) {
  PF_REQUIRE(edge_index && perm && status && E > 0, "pfsgnn_layout_analyze", "null/empty");
  PF_REQUIRE(E == (long long)G * NF * NC, "pfsgnn_layout_analyze",
             "E != G*NF*NC: not a complete bipartite batch");
  PF_REQUIRE(E < (1ll << 31), "pfsgnn_layout_analyze", "E too large for int32 permutation");
  PF_REQUIRE(ws && ws_bytes >= (size_t)E * sizeof(int32_t), "pfsgnn_layout_analyze",
             "workspace too small");
  hipStream_t st = as_stream(stream);
  int32_t* cnt = reinterpret_cast<int32_t*>(ws);
  if (hipMemsetAsync(cnt, 0, (size_t)E * sizeof(int32_t), st) != hipSuccess)
    return pf::fail("pfsgnn_layout_analyze", "memset");
  hipLaunchKernelGGL(k_layout_init, dim3(1), dim3(64), 0, st, status);
  const unsigned nbk = (unsigned)((E + 255) / 256);
  hipLaunchKernelGGL(k_layout_scatter, dim3(nbk), dim3(256), 0, st, edge_index, E, G, NF, NC, perm,
                     cnt, status);
  hipLaunchKernelGGL(k_layout_check, dim3(nbk), dim3(256), 0, st, cnt, E, status);
  return pf::check_launch("pfsgnn_layout_analyze");
}

extern "C" int pfsgnn_edges_to_canonical(const float* src, int G, int NF, int NC, int F, int mode,
                                         const int32_t* perm, float* dst, void* stream) {
  const long long E = (long long)G * NF * NC;
  PF_REQUIRE(src && dst && E > 0 && F > 0 && mode >= 0 && mode <= 2 && (mode != 0 || perm),
             "pfsgnn_edges_to_canonical", "bad arguments");
  hipLaunchKernelGGL(k_to_canonical, dim3((unsigned)((E + 255) / 256)), dim3(256), 0,
                     as_stream(stream), src, E, NF, NC, F, mode, perm, dst);
  return pf::check_launch("pfsgnn_edges_to_canonical");
}

extern "C" int pfsgnn_edges_from_canonical(const float* y, const float* sc, const float* sh, int G,
                                           int NF, int NC, int F, int mode, const int32_t* perm,
                                           int rowmajor, float* dst, void* stream) {
  const long long E = (long long)G * NF * NC;
  PF_REQUIRE(y && dst && E > 0 && F > 0 && mode >= 0 && mode <= 2 && (mode != 0 || perm),
             "pfsgnn_edges_from_canonical", "bad arguments");
  if (mode == 1 && rowmajor && (F == 8 || F == 10 || F == 16)) {
    const unsigned nb = (unsigned)((long long)G * ((NF + 63) / 64) * ((NC + FC_CT - 1) / FC_CT));
    switch (F) {
      case 8: hipLaunchKernelGGL(k_from_canonical_fm<8>, dim3(nb), dim3(256), 0,
                                 as_stream(stream), y, sc, sh, G, NF, NC, dst); break;
      case 10: hipLaunchKernelGGL(k_from_canonical_fm<10>, dim3(nb), dim3(256), 0,
                                  as_stream(stream), y, sc, sh, G, NF, NC, dst); break;
      default: hipLaunchKernelGGL(k_from_canonical_fm<16>, dim3(nb), dim3(256), 0,
                                  as_stream(stream), y, sc, sh, G, NF, NC, dst); break;
    }
    return pf::check_launch("pfsgnn_edges_from_canonical");
  }
  hipLaunchKernelGGL(k_from_canonical, dim3((unsigned)((E + 255) / 256)), dim3(256), 0,
                     as_stream(stream), y, sc, sh, E, NF, NC, F, mode, perm, rowmajor, dst);
  return pf::check_launch("pfsgnn_edges_from_canonical");
}
