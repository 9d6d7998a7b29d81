// pfsgnn_sparse.hip -- general (non-complete) bipartite graphs.
//
// The reference's data model takes any edge_index (gnn.py:32-63), and its
// scatters reduce over arbitrary src / tgt (gnn.py:140-144 per fiber, 190 per
// class).  A general batch is laid out once (pfsgnn_sparse_layout): edges
// sorted stably by fiber (CSR by fiber: fib_ptr) -- every edge tensor of the
// step lives in that order -- plus the positions sorted stably by class (CSR
// by class: cls_ord / cls_ptr).  The per-edge MLPs then run as gathers of the
// per-node parts + the node-level Linear kernels over E columns, and the
// scatters as deterministic segment kernels (block per segment, fixed-order
// tree: bitwise reproducible), all in this file:
//   gather_cols      per-edge copy / add / (x) lrelu' of node-table columns
//   segment_sum      per-fiber or per-class sums (optionally of lrelu(x))
//   segment_moments  per-fiber mean + central moments -> SModel features
//   segment_moment_grad  d loss / d message from the per-fiber coefficients
//   rows_stats / rows_bn_sums / rows_axpby   the EdgeModel BatchNorm pieces
#include "pfsgnn_common.h"
#include "../../include/pfsgnn.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>

namespace {

// ------------------------------------------------------------ layout
__global__ void k_sp_prepare(const long long* __restrict__ ei, long long E, int G, int NF, int NC,
                             int* __restrict__ key, int* __restrict__ val,
                             int* __restrict__ bad) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < E;
       e += (long long)gridDim.x * 256) {
    const long long s = ei[e], t = ei[E + e];
    const bool ok = s >= 0 && s < (long long)G * NF && t >= 0 && t < (long long)G * NC &&
                    s / NF == t / NC;
    if (!ok) bad[0] = 1;  // any writer: a flag, the value is the same
    key[e] = ok ? (int)s : 0;
    val[e] = (int)e;
  }
}

// after the sort by fiber: user_of[p] = the caller's edge at position p
__global__ void k_sp_scatter(const long long* __restrict__ ei, long long E,
                             const int* __restrict__ user_of, int* __restrict__ tgt_p,
                             int* __restrict__ iota) {
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < E;
       p += (long long)gridDim.x * 256) {
    tgt_p[p] = (int)ei[E + user_of[p]];
    iota[p] = (int)p;
  }
}

// ptr[k] = first position whose (sorted) key is >= k, k = 0..n
__global__ void k_sp_ptr(const int* __restrict__ keys, long long E, int n, int* __restrict__ ptr) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k > n) return;
  long long lo = 0, hi = E;
  while (lo < hi) {
    const long long mid = (lo + hi) >> 1;
    if (keys[mid] < k) lo = mid + 1; else hi = mid;
  }
  ptr[k] = (int)lo;
}

// ------------------------------------------------------------ sliced layout
// (pfsgnn_sliced.hip) key per fiber: its graph in the high word, 2^32-1 minus its
// degree in the low one -- one stable ascending sort orders the fibers by
// graph, then by degree descending, ties in fiber order
__global__ void k_sl_keys(const int* __restrict__ fib_ptr, int NS, int NF,
                          unsigned long long* __restrict__ key, int* __restrict__ val) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= NS) return;
  const unsigned deg = (unsigned)(fib_ptr[n + 1] - fib_ptr[n]);
  key[n] = ((unsigned long long)(unsigned)(n / NF) << 32) | (0xFFFFFFFFu - deg);
  val[n] = n;
}

// thread per slice: lane j of slice q of graph g takes the (16 q + j)-th fiber
// of g in degree order; the slice runs for its largest degree (lane 0's)
__global__ void k_sl_slices(const int* __restrict__ sorted, const int* __restrict__ fib_ptr,
                            int G, int NF, int SPG, int* __restrict__ fib, int* __restrict__ len,
                            long long* __restrict__ cnt, int* __restrict__ slot_of) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= G * SPG) return;
  const int g = s / SPG, q = s - g * SPG;
  int L = 0;
  for (int j = 0; j < 16; ++j) {
    const int i = 16 * q + j;
    const int f = i < NF ? sorted[(long long)g * NF + i] : -1;
    fib[s * 16 + j] = f;
    if (f >= 0) {
      slot_of[f] = s * 16 + j;
      L = max(L, fib_ptr[f + 1] - fib_ptr[f]);
    }
  }
  len[s] = L;
  cnt[s] = 16ll * L;
}

__global__ void k_sl_info(const long long* __restrict__ base64, const long long* __restrict__ cnt,
                          int nsl, const int* __restrict__ maxd, int* __restrict__ base,
                          long long* __restrict__ info) {
  for (int s = blockIdx.x * 256 + threadIdx.x; s < nsl; s += gridDim.x * 256)
    base[s] = (int)base64[s];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    info[0] = base64[nsl - 1] + cnt[nsl - 1];
    info[1] = maxd[0];
  }
}

// thread per fiber-sorted position p: its slot position base + 16 k + lane
__global__ void k_sl_fill(const int* __restrict__ src_p, const int* __restrict__ tgt_p,
                          const int* __restrict__ user_of, const int* __restrict__ fib_ptr,
                          long long E, int NF, int NC, const int* __restrict__ slot_of,
                          const int* __restrict__ base, unsigned char* __restrict__ cls,
                          int* __restrict__ pos_user) {
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < E;
       p += (long long)gridDim.x * 256) {
    const int n = src_p[p];
    const int k = (int)(p - fib_ptr[n]);
    const int sl = slot_of[n];
    const long long q = (long long)base[sl >> 4] + 16ll * k + (sl & 15);
    cls[q] = (unsigned char)(tgt_p[p] - (n / NF) * NC);
    pos_user[q] = user_of[p];
  }
}

// Pebay's count-only coefficients of the n-th message (pfsgnn_mfma.hip
// km_source_fwd's table), n = k + 1
__global__ void k_sl_pco(int maxdeg, float* __restrict__ pco) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= maxdeg) return;
  const double nn = k + 1, r = 1.0 / nn;
  float* p = pco + 8 * k;
  p[0] = (float)((nn - 1) * r);
  p[1] = (float)((nn - 1) * (nn - 2) * r * r);
  p[2] = (float)((nn - 1) * (nn * nn - 3 * nn + 3) * r * r * r);
  p[3] = (float)r;
  p[4] = (float)(6 * r * r);
  p[5] = (float)(-4 * r);
  p[6] = (float)(-3 * r);
  p[7] = 0.f;
}

// caller-order rows [E][F] <-> slot tensors [F][EP] (0 at padding): thread per
// position, the slot side coalesced; the caller's row (F floats at a random
// row: 8-byte aligned for even F) moves as F/2 float2 accesses
template <int F>
__global__ void k_to_slots(const float* __restrict__ src, long long EP,
                           const int* __restrict__ pos_user, float* __restrict__ dst) {
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < EP;
       p += (long long)gridDim.x * 256) {
    const int u = pos_user[p];
    float v[F];
    if (F % 2 == 0) {
      const float2* r = reinterpret_cast<const float2*>(src + (long long)(u >= 0 ? u : 0) * F);
#pragma unroll
      for (int j = 0; j < F / 2; ++j) {
        const float2 q = r[j];
        v[2 * j] = q.x;
        v[2 * j + 1] = q.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < F; ++j) v[j] = src[(long long)(u >= 0 ? u : 0) * F + j];
    }
#pragma unroll
    for (int j = 0; j < F; ++j) dst[(long long)j * EP + p] = u >= 0 ? v[j] : 0.f;
  }
}
template <int F>
__global__ void k_from_slots(const float* __restrict__ y, const float* __restrict__ sc,
                             const float* __restrict__ sh, long long E, long long EP,
                             const int* __restrict__ pos_user, int rowmajor,
                             float* __restrict__ dst) {
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < EP;
       p += (long long)gridDim.x * 256) {
    const int u = pos_user[p];
    if (u < 0) continue;
    float v[F];
#pragma unroll
    for (int j = 0; j < F; ++j) {
      v[j] = y[(long long)j * EP + p];
      if (sc) v[j] = fmaf(v[j], sc[j], sh[j]);
    }
    if (rowmajor && F % 2 == 0) {
      float2* r = reinterpret_cast<float2*>(dst + (long long)u * F);
#pragma unroll
      for (int j = 0; j < F / 2; ++j) r[j] = make_float2(v[2 * j], v[2 * j + 1]);
    } else {
#pragma unroll
      for (int j = 0; j < F; ++j) {
        if (rowmajor) dst[(long long)u * F + j] = v[j];
        else dst[(long long)j * E + u] = v[j];
      }
    }
  }
}

// ------------------------------------------------------------ gathers
// thread per position e (idx[e] read once), every channel: coalesced writes
// out[c][e]; mode 0: = X[c][idx[e]], 1: += X[c][idx[e]], 2: = X[c][idx[e]] *
// lrelu'(Z[c][e])
__global__ __launch_bounds__(256) void k_gather_cols(const float* __restrict__ X, int C, int N,
                                                     const int* __restrict__ idx, long long E,
                                                     const float* __restrict__ Z, int mode,
                                                     float* __restrict__ out) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < E;
       e += (long long)gridDim.x * 256) {
    const float* xr = X + idx[e];
    for (int c = 0; c < C; ++c) {
      const float v = xr[(size_t)c * N];
      const size_t i = (size_t)c * E + e;
      if (mode == 0) out[i] = v;
      else if (mode == 1) out[i] += v;
      else out[i] = v * dlrelu(Z[i]);
    }
  }
}

// ------------------------------------------------------------ segment sums
// one wave per segment: lane l takes positions p0 + l, p0 + l + 64, ... and
// keeps every channel's running sum in registers (CM >= C); a fixed DPP tree
// per channel finishes it (deterministic).  Fiber segments are contiguous
// runs of positions (coalesced); class segments gather through ord.
template <int CM>
__global__ __launch_bounds__(256) void k_segment_sum(const float* __restrict__ X, int C, long long E,
                                                     const int* __restrict__ ord,
                                                     const int* __restrict__ ptr, int act,
                                                     float* __restrict__ out, int nseg, int add) {
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;  // the whole wave
  const int p0 = ptr[s], p1 = ptr[s + 1];
  float acc[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) acc[c] = 0.f;
  for (int p = p0 + lane; p < p1; p += 64) {
    const size_t e = ord ? (size_t)ord[p] : (size_t)p;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) {
        const float x = X[(size_t)c * E + e];
        acc[c] += act ? lrelu(x) : x;
      }
  }
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) {
      const float v = wave_sum(acc[c]);
      if (lane == 0) {
        float* o = out + (size_t)c * nseg + s;
        *o = add ? *o + v : v;
      }
    }
}

// ------------------------------------------------------------ moments
// one wave per fiber segment (contiguous positions): the mean, then the
// central moments (two passes over the segment, fp32 as the reference's
// scatter means, gnn.py:140-144); torch_scatter's mean clamps the count at 1,
// so an empty segment gives mean 0 and moments 0
template <int CM>
__global__ __launch_bounds__(256) void k_segment_moments(const float* __restrict__ M, int C,
                                                         long long E,
                                                         const int* __restrict__ ptr, int nseg,
                                                         float* __restrict__ mom,
                                                         float* __restrict__ hs) {
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;
  const int p0 = ptr[s], p1 = ptr[s + 1];
  const float inv_n = 1.0f / (float)(p1 > p0 ? p1 - p0 : 1);
  float mean[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) mean[c] = 0.f;
  for (int p = p0 + lane; p < p1; p += 64)
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) mean[c] += M[(size_t)c * E + p];
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) mean[c] = wave_sum(mean[c]) * inv_n;
  float s2[CM], s3[CM], s4[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) s2[c] = s3[c] = s4[c] = 0.f;
  for (int p = p0 + lane; p < p1; p += 64)
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) {
        const float d = M[(size_t)c * E + p] - mean[c], d2 = d * d;
        s2[c] += d2;
        s3[c] += d2 * d;
        s4[c] += d2 * d2;
      }
  const size_t CN = (size_t)C * nseg;
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) {
      const float c2 = wave_sum(s2[c]) * inv_n, c3 = wave_sum(s3[c]) * inv_n,
                  c4 = wave_sum(s4[c]) * inv_n;
      if (lane == 0) {
        const size_t idx = (size_t)c * nseg + s;
        mom[idx] = mean[c];
        mom[CN + idx] = c2;
        mom[2 * CN + idx] = c3;
        mom[3 * CN + idx] = c4;
        const float var = c2 > 0.f ? c2 : 0.01f * c2;  // F.leaky_relu (slope 0.01), gnn.py:141
        const float sd = sqrtf(var + 1e-6f);
        hs[idx] = mean[c];
        hs[CN + idx] = sd;
        hs[2 * CN + idx] = c3 / (sd * sd * sd);
        hs[3 * CN + idx] = c4 / ((sd * sd) * (sd * sd));
      }
    }
}

// g_m[c][e] = C0 + d (C1 + d (C2 + d C3)), d = m - mean, per-fiber coefficients
// (thread per position, every channel)
__global__ __launch_bounds__(256) void k_segment_moment_grad(const float* __restrict__ M, int C,
                                                             long long E,
                                                             const int* __restrict__ seg,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ coef,
                                                             int nseg, float* __restrict__ gm) {
  const size_t CN = (size_t)C * nseg;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < E;
       e += (long long)gridDim.x * 256) {
    const int sg = seg[e];
    for (int c = 0; c < C; ++c) {
      const size_t i = (size_t)c * E + e, j = (size_t)c * nseg + sg;
      const float d = M[i] - mean[j];
      gm[i] = fmaf(d, fmaf(d, fmaf(d, coef[3 * CN + j], coef[2 * CN + j]), coef[CN + j]), coef[j]);
    }
  }
}

// ------------------------------------------------------------ row statistics
// per-(channel, chunk) Welford partials -> per-channel mean / biased variance
__global__ __launch_bounds__(256) void k_rows_stats_part(const float* __restrict__ X, long long N,
                                                         int S, float* __restrict__ part) {
  const int c = blockIdx.x, sidx = blockIdx.y, t = threadIdx.x;
  const long long chunk = (N + S - 1) / S;
  const long long n0 = (long long)sidx * chunk, n1 = std::min<long long>(N, n0 + chunk);
  float cnt = 0.f, mean = 0.f, m2 = 0.f;
  for (long long n = n0 + t; n < n1; n += 256) {
    const float x = X[(long long)c * N + n];
    cnt += 1.f;
    const float d = x - mean;
    mean += d / cnt;
    m2 += d * (x - mean);
  }
  __shared__ float sc[256], sm[256], sq[256];
  sc[t] = cnt; sm[t] = mean; sq[t] = m2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      const float ca = sc[t], cb = sc[t + w], tot = ca + cb;
      if (tot > 0.f) {
        const float d = sm[t + w] - sm[t];
        sm[t] = sm[t] + d * (cb / tot);
        sq[t] = sq[t] + sq[t + w] + d * d * (ca * cb / tot);
      }
      sc[t] = tot;
    }
    __syncthreads();
  }
  if (t == 0) {
    float* p = part + ((long long)c * S + sidx) * 3;
    p[0] = sc[0]; p[1] = sm[0]; p[2] = sq[0];
  }
}

__global__ void k_rows_stats_fin(const float* __restrict__ part, int C, int S, long long N,
                                 float* __restrict__ mu, float* __restrict__ var) {
  const int c = threadIdx.x;
  if (c >= C) return;
  double n = 0, mean = 0, m2 = 0;
  for (int s = 0; s < S; ++s) {
    const float* p = part + ((long long)c * S + s) * 3;
    const double cb = p[0], tot = n + cb;
    if (tot > 0) {
      const double d = p[1] - mean;
      mean += d * (cb / tot);
      m2 += p[2] + d * d * (n * cb / tot);
    }
    n = tot;
  }
  mu[c] = (float)mean;
  var[c] = (float)(m2 / (double)N);
}

// Sg[c] = sum_n g, Sgx[c] = sum_n g * (y - mu) * inv  (block partials, fixed order)
__global__ __launch_bounds__(256) void k_rows_bn_sums_part(const float* __restrict__ g,
                                                           const float* __restrict__ y,
                                                           long long N, int S,
                                                           const float* __restrict__ mu,
                                                           const float* __restrict__ inv,
                                                           float* __restrict__ part) {
  const int c = blockIdx.x, sidx = blockIdx.y, t = threadIdx.x;
  const long long chunk = (N + S - 1) / S;
  const long long n0 = (long long)sidx * chunk, n1 = std::min<long long>(N, n0 + chunk);
  const float m = mu[c], iv = inv[c];
  float a = 0.f, b = 0.f;
  for (long long n = n0 + t; n < n1; n += 256) {
    const float gv = g[(long long)c * N + n];
    a += gv;
    b += gv * ((y[(long long)c * N + n] - m) * iv);
  }
  __shared__ float ra[256], rb[256];
  ra[t] = a; rb[t] = b;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) { ra[t] += ra[t + w]; rb[t] += rb[t + w]; }
    __syncthreads();
  }
  if (t == 0) {
    part[((long long)c * S + sidx) * 2] = ra[0];
    part[((long long)c * S + sidx) * 2 + 1] = rb[0];
  }
}

__global__ void k_rows_bn_sums_fin(const float* __restrict__ part, int C, int S,
                                   float* __restrict__ Sg, float* __restrict__ Sgx) {
  const int c = threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int s = 0; s < S; ++s) {
    a += part[((long long)c * S + s) * 2];
    b += part[((long long)c * S + s) * 2 + 1];
  }
  Sg[c] = a;
  Sgx[c] = b;
}

// out may alias g or y (elementwise); thread per column, every channel
__global__ __launch_bounds__(256) void k_rows_axpby(const float* g, const float* y, int C,
                                                    long long N,
                                                    const float* __restrict__ alpha,
                                                    const float* __restrict__ gam1,
                                                    const float* __restrict__ gam0, float* out) {
  for (long long n = (long long)blockIdx.x * 256 + threadIdx.x; n < N;
       n += (long long)gridDim.x * 256)
    for (int c = 0; c < C; ++c) {
      const size_t i = (size_t)c * N + n;
      out[i] = fmaf(gam1[c], y[i], fmaf(alpha[c], g[i], gam0[c]));
    }
}

unsigned grid_of(long long n) { return (unsigned)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192)); }
int row_splits(long long N) { return (int)std::max<long long>(1, std::min<long long>(64, (N + 8191) / 8192)); }

}  // namespace

// ================================================================ ABI
extern "C" size_t pfsgnn_sparse_layout_ws_bytes(long long E) {
  if (E <= 0 || E >= INT32_MAX) return 256;
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const int*)nullptr, (int*)nullptr,
                                           (const int*)nullptr, (int*)nullptr, (int)E);
  return align256(tmp) + 4 * align256((size_t)E * sizeof(int)) + 256;
}

static int key_bits(int n) {  // keys are 0..n-1
  int b = 1;
  while (b < 31 && (1 << b) < n) ++b;
  return b;
}

extern "C" int pfsgnn_sparse_layout(const long long* edge_index, long long E, int G, int NF, int NC,
                                    int* src_p, int* tgt_p, int* user_of, int* fib_ptr,
                                    int* cls_ord, int* cls_ptr, int* status, void* ws,
                                    size_t ws_bytes, void* stream) {
  const char* where = "pfsgnn_sparse_layout";
  PF_REQUIRE(edge_index && E > 0 && E < INT32_MAX && G > 0 && NF > 0 && NC > 0 && src_p &&
                 tgt_p && user_of && fib_ptr && cls_ord && cls_ptr && status,
             where, "bad arguments");
  PF_REQUIRE((long long)G * NF < INT32_MAX && (long long)G * NC < INT32_MAX, where,
             "too many nodes for int32 indices");
  PF_REQUIRE(ws && ws_bytes >= pfsgnn_sparse_layout_ws_bytes(E), where, "workspace too small");
  hipStream_t st = as_stream(stream);
  char* w = static_cast<char*>(ws);
  const size_t eb = align256((size_t)E * sizeof(int));
  int* key = reinterpret_cast<int*>(w);
  int* val = reinterpret_cast<int*>(w + eb);
  int* iota = reinterpret_cast<int*>(w + 2 * eb);
  int* ckey = reinterpret_cast<int*>(w + 3 * eb);
  void* tmp = w + 4 * eb;
  size_t tmpb = ws_bytes - 4 * eb;
  const int NS = G * NF, NT = G * NC;
  if (hipMemsetAsync(status, 0, sizeof(int), st) != hipSuccess) return pf::fail(where, "memset");
  hipLaunchKernelGGL(k_sp_prepare, dim3(grid_of(E)), dim3(256), 0, st, edge_index, E, G, NF, NC,
                     key, val, status);
  // stable LSD radix sorts: the edges by fiber (ties keep the caller's order),
  // then the fiber-sorted positions by class (ties keep position order)
  if (hipcub::DeviceRadixSort::SortPairs(tmp, tmpb, key, src_p, val, user_of, (int)E, 0,
                                         key_bits(NS), st) != hipSuccess)
    return pf::fail(where, "radix sort (fibers)");
  hipLaunchKernelGGL(k_sp_scatter, dim3(grid_of(E)), dim3(256), 0, st, edge_index, E, user_of,
                     tgt_p, iota);
  if (hipcub::DeviceRadixSort::SortPairs(tmp, tmpb, tgt_p, ckey, iota, cls_ord, (int)E, 0,
                                         key_bits(NT), st) != hipSuccess)
    return pf::fail(where, "radix sort (classes)");
  hipLaunchKernelGGL(k_sp_ptr, dim3((NS + 256) / 256), dim3(256), 0, st, src_p, E, NS, fib_ptr);
  hipLaunchKernelGGL(k_sp_ptr, dim3((NT + 256) / 256), dim3(256), 0, st, ckey, E, NT, cls_ptr);
  return pf::check_launch(where);
}

extern "C" int pfsgnn_gather_cols(const float* X, int C, int N, const int* idx, long long E,
                                  const float* Z, int mode, float* out, void* stream) {
  PF_REQUIRE(X && idx && out && C > 0 && N > 0 && E > 0 && mode >= 0 && mode <= 2 &&
                 (mode != 2 || Z),
             "pfsgnn_gather_cols", "bad arguments");
  hipLaunchKernelGGL(k_gather_cols, dim3(grid_of(E)), dim3(256), 0, as_stream(stream), X, C, N,
                     idx, E, Z, mode, out);
  return pf::check_launch("pfsgnn_gather_cols");
}

extern "C" int pfsgnn_segment_sum(const float* X, int C, long long E, const int* ord,
                                  const int* ptr, int nseg, int act, float* out, int add,
                                  void* stream) {
  PF_REQUIRE(X && ptr && out && C > 0 && C <= 64 && E > 0 && nseg > 0, "pfsgnn_segment_sum",
             "bad arguments (C <= 64)");
  const dim3 grid((nseg + 3) / 4);
  hipStream_t st = as_stream(stream);
  if (C <= 16)
    hipLaunchKernelGGL(k_segment_sum<16>, grid, dim3(256), 0, st, X, C, E, ord, ptr, act, out, nseg, add);
  else if (C <= 24)
    hipLaunchKernelGGL(k_segment_sum<24>, grid, dim3(256), 0, st, X, C, E, ord, ptr, act, out, nseg, add);
  else if (C <= 40)
    hipLaunchKernelGGL(k_segment_sum<40>, grid, dim3(256), 0, st, X, C, E, ord, ptr, act, out, nseg, add);
  else
    hipLaunchKernelGGL(k_segment_sum<64>, grid, dim3(256), 0, st, X, C, E, ord, ptr, act, out, nseg, add);
  return pf::check_launch("pfsgnn_segment_sum");
}

extern "C" int pfsgnn_segment_moments(const float* M, int C, long long E, const int* ptr, int nseg,
                                      float* mom, float* hs, void* stream) {
  PF_REQUIRE(M && ptr && mom && hs && C > 0 && C <= 32 && E > 0 && nseg > 0,
             "pfsgnn_segment_moments", "bad arguments (C <= 32)");
  const dim3 grid((nseg + 3) / 4);
  hipStream_t st = as_stream(stream);
  if (C <= 16)
    hipLaunchKernelGGL(k_segment_moments<16>, grid, dim3(256), 0, st, M, C, E, ptr, nseg, mom, hs);
  else if (C <= 20)
    hipLaunchKernelGGL(k_segment_moments<20>, grid, dim3(256), 0, st, M, C, E, ptr, nseg, mom, hs);
  else
    hipLaunchKernelGGL(k_segment_moments<32>, grid, dim3(256), 0, st, M, C, E, ptr, nseg, mom, hs);
  return pf::check_launch("pfsgnn_segment_moments");
}

extern "C" int pfsgnn_segment_moment_grad(const float* M, int C, long long E, const int* seg,
                                          const float* mean, const float* coef, int nseg,
                                          float* gm, void* stream) {
  PF_REQUIRE(M && seg && mean && coef && gm && C > 0 && E > 0 && nseg > 0,
             "pfsgnn_segment_moment_grad", "bad arguments");
  hipLaunchKernelGGL(k_segment_moment_grad, dim3(grid_of(E)), dim3(256), 0, as_stream(stream), M,
                     C, E, seg, mean, coef, nseg, gm);
  return pf::check_launch("pfsgnn_segment_moment_grad");
}

extern "C" size_t pfsgnn_rows_ws_bytes(int C, long long N) {
  return align256((size_t)C * row_splits(N) * 3 * sizeof(float));
}

extern "C" int pfsgnn_rows_stats(const float* X, int C, long long N, float* mu, float* var,
                                 void* ws, size_t ws_bytes, void* stream) {
  PF_REQUIRE(X && mu && var && C > 0 && C <= 256 && N > 0, "pfsgnn_rows_stats", "bad arguments");
  PF_REQUIRE(ws && ws_bytes >= pfsgnn_rows_ws_bytes(C, N), "pfsgnn_rows_stats",
             "workspace too small");
  const int S = row_splits(N);
  hipStream_t st = as_stream(stream);
  float* part = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_rows_stats_part, dim3(C, S), dim3(256), 0, st, X, N, S, part);
  hipLaunchKernelGGL(k_rows_stats_fin, dim3(1), dim3(256), 0, st, part, C, S, N, mu, var);
  return pf::check_launch("pfsgnn_rows_stats");
}

extern "C" int pfsgnn_rows_bn_sums(const float* g, const float* y, int C, long long N,
                                   const float* mu, const float* inv, float* Sg, float* Sgx,
                                   void* ws, size_t ws_bytes, void* stream) {
  PF_REQUIRE(g && y && mu && inv && Sg && Sgx && C > 0 && C <= 256 && N > 0,
             "pfsgnn_rows_bn_sums", "bad arguments");
  PF_REQUIRE(ws && ws_bytes >= pfsgnn_rows_ws_bytes(C, N), "pfsgnn_rows_bn_sums",
             "workspace too small");
  const int S = row_splits(N);
  hipStream_t st = as_stream(stream);
  float* part = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_rows_bn_sums_part, dim3(C, S), dim3(256), 0, st, g, y, N, S, mu, inv, part);
  hipLaunchKernelGGL(k_rows_bn_sums_fin, dim3(1), dim3(256), 0, st, part, C, S, Sg, Sgx);
  return pf::check_launch("pfsgnn_rows_bn_sums");
}

extern "C" int pfsgnn_rows_axpby(const float* g, const float* y, int C, long long N,
                                 const float* alpha, const float* gam1, const float* gam0,
                                 float* out, void* stream) {
  PF_REQUIRE(g && y && alpha && gam1 && gam0 && out && C > 0 && N > 0, "pfsgnn_rows_axpby",
             "bad arguments");
  hipLaunchKernelGGL(k_rows_axpby, dim3(grid_of(N)), dim3(256), 0, as_stream(stream), g, y, C, N,
                     alpha, gam1, gam0, out);
  return pf::check_launch("pfsgnn_rows_axpby");
}

// ---------------------------------------------------------------- sliced layout
namespace {
struct SlPlanWs {
  size_t keys, vals, cnt, tmp, total;
};
SlPlanWs sl_plan_ws(int G, int NF) {
  const int NS = G * NF, nsl = G * ((NF + 63) / 64) * 4;
  size_t ts = 0, tc = 0, tr = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, ts, (const unsigned long long*)nullptr,
                                           (unsigned long long*)nullptr, (const int*)nullptr,
                                           (int*)nullptr, NS);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tc, (const long long*)nullptr,
                                         (long long*)nullptr, nsl);
  (void)hipcub::DeviceReduce::Max(nullptr, tr, (const int*)nullptr, (int*)nullptr, nsl);
  SlPlanWs w;
  w.keys = 2 * align256((size_t)NS * 8);
  w.vals = 2 * align256((size_t)NS * 4);
  w.cnt = 2 * align256((size_t)nsl * 8) + 256;
  w.tmp = align256(std::max(ts, std::max(tc, tr)));
  w.total = w.keys + w.vals + w.cnt + w.tmp;
  return w;
}
}  // namespace

extern "C" size_t pfsgnn_sliced_plan_ws_bytes(int G, int NF) {
  if (G <= 0 || NF <= 0) return 256;
  return sl_plan_ws(G, NF).total;
}

extern "C" int pfsgnn_sliced_plan(const int* fib_ptr, int G, int NF, int* fib, int* base, int* len,
                                  int* slot_of, long long* info, void* ws, size_t ws_bytes,
                                  void* stream) {
  const char* where = "pfsgnn_sliced_plan";
  PF_REQUIRE(fib_ptr && G > 0 && NF > 0 && fib && base && len && slot_of && info, where,
             "bad arguments");
  PF_REQUIRE((long long)G * NF < INT32_MAX, where, "too many fibers for int32 indices");
  const SlPlanWs p = sl_plan_ws(G, NF);
  PF_REQUIRE(ws && ws_bytes >= p.total, where, "workspace too small");
  hipStream_t st = as_stream(stream);
  const int NS = G * NF, SPG = ((NF + 63) / 64) * 4, nsl = G * SPG;
  char* w = static_cast<char*>(ws);
  auto* key = reinterpret_cast<unsigned long long*>(w);
  auto* key2 = reinterpret_cast<unsigned long long*>(w + p.keys / 2);
  int* val = reinterpret_cast<int*>(w + p.keys);
  int* sorted = reinterpret_cast<int*>(w + p.keys + p.vals / 2);
  auto* cnt = reinterpret_cast<long long*>(w + p.keys + p.vals);
  auto* base64 = reinterpret_cast<long long*>(w + p.keys + p.vals + (p.cnt - 256) / 2);
  int* maxd = reinterpret_cast<int*>(w + p.keys + p.vals + p.cnt - 256);
  void* tmp = w + p.keys + p.vals + p.cnt;
  size_t tmpb = p.tmp;
  hipLaunchKernelGGL(k_sl_keys, dim3((NS + 255) / 256), dim3(256), 0, st, fib_ptr, NS, NF, key, val);
  if (hipcub::DeviceRadixSort::SortPairs(tmp, tmpb, key, key2, val, sorted, NS, 0,
                                         32 + key_bits(G), st) != hipSuccess)
    return pf::fail(where, "radix sort (fiber degrees)");
  hipLaunchKernelGGL(k_sl_slices, dim3((nsl + 255) / 256), dim3(256), 0, st, sorted, fib_ptr, G,
                     NF, SPG, fib, len, cnt, slot_of);
  tmpb = p.tmp;
  if (hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, cnt, base64, nsl, st) != hipSuccess)
    return pf::fail(where, "scan (slice bases)");
  tmpb = p.tmp;
  if (hipcub::DeviceReduce::Max(tmp, tmpb, len, maxd, nsl, st) != hipSuccess)
    return pf::fail(where, "reduce (largest degree)");
  hipLaunchKernelGGL(k_sl_info, dim3((nsl + 255) / 256), dim3(256), 0, st, base64, cnt, nsl, maxd,
                     base, info);
  return pf::check_launch(where);
}

extern "C" int pfsgnn_sliced_fill(const int* src_p, const int* tgt_p, const int* user_of,
                                  const int* fib_ptr, long long E, int NF, int NC,
                                  const int* slot_of, const int* base, long long EP, int maxdeg,
                                  unsigned char* cls, int* pos_user, float* pco, void* stream) {
  const char* where = "pfsgnn_sliced_fill";
  PF_REQUIRE(src_p && tgt_p && user_of && fib_ptr && slot_of && base && cls && pos_user && pco &&
                 E > 0 && EP >= E && NF > 0 && NC > 0 && NC < 255 && maxdeg >= 0,
             where, "bad arguments (NC < 255)");
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(cls, 0xFF, (size_t)EP, st) != hipSuccess ||
      hipMemsetAsync(pos_user, 0xFF, (size_t)EP * sizeof(int), st) != hipSuccess)
    return pf::fail(where, "memset");
  hipLaunchKernelGGL(k_sl_fill, dim3(grid_of(E)), dim3(256), 0, st, src_p, tgt_p, user_of, fib_ptr,
                     E, NF, NC, slot_of, base, cls, pos_user);
  if (maxdeg > 0)
    hipLaunchKernelGGL(k_sl_pco, dim3((maxdeg + 255) / 256), dim3(256), 0, st, maxdeg, pco);
  return pf::check_launch(where);
}

extern "C" int pfsgnn_edges_to_slots(const float* src, long long E, long long EP, int F,
                                     const int* pos_user, float* dst, void* stream) {
  PF_REQUIRE(src && pos_user && dst && E > 0 && EP >= E && F > 0, "pfsgnn_edges_to_slots",
             "bad arguments");
  hipStream_t st = as_stream(stream);
  switch (F) {
#define TS(FF) case FF: hipLaunchKernelGGL(k_to_slots<FF>, dim3(grid_of(EP)), dim3(256), 0, st, src, EP, pos_user, dst); break;
    TS(8) TS(10) TS(16)
#undef TS
    default: return pf::fail("pfsgnn_edges_to_slots", "F must be 8, 10 or 16");
  }
  return pf::check_launch("pfsgnn_edges_to_slots");
}

extern "C" int pfsgnn_edges_from_slots(const float* y, const float* sc, const float* sh,
                                       long long E, long long EP, int F, const int* pos_user,
                                       int rowmajor, float* dst, void* stream) {
  PF_REQUIRE(y && pos_user && dst && E > 0 && EP >= E && F > 0 && (!sc == !sh),
             "pfsgnn_edges_from_slots", "bad arguments");
  hipStream_t st = as_stream(stream);
  switch (F) {
#define FS(FF) case FF: hipLaunchKernelGGL(k_from_slots<FF>, dim3(grid_of(EP)), dim3(256), 0, st, y, sc, sh, E, EP, pos_user, rowmajor, dst); break;
    FS(8) FS(10) FS(16)
#undef FS
    default: return pf::fail("pfsgnn_edges_from_slots", "F must be 8, 10 or 16");
  }
  return pf::check_launch("pfsgnn_edges_from_slots");
}
