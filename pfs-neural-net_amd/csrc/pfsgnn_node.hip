// pfsgnn_node.hip -- node-level ops (channel-major [C][N] tensors).
//
// These carry the per-node / per-graph parts of the reference modules:
// the MLPs (gnn.py:65), BatchNorm1d over fibers / classes (gnn.py:154, 192),
// the GlobalModel means + double RMSNorm (gnn.py:218-223) and the
// per-graph broadcast of u (gnn.py:100/153/191).  Node tensors are small
// (G*NF fibers, G*NC classes) and L2-resident; the hot path is the edge ops.
#include "pfsgnn_common.h"
#include <cstdlib>
#include "../../include/pfsgnn.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cmath>
#include <map>
#include <vector>

namespace pf {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int fail(const char* where, const char* what) {
  g_err = std::string(where) + ": " + what;
  return -1;
}
// A failure found by a void launcher deep in a call (launch_reduce_multi's
// descriptor limits): recorded here, returned by the C entry point's closing
// check_launch, so no caller reports success with work silently skipped.
static bool g_fail_pending = false;
int fail_pending(const char* where, const char* what) {
  g_fail_pending = true;
  return fail(where, what);
}
// a caller that returns the launcher's error itself takes it off the pending slot
int take_pending(int rc) {
  g_fail_pending = false;
  return rc;
}
int check_launch(const char* where) {
  if (g_fail_pending) {
    g_fail_pending = false;
    return -1;   // (g_err already names the failing launcher)
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(where) + ": " + hipGetErrorString(e);
    return -2;
  }
  return 0;
}
}  // namespace pf

// ---------------------------------------------------------------- timing
// Optional per-kernel HIP-event timing (off by default; never enabled while a
// stream is being captured).  Each main edge kernel launch is bracketed by two
// events on its own stream; pfsgnn_timing_query() resolves them.
namespace pf {
struct TimerRec {
  hipEvent_t a, b;
};
static int g_timing = 0;   // 0 off, 1 events around each launch, 2 + a lead-in spin
static std::map<std::string, std::vector<TimerRec>> g_pending;
static std::map<std::string, std::pair<double, long long>> g_done;
static std::vector<hipEvent_t> g_pool;

static hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Mode 2: a ~0.1 ms single-wave spin kernel goes on the stream before the
// start event.  In eager launching the GPU otherwise idles between kernels
// while the host enqueues the next one, and the start event would time-stamp
// that idle gap (host launch latency) into the kernel's interval; behind the
// spin the start event, the kernel and the end event are all enqueued before
// the GPU reaches them, so the interval is the kernel's own, as in a replayed
// graph (bench.py; rocprofv3's kernel trace of the same command agrees).
__global__ void k_timing_spin(float* sink, int iters) {
  float a = (float)threadIdx.x, b = 1.0000001f;
  for (int i = 0; i < iters; ++i) a = fmaf(a, b, 1e-7f);
  if (a == -1.f) sink[threadIdx.x] = a;   // (never true: keeps the loop)
}
static float* g_sink = nullptr;

Timer::Timer(const char* name, hipStream_t st) : name_(name), st_(st), a_(nullptr) {
  if (!g_timing) return;
  a_ = take_event();
  if (!a_) return;
  if (g_timing == 2) {
    if (!g_sink && hipMalloc(&g_sink, 256) != hipSuccess) g_sink = nullptr;
    if (g_sink) hipLaunchKernelGGL(k_timing_spin, dim3(1), dim3(64), 0, st_, g_sink, 50000);
  }
  (void)hipEventRecord(a_, st_);
}

void Timer::end() {
  if (!g_timing || !a_) return;
  hipEvent_t b = take_event();
  if (!b) return;
  (void)hipEventRecord(b, st_);
  g_pending[name_].push_back({a_, b});
  a_ = nullptr;
}

static void resolve(const std::string& name) {
  auto it = g_pending.find(name);
  if (it == g_pending.end()) return;
  for (auto& r : it->second) {
    float ms = 0.f;
    (void)hipEventSynchronize(r.b);
    (void)hipEventElapsedTime(&ms, r.a, r.b);
    auto& d = g_done[name];
    d.first += ms;
    d.second += 1;
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  it->second.clear();
}
}  // namespace pf

namespace pf {
static std::map<std::string, int> g_repeat;
int repeats(const char* name) {
  if (g_repeat.empty()) return 0;
  auto it = g_repeat.find(name);
  return it == g_repeat.end() ? 0 : it->second;
}
}  // namespace pf

extern "C" int pfsgnn_timing_repeat(const char* name, int extra) {
  PF_REQUIRE(name && extra >= 0 && extra <= 16, "pfsgnn_timing_repeat", "bad arguments");
  if (extra == 0)
    pf::g_repeat.erase(name);
  else
    pf::g_repeat[name] = extra;
  return 0;
}

extern "C" int pfsgnn_timing_enable(int on) {
  pf::g_timing = on == 2 ? 2 : (on != 0 ? 1 : 0);
  return 0;
}

extern "C" int pfsgnn_timing_reset(void) {
  for (auto& kv : pf::g_pending) pf::resolve(kv.first);
  pf::g_done.clear();
  return 0;
}

extern "C" int pfsgnn_timing_query(const char* name, double* total_ms, long long* count) {
  pf::resolve(name);
  auto it = pf::g_done.find(name);
  *total_ms = it == pf::g_done.end() ? 0.0 : it->second.first;
  *count = it == pf::g_done.end() ? 0 : it->second.second;
  return 0;
}

extern "C" const char* pfsgnn_last_error(void) { return pf::g_err.c_str(); }
extern "C" const char* pfsgnn_version(void) { return "pfsgnn 0.1 gfx950"; }

// ---------------------------------------------------------------- reduce
// Partial reductions out[r][c] (+)= scale * sum_b part[b*plen + r*ldp + c],
// up to PF_MAX_RED (96) independent ones per launch (blockIdx.z picks one; block
// layout below).  Long lists (nb > 2 RED_SEG) first take an in-place stage: segment s of RED_SEG
// partials is summed into the segment's first row (each block touches only its
// own cells; the descriptors of one launch never share cells).
#ifndef RED_SEG
#define RED_SEG 256   // (128: +0.01 ms per step, 64: +0.06; profiles/r05as_red_seg_ab.txt)
#endif
// a RedDesc as the kernels read it: 40 bytes, so that 96 share one launch's
// 4 KB of kernel arguments (a backward pass's ~200 weight-gradient
// reductions in 3 launches, not 5); the add flag rides in cols' top bit
#define PF_PACK_RED PF_MAX_RED
struct RedDev {
  const float* part;
  float* out;
  uint32_t plen;
  int nb, ldp, ldo;
  uint16_t rows, colsa;
  float scale;
  __device__ __host__ int cols() const { return colsa & 0x7fff; }
  __device__ __host__ bool add() const { return (colsa >> 15) != 0; }
};
static_assert(sizeof(RedDev) == 40, "RedDev layout");
struct RedPack {
  RedDev d[PF_PACK_RED];
};
static_assert(sizeof(RedPack) <= 4096, "k_reduce_rows' descriptor pack must fit the kernel arguments");

// k_reduce_rows: a block owns 16 consecutive outputs x 16 partial lanes; lane
// (o, pl) sums partials b = pl, pl + 16, ... with 4 independent accumulators
// (4 loads in flight), the 16 lanes combined in a fixed order -- deterministic
// for a given nb.  k_reduce_seg (a segment of RED_SEG partials per block): RED_O
// consecutive outputs x RED_P lanes, so a wave reads 256 contiguous bytes of a
// partial row per load (16 x 16 read 64-byte runs: the deferred flush's 48-way
// segment stage took 55 us; measured 74 -> 57 us per step.  The same layout in
// k_reduce_rows, whose lists are short, was slower: 82 -> 109 us).
#define RED_O 64
#define RED_P 4
__global__ __launch_bounds__(256) void k_reduce_rows(RedPack pk) {
  const RedDev& D = pk.d[blockIdx.z];
  const int t = threadIdx.x, o = t & 15, pl = t >> 4;
  const int idx = blockIdx.x * 16 + o;
  const int cols = D.cols();
  if (blockIdx.x * 16 >= D.rows * cols) return;
  const bool v = idx < D.rows * cols;
  const int r = v ? idx / cols : 0, c = v ? idx - r * cols : 0;
  const float* p = D.part + (size_t)r * D.ldp + c;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = pl;
  for (; b + 48 < D.nb; b += 64) {
    s0 += p[(size_t)b * D.plen];
    s1 += p[(size_t)(b + 16) * D.plen];
    s2 += p[(size_t)(b + 32) * D.plen];
    s3 += p[(size_t)(b + 48) * D.plen];
  }
  for (; b < D.nb; b += 16) s0 += p[(size_t)b * D.plen];
  __shared__ float sh[16][17];
  sh[pl][o] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (t < 16 && v) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += sh[i][t];
    float* op = D.out + (size_t)r * D.ldo + c;
    *op = D.add() ? (*op + D.scale * s) : D.scale * s;
  }
}

__global__ __launch_bounds__(256) void k_reduce_seg(RedPack pk) {
  const RedDev& D = pk.d[blockIdx.z];
  const int t = threadIdx.x, o = t & (RED_O - 1), pl = t / RED_O;
  const int idx = blockIdx.x * RED_O + o;
  const int b0 = blockIdx.y * RED_SEG;
  const int cols = D.cols();
  if (blockIdx.x * RED_O >= D.rows * cols || b0 >= D.nb || D.nb <= 2 * RED_SEG) return;
  const bool v = idx < D.rows * cols;
  const int r = v ? idx / cols : 0, c = v ? idx - r * cols : 0;
  const int b1 = min(D.nb, b0 + RED_SEG);
  float* p = const_cast<float*>(D.part) + (size_t)r * D.ldp + c;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = b0 + pl;
  for (; b + 3 * RED_P < b1; b += 4 * RED_P) {
    s0 += p[(size_t)b * D.plen];
    s1 += p[(size_t)(b + RED_P) * D.plen];
    s2 += p[(size_t)(b + 2 * RED_P) * D.plen];
    s3 += p[(size_t)(b + 3 * RED_P) * D.plen];
  }
  for (; b < b1; b += RED_P) s0 += p[(size_t)b * D.plen];
  __shared__ float sh[RED_P][RED_O];
  sh[pl][o] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (t < RED_O && v) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < RED_P; ++i) s += sh[i][t];
    p[(size_t)b0 * D.plen] = s;
  }
}

static bool red_fits(const RedDesc& a) {
  return a.rows >= 0 && a.rows <= 65535 && a.cols >= 0 && a.cols <= 32767 &&
         a.plen * (a.nb > 2 * RED_SEG ? RED_SEG : 1) <= 0xffffffffull;
}
static RedDev red_dev(const RedDesc& a) {
  return RedDev{a.part, a.out, (uint32_t)a.plen, a.nb, a.ldp, a.ldo, (uint16_t)a.rows,
                (uint16_t)(a.cols | (a.add ? 0x8000 : 0)), a.scale};
}

// -> 0, or -1 with nothing launched when a descriptor does not fit the packed
// 40-byte RedDev (rows > 65535, cols > 32767 or a segment stride past 32 bits);
// the failure is also left pending for the entry point's check_launch
int launch_reduce_multi(const RedDesc* d, int n, hipStream_t st) {
  for (int i = 0; i < n; ++i)
    if (!red_fits(d[i]))
      return pf::fail_pending("launch_reduce_multi", "reduction wider than the packed descriptor");
  for (int i0 = 0; i0 < n; i0 += PF_PACK_RED) {
    const int m = std::min(PF_PACK_RED, n - i0);
    RedPack pk{};
    int gx = 1, gxs = 1, gy = 1;
    bool seg = false;
    for (int i = 0; i < m; ++i) {
      pk.d[i] = red_dev(d[i0 + i]);
      gx = std::max(gx, (pk.d[i].rows * pk.d[i].cols() + 15) / 16);
      gxs = std::max(gxs, (pk.d[i].rows * pk.d[i].cols() + RED_O - 1) / RED_O);
      if (pk.d[i].nb > 2 * RED_SEG) {
        seg = true;
        gy = std::max(gy, (pk.d[i].nb + RED_SEG - 1) / RED_SEG);
      }
    }
    if (seg) {
      hipLaunchKernelGGL(k_reduce_seg, dim3(gxs, gy, m), dim3(256), 0, st, pk);
      for (int i = 0; i < m; ++i)
        if (pk.d[i].nb > 2 * RED_SEG) {
          pk.d[i].nb = (pk.d[i].nb + RED_SEG - 1) / RED_SEG;
          pk.d[i].plen *= RED_SEG;
        }
    }
    hipLaunchKernelGGL(k_reduce_rows, dim3(gx, 1, m), dim3(256), 0, st, pk);
  }
  return 0;
}

int launch_reduce_rows(const float* part, int nb, size_t plen, int ldp, int rows, int cols,
                        float* out, int ldo, int add, float scale, hipStream_t st) {
  RedDesc d{part, nb, plen, ldp, rows, cols, out, ldo, add, scale};
  return launch_reduce_multi(&d, 1, st);
}

// per-class sums over the BPG fiber groups of a graph: out[i][g*NC + c] =
// sum_b part[((g*BPG + b)*NC + c)*C + i]; 16 outputs x 16 partial lanes per
// block, fixed-order combine (deterministic)
__global__ __launch_bounds__(256) void k_reduce_columns(const float* __restrict__ part, int G,
                                                        int BPG, int NC, int C,
                                                        float* __restrict__ out) {
  const int t = threadIdx.x, o = t & 15, pl = t >> 4;
  const int idx = blockIdx.x * 16 + o;  // over G*NC*C, i fastest
  const int total = G * NC * C;
  const bool v = idx < total;
  const int ii = v ? idx : 0;
  const int g = ii / (NC * C);
  const int rem = ii - g * NC * C;
  const float* p = part + (size_t)g * BPG * NC * C + rem;
  float s0 = 0.f, s1 = 0.f;
  int b = pl;
  for (; b + 16 < BPG; b += 32) {
    s0 += p[(size_t)b * NC * C];
    s1 += p[(size_t)(b + 16) * NC * C];
  }
  if (b < BPG) s0 += p[(size_t)b * NC * C];
  __shared__ float sh[16][17];
  sh[pl][o] = s0 + s1;
  __syncthreads();
  if (t < 16 && v) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += sh[k][t];
    const int c = rem / C, i = rem - c * C;
    out[(size_t)i * G * NC + (size_t)g * NC + c] = s;
  }
}

void launch_reduce_columns(const float* part, int G, int BPG, int NC, int C, float* out,
                           hipStream_t st) {
  const int total = G * NC * C;
  hipLaunchKernelGGL(k_reduce_columns, dim3((total + 15) / 16), dim3(256), 0, st, part, G, BPG,
                     NC, C, out);
}

// ---------------------------------------------------------------- node inputs
// A node-op input is up to PF_MAX_SEG row blocks of a virtual concatenation
// (the torch.cat of gnn.py:100/136/153/188/191/220) -- never materialised.
// Block s covers input rows [k0[s], k0[s+1]); its row k reads p[s] row
// k - k0[s], either a [rows][N] node tensor or, when bc[s], a per-graph
// [rows][N / npg] tensor whose column n / npg is broadcast to the npg nodes of
// graph n / npg (the u[batch] gathers).  wcol[s] is the weight column of the
// block's first row.  Unused blocks have k0 = INT_MAX.
#define PF_MAX_SEG 4
struct XSegs {
  const float* p[PF_MAX_SEG];
  int k0[PF_MAX_SEG + 1];
  int wcol[PF_MAX_SEG];
  int bc[PF_MAX_SEG];
  int npg;
};

__device__ __forceinline__ int seg_of(const XSegs& S, int k) {
  int s = 0;
#pragma unroll
  for (int i = 1; i < PF_MAX_SEG; ++i) s += k >= S.k0[i] ? 1 : 0;
  return s;
}

// row k of the concatenation at node n (ng = n / npg)
__device__ __forceinline__ float seg_load(const XSegs& S, int k, int n, int ng, int N, int Gc) {
  const int s = seg_of(S, k);
  const float* p = S.p[0];
  int kb = S.k0[0], bc = S.bc[0];
#pragma unroll
  for (int i = 1; i < PF_MAX_SEG; ++i)
    if (s == i) {
      p = S.p[i];
      kb = S.k0[i];
      bc = S.bc[i];
    }
  return bc ? p[(size_t)(k - kb) * Gc + ng] : p[(size_t)(k - kb) * N + n];
}

__device__ __forceinline__ int seg_wcol(const XSegs& S, int k) {
  const int s = seg_of(S, k);
  int kb = S.k0[0], wc = S.wcol[0];
#pragma unroll
  for (int i = 1; i < PF_MAX_SEG; ++i)
    if (s == i) {
      kb = S.k0[i];
      wc = S.wcol[i];
    }
  return wc + (k - kb);
}

static XSegs one_seg(const float* X, int wcol) {
  XSegs S{};
  S.p[0] = X;
  S.k0[0] = 0;
  S.wcol[0] = wcol;
  for (int i = 1; i <= PF_MAX_SEG; ++i) S.k0[i] = INT_MAX;
  S.npg = 0;
  return S;
}

// Builds XSegs from the ABI's pfsgnn_seg list; returns the total row count or
// -1 on a malformed list.
static int make_segs(const pfsgnn_seg* segs, int nseg, int N, XSegs& S) {
  if (!segs || nseg < 1 || nseg > PF_MAX_SEG) return -1;
  S = XSegs{};
  int k = 0, npg = 0;
  for (int i = 0; i < nseg; ++i) {
    if (!segs[i].x || segs[i].rows <= 0 || segs[i].col < 0 || segs[i].per_graph < 0) return -1;
    if (segs[i].per_graph) {
      if (N % segs[i].per_graph) return -1;
      if (npg && npg != segs[i].per_graph) return -1;
      npg = segs[i].per_graph;
    }
    S.p[i] = segs[i].x;
    S.k0[i] = k;
    S.wcol[i] = segs[i].col;
    S.bc[i] = segs[i].per_graph ? 1 : 0;
    k += segs[i].rows;
  }
  for (int i = nseg; i <= PF_MAX_SEG; ++i) S.k0[i] = INT_MAX;
  S.npg = npg;
  return k;
}

// ---------------------------------------------------------------- lin / lin_t
// Y[Mo][N] (+)= op(W)[Mo][Ki] . act(X)[Ki][N] (+ bscale*b) (* lrelu'(Z)) on
// v_mfma_f32_16x16x4_f32: a wave owns 16 node columns and every output row
// (MT tiles of 16), the node column is the MFMA N index, the input channel
// the K index.  Each lane first issues ALL its X loads (KSM >= ceil(Ki/4)
// slots, held in registers), then the block stages the whole op(W) -- W for
// lin, W^T for lin_t -- in LDS once ([MT*16][4*KSM+1], odd stride), so the X
// latency overlaps the staging and the MFMA chain runs without a wait.
// Optional epilogue gathers of lin: Y[m][n] += g[j][m*ld[j] + idx[j][n]] --
// per-node tables indexed per column (the general-graph path adds the gathered
// node parts of a first Linear, gnn.py:100/136/188, in the same pass)
struct GatherAdd {
  const float* g[2];
  const int* idx[2];
  int ld[2];
};

template <int MT, int KSM>
__device__ __forceinline__ void gemm_block(const float* __restrict__ W, int ldw, int trans, int Mo,
                                           int Ki, const XSegs& S, int N,
                                           const float* __restrict__ b, float bscale, int act_in,
                                           const float* __restrict__ Z, float* __restrict__ Y,
                                           int add, int bid, const GatherAdd& GA) {
  extern __shared__ float Ws[];
  // KSM K-steps of 4 always run (no per-step branch: the accumulators stay in
  // AGPRs across the chain); rows Ki..4*KSM of op(W) and X are zero
  constexpr int K4 = 4 * KSM, LDK = K4 + 1;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, col = lane & 15, kq = lane >> 4;
  const int n = bid * 64 + wave * 16 + col;
  const bool nv = n < N;
  const int nc = nv ? n : N - 1;
  const int Gc = S.npg ? N / S.npg : 1, ng = S.npg ? nc / S.npg : 0;
  float bv[KSM];
#pragma unroll
  for (int s = 0; s < KSM; ++s) {
    const int kk = 4 * s + kq;
    bv[s] = kk < Ki ? seg_load(S, kk, nc, ng, N, Gc) : 0.f;
  }
  // op(W) staging: up to 48 loads per thread in flight (the whole op(W) in one
  // L2 round trip for every shape up to 100 x 100), then their LDS stores; the
  // (m, kk) split is recomputed for the stores instead of held in registers
  constexpr int MR = MT * 16, TOT = MR * K4;
  // (a power-of-two batch: odd-sized register arrays here went to scratch)
  constexpr int PER = (TOT + 255) / 256;
  constexpr int BATCH = PER <= 1 ? 1 : PER <= 2 ? 2 : PER <= 4 ? 4 : PER <= 8 ? 8 : PER <= 16 ? 16 : 32;
  // (m, kk) of staging item idx, returned by value (reference out-parameters
  // here were kept in scratch memory)
  auto split = [&](int idx) -> int2 {
    if (!trans) {
      const int m = idx / K4;
      return make_int2(m, idx - m * K4);
    }
    // op(W) = W^T: walk W's rows so the reads stay contiguous
    const int kk = idx / MR;
    return make_int2(idx - kk * MR, kk);
  };
  for (int base = t; base < TOT; base += BATCH * 256) {
    float v[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int idx = base + u * 256;
      const int2 mk = split(idx);
      v[u] = 0.f;
      if (idx < TOT && mk.x < Mo && mk.y < Ki)
        v[u] = trans ? W[(size_t)mk.y * ldw + mk.x] : W[(size_t)mk.x * ldw + seg_wcol(S, mk.y)];
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int idx = base + u * 256;
      const int2 mk = split(idx);
      if (idx < TOT) Ws[mk.x * LDK + mk.y] = v[u];
    }
  }
  __syncthreads();
  const float* wr = Ws + col * LDK + kq;
  if (act_in) {
#pragma unroll
    for (int s = 0; s < KSM; ++s) bv[s] = lrelu(bv[s]);
  }
  floatx4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KSM; ++s) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[16 * mt * LDK + 4 * s], bv[s], acc[mt],
                                                     0, 0, 0);
  }
  if (!nv) return;
  // (epilogue gathers only in the small shapes that take them)
  constexpr bool GATH = MT <= 4 && KSM <= 16;
  const int gi0 = GATH && GA.g[0] ? GA.idx[0][n] : 0;
  const int gi1 = GATH && GA.g[1] ? GA.idx[1][n] : 0;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * mt + 4 * kq + r;
      if (row < Mo) {
        float v = acc[mt][r];
        if (b) v += bscale * b[row];
        if (GATH && GA.g[0]) v += GA.g[0][(size_t)row * GA.ld[0] + gi0];
        if (GATH && GA.g[1]) v += GA.g[1][(size_t)row * GA.ld[1] + gi1];
        if (Z) v *= dlrelu(Z[(size_t)row * N + n]);
        float* o = Y + (size_t)row * N + n;
        *o = add ? (*o + v) : v;
      }
    }
}

template <int MT, int KSM>
__global__ __launch_bounds__(256) void k_gemm(const float* __restrict__ W, int ldw, int trans,
                                              int Mo, int Ki, XSegs S, int N,
                                              const float* __restrict__ b, float bscale,
                                              int act_in, const float* __restrict__ Z,
                                              float* __restrict__ Y, int add, GatherAdd GA) {
  gemm_block<MT, KSM>(W, ldw, trans, Mo, Ki, S, N, b, bscale, act_in, Z, Y, add, blockIdx.x, GA);
}

// Several independent small products in one launch (pfsgnn_gemm_multi): job j
// owns blocks [blk0_j, blk0_j + ceil(N_j / 64)); the table rides in the kernel
// arguments; the instantiation covers the widest job (MT, KSM), narrower jobs
// run zero padding.
#define GM_MULTI 4
struct GemmJob {
  const float* W;
  XSegs S;
  const float* b;
  const float* Z;
  float* Y;
  int ldw, trans, Mo, Ki, N, act_in, add, blk0;
  float bscale;
};
struct GemmTable {
  GemmJob j[GM_MULTI];
  int njob;
};

template <int MT, int KSM>
__global__ __launch_bounds__(256) void k_gemm_multi(GemmTable T) {
  const int bx = blockIdx.x;
  int jj = 0;
#pragma unroll
  for (int u = 1; u < GM_MULTI; ++u)
    if (u < T.njob && bx >= T.j[u].blk0) jj = u;
  const GemmJob& J = T.j[jj];   // read in place from the kernel arguments
  const GatherAdd none{};
  gemm_block<MT, KSM>(J.W, J.ldw, J.trans, J.Mo, J.Ki, J.S, J.N, J.b, J.bscale, J.act_in, J.Z,
                      J.Y, J.add, bx - J.blk0, none);
}

// K-step counts instantiated (Ki = 1..4, 9..12, 17..20, 29..32, 37..40, 97..100
// and 157..160 run without padding steps: the encoders, F, 2F, 3F, 4F, 10F)
#define PF_GEMM_KSM(X) X(1) X(3) X(5) X(8) X(10) X(16) X(25) X(40)
static int gemm_ksm(int Ki) {
  const int ks = (Ki + 3) / 4;
  for (int v : {1, 3, 5, 8, 10, 16, 25, 40})
    if (ks <= v) return v;
  return -1;
}

template <int MT>
static void gemm_attr() {
#define PF_ATTR(KSM)                                                                       \
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<MT, KSM>),               \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  PF_GEMM_KSM(PF_ATTR)
#undef PF_ATTR
}

template <int MT>
static void gemm_launch(int ksm, dim3 grid, size_t lds, hipStream_t st, const float* W, int ldw,
                        int trans, int Mo, int Ki, const XSegs& S, int N, const float* b,
                        float bscale, int act_in, const float* Z, float* Y, int add,
                        const GatherAdd& GA) {
  switch (ksm) {
#define PF_CASE(KSM)                                                                           \
  case KSM:                                                                                    \
    hipLaunchKernelGGL((k_gemm<MT, KSM>), grid, dim3(256), lds, st, W, ldw, trans, Mo, Ki, S, \
                       N, b, bscale, act_in, Z, Y, add, GA);                                   \
    break;
    PF_GEMM_KSM(PF_CASE)
#undef PF_CASE
  }
}

static int launch_gemm(const float* W, int ldw, int trans, int Mo, int Ki, const XSegs& S, int N,
                       const float* b, float bscale, int act_in, const float* Z, float* Y, int add,
                       hipStream_t st, const char* where, const GatherAdd& GA = GatherAdd{}) {
  const int MT = (Mo + 15) / 16;
  const int ksm = gemm_ksm(Ki);
  if (ksm < 0) return pf::fail(where, "input width > 160 not supported");
  if (MT > 11) return pf::fail(where, "output width > 176 not supported");
  static bool attr_set = false;
  if (!attr_set) {  // the widest op(W) (176 x 161) stages 113 KB of the CU's 160 KB LDS
    gemm_attr<1>(); gemm_attr<2>(); gemm_attr<3>(); gemm_attr<4>(); gemm_attr<5>();
    gemm_attr<6>(); gemm_attr<7>(); gemm_attr<8>(); gemm_attr<9>(); gemm_attr<10>();
    gemm_attr<11>();
    attr_set = true;
  }
  const dim3 grid((N + 63) / 64);
  const size_t lds = (size_t)MT * 16 * (4 * ksm + 1) * sizeof(float);
  switch (MT) {
#define PF_MT(T) \
  case T: gemm_launch<T>(ksm, grid, lds, st, W, ldw, trans, Mo, Ki, S, N, b, bscale, act_in, Z, Y, add, GA); break;
    PF_MT(1) PF_MT(2) PF_MT(3) PF_MT(4) PF_MT(5) PF_MT(6) PF_MT(7) PF_MT(8) PF_MT(9) PF_MT(10)
    PF_MT(11)
#undef PF_MT
  }
  return pf::check_launch(where);
}

extern "C" int pfsgnn_lin(const float* W, int ldw, int M, int K, const float* X, int N,
                          const float* b, float bscale, int act_in, float* Y, int add,
                          void* stream) {
  PF_REQUIRE(W && X && Y && M > 0 && K > 0 && N > 0, "pfsgnn_lin", "bad arguments");
  return launch_gemm(W, ldw, 0, M, K, one_seg(X, 0), N, b, bscale, act_in, nullptr, Y, add,
                     as_stream(stream), "pfsgnn_lin");
}

extern "C" int pfsgnn_lin_gather(const float* W, int ldw, int M, int K, const float* X, int N,
                                 const float* b, float bscale, int act_in, float* Y, int add,
                                 const float* G1, const int* idx1, int ld1, const float* G2,
                                 const int* idx2, int ld2, void* stream) {
  PF_REQUIRE(W && X && Y && M > 0 && K > 0 && N > 0 && (!G1 || idx1) && (!G2 || idx2),
             "pfsgnn_lin_gather", "bad arguments");
  PF_REQUIRE((!G1 && !G2) || (M <= 64 && K <= 64), "pfsgnn_lin_gather",
             "gathers need M, K <= 64");
  const GatherAdd GA{{G1, G2}, {idx1, idx2}, {ld1, ld2}};
  return launch_gemm(W, ldw, 0, M, K, one_seg(X, 0), N, b, bscale, act_in, nullptr, Y, add,
                     as_stream(stream), "pfsgnn_lin_gather", GA);
}

extern "C" int pfsgnn_lin_cat(const float* W, int ldw, int M, const pfsgnn_seg* segs, int nseg,
                              int N, const float* b, float bscale, int act_in, float* Y, int add,
                              void* stream) {
  PF_REQUIRE(W && Y && M > 0 && N > 0, "pfsgnn_lin_cat", "bad arguments");
  XSegs S;
  const int K = make_segs(segs, nseg, N, S);
  PF_REQUIRE(K > 0, "pfsgnn_lin_cat", "bad segment list");
  return launch_gemm(W, ldw, 0, M, K, S, N, b, bscale, act_in, nullptr, Y, add, as_stream(stream),
                     "pfsgnn_lin_cat");
}

extern "C" int pfsgnn_lin_t(const float* W, int ldw, int M, int K, const float* dY, int N,
                            const float* Z, float* out, int add, void* stream) {
  PF_REQUIRE(W && dY && out && M > 0 && K > 0 && N > 0, "pfsgnn_lin_t", "bad arguments");
  // out[K][N] = W^T[K][M] . dY[M][N]
  return launch_gemm(W, ldw, 1, K, M, one_seg(dY, 0), N, nullptr, 1.f, 0, Z, out, add,
                     as_stream(stream), "pfsgnn_lin_t");
}

// Batched small products (the node-side Linear layers of one block that have
// no data dependence on each other): up to GM_MULTI jobs per launch, each a
// pfsgnn_lin_cat (trans 0) or pfsgnn_lin_t (trans 1); same per-output
// arithmetic as the single launches (zero padding adds exact zeros).
#define PF_GMM_ALL(X) \
  X(1, 3) X(1, 5) X(1, 10) X(2, 3) X(2, 5) X(2, 10) X(3, 3) X(3, 5) X(3, 10) X(4, 3) X(4, 5) \
  X(4, 10)
extern "C" int pfsgnn_gemm_multi(const pfsgnn_gemm_job* jobs, int n, void* stream) {
  const char* where = "pfsgnn_gemm_multi";
  PF_REQUIRE(n >= 0 && (jobs || n == 0), where, "bad arguments");
  hipStream_t st = as_stream(stream);
  static bool attr = false;
  if (!attr) {
#define PF_GMA(T, K)                                                                           \
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_multi<T, K>),                \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    PF_GMM_ALL(PF_GMA)
#undef PF_GMA
    attr = true;
  }
  for (int i0 = 0; i0 < n; i0 += GM_MULTI) {
    const int m = std::min(GM_MULTI, n - i0);
    GemmTable T{};
    int blocks = 0, mt = 1, ks = 3;
    for (int u = 0; u < m; ++u) {
      const pfsgnn_gemm_job& jb = jobs[i0 + u];
      PF_REQUIRE(jb.W && jb.Y && jb.M > 0 && jb.N > 0 && (jb.trans == 0 || jb.trans == 1), where,
                 "bad job");
      GemmJob& J = T.j[u];
      int Ki;
      if (jb.trans) {
        PF_REQUIRE(jb.nseg == 1 && jb.segs && jb.segs[0].x && !jb.segs[0].per_graph, where,
                   "lin_t job takes one plain input block");
        J.S = one_seg(jb.segs[0].x, 0);
        Ki = jb.K;
      } else {
        Ki = make_segs(jb.segs, jb.nseg, jb.N, J.S);
        PF_REQUIRE(Ki > 0, where, "bad segment list");
      }
      PF_REQUIRE(Ki <= 40 && jb.M <= 64, where, "job wider than the batched kernels (K 40, M 64)");
      J.W = jb.W;
      J.b = jb.b;
      J.Z = jb.Z;
      J.Y = jb.Y;
      J.ldw = jb.ldw;
      J.trans = jb.trans;
      J.Mo = jb.M;
      J.Ki = Ki;
      J.N = jb.N;
      J.act_in = jb.act_in;
      J.add = jb.add;
      J.bscale = jb.bscale;
      J.blk0 = blocks;
      blocks += (jb.N + 63) / 64;
      mt = std::max(mt, (jb.M + 15) / 16);
      const int k4 = (Ki + 3) / 4;
      ks = std::max(ks, k4 <= 3 ? 3 : k4 <= 5 ? 5 : 10);
    }
    T.njob = m;
    const size_t lds = (size_t)mt * 16 * (4 * ks + 1) * sizeof(float);
    bool launched = false;
#define PF_GMM(TT, KK)                                                                       \
  if (!launched && mt == TT && ks == KK) {                                                   \
    hipLaunchKernelGGL((k_gemm_multi<TT, KK>), dim3(blocks), dim3(256), lds, st, T);         \
    launched = true;                                                                         \
  }
    PF_GMM_ALL(PF_GMM)
#undef PF_GMM
    PF_REQUIRE(launched, where, "no kernel for this shape");
  }
  return pf::check_launch(where);
}

// ---------------------------------------------------------------- wgrad
// dW[m][col(k)] += sum_n dY[m][n] act(X[k][n]) and (optionally) db[m] +=
// s*sum_n dY[m][n] as one more row k = K of ones.  A block owns a node range
// and walks it in chunks of 64 nodes, staged ROW-major in LDS ([row][68]:
// straight float4 copies of dY and X rows, no transpose).  The MFMA reduction
// index is a permutation of the chunk's nodes -- step s of lane quad kq takes
// node 16*kq + s for both operands -- so each lane reads its A and B values as
// float4 runs (ds_read_b128; a 68-float row stride puts 16 rows on 64 distinct
// banks).  The next chunk's global loads are issued before the current
// chunk's MFMAs.  8 waves own output tiles wave, wave+8, ...; per-block
// partials + a fixed-order reduce (deterministic).
#define WG_WAVES 8
#define WG_LD 68
// staged row kinds (per float4 item of a thread; fixed over the chunks)
#define WG_DY 0
#define WG_X 1
#define WG_XBC 2
#define WG_ONE 3
#define WG_NONE 4
// X3 (bf16x3): the chunk is staged as split bf16 planes instead -- row =
// [64 hi | 64 lo] bf16 in the same 272-byte stride, node 32s + 8kq + q at step
// s (two v_mfma_f32_16x16x32_bf16 K-steps per chunk, three products each:
// Ah Bl + Al Bh + Ah Bh, ~2^-16 relative per product, fp32 accumulation;
// 6 x 16 instead of 16 x 32 MFMA cycles per tile and chunk).  A wave owns a
// contiguous run of tiles (one dY row tile for many X tiles: its A operand is
// read once), and db -- a bias gradient a following BatchNorm cancels to ~0 --
// stays an exact fp32 sum of the staged dY values.
template <int TMAX, int PER, bool X3 = false>
__device__ __forceinline__ void wgrad_block(const float* __restrict__ dY, int M, const XSegs& S,
                                            int K, int K1, int N, int act_in, int chunk, int vec,
                                            float* __restrict__ part, int bid) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int MR = (M + 15) & ~15, KR = (K1 + 15) & ~15;
  float* Sd = sm;
  float* Sx = sm + MR * WG_LD;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, col = lane & 15, kq = lane >> 4;
  const int KT = KR / 16, NTILE = (MR / 16) * KT;
  const int n0 = bid * chunk, n1 = min(N, n0 + chunk);
  const int Gc = S.npg ? N / S.npg : 1;
  floatx4 acc[TMAX];
#pragma unroll
  for (int j = 0; j < TMAX; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // padding rows (M..MR, K1..KR) are zero once; the chunk loop never writes them
  for (int idx = t; idx < (MR - M) * WG_LD; idx += 64 * WG_WAVES) Sd[M * WG_LD + idx] = 0.f;
  for (int idx = t; idx < (KR - K1) * WG_LD; idx += 64 * WG_WAVES) Sx[K1 * WG_LD + idx] = 0.f;
  // item it = row (it >> 4: dY rows, then X rows, then the ones row) x float4 q
  const int items = (M + K1) * 16;
  const float* rp[PER];
  int kind[PER];
  float* lp[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int it = t + i * 64 * WG_WAVES, r = it >> 4, q = it & 15;
    rp[i] = nullptr;
    kind[i] = WG_NONE;
    lp[i] = (r < M ? Sd + r * WG_LD : Sx + (r - M) * WG_LD) + 4 * q;
    if (it >= items) continue;
    if (r < M) {
      rp[i] = dY + (size_t)r * N + 4 * q;
      kind[i] = WG_DY;
    } else if (r - M < K) {
      const int k = r - M, s = seg_of(S, k);
      const float* p = S.p[0];
      int kb = S.k0[0], bc = S.bc[0];
#pragma unroll
      for (int u = 1; u < PF_MAX_SEG; ++u)
        if (s == u) {
          p = S.p[u];
          kb = S.k0[u];
          bc = S.bc[u];
        }
      rp[i] = bc ? p + (size_t)(k - kb) * Gc : p + (size_t)(k - kb) * N + 4 * q;
      kind[i] = bc ? WG_XBC : WG_X;
    } else {
      kind[i] = WG_ONE;
    }
  }
  auto fetch = [&](int c, int i) -> float4 {
    const int q = (t + i * 64 * WG_WAVES) & 15;
    const int nn = c + 4 * q;  // first node of the item
    float4 v = {0.f, 0.f, 0.f, 0.f};
    const int k = kind[i];
    if (k == WG_DY || k == WG_X) {
      const float* p = rp[i] + c;
      if (vec && nn + 3 < n1) {
        v = *reinterpret_cast<const float4*>(p);
      } else {
        v.x = nn < n1 ? p[0] : 0.f;
        v.y = nn + 1 < n1 ? p[1] : 0.f;
        v.z = nn + 2 < n1 ? p[2] : 0.f;
        v.w = nn + 3 < n1 ? p[3] : 0.f;
      }
    } else if (k == WG_XBC) {
      const float* p = rp[i];
      v.x = nn < n1 ? p[nn / S.npg] : 0.f;
      v.y = nn + 1 < n1 ? p[(nn + 1) / S.npg] : 0.f;
      v.z = nn + 2 < n1 ? p[(nn + 2) / S.npg] : 0.f;
      v.w = nn + 3 < n1 ? p[(nn + 3) / S.npg] : 0.f;
    } else if (k == WG_ONE) {
      v.x = nn < n1 ? 1.f : 0.f;
      v.y = nn + 1 < n1 ? 1.f : 0.f;
      v.z = nn + 2 < n1 ? 1.f : 0.f;
      v.w = nn + 3 < n1 ? 1.f : 0.f;
    }
    if (act_in && (k == WG_X || k == WG_XBC)) {
      v.x = lrelu(v.x); v.y = lrelu(v.y); v.z = lrelu(v.z); v.w = lrelu(v.w);
    }
    return v;
  };
  float4 buf[PER];
  float dbs[PER];   // X3: this thread's share of db (its dY items), exact fp32
#pragma unroll
  for (int i = 0; i < PER; ++i) dbs[i] = 0.f;
  const bool xdb = X3 && K1 > K;
  // tile of (wave, j): X3 contiguous runs, else wave + 8 j
  const int tpw = (NTILE + WG_WAVES - 1) / WG_WAVES;
  auto tile_of = [&](int j) { return X3 ? (j < tpw ? wave * tpw + j : NTILE) : wave + WG_WAVES * j; };
  // the bf16x3 form keeps two chunks of loads in flight, not one (<8, 8>:
  // 139 -> 114 us at the bench batch, 1525 -> 915 us at configs[2]); the fp32
  // form measured slower so (<1, 4>: 37 -> 47 us, profiles/r04ah_*)
  constexpr bool DEEP = X3 && PER <= 8 && TMAX <= 8;
  float4 buf2[DEEP ? PER : 1];
  if (n0 < n1) {
#pragma unroll
    for (int i = 0; i < PER; ++i) buf[i] = fetch(n0, i);
  }
  if constexpr (DEEP) {
    if (n0 + 64 < n1) {
#pragma unroll
      for (int i = 0; i < PER; ++i) buf2[i] = fetch(n0 + 64, i);
    }
  }
  for (int c = n0; c < n1; c += 64) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (kind[i] != WG_NONE) {
        if constexpr (X3) {
          const int q = t & 15;
          short* row = reinterpret_cast<short*>(lp[i] - 4 * q);
          pf_s16x4 h, l;
          pf_split4(buf[i].x, buf[i].y, buf[i].z, buf[i].w, h, l);
          *reinterpret_cast<pf_s16x4*>(row + 4 * q) = h;
          *reinterpret_cast<pf_s16x4*>(row + 64 + 4 * q) = l;
          if (xdb && kind[i] == WG_DY) dbs[i] += (buf[i].x + buf[i].y) + (buf[i].z + buf[i].w);
        } else {
          *reinterpret_cast<float4*>(lp[i]) = buf[i];
        }
      }
    __syncthreads();
    if constexpr (DEEP) {   // chunk c + 2's loads join c + 1's in flight
#pragma unroll
      for (int i = 0; i < PER; ++i) buf[i] = buf2[i];
      if (c + 128 < n1) {
#pragma unroll
        for (int i = 0; i < PER; ++i) buf2[i] = fetch(c + 128, i);
      }
    } else if (c + 64 < n1) {  // next chunk's loads in flight during this chunk's MFMAs
#pragma unroll
      for (int i = 0; i < PER; ++i) buf[i] = fetch(c + 64, i);
    }
    if constexpr (X3) {
      int mprev = -1;
      pf_s16x8 ah0, al0, ah1, al1;
#pragma unroll
      for (int j = 0; j < TMAX; ++j) {
        const int tile = tile_of(j);
        if (tile < NTILE) {
          const int mt = tile / KT, kt = tile - mt * KT;
          if (mt != mprev) {
            const short* pa = reinterpret_cast<const short*>(Sd + (16 * mt + col) * WG_LD) + 8 * kq;
            ah0 = *reinterpret_cast<const pf_s16x8*>(pa);
            ah1 = *reinterpret_cast<const pf_s16x8*>(pa + 32);
            al0 = *reinterpret_cast<const pf_s16x8*>(pa + 64);
            al1 = *reinterpret_cast<const pf_s16x8*>(pa + 96);
            mprev = mt;
          }
          const short* pb = reinterpret_cast<const short*>(Sx + (16 * kt + col) * WG_LD) + 8 * kq;
          const pf_s16x8 bh0 = *reinterpret_cast<const pf_s16x8*>(pb);
          const pf_s16x8 bh1 = *reinterpret_cast<const pf_s16x8*>(pb + 32);
          const pf_s16x8 bl0 = *reinterpret_cast<const pf_s16x8*>(pb + 64);
          const pf_s16x8 bl1 = *reinterpret_cast<const pf_s16x8*>(pb + 96);
          acc[j] = pf_mf8(ah0, bl0, acc[j]);
          acc[j] = pf_mf8(al0, bh0, acc[j]);
          acc[j] = pf_mf8(ah0, bh0, acc[j]);
          acc[j] = pf_mf8(ah1, bl1, acc[j]);
          acc[j] = pf_mf8(al1, bh1, acc[j]);
          acc[j] = pf_mf8(ah1, bh1, acc[j]);
        }
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      const int tile = wave + WG_WAVES * j;
      if (tile < NTILE) {
        const int mt = tile / KT, kt = tile - mt * KT;
        const float* pa = Sd + (16 * mt + col) * WG_LD + 16 * kq;
        const float* pb = Sx + (16 * kt + col) * WG_LD + 16 * kq;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const float4 a = *reinterpret_cast<const float4*>(pa + 4 * q4);
          const float4 bq = *reinterpret_cast<const float4*>(pb + 4 * q4);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bq.x, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bq.y, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bq.z, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bq.w, acc[j], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TMAX; ++j) {
    const int tile = tile_of(j);
    if (tile < NTILE) {
      const int mt = tile / KT, kt = tile - mt * KT;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * mt + 4 * kq + r, k = 16 * kt + col;
        if (m < M && k < (xdb ? K : K1))
          part[(size_t)bid * M * K1 + (size_t)m * K1 + k] = acc[j][r];
      }
    }
  }
  if (xdb) {   // db column: the 16 threads of a dY row, fixed xor tree
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      float v = dbs[i];
      v += __shfl_xor(v, 8, 16);
      v += __shfl_xor(v, 4, 16);
      v += __shfl_xor(v, 2, 16);
      v += __shfl_xor(v, 1, 16);
      const int r = (t + i * 64 * WG_WAVES) >> 4;
      if ((t & 15) == 0 && kind[i] == WG_DY) part[(size_t)bid * M * K1 + (size_t)r * K1 + K] = v;
    }
  }
}

template <int TMAX, int PER, bool X3>
__global__ __launch_bounds__(512) void k_wgrad(const float* __restrict__ dY, int M, XSegs S, int K,
                                               int K1, int N, int act_in, int chunk, int vec,
                                               float* __restrict__ part) {
  wgrad_block<TMAX, PER, X3>(dY, M, S, K, K1, N, act_in, chunk, vec, part, blockIdx.x);
}

// Several independent weight gradients in one launch (pfsgnn_wgrad_multi):
// job j owns blocks [blk0_j, blk0_j + nblk_j); the table rides in the kernel
// arguments and a block selects its job with constant indices (uniform).
#define WG_MULTI 24   // (24 jobs x 144 B: the table stays under the 4 KB kernel-argument limit)
struct WgJob {
  const float* dY;
  XSegs S;
  float* part;
  int M, K, K1, N, act_in, chunk, vec, blk0;
};
struct WgTable {
  WgJob j[WG_MULTI];
  int njob;
};
static_assert(sizeof(WgTable) <= 4096, "k_wgrad_multi's job table must fit the kernel arguments");

template <int TMAX, int PER, bool X3>
__global__ __launch_bounds__(512) void k_wgrad_multi(WgTable T) {
  const int b = blockIdx.x;
  int jj = 0;
#pragma unroll
  for (int u = 1; u < WG_MULTI; ++u)
    if (u < T.njob && b >= T.j[u].blk0) jj = u;
  const WgJob& J = T.j[jj];   // read in place from the kernel arguments (a copy spills)
  wgrad_block<TMAX, PER, X3>(J.dY, J.M, J.S, J.K, J.K1, J.N, J.act_in, J.chunk, J.vec, J.part,
                             b - J.blk0);
}

// Node-level weight gradients in bf16x3 (wgrad_block's X3 form) on every edge
// path except the exact-fp32 ones (PFSGNN_EDGE_MFMA_F32, _VALU, _BF16Y);
// PFSGNN_NODE_WG_X3=0 keeps the fp32 MFMA form everywhere.
// Only where the MFMAs dominate: >= 4 output tiles per wave (the narrow ones
// -- a tile or two per wave -- are staging-bound and the operand split costs
// more than it saves: <1, 4> 36.8 -> 44.4 us, <8, 8> 148 -> 134.5 us,
// profiles/r04z_step_trace.txt); <16, 16> X3 spills.
static bool wg_x3_for(int tm, int per) {
  static const int min_tm = [] {   // A/B knob PFSGNN_WG_X3_MIN_TM
    const char* e = std::getenv("PFSGNN_WG_X3_MIN_TM");
    return e ? std::max(1, std::atoi(e)) : 4;
  }();
  return tm >= min_tm && !(tm == 16 && per == 16) && pf::node_x3("PFSGNN_NODE_WG_X3");
}

static int wgrad_blocks(int N) {
  static const int cap = [] {   // tuning knob: PFSGNN_WG_BLOCKS (blocks per weight gradient)
    const char* e = std::getenv("PFSGNN_WG_BLOCKS");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? std::min(v, 256) : 256;
  }();
  // >= ~400 nodes per block: at the bench shape (38k nodes) 96 blocks, not 256,
  // -0.035 ms per step (profiles/r05af_wg_blocks_ab.txt); configs[2]'s 613k
  // nodes keep 256 (96 there: +0.12 ms, r05ag_wg_blocks_configs2_ab.txt)
  int s = (N + 399) / 400;
  return std::max(1, std::min(s, cap));   // <= 2*RED_SEG: one reduce launch
}

static size_t wgrad_part_bytes(int M, int K1, int N) {
  return (size_t)wgrad_blocks(N) * M * K1 * sizeof(float);
}

// Launch geometry of one weight gradient (shared by the single and the
// batched launches).
struct WgPlan {
  int K1, nblk, chunk, tm, per, vec;
  size_t lds, part_bytes;
};

static int wgrad_plan(const float* dY, int M, const XSegs& S, int nseg, int K, int N, bool has_db,
                      const char* where, WgPlan& P) {
  PF_REQUIRE(M <= 256 && K <= 256, where, "M, K too large");
  const int nbk = wgrad_blocks(N);
  P.K1 = K + (has_db ? 1 : 0);
  P.chunk = ((N + nbk - 1) / nbk + 63) / 64 * 64;
  P.nblk = (N + P.chunk - 1) / P.chunk;
  P.part_bytes = (size_t)P.nblk * M * P.K1 * sizeof(float);
  const int MR = (M + 15) & ~15, KR = (P.K1 + 15) & ~15;
  P.lds = (size_t)(MR + KR) * WG_LD * sizeof(float);
  const int ntile = (MR / 16) * (KR / 16);
  // float4 staging when every row starts 16-byte aligned
  bool vec = (N % 4 == 0) && ((uintptr_t)dY % 16 == 0);
  for (int i = 0; i < nseg; ++i)
    if (!S.bc[i] && (uintptr_t)S.p[i] % 16 != 0) vec = false;
  P.vec = vec ? 1 : 0;
  const int items = (M + P.K1) * 16;
  P.per = items <= 512 ? 1 : items <= 1024 ? 2 : items <= 2048 ? 4 : items <= 4096 ? 8 : 16;
  PF_REQUIRE(items <= 16 * 64 * WG_WAVES, where, "M + K too large");
  P.tm = ntile <= WG_WAVES ? 1 : ntile <= 2 * WG_WAVES ? 2 : ntile <= 4 * WG_WAVES ? 4
       : ntile <= 8 * WG_WAVES ? 8 : ntile <= 16 * WG_WAVES ? 16 : -1;
  PF_REQUIRE(P.tm > 0, where, "too many output tiles");
  return 0;
}

// the reductions finishing one weight gradient's partials: each input block's
// dW columns, plus db
static int wgrad_reds(const XSegs& S, int nseg, int K, int M, const WgPlan& P, float* part,
                      float* dW, int lddw, float* db, float dbscale, RedDesc* rd) {
  int nr = 0;
  for (int i = 0; i < nseg; ++i) {
    const int k0 = S.k0[i], k1 = (i + 1 < nseg) ? S.k0[i + 1] : K;
    rd[nr++] = {part + k0, P.nblk, (size_t)M * P.K1, P.K1, M, k1 - k0, dW + S.wcol[i], lddw, 1,
                1.f};
  }
  if (db) rd[nr++] = {part + K, P.nblk, (size_t)M * P.K1, P.K1, M, 1, db, 1, 1, dbscale};
  return nr;
}

// Dynamic LDS above 64 KB needs the attribute once per instantiation.
template <typename Fn>
static bool wg_allow_lds(Fn fn) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
}

#define PF_WG_ALL(X) \
  X(1, 1) X(1, 2) X(1, 4) X(1, 8) X(2, 1) X(2, 2) X(2, 4) X(2, 8) X(4, 1) X(4, 2) X(4, 4) \
  X(4, 8) X(8, 1) X(8, 2) X(8, 4) X(8, 8) X(16, 1) X(16, 2) X(16, 4) X(16, 8) X(16, 16)

// Launches the per-block partials of dW (and db) into ws and describes the
// reduction that finishes them (rd[0..*nr)); the caller launches it now or
// batches it with others (pfsgnn_reduce_batch).
static int wgrad_launch(const float* dY, int M, const XSegs& S, int nseg, int K, int N, int act_in,
                        float* dW, int lddw, float* db, float dbscale, void* ws, size_t ws_bytes,
                        hipStream_t st, const char* where, RedDesc* rd, int* nr_out) {
  WgPlan P;
  if (int rc = wgrad_plan(dY, M, S, nseg, K, N, db != nullptr, where, P)) return rc;
  PF_REQUIRE(ws && ws_bytes >= P.part_bytes, where, "workspace too small");
  float* part = reinterpret_cast<float*>(ws);
  const dim3 grid(P.nblk), blk(64 * WG_WAVES);
  bool launched = false;
  const bool x3 = wg_x3_for(P.tm, P.per);
#define PF_WG(T, PP)                                                                           \
  if (P.tm == T && P.per == PP) {                                                              \
    auto fn = x3 ? &k_wgrad<T, PP, true> : &k_wgrad<T, PP, false>;                             \
    static bool attr[2] = {false, false};                                                      \
    if (!attr[x3]) {                                                                           \
      if (!wg_allow_lds(fn)) return pf::fail(where, "hipFuncSetAttribute");                    \
      attr[x3] = true;                                                                         \
    }                                                                                          \
    hipLaunchKernelGGL(fn, grid, blk, P.lds, st, dY, M, S, K, P.K1, N, act_in, P.chunk, P.vec, \
                       part);                                                                  \
    launched = true;                                                                           \
  }
  PF_WG_ALL(PF_WG)
#undef PF_WG
  if (!launched) return pf::fail(where, "no kernel for this shape");
  *nr_out = wgrad_reds(S, nseg, K, M, P, part, dW, lddw, db, dbscale, rd);
  return pf::check_launch(where);
}

static int wgrad_impl(const float* dY, int M, const XSegs& S, int nseg, int K, int N, int act_in,
                      float* dW, int lddw, float* db, float dbscale, void* ws, size_t ws_bytes,
                      hipStream_t st, const char* where) {
  RedDesc rd[PF_MAX_SEG + 1];
  int nr = 0;
  const int rc = wgrad_launch(dY, M, S, nseg, K, N, act_in, dW, lddw, db, dbscale, ws, ws_bytes,
                              st, where, rd, &nr);
  if (rc) return rc;
  launch_reduce_multi(rd, nr, st);
  return pf::check_launch(where);
}

extern "C" int pfsgnn_wgrad(const float* dY, int M, const float* X, int K, int N, int act_in,
                            float* dW, int lddw, float* db, float dbscale, void* ws,
                            size_t ws_bytes, void* stream) {
  PF_REQUIRE(dY && X && dW && M > 0 && K > 0 && N > 0, "pfsgnn_wgrad", "bad arguments");
  return wgrad_impl(dY, M, one_seg(X, 0), 1, K, N, act_in, dW, lddw, db, dbscale, ws, ws_bytes,
                    as_stream(stream), "pfsgnn_wgrad");
}

extern "C" int pfsgnn_wgrad_cat(const float* dY, int M, const pfsgnn_seg* segs, int nseg, int N,
                                int act_in, float* dW, int lddw, float* db, float dbscale,
                                void* ws, size_t ws_bytes, void* stream) {
  PF_REQUIRE(dY && dW && M > 0 && N > 0, "pfsgnn_wgrad_cat", "bad arguments");
  XSegs S;
  const int K = make_segs(segs, nseg, N, S);
  PF_REQUIRE(K > 0, "pfsgnn_wgrad_cat", "bad segment list");
  return wgrad_impl(dY, M, S, nseg, K, N, act_in, dW, lddw, db, dbscale, ws, ws_bytes,
                    as_stream(stream), "pfsgnn_wgrad_cat");
}

extern "C" size_t pfsgnn_wgrad_part_bytes(int M, int K, int N, int has_db) {
  if (M <= 0 || K <= 0 || N <= 0) return 0;
  return wgrad_part_bytes(M, K + (has_db ? 1 : 0), N);
}

extern "C" int pfsgnn_wgrad_cat_part(const float* dY, int M, const pfsgnn_seg* segs, int nseg,
                                     int N, int act_in, float* dW, int lddw, float* db,
                                     float dbscale, void* part, size_t part_bytes,
                                     pfsgnn_red* red_out, int* nred_out, void* stream) {
  PF_REQUIRE(dY && dW && M > 0 && N > 0 && red_out && nred_out, "pfsgnn_wgrad_cat_part",
             "bad arguments");
  XSegs S;
  const int K = make_segs(segs, nseg, N, S);
  PF_REQUIRE(K > 0, "pfsgnn_wgrad_cat_part", "bad segment list");
  RedDesc rd[PF_MAX_SEG + 1];
  int nr = 0;
  const int rc = wgrad_launch(dY, M, S, nseg, K, N, act_in, dW, lddw, db, dbscale, part,
                              part_bytes, as_stream(stream), "pfsgnn_wgrad_cat_part", rd, &nr);
  if (rc) return rc;
  for (int i = 0; i < nr; ++i)
    red_out[i] = {rd[i].part, rd[i].nb, rd[i].plen, rd[i].ldp, rd[i].rows, rd[i].cols, rd[i].out,
                  rd[i].ldo, rd[i].add, rd[i].scale};
  *nred_out = nr;
  return 0;
}

// ------------------------------------------------- batched weight gradients
// Many independent weight gradients (a backward pass's worth, deferred by the
// host) in a few launches: jobs with the same kernel shape share a launch (up
// to WG_MULTI per launch), then all their reductions go through the batched
// reduce.  Per job the partials and the reduction order are those of
// pfsgnn_wgrad_cat: results are bitwise identical.
static int wgrad_job_prep(const pfsgnn_wgrad_job& jb, XSegs& S, int& K, WgPlan& P,
                          const char* where) {
  PF_REQUIRE(jb.dY && jb.dW && jb.M > 0 && jb.N > 0, where, "bad job");
  K = make_segs(jb.segs, jb.nseg, jb.N, S);
  PF_REQUIRE(K > 0, where, "bad segment list");
  return wgrad_plan(jb.dY, jb.M, S, jb.nseg, K, jb.N, jb.db != nullptr, where, P);
}

extern "C" size_t pfsgnn_wgrad_multi_bytes(const pfsgnn_wgrad_job* jobs, int n) {
  size_t tot = 0;
  for (int i = 0; i < n; ++i) {
    XSegs S;
    int K;
    WgPlan P;
    if (wgrad_job_prep(jobs[i], S, K, P, "pfsgnn_wgrad_multi_bytes")) return 0;
    tot += align256(P.part_bytes);
  }
  return tot + 256;
}

static int reduce_batch_desc(const std::vector<RedDesc>& reds, hipStream_t st);

// the jobs' kernels; their reductions are appended to `reds`
static int wgrad_multi_launch(const pfsgnn_wgrad_job* jobs, int n, void* part, size_t part_bytes,
                              hipStream_t st, std::vector<RedDesc>& reds, const char* where) {
  std::vector<WgJob> J(n);
  std::vector<WgPlan> PL(n);
  size_t off = 0;
  char* base = static_cast<char*>(part);
  for (int i = 0; i < n; ++i) {
    int K;
    if (int rc = wgrad_job_prep(jobs[i], J[i].S, K, PL[i], where)) return rc;
    PF_REQUIRE(part && off + PL[i].part_bytes <= part_bytes, where, "partial arena too small");
    float* p = reinterpret_cast<float*>(base + off);
    off += align256(PL[i].part_bytes);
    const pfsgnn_wgrad_job& jb = jobs[i];
    J[i].dY = jb.dY;
    J[i].part = p;
    J[i].M = jb.M;
    J[i].K = K;
    J[i].K1 = PL[i].K1;
    J[i].N = jb.N;
    J[i].act_in = jb.act_in;
    J[i].chunk = PL[i].chunk;
    J[i].vec = PL[i].vec;
    RedDesc rd[PF_MAX_SEG + 1];
    const int nr = wgrad_reds(J[i].S, jb.nseg, K, jb.M, PL[i], p, jb.dW, jb.lddw, jb.db,
                              jb.dbscale, rd);
    reds.insert(reds.end(), rd, rd + nr);
  }
  // group by kernel shape, in job order; launch WG_MULTI at a time
  std::vector<bool> done(n, false);
  for (int i = 0; i < n; ++i) {
    if (done[i]) continue;
    std::vector<int> grp;
    for (int k = i; k < n; ++k)
      if (!done[k] && PL[k].tm == PL[i].tm && PL[k].per == PL[i].per) {
        grp.push_back(k);
        done[k] = true;
      }
    for (size_t g0 = 0; g0 < grp.size(); g0 += WG_MULTI) {
      WgTable T{};
      int blocks = 0;
      size_t lds = 0;
      const int m = (int)std::min<size_t>(WG_MULTI, grp.size() - g0);
      for (int u = 0; u < m; ++u) {
        T.j[u] = J[grp[g0 + u]];
        T.j[u].blk0 = blocks;
        blocks += PL[grp[g0 + u]].nblk;
        lds = std::max(lds, PL[grp[g0 + u]].lds);
      }
      T.njob = m;
      bool launched = false;
      const int tm = PL[i].tm, per = PL[i].per;
      const bool x3 = wg_x3_for(tm, per);
#define PF_WGM(TT, PP)                                                                    \
  if (tm == TT && per == PP) {                                                            \
    auto fn = x3 ? &k_wgrad_multi<TT, PP, true> : &k_wgrad_multi<TT, PP, false>;          \
    static bool attr[2] = {false, false};                                                 \
    if (!attr[x3]) {                                                                      \
      if (!wg_allow_lds(fn)) return pf::fail(where, "hipFuncSetAttribute");               \
      attr[x3] = true;                                                                    \
    }                                                                                     \
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(64 * WG_WAVES), lds, st, T);                \
    launched = true;                                                                      \
  }
      PF_WG_ALL(PF_WGM)
#undef PF_WGM
      if (!launched) return pf::fail(where, "no kernel for this shape");
    }
  }
  return 0;
}

extern "C" int pfsgnn_wgrad_multi(const pfsgnn_wgrad_job* jobs, int n, void* part,
                                  size_t part_bytes, void* stream) {
  const char* where = "pfsgnn_wgrad_multi";
  PF_REQUIRE(n >= 0 && (jobs || n == 0), where, "bad arguments");
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  std::vector<RedDesc> reds;
  if (int rc = wgrad_multi_launch(jobs, n, part, part_bytes, st, reds, where)) return rc;
  // the reductions, batched (a launch never holds two into the same cells)
  if (int rc = reduce_batch_desc(reds, st)) return rc;
  return pf::check_launch(where);
}

namespace pf {
bool node_x3(const char* knob) {
  const char* e = std::getenv(knob);
  if (e) return std::atoi(e) != 0;
  const int p = pfsgnn_get_edge_path();
  return p != PFSGNN_EDGE_MFMA_F32 && p != PFSGNN_EDGE_VALU && p != PFSGNN_EDGE_BF16Y;
}
}  // namespace pf

// ------------------------------------------------- deferred reductions
namespace pf {
namespace {
struct DeferCtx {
  char* base = nullptr;
  size_t cap = 0, off = 0, need = 0;
  bool on = false;
  std::vector<RedDesc> q;
};
DeferCtx g_defer;
}  // namespace

float* defer_take(size_t nfloats) {
  DeferCtx& D = g_defer;
  if (!D.on) return nullptr;
  const size_t b = align256(nfloats * sizeof(float));
  D.need += b;
  if (D.off + b > D.cap) return nullptr;
  float* r = reinterpret_cast<float*>(D.base + D.off);
  D.off += b;
  return r;
}

void defer_push(const RedDesc* d, int n) { g_defer.q.insert(g_defer.q.end(), d, d + n); }

// the in-launch hand-off counters (pfsgnn_common.h): a caller-owned, zeroed
// device buffer; every launch leaves its counters at zero again
namespace {
unsigned* g_sync = nullptr;
size_t g_sync_n = 0;
}  // namespace
unsigned* sync_counters(size_t n) { return (g_sync && n <= g_sync_n) ? g_sync : nullptr; }
unsigned* sync_slot(size_t n) {
  // contiguous runs of 128-counter slots, handed out round robin over the
  // buffer (slot 0 is sync_counters' own), so that launches in flight at once
  // never share a counter
  constexpr size_t SLOT = 128;
  static size_t next = 1;
  const size_t nslots = g_sync ? g_sync_n / SLOT : 0;
  const size_t need = (n + SLOT - 1) / SLOT;
  if (n == 0 || nslots < 2 || need > (nslots - 1) / 4) return nullptr;
  if (next + need > nslots) next = 1;
  unsigned* p = g_sync + next * SLOT;
  next += need;
  return p;
}
}  // namespace pf

extern "C" size_t pfsgnn_sync_bytes(void) { return (size_t)1 << 20; }

extern "C" int pfsgnn_set_sync_buffer(void* buf, size_t bytes) {
  PF_REQUIRE(!buf || bytes >= sizeof(unsigned), "pfsgnn_set_sync_buffer", "buffer too small");
  pf::g_sync = static_cast<unsigned*>(buf);
  pf::g_sync_n = buf ? bytes / sizeof(unsigned) : 0;
  return 0;
}

extern "C" int pfsgnn_defer_begin(void* arena, size_t bytes) {
  pf::DeferCtx& D = pf::g_defer;
  PF_REQUIRE(!D.on, "pfsgnn_defer_begin", "a deferred pass is already open");
  D.base = static_cast<char*>(arena);
  D.cap = arena ? bytes : 0;
  D.off = D.need = 0;
  D.q.clear();
  D.on = true;
  return 0;
}

extern "C" size_t pfsgnn_defer_need(void) { return pf::g_defer.need; }

extern "C" int pfsgnn_defer_end(void* stream) {
  pf::DeferCtx& D = pf::g_defer;
  PF_REQUIRE(D.on, "pfsgnn_defer_end", "no deferred pass is open");
  D.on = false;
  std::vector<RedDesc> reds;
  reds.swap(D.q);
  if (int rc = reduce_batch_desc(reds, as_stream(stream))) return rc;
  return pf::check_launch("pfsgnn_defer_end");
}

extern "C" int pfsgnn_defer_end_multi(const pfsgnn_wgrad_job* jobs, int n, void* part,
                                      size_t part_bytes, void* stream) {
  const char* where = "pfsgnn_defer_end_multi";
  pf::DeferCtx& D = pf::g_defer;
  PF_REQUIRE(D.on, where, "no deferred pass is open");
  PF_REQUIRE(n >= 0 && (jobs || n == 0), where, "bad arguments");
  D.on = false;
  std::vector<RedDesc> reds;
  reds.swap(D.q);
  hipStream_t st = as_stream(stream);
  // the jobs' kernels first (they read activations and gradients, never a
  // weight gradient), then the pass's deferred edge reductions and the jobs'
  // own in one batch
  if (n > 0)
    if (int rc = wgrad_multi_launch(jobs, n, part, part_bytes, st, reds, where)) return rc;
  if (int rc = reduce_batch_desc(reds, st)) return rc;
  return pf::check_launch(where);
}

// Output rectangles of two reductions intersect?  Exact when both write rows
// of the same row pitch without wrapping; conservative (true) otherwise.
static bool red_overlap(const RedDesc& a, const RedDesc& b) {
  const intptr_t ea = ((intptr_t)(a.rows - 1) * a.ldo + a.cols) * 4;
  const intptr_t eb = ((intptr_t)(b.rows - 1) * b.ldo + b.cols) * 4;
  const intptr_t pa = (intptr_t)a.out, pb = (intptr_t)b.out;
  if (pa + ea <= pb || pb + eb <= pa) return false;  // disjoint address ranges
  if (a.ldo != b.ldo || (pb - pa) % 4) return true;
  const intptr_t d = (pb - pa) / 4;  // b's origin relative to a's, in floats
  const intptr_t ld = a.ldo;
  intptr_t dr = d / ld, dc = d % ld;
  if (dc < 0) {
    dc += ld;
    dr -= 1;
  }
  if (a.cols > ld || dc + b.cols > ld) return true;
  const bool rows_meet = dr < a.rows && dr + b.rows > 0;
  const bool cols_meet = dc < a.cols && dc + b.cols > 0;
  return rows_meet && cols_meet;
}

static int reduce_batch_desc(const std::vector<RedDesc>& reds, hipStream_t st) {
  std::vector<RedDesc> group;
  for (const RedDesc& d : reds) {
    PF_REQUIRE(d.part && d.out && d.nb > 0 && d.rows > 0 && d.cols > 0, "pfsgnn_reduce_batch",
               "bad reduction");
    bool clash = (int)group.size() == PF_MAX_RED;
    for (const RedDesc& g : group) clash = clash || red_overlap(g, d);
    if (clash) {  // a launch never holds two reductions into the same cells
      if (int rc = launch_reduce_multi(group.data(), (int)group.size(), st))
        return pf::take_pending(rc);
      group.clear();
    }
    group.push_back(d);
  }
  if (!group.empty())
    if (int rc = launch_reduce_multi(group.data(), (int)group.size(), st)) return pf::take_pending(rc);
  return 0;
}

extern "C" int pfsgnn_reduce_batch(const pfsgnn_red* reds, int n, void* stream) {
  PF_REQUIRE(n >= 0 && (reds || n == 0), "pfsgnn_reduce_batch", "bad arguments");
  std::vector<RedDesc> v(n);
  for (int i = 0; i < n; ++i) {
    const pfsgnn_red& r = reds[i];
    v[i] = RedDesc{r.part, r.nb, r.plen, r.ldp, r.rows, r.cols, r.out, r.ldo, r.add, r.scale};
  }
  if (int rc = reduce_batch_desc(v, as_stream(stream))) return rc;
  return pf::check_launch("pfsgnn_reduce_batch");
}

// ---------------------------------------------------------------- batchnorm
// Per-channel Welford partials: grid (C, S); part[c][s] = (count, mean, M2).
__global__ __launch_bounds__(256) void k_bn_stats(const float* __restrict__ X, int N, int S,
                                                  float* __restrict__ part) {
  const int c = blockIdx.x, s = blockIdx.y;
  const int chunk = (N + S - 1) / S;
  const int n0 = s * chunk, n1 = min(N, n0 + chunk);
  float cnt = 0.f, mean = 0.f, m2 = 0.f;
  for (int n = n0 + threadIdx.x; n < n1; n += 256) {
    const float x = X[(size_t)c * N + n];
    cnt += 1.f;
    const float d = x - mean;
    mean += d / cnt;
    m2 += d * (x - mean);
  }
  // merge across the block (Chan), tree over lanes then waves
  for (int o = 32; o > 0; o >>= 1) {
    const float cb = __shfl_xor(cnt, o), mb = __shfl_xor(mean, o), qb = __shfl_xor(m2, o);
    const float tot = cnt + cb;
    if (tot > 0.f) {
      const float d = mb - mean;
      mean = mean + d * (cb / tot);
      m2 = m2 + qb + d * d * (cnt * cb / tot);
    }
    cnt = tot;
  }
  __shared__ float sh[4][3];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { sh[wave][0] = cnt; sh[wave][1] = mean; sh[wave][2] = m2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float C0 = sh[0][0], M0 = sh[0][1], Q0 = sh[0][2];
    for (int w = 1; w < 4; ++w) {
      const float cb = sh[w][0], mb = sh[w][1], qb = sh[w][2];
      const float tot = C0 + cb;
      if (tot > 0.f) {
        const float d = mb - M0;
        M0 = M0 + d * (cb / tot);
        Q0 = Q0 + qb + d * d * (C0 * cb / tot);
      }
      C0 = tot;
    }
    float* p = part + ((size_t)c * S + s) * 3;
    p[0] = C0; p[1] = M0; p[2] = Q0;
  }
}

// merge S partials per channel (double), write mu/var, update running stats
__global__ void k_bn_finalize(const float* __restrict__ part, int C, int S, long long N,
                              float* __restrict__ mu, float* __restrict__ var,
                              float* __restrict__ rm, float* __restrict__ rv, float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double cnt = 0, mean = 0, m2 = 0;
  for (int s = 0; s < S; ++s) {
    const float* p = part + ((size_t)c * S + s) * 3;
    const double cb = p[0], mb = p[1], qb = p[2];
    const double tot = cnt + cb;
    if (tot > 0) {
      const double d = mb - mean;
      mean += d * (cb / tot);
      m2 += qb + d * d * (cnt * cb / tot);
    }
    cnt = tot;
  }
  const double v = m2 / (double)N;
  mu[c] = (float)mean;
  var[c] = (float)v;
  if (rm) {
    const double unb = N > 1 ? m2 / (double)(N - 1) : v;
    rm[c] = (float)((1.0 - momentum) * rm[c] + momentum * mean);
    rv[c] = (float)((1.0 - momentum) * rv[c] + momentum * unb);
  }
}

__global__ void k_bn_apply(const float* __restrict__ X, int C, int N, const float* __restrict__ mu,
                           const float* __restrict__ var, const float* __restrict__ gamma,
                           const float* __restrict__ beta, float eps, float* __restrict__ Y) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)C * N) return;
  const int c = (int)(idx / N);
  const float inv = 1.0f / sqrtf(var[c] + eps);
  Y[idx] = (X[idx] - mu[c]) * inv * gamma[c] + beta[c];
}

static int bn_splits(int N) { return std::max(1, std::min(64, (N + 4095) / 4096)); }

extern "C" int pfsgnn_bn_fwd(const float* X, int C, int N, const float* gamma, const float* beta,
                             float* rm, float* rv, float momentum, float eps, float* Y, float* mu,
                             float* var, void* ws, size_t ws_bytes, void* stream) {
  PF_REQUIRE(X && Y && mu && var && gamma && beta && C > 0 && N > 1, "pfsgnn_bn_fwd",
             "bad arguments (BatchNorm needs more than one value per channel)");
  hipStream_t st = as_stream(stream);
  const int S = bn_splits(N);
  const size_t need = (size_t)C * S * 3 * sizeof(float);
  PF_REQUIRE(ws && ws_bytes >= need, "pfsgnn_bn_fwd", "workspace too small");
  float* pool = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_bn_stats, dim3(C, S), dim3(256), 0, st, X, N, S, pool);
  hipLaunchKernelGGL(k_bn_finalize, dim3(1), dim3(64), 0, st, pool, C, S, (long long)N, mu, var,
                     rm, rv, momentum);
  const size_t tot = (size_t)C * N;
  hipLaunchKernelGGL(k_bn_apply, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, X, C, N,
                     mu, var, gamma, beta, eps, Y);
  return pf::check_launch("pfsgnn_bn_fwd");
}

// backward sums per channel: Sg = sum dY, Sgx = sum dY*xhat -- grid (C, S)
// partials over node chunks; the apply kernel finishes them in fixed order
__global__ __launch_bounds__(256) void k_bn_bwd_sums(const float* __restrict__ dY,
                                                     const float* __restrict__ X, int N, int S,
                                                     const float* __restrict__ mu,
                                                     const float* __restrict__ var, float eps,
                                                     float* __restrict__ part) {
  const int c = blockIdx.x, s = blockIdx.y;
  const int chunk = (N + S - 1) / S;
  const int n0 = s * chunk, n1 = min(N, n0 + chunk);
  const float m = mu[c], inv = 1.0f / sqrtf(var[c] + eps);
  float v[2] = {0.f, 0.f};
  for (int n = n0 + threadIdx.x; n < n1; n += 256) {
    const float g = dY[(size_t)c * N + n];
    v[0] += g;
    v[1] += g * (X[(size_t)c * N + n] - m) * inv;
  }
  __shared__ float scratch[8];
  block_sum<2>(v, scratch);
  if (threadIdx.x == 0) {
    part[((size_t)c * S + s) * 2] = v[0];
    part[((size_t)c * S + s) * 2 + 1] = v[1];
  }
}

// grid (C, ceil(N/1024)): every block re-derives its channel's two sums from
// the S partials (fixed order), block (c, 0) also accumulates dgamma/dbeta
__global__ __launch_bounds__(256) void k_bn_bwd_apply(const float* __restrict__ dY,
                                                      const float* __restrict__ X, int N, int S,
                                                      const float* __restrict__ mu,
                                                      const float* __restrict__ var,
                                                      const float* __restrict__ gamma, float eps,
                                                      const float* __restrict__ part,
                                                      float* __restrict__ dX,
                                                      float* __restrict__ dgamma,
                                                      float* __restrict__ dbeta) {
  const int c = blockIdx.x;
  __shared__ float sums[2];
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int s = 0; s < S; ++s) {
      a += part[((size_t)c * S + s) * 2];
      b += part[((size_t)c * S + s) * 2 + 1];
    }
    sums[0] = a;
    sums[1] = b;
    if (blockIdx.y == 0) {
      dgamma[c] += b;
      dbeta[c] += a;
    }
  }
  __syncthreads();
  const float inv = 1.0f / sqrtf(var[c] + eps), m = mu[c];
  const float k0 = sums[0] / N, k1 = sums[1] / N, gi = gamma[c] * inv;
  const int base = blockIdx.y * 1024;
  for (int i = threadIdx.x; i < 1024; i += 256) {
    const int n = base + i;
    if (n < N) {
      const size_t idx = (size_t)c * N + n;
      const float xh = (X[idx] - m) * inv;
      dX[idx] = gi * (dY[idx] - k0 - xh * k1);
    }
  }
}

extern "C" int pfsgnn_bn_bwd(const float* dY, const float* X, const float* mu, const float* var,
                             const float* gamma, float eps, int C, int N, float* dX, float* dgamma,
                             float* dbeta, void* ws, size_t ws_bytes, void* stream) {
  PF_REQUIRE(dY && X && dX && C > 0 && N > 0, "pfsgnn_bn_bwd", "bad arguments");
  const int S = bn_splits(N);
  PF_REQUIRE(ws && ws_bytes >= (size_t)2 * C * S * sizeof(float), "pfsgnn_bn_bwd",
             "workspace too small");
  hipStream_t st = as_stream(stream);
  float* part = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_bn_bwd_sums, dim3(C, S), dim3(256), 0, st, dY, X, N, S, mu, var, eps, part);
  hipLaunchKernelGGL(k_bn_bwd_apply, dim3(C, (N + 1023) / 1024), dim3(256), 0, st, dY, X, N, S, mu,
                     var, gamma, eps, part, dX, dgamma, dbeta);
  return pf::check_launch("pfsgnn_bn_bwd");
}

// ---------------------------------------------------------------- graph ops
__global__ void k_graph_reduce(const float* __restrict__ X, int C, int G, int n, int mean,
                               float* __restrict__ out, int add) {
  const int cg = blockIdx.x;  // c*G + g
  const int c = cg / G, g = cg - c * G;
  float v[1] = {0.f};
  const float* p = X + (size_t)c * G * n + (size_t)g * n;
  for (int i = threadIdx.x; i < n; i += 256) v[0] += p[i];
  __shared__ float scratch[4];
  block_sum<1>(v, scratch);
  if (threadIdx.x == 0) {
    const float r = mean ? v[0] / (float)n : v[0];
    float* o = out + (size_t)c * G + g;
    *o = add ? *o + r : r;
  }
}

extern "C" int pfsgnn_graph_reduce(const float* X, int C, int G, int n, int mean, float* out,
                                   void* stream) {
  PF_REQUIRE(X && out && C > 0 && G > 0 && n > 0, "pfsgnn_graph_reduce", "bad arguments");
  hipLaunchKernelGGL(k_graph_reduce, dim3(C * G), dim3(256), 0, as_stream(stream), X, C, G, n,
                     mean, out, 0);
  return pf::check_launch("pfsgnn_graph_reduce");
}

extern "C" int pfsgnn_graph_reduce_add(const float* X, int C, int G, int n, int mean, float* out,
                                       void* stream) {
  PF_REQUIRE(X && out && C > 0 && G > 0 && n > 0, "pfsgnn_graph_reduce_add", "bad arguments");
  hipLaunchKernelGGL(k_graph_reduce, dim3(C * G), dim3(256), 0, as_stream(stream), X, C, G, n,
                     mean, out, 1);
  return pf::check_launch("pfsgnn_graph_reduce_add");
}

// Several per-graph sums into one accumulator in one launch (the u[batch]
// gradients of a block's SModel, TModel and EdgeModel, gnn.py:100/153/191):
// out[c][g] += sum_j sum_i X_j[c][g*n_j + i], j in order, one block per (c, g).
#define GR_MAX 4
struct GrPack {
  const float* x[GR_MAX];
  int n[GR_MAX];
};
__global__ void k_graph_reduce_multi(GrPack pk, int m, int C, int G, float* __restrict__ out) {
  const int cg = blockIdx.x;  // c*G + g
  const int c = cg / G, g = cg - c * G;
  float v[1] = {0.f};
  for (int j = 0; j < m; ++j) {
    const int n = pk.n[j];
    const float* p = pk.x[j] + (size_t)c * G * n + (size_t)g * n;
    for (int i = threadIdx.x; i < n; i += 256) v[0] += p[i];
  }
  __shared__ float scratch[4];
  block_sum<1>(v, scratch);
  if (threadIdx.x == 0) out[(size_t)c * G + g] += v[0];
}

extern "C" int pfsgnn_graph_reduce_multi(const float* const* X, const int* n, int m, int C, int G,
                                         float* out, void* stream) {
  PF_REQUIRE(X && n && out && m >= 1 && m <= GR_MAX && C > 0 && G > 0,
             "pfsgnn_graph_reduce_multi", "bad arguments (1..4 inputs)");
  GrPack pk{};
  for (int j = 0; j < m; ++j) {
    PF_REQUIRE(X[j] && n[j] > 0, "pfsgnn_graph_reduce_multi", "bad input");
    pk.x[j] = X[j];
    pk.n[j] = n[j];
  }
  hipLaunchKernelGGL(k_graph_reduce_multi, dim3(C * G), dim3(256), 0, as_stream(stream), pk, m, C,
                     G, out);
  return pf::check_launch("pfsgnn_graph_reduce_multi");
}

// Two per-graph means in one launch (GlobalModel's x_s.mean / x_t.mean,
// gnn.py:218-219): out rows [0, C) from X1 (n1 nodes per graph), [C, 2C) from X2.
__global__ void k_graph_mean2(const float* __restrict__ X1, int n1, const float* __restrict__ X2,
                              int n2, int C, int G, float* __restrict__ out) {
  const int cg = blockIdx.x, which = blockIdx.y;
  const int c = cg / G, g = cg - c * G;
  const int n = which ? n2 : n1;
  const float* p = (which ? X2 : X1) + (size_t)c * G * n + (size_t)g * n;
  float v[1] = {0.f};
  for (int i = threadIdx.x; i < n; i += 256) v[0] += p[i];
  __shared__ float scratch[4];
  block_sum<1>(v, scratch);
  if (threadIdx.x == 0) out[(size_t)(which * C + c) * G + g] = v[0] / (float)n;
}

extern "C" int pfsgnn_graph_mean2(const float* X1, int n1, const float* X2, int n2, int C, int G,
                                  float* out, void* stream) {
  PF_REQUIRE(X1 && X2 && out && C > 0 && G > 0 && n1 > 0 && n2 > 0, "pfsgnn_graph_mean2",
             "bad arguments");
  hipLaunchKernelGGL(k_graph_mean2, dim3(C * G, 2), dim3(256), 0, as_stream(stream), X1, n1, X2,
                     n2, C, G, out);
  return pf::check_launch("pfsgnn_graph_mean2");
}

// Its backward in one launch: out1[c][g*n1 + i] += s1 src[c][g], out2 likewise
// with src rows [C, 2C).
__global__ void k_graph_bcast_add2(float* __restrict__ out1, int n1, float s1,
                                   float* __restrict__ out2, int n2, float s2, int C, int G,
                                   const float* __restrict__ src) {
  const size_t t1 = (size_t)C * G * n1, t2 = (size_t)C * G * n2;
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < t1) {
    const size_t c = idx / ((size_t)G * n1), g = (idx - c * G * n1) / n1;
    out1[idx] += s1 * src[c * G + g];
  } else if ((idx -= t1) < t2) {
    const size_t c = idx / ((size_t)G * n2), g = (idx - c * G * n2) / n2;
    out2[idx] += s2 * src[(C + c) * G + g];
  }
}

extern "C" int pfsgnn_graph_bcast_add2(float* out1, int n1, float s1, float* out2, int n2,
                                       float s2, int C, int G, const float* src, void* stream) {
  PF_REQUIRE(out1 && out2 && src && C > 0 && G > 0 && n1 > 0 && n2 > 0,
             "pfsgnn_graph_bcast_add2", "bad arguments");
  const size_t tot = (size_t)C * G * ((size_t)n1 + n2);
  hipLaunchKernelGGL(k_graph_bcast_add2, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), out1, n1, s1, out2, n2, s2, C, G, src);
  return pf::check_launch("pfsgnn_graph_bcast_add2");
}

__global__ void k_graph_bcast_add(float* __restrict__ out, int C, int G, int n,
                                  const float* __restrict__ src, float scale) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t tot = (size_t)C * G * n;
  if (idx >= tot) return;
  const size_t c = idx / ((size_t)G * n);
  const size_t g = (idx - c * G * n) / n;
  out[idx] += scale * src[c * G + g];
}

extern "C" int pfsgnn_graph_bcast_add(float* out, int C, int G, int n, const float* src,
                                      float scale, void* stream) {
  PF_REQUIRE(out && src && C > 0 && G > 0 && n > 0, "pfsgnn_graph_bcast_add", "bad arguments");
  const size_t tot = (size_t)C * G * n;
  hipLaunchKernelGGL(k_graph_bcast_add, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), out, C, G, n, src, scale);
  return pf::check_launch("pfsgnn_graph_bcast_add");
}

// ---------------------------------------------------------------- RMSNorm x2
// y = x * rsqrt(mean_c x^2 + eps) * w, applied twice (thread per graph row).
__global__ void k_rms2_fwd(const float* __restrict__ X, int C, int G, const float* __restrict__ w,
                           float eps, float* __restrict__ Y, float* __restrict__ y1,
                           float* __restrict__ r1, float* __restrict__ r2) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  float s = 0.f;
  for (int c = 0; c < C; ++c) { const float x = X[(size_t)c * G + g]; s += x * x; }
  const float a = rsqrtf(s / C + eps);
  float s2 = 0.f;
  for (int c = 0; c < C; ++c) {
    const float v = X[(size_t)c * G + g] * a * w[c];
    y1[(size_t)c * G + g] = v;
    s2 += v * v;
  }
  const float b = rsqrtf(s2 / C + eps);
  for (int c = 0; c < C; ++c) Y[(size_t)c * G + g] = y1[(size_t)c * G + g] * b * w[c];
  r1[g] = a;
  r2[g] = b;
}

extern "C" int pfsgnn_rms2_fwd(const float* X, int C, int G, const float* w, float eps, float* Y,
                               float* y1, float* r1, float* r2, void* stream) {
  PF_REQUIRE(X && w && Y && y1 && r1 && r2 && C > 0 && G > 0, "pfsgnn_rms2_fwd", "bad arguments");
  hipLaunchKernelGGL(k_rms2_fwd, dim3((G + 63) / 64), dim3(64), 0, as_stream(stream), X, C, G, w,
                     eps, Y, y1, r1, r2);
  return pf::check_launch("pfsgnn_rms2_fwd");
}

// backward: one block, thread per graph row computes dX; dw reduced over rows
__global__ void k_rms2_bwd(const float* __restrict__ dY, const float* __restrict__ X,
                           const float* __restrict__ w, const float* __restrict__ y1,
                           const float* __restrict__ r1, const float* __restrict__ r2, int C,
                           int G, float* __restrict__ dX, float* __restrict__ dwpart) {
  // dwpart [G][C] per-row contributions, summed by the host-side reduce
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const float a = r1[g], b = r2[g];
  // second application: y = y1 * b * w
  float dot = 0.f;
  for (int c = 0; c < C; ++c) {
    const float dy = dY[(size_t)c * G + g];
    const float x = y1[(size_t)c * G + g];
    dwpart[(size_t)g * C + c] = dy * x * b;
    dot += dy * w[c] * x;
  }
  // d1 = b*dxn - x*b^3*dot/C, dxn = dy*w ; then first application on X
  float dot2 = 0.f;
  for (int c = 0; c < C; ++c) {
    const float dy = dY[(size_t)c * G + g];
    const float x1 = y1[(size_t)c * G + g];
    const float d1 = b * dy * w[c] - x1 * b * b * b * dot / C;
    dX[(size_t)c * G + g] = d1;  // temp
    const float x0 = X[(size_t)c * G + g];
    dwpart[(size_t)g * C + c] += d1 * x0 * a;
    dot2 += d1 * w[c] * x0;
  }
  for (int c = 0; c < C; ++c) {
    const float d1 = dX[(size_t)c * G + g];
    const float x0 = X[(size_t)c * G + g];
    dX[(size_t)c * G + g] = a * d1 * w[c] - x0 * a * a * a * dot2 / C;
  }
}

extern "C" int pfsgnn_rms2_bwd(const float* dY, const float* X, const float* w, const float* y1,
                               const float* r1, const float* r2, int C, int G, float eps,
                               float* dX, float* dw, void* ws, size_t ws_bytes, void* stream) {
  (void)eps;
  PF_REQUIRE(dY && X && w && dX && dw && C > 0 && G > 0, "pfsgnn_rms2_bwd", "bad arguments");
  hipStream_t st = as_stream(stream);
  const size_t need = (size_t)G * C * sizeof(float);
  PF_REQUIRE(ws && ws_bytes >= need, "pfsgnn_rms2_bwd", "workspace too small");
  float* part = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_rms2_bwd, dim3((G + 63) / 64), dim3(64), 0, st, dY, X, w, y1, r1, r2, C, G,
                     dX, part);
  launch_reduce_rows(part, G, (size_t)C, C, 1, C, dw, C, 1, 1.f, st);
  return pf::check_launch("pfsgnn_rms2_bwd");
}

// ---------------------------------------------------------------- GlobalModel, fused
// GlobalModel (gnn.py:208-223): the node means (gnn.py:218-219) by the wide
// k_graph_mean2, then one block per graph does the MLP(3F -> H -> F) on
// [u, mean x_s, mean x_t] and the double RMSNorm (the arithmetic of k_rms2_fwd,
// serial over the F features): two launches for what was mean2 + mlp + rms2.
constexpr int GL_MAXK = 192;  // 3F and H <= 192 (F <= 64)
__global__ __launch_bounds__(256) void k_global_fwd(
    const float* __restrict__ xs, int n1, const float* __restrict__ xt, int n2,
    const float* __restrict__ u, int F, int G, const float* __restrict__ W1, int H,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    const float* __restrict__ w, float eps, float* __restrict__ means, float* __restrict__ Z,
    float* __restrict__ V, float* __restrict__ Y, float* __restrict__ y1,
    float* __restrict__ r1, float* __restrict__ r2) {
  __shared__ float h[GL_MAXK], z[GL_MAXK], v[GL_MAXK];
  const int g = blockIdx.x, t = threadIdx.x;
  const int K = 3 * F;
  (void)xs; (void)xt; (void)n1; (void)n2;
  if (t < F) h[t] = u[(size_t)t * G + g];
  else if (t < K) h[t] = means[(size_t)(t - F) * G + g];
  __syncthreads();
  for (int j = t; j < H; j += 256) {
    float acc = b1[j];
    for (int k = 0; k < K; ++k) acc = fmaf(W1[(size_t)j * K + k], h[k], acc);
    z[j] = acc;
    Z[(size_t)j * G + g] = acc;
  }
  __syncthreads();
  for (int o = t; o < F; o += 256) {
    float acc = b2[o];
    for (int j = 0; j < H; ++j) acc = fmaf(W2[(size_t)o * H + j], lrelu(z[j]), acc);
    v[o] = acc;
    V[(size_t)o * G + g] = acc;
  }
  __syncthreads();
  if (!w) {  // unnormed GNN: u_new = v
    if (t < F) Y[(size_t)t * G + g] = v[t];
    return;
  }
  if (t == 0) {
    float s = 0.f;
    for (int c = 0; c < F; ++c) s += v[c] * v[c];
    const float a = rsqrtf(s / F + eps);
    float s2 = 0.f;
    for (int c = 0; c < F; ++c) {
      const float q = v[c] * a * w[c];
      h[c] = q;
      y1[(size_t)c * G + g] = q;
      s2 += q * q;
    }
    const float b = rsqrtf(s2 / F + eps);
    for (int c = 0; c < F; ++c) Y[(size_t)c * G + g] = h[c] * b * w[c];
    r1[g] = a;
    r2[g] = b;
  }
}

// Its backward, one block per graph: the double RMSNorm backward (k_rms2_bwd's
// arithmetic; dw per graph into dwp [F][G], summed by the caller), then
// dZ = (W2^T gV) lrelu'(Z), dh = W1^T dZ, gU += dh[0:F], gm = dh[F:3F]; the
// wide k_graph_bcast_add2 then broadcasts gm over the graphs' nodes (gnn.py:
// 218-219).  Two launches for rms2_bwd + reduce + mlp_bwd + graph_bcast_add2.
__global__ __launch_bounds__(256) void k_global_bwd(
    const float* __restrict__ dY, const float* __restrict__ V, const float* __restrict__ w,
    const float* __restrict__ y1, const float* __restrict__ r1, const float* __restrict__ r2,
    int F, int G, const float* __restrict__ Z, int H, const float* __restrict__ W1,
    const float* __restrict__ W2, float* __restrict__ gV, float* __restrict__ dZ,
    float* __restrict__ dwp, float* __restrict__ gU, float* __restrict__ gm) {
  __shared__ float gv[GL_MAXK], dz[GL_MAXK], dh[GL_MAXK], d1[GL_MAXK];
  __shared__ float sdy[GL_MAXK], sy1[GL_MAXK], sv[GL_MAXK], sw[GL_MAXK], sdw[GL_MAXK];
  const int g = blockIdx.x, t = threadIdx.x;
  const int K = 3 * F;
  // the graph's vectors staged in parallel; the serial RMSNorm math reads LDS
  if (t < F) {
    sdy[t] = dY[(size_t)t * G + g];
    if (w) {
      sy1[t] = y1[(size_t)t * G + g];
      sv[t] = V[(size_t)t * G + g];
      sw[t] = w[t];
    }
  }
  __syncthreads();
  if (!w) {
    if (t < F) gv[t] = sdy[t];
  } else if (t == 0) {
    const float a = r1[g], b = r2[g];
    float dot = 0.f;
    for (int c = 0; c < F; ++c) {
      const float dy = sdy[c], x = sy1[c];
      sdw[c] = dy * x * b;
      dot += dy * sw[c] * x;
    }
    float dot2 = 0.f;
    for (int c = 0; c < F; ++c) {
      const float dy = sdy[c], x1 = sy1[c];
      const float q = b * dy * sw[c] - x1 * b * b * b * dot / F;
      d1[c] = q;
      const float x0 = sv[c];
      sdw[c] += q * x0 * a;
      dot2 += q * sw[c] * x0;
    }
    for (int c = 0; c < F; ++c) {
      const float x0 = sv[c];
      gv[c] = a * d1[c] * sw[c] - x0 * a * a * a * dot2 / F;
    }
  }
  __syncthreads();
  if (w && t < F) dwp[(size_t)t * G + g] = sdw[t];
  if (t < F) gV[(size_t)t * G + g] = gv[t];
  for (int j = t; j < H; j += 256) {
    float acc = 0.f;
    for (int o = 0; o < F; ++o) acc = fmaf(W2[(size_t)o * H + j], gv[o], acc);
    const float q = acc * dlrelu(Z[(size_t)j * G + g]);
    dz[j] = q;
    dZ[(size_t)j * G + g] = q;
  }
  __syncthreads();
  for (int k = t; k < K; k += 256) {
    float acc = 0.f;
    for (int j = 0; j < H; ++j) acc = fmaf(W1[(size_t)j * K + k], dz[j], acc);
    dh[k] = acc;
  }
  __syncthreads();
  if (t < F) gU[(size_t)t * G + g] += dh[t];
  else if (t < K) gm[(size_t)(t - F) * G + g] = dh[t];
}

extern "C" int pfsgnn_global_fwd(const float* xs, int n1, const float* xt, int n2, const float* u,
                                 int F, int G, const float* W1, int H, const float* b1,
                                 const float* W2, const float* b2, const float* w, float eps,
                                 float* means, float* Z, float* V, float* Y, float* y1, float* r1,
                                 float* r2, void* stream) {
  PF_REQUIRE(xs && xt && u && W1 && b1 && W2 && b2 && means && Z && V && Y && F > 0 && G > 0 &&
                 n1 > 0 && n2 > 0 && H > 0 && 3 * F <= GL_MAXK && H <= GL_MAXK,
             "pfsgnn_global_fwd", "bad arguments (3F, H <= 192)");
  PF_REQUIRE(!w || (y1 && r1 && r2), "pfsgnn_global_fwd", "RMSNorm needs y1, r1, r2");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_graph_mean2, dim3(F * G, 2), dim3(256), 0, st, xs, n1, xt, n2, F, G, means);
  hipLaunchKernelGGL(k_global_fwd, dim3(G), dim3(256), 0, st, xs, n1, xt, n2, u, F, G, W1, H, b1,
                     W2, b2, w, eps, means, Z, V, Y, y1, r1, r2);
  return pf::check_launch("pfsgnn_global_fwd");
}

extern "C" int pfsgnn_global_bwd(const float* dY, const float* V, const float* w, const float* y1,
                                 const float* r1, const float* r2, int F, int G, const float* Z,
                                 int H, const float* W1, const float* W2, float* gV, float* dZ,
                                 float* dwp, float* gU, float* gm, float* gxs, int n1, float s1,
                                 float* gxt, int n2, float s2, void* stream) {
  PF_REQUIRE(dY && V && Z && W1 && W2 && gV && dZ && gU && gm && gxs && gxt && F > 0 && G > 0 &&
                 n1 > 0 && n2 > 0 && H > 0 && 3 * F <= GL_MAXK && H <= GL_MAXK,
             "pfsgnn_global_bwd", "bad arguments (3F, H <= 192)");
  PF_REQUIRE(!w || (y1 && r1 && r2 && dwp), "pfsgnn_global_bwd", "RMSNorm needs y1, r1, r2, dwp");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_global_bwd, dim3(G), dim3(256), 0, st, dY, V, w, y1, r1, r2, F, G, Z, H, W1,
                     W2, gV, dZ, dwp, gU, gm);
  const size_t tot = (size_t)F * G * ((size_t)n1 + n2);
  hipLaunchKernelGGL(k_graph_bcast_add2, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                     gxs, n1, s1, gxt, n2, s2, F, G, gm);
  return pf::check_launch("pfsgnn_global_bwd");
}

// ---------------------------------------------------------------- BN x2 (edges)
__global__ void k_bn2_finalize(const float* __restrict__ mu1, const float* __restrict__ var1,
                               const float* __restrict__ gamma, const float* __restrict__ beta,
                               float* __restrict__ rm, float* __restrict__ rv, int C, long long n,
                               float momentum, float eps, float* __restrict__ sc,
                               float* __restrict__ sh, float* __restrict__ inv1o,
                               float* __restrict__ inv2o) {
  const int c = threadIdx.x;
  if (c >= C) return;
  bn2_coef(gamma, beta, rm, rv, c, n, momentum, eps, mu1[c], var1[c], sc, sh, inv1o, inv2o);
}

extern "C" int pfsgnn_bn2_finalize(const float* mu1, const float* var1, const float* gamma,
                                   const float* beta, float* rm, float* rv, int C, long long n,
                                   float momentum, float eps, float* sc, float* sh, float* inv1,
                                   float* inv2, void* stream) {
  PF_REQUIRE(mu1 && var1 && gamma && beta && sc && sh && inv1 && inv2 && C > 0 && C <= 64,
             "pfsgnn_bn2_finalize", "bad arguments");
  hipLaunchKernelGGL(k_bn2_finalize, dim3(1), dim3(64), 0, as_stream(stream), mu1, var1, gamma,
                     beta, rm, rv, C, n, momentum, eps, sc, sh, inv1, inv2);
  return pf::check_launch("pfsgnn_bn2_finalize");
}

// eval-mode BatchNorm1d (running statistics, nothing updated), applied
// `times` times (2 for EdgeModel, gnn.py:101; 1 for S/T, gnn.py:154/192):
// each application is y -> a*y + b with a = gamma/sqrt(rv+eps), b = beta - rm*a
__global__ void k_bn_eval_coef(const float* __restrict__ gamma, const float* __restrict__ beta,
                               const float* __restrict__ rm, const float* __restrict__ rv, int C,
                               float eps, int times, float* __restrict__ sc,
                               float* __restrict__ sh) {
  const int c = threadIdx.x;
  if (c >= C) return;
  const float a = gamma[c] / sqrtf(rv[c] + eps), b = beta[c] - rm[c] * a;
  float s = 1.f, t = 0.f;
  for (int i = 0; i < times; ++i) {
    t = a * t + b;
    s = a * s;
  }
  sc[c] = s;
  sh[c] = t;
}

// Backward of eval-mode BatchNorm1d applied `times` times (pfsgnn_bn_eval_coef's
// affine): y1 = a (y - rm) + beta, a = gamma / sqrt(rv + eps), [y2 = a (y1 - rm)
// + beta].  d out / d y = a^times; with Sg = sum g, Sgx = sum g (y - rm) inv:
//   times 1: dgamma += Sgx,                         dbeta += Sg
//   times 2: dgamma += 2 a Sgx + inv (beta - rm) Sg, dbeta += (a + 1) Sg
// (d y2 / d gamma = inv (y1 - rm) + a inv (y - rm), d y2 / d beta = a + 1).
__global__ void k_bn_eval_bwd_coef(const float* __restrict__ gamma, const float* __restrict__ beta,
                                   const float* __restrict__ rm, const float* __restrict__ rv,
                                   int C, float eps, int times, const float* __restrict__ Sg,
                                   const float* __restrict__ Sgx, float* __restrict__ inv,
                                   float* __restrict__ scale, float* __restrict__ dgamma,
                                   float* __restrict__ dbeta) {
  const int c = threadIdx.x;
  if (c >= C) return;
  const float sd = sqrtf(rv[c] + eps);
  const float iv = 1.f / sd, a = gamma[c] / sd;
  if (inv) inv[c] = iv;
  if (scale) scale[c] = times == 2 ? a * a : a;
  if (!Sg) return;
  if (times == 2) {
    dgamma[c] += 2.f * a * Sgx[c] + iv * (beta[c] - rm[c]) * Sg[c];
    dbeta[c] += (a + 1.f) * Sg[c];
  } else {
    dgamma[c] += Sgx[c];
    dbeta[c] += Sg[c];
  }
}

extern "C" int pfsgnn_bn_eval_bwd_coef(const float* gamma, const float* beta, const float* rm,
                                       const float* rv, int C, float eps, int times,
                                       const float* Sg, const float* Sgx, float* inv,
                                       float* scale, float* dgamma, float* dbeta, void* stream) {
  PF_REQUIRE(gamma && beta && rm && rv && C > 0 && C <= 64 && times >= 1 && times <= 2 &&
                 (!Sg || (Sgx && dgamma && dbeta)),
             "pfsgnn_bn_eval_bwd_coef", "bad arguments");
  hipLaunchKernelGGL(k_bn_eval_bwd_coef, dim3(1), dim3(64), 0, as_stream(stream), gamma, beta, rm,
                     rv, C, eps, times, Sg, Sgx, inv, scale, dgamma, dbeta);
  return pf::check_launch("pfsgnn_bn_eval_bwd_coef");
}

extern "C" int pfsgnn_bn_eval_coef(const float* gamma, const float* beta, const float* rm,
                                   const float* rv, int C, float eps, int times, float* sc,
                                   float* sh, void* stream) {
  PF_REQUIRE(gamma && beta && rm && rv && sc && sh && C > 0 && C <= 64 && times >= 1 &&
                 times <= 2,
             "pfsgnn_bn_eval_coef", "bad arguments");
  hipLaunchKernelGGL(k_bn_eval_coef, dim3(1), dim3(64), 0, as_stream(stream), gamma, beta, rm,
                     rv, C, eps, times, sc, sh);
  return pf::check_launch("pfsgnn_bn_eval_coef");
}

// Y[c][n] = sc[c]*X[c][n] + sh[c]; grid-stride over the flat [C][N] array
__global__ __launch_bounds__(256) void k_affine_rows(const float* __restrict__ X, int C, int N,
                                                     const float* __restrict__ sc,
                                                     const float* __restrict__ sh,
                                                     float* __restrict__ Y) {
  const size_t tot = (size_t)C * N;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < tot; i += (size_t)gridDim.x * 256) {
    const int c = (int)(i / (size_t)N);
    Y[i] = fmaf(sc[c], X[i], sh[c]);
  }
}

extern "C" int pfsgnn_affine_rows(const float* X, int C, int N, const float* sc, const float* sh,
                                  float* Y, void* stream) {
  PF_REQUIRE(X && Y && sc && sh && C > 0 && N > 0, "pfsgnn_affine_rows", "bad arguments");
  const size_t tot = (size_t)C * N;
  const unsigned blocks = (unsigned)std::min<size_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(k_affine_rows, dim3(blocks), dim3(256), 0, as_stream(stream), X, C, N, sc,
                     sh, Y);
  return pf::check_launch("pfsgnn_affine_rows");
}

__global__ void k_bn2_bwd_coef(const float* __restrict__ Sg, const float* __restrict__ Sgx,
                               const float* __restrict__ mu1, const float* __restrict__ var1,
                               const float* __restrict__ gamma, int C, long long n, float eps,
                               float* __restrict__ alpha, float* __restrict__ gam0,
                               float* __restrict__ gam1, float* __restrict__ dgamma,
                               float* __restrict__ dbeta) {
  const int c = threadIdx.x;
  if (c >= C) return;
  bn2_bwd_coef_one(c, Sg[c], Sgx[c], mu1, var1, gamma, n, eps, alpha, gam0, gam1, dgamma, dbeta);
}

extern "C" int pfsgnn_bn2_bwd_coef(const float* Sg, const float* Sgx, const float* mu1,
                                   const float* var1, const float* gamma, int C, long long n,
                                   float eps, float* alpha, float* gam0, float* gam1,
                                   float* dgamma, float* dbeta, void* stream) {
  PF_REQUIRE(Sg && Sgx && mu1 && var1 && gamma && alpha && gam0 && gam1 && dgamma && dbeta &&
                 C > 0 && C <= 64,
             "pfsgnn_bn2_bwd_coef", "bad arguments");
  hipLaunchKernelGGL(k_bn2_bwd_coef, dim3(1), dim3(64), 0, as_stream(stream), Sg, Sgx, mu1, var1,
                     gamma, C, n, eps, alpha, gam0, gam1, dgamma, dbeta);
  return pf::check_launch("pfsgnn_bn2_bwd_coef");
}

// ---------------------------------------------------------------- moments
__global__ void k_moment_coef(const float* __restrict__ mom, const float* __restrict__ gst, int C,
                              int NS, int n, const int* __restrict__ ptr,
                              float* __restrict__ coef) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // over C*NS
  const size_t CN = (size_t)C * NS;
  if (idx >= CN) return;
  if (ptr) {  // general graph: this fiber's degree (count clamped at 1, as scatter mean)
    const int s = (int)(idx % NS);
    n = max(ptr[s + 1] - ptr[s], 1);
  }
  const float c2 = mom[CN + idx], c3 = mom[2 * CN + idx], c4 = mom[3 * CN + idx];
  const float gmean = gst[idx], gstd = gst[CN + idx], gskew = gst[2 * CN + idx],
              gkurt = gst[3 * CN + idx];
  const float var = c2 > 0.f ? c2 : 0.01f * c2;
  const float sd = sqrtf(var + 1e-6f);
  const float sd2 = sd * sd, sd3 = sd2 * sd, sd4 = sd2 * sd2;
  const float A3 = gskew / sd3;
  const float A4 = gkurt / sd4;
  const float gstd_tot = gstd - 3.f * gskew * c3 / sd4 - 4.f * gkurt * c4 / (sd4 * sd);
  const float gvr = gstd_tot / (2.f * sd) * (c2 > 0.f ? 1.f : 0.01f);
  const float invn = 1.0f / (float)n;
  coef[idx] = (gmean - 3.f * c2 * A3 - 4.f * c3 * A4) * invn;
  coef[CN + idx] = 2.f * gvr * invn;
  coef[2 * CN + idx] = 3.f * A3 * invn;
  coef[3 * CN + idx] = 4.f * A4 * invn;
}

extern "C" int pfsgnn_moment_coef(const float* mom, const float* gst, int C, int NS, int n,
                                  float* coef, void* stream) {
  PF_REQUIRE(mom && gst && coef && C > 0 && NS > 0 && n > 0, "pfsgnn_moment_coef",
             "bad arguments");
  const size_t tot = (size_t)C * NS;
  hipLaunchKernelGGL(k_moment_coef, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), mom, gst, C, NS, n, nullptr, coef);
  return pf::check_launch("pfsgnn_moment_coef");
}

extern "C" int pfsgnn_moment_coef_seg(const float* mom, const float* gst, int C, int NS,
                                      const int* fib_ptr, float* coef, void* stream) {
  PF_REQUIRE(mom && gst && coef && fib_ptr && C > 0 && NS > 0, "pfsgnn_moment_coef_seg",
             "bad arguments");
  const size_t tot = (size_t)C * NS;
  hipLaunchKernelGGL(k_moment_coef, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), mom, gst, C, NS, 1, fib_ptr, coef);
  return pf::check_launch("pfsgnn_moment_coef_seg");
}

// ---------------------------------------------------------------- adam
// torch.optim.Adam as the reference runs it on a GPU with capturable=False
// (torch/optim/adam.py _multi_tensor_adam, the default for device tensors;
// _single_tensor_adam forms the same scalars; amsgrad=False): the scalars torch
// forms from the Python-float step in double (1 - beta1, 1 - beta2,
// lr / bias_correction1, sqrt(bias_correction2)) are formed in double here too
// and rounded to fp32 once, and the element arithmetic is fp32 in the order of
// torch's device kernels, fused multiply-adds where they contract.  The
// step_dev form (our capturable graphs: the count lives on the device) keeps
// these double-scalar semantics -- one double pow per block from the device
// count -- and so matches torch's NON-capturable update at that step; torch's
// own capturable=True variant forms the corrections from fp32 step tensors
// and can differ from both in the last ulp.
//   exp_avg.lerp_(g, 1 - beta1)          m = fma(1 - beta1, g - m, m)
//   exp_avg_sq.mul_(beta2)               v = v * beta2
//   .addcmul_(g, g, 1 - beta2)           v = fma(1 - beta2, g * g, v)
//   denom = sqrt(v) / sqrt(bc2) + eps    (three roundings)
//   p.addcdiv_(m, denom, -step_size)     p = fma(-step_size, m / denom, p)
struct AdamK {
  float omb1, omb2, b2, eps, wd;   // fp32 scalars as torch rounds them
  float neg_step, bc2_sqrt;        // host step
  double beta1, beta2, lr;         // capturable: bias corrections on the device
};
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, long long n, AdamK k,
                       const float* __restrict__ step_dev, const unsigned char* __restrict__ live) {
  float neg_step = k.neg_step, bc2_sqrt = k.bc2_sqrt;
  if (step_dev) {  // device step count: the corrections once per block
    __shared__ float sc[2];
    if (threadIdx.x == 0) {
      const double st = (double)*step_dev;
      const double bc1 = 1.0 - pow(k.beta1, st);
      const double bc2 = 1.0 - pow(k.beta2, st);
      sc[0] = (float)(-(k.lr / bc1));
      sc[1] = (float)sqrt(bc2);
    }
    __syncthreads();
    neg_step = sc[0];
    bc2_sqrt = sc[1];
  }
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // a parameter whose .grad the reference leaves None is skipped by
  // torch.optim.Adam: no decay, moments and value untouched
  if (live && !live[i]) return;
  float gi = g[i];
  if (k.wd != 0.f) gi = fmaf(k.wd, p[i], gi);              // grad.add(param, alpha=wd)
  const float mo = m[i];
  const float mi = fmaf(k.omb1, gi - mo, mo);              // exp_avg.lerp_(grad, 1-beta1)
  const float vb = __fmul_rn(v[i], k.b2);                  // exp_avg_sq.mul_(beta2)
  const float vi = fmaf(k.omb2, __fmul_rn(gi, gi), vb);    // .addcmul_(g, g, 1-beta2)
  m[i] = mi;
  v[i] = vi;
  // sqrt(v)/sqrt(bc2) + eps.  The square root is taken in double and rounded
  // once: correctly rounded (53 >= 2*24 + 2), as torch's is, where the fp32
  // hardware square root (v_sqrt_f32, which __fsqrt_rn lowers to here) is
  // 1-ulp accurate and changed 2 of 10000 updates of a checkpoint resume by
  // one ulp (tests/test_gpu_adam_resume.py)
  const float sq = (float)sqrt((double)vi);
  const float denom = __fadd_rn(__fdiv_rn(sq, bc2_sqrt), k.eps);
  p[i] = fmaf(neg_step, __fdiv_rn(mi, denom), p[i]);       // addcdiv_(m, denom, -lr/bc1)
}

extern "C" int pfsgnn_adam(float* p, const float* g, float* m, float* v, long long n, int step,
                           const float* step_dev, double lr, double beta1, double beta2,
                           double eps, double weight_decay, const unsigned char* live,
                           void* stream) {
  PF_REQUIRE(p && g && m && v && n > 0 && (step >= 1 || step_dev), "pfsgnn_adam",
             "bad arguments");
  const int st = step >= 1 ? step : 1;
  const double bc1 = 1.0 - std::pow(beta1, st);
  const double bc2 = 1.0 - std::pow(beta2, st);
  AdamK k;
  k.omb1 = (float)(1.0 - beta1);
  k.omb2 = (float)(1.0 - beta2);
  k.b2 = (float)beta2;
  k.eps = (float)eps;
  k.wd = (float)weight_decay;
  k.neg_step = (float)(-(lr / bc1));
  k.bc2_sqrt = (float)std::sqrt(bc2);
  k.beta1 = beta1;
  k.beta2 = beta2;
  k.lr = lr;
  hipLaunchKernelGGL(k_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                     p, g, m, v, n, k, step_dev, live);
  return pf::check_launch("pfsgnn_adam");
}
