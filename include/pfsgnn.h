/*
 * pfsgnn.h -- C ABI of libpfsgnn.so, the MI355X (gfx950) bipartite
 * message-passing engine that drops in behind the reference's
 * EdgeModel / SModel / TModel / GlobalModel operator surface
 * (joshua-lintropic/pfs-neural-net, src/gnn.py) and its training objective
 * (src/train.py).
 *
 * Conventions
 *   - every pointer is a DEVICE pointer (HBM) unless noted; float = fp32;
 *   - node tensors are channel-major [C][N] (row stride N);
 *   - edge tensors are channel-major [C][E] over the canonical CLASS-major
 *     order e = (g*NC + c)*NF + f of a batch of G complete bipartite graphs
 *     with NF fibers (source nodes) and NC classes (target nodes) each (the
 *     caller's edge order is mapped by pfsgnn_layout_analyze);
 *     NS = G*NF, NT = G*NC, E = G*NF*NC;
 *   - weights are torch.nn.Linear matrices [out][in] with row stride `ldw`;
 *     a column block is passed as (W + col0, ldw);
 *   - (sc, sh) optional per-channel affine applied to an edge tensor on read
 *     (lazy BatchNorm output); NULL means identity;
 *   - gradient outputs named d* ACCUMULATE (+=); other outputs overwrite;
 *   - `ws`/`ws_bytes` is caller-owned device scratch, at least
 *     pfsgnn_workspace_bytes(G, NF, NC, F) bytes;
 *   - `stream` is a hipStream_t; every call is asynchronous on it and
 *     graph-capturable (no allocation, no synchronisation inside);
 *   - return 0 on success, <0 on error (pfsgnn_last_error() has the text);
 *   - calls come from ONE host thread at a time (the error text, the
 *     deferred-reduction queue and the device-wide barrier slots' round robin
 *     are plain process state), as from the reference's training loop.
 *
 * Supported feature widths F (Fdim): 8, 10, 16.
 */
#ifndef PFSGNN_H
#define PFSGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* pfsgnn_version(void);
const char* pfsgnn_last_error(void);
size_t pfsgnn_workspace_bytes(int G, int NF, int NC, int F);

/* Implementation of the per-edge kernels (process-wide, read at launch, so a
 * captured graph keeps the path it was captured with):
 *   PFSGNN_EDGE_MFMA (default) -- matrix cores (pfsgnn_mfma.hip): forward
 *       layer contractions and their backward recompute on
 *       v_mfma_f32_16x16x4_f32 (exact fp32 products); the backward's gradient
 *       chains (W^T g) and the weight gradients on v_mfma_f32_16x16x16_bf16
 *       with split operands (bf16 hi + lo, ~2^-16 relative per product);
 *   PFSGNN_EDGE_MFMA_F32 -- the same with the gradient chains in exact fp32;
 *   PFSGNN_EDGE_VALU -- fp32 fmaf chains on the vector ALU (pfsgnn_edge.hip);
 *   PFSGNN_EDGE_BF16Y -- MFMA_F32 arithmetic with the edge state y rounded to
 *       bf16 where it is stored (the numerics of bf16 edge-state storage);
 *   PFSGNN_EDGE_BF16 -- every per-edge contraction a single bf16 MFMA (fp32
 *       accumulation) + bf16 edge state (Fdim 10; 13-132x over the fp32 bar);
 *   PFSGNN_EDGE_BF16_MFMA -- the bf16 contractions with the fp32 edge state;
 *   PFSGNN_EDGE_BF16X3 -- every per-edge contraction, the forward ones and
 *       their backward recompute included, on v_mfma_f32_16x16x32_bf16 with
 *       split operands (bf16 hi + lo, ~2^-16 relative per product, fp32
 *       accumulation and edge state; inside the fp32 bar at the bench
 *       geometry, up to 8.3x over it on small graphs: not a configs[4] answer);
 *   PFSGNN_EDGE_BF16X6 -- the forward contractions and their
 *       backward recompute on v_mfma_f32_16x16x32_bf16 with three-way split
 *       operands (hi + mid + lo, the six products down to ~2^-18: fp32-class
 *       products), the gradient chains and weight gradients as
 *       PFSGNN_EDGE_MFMA: BASELINE configs[4] at fp32 tolerance (every parity
 *       case).  Built for Fdim 10; at other Fdims this path runs
 *       the PFSGNN_EDGE_MFMA arithmetic.
 * The fp32-class paths (MFMA, MFMA_F32, VALU, BF16X6) produce the same outputs to the
 * parity tolerance; the bf16 paths' deviation is measured, not bounded
 * (DESIGN.md §Numerics).  Node-level ops, reductions and the loss are shared. */
#define PFSGNN_EDGE_VALU 0
#define PFSGNN_EDGE_MFMA 1
#define PFSGNN_EDGE_MFMA_F32 2
#define PFSGNN_EDGE_BF16Y 3
#define PFSGNN_EDGE_BF16 4
#define PFSGNN_EDGE_BF16_MFMA 5
#define PFSGNN_EDGE_BF16X3 6
#define PFSGNN_EDGE_BF16X6 7
int pfsgnn_set_edge_path(int path);
int pfsgnn_get_edge_path(void);
/* Sync buffer of the in-launch reductions: a device buffer of
 * pfsgnn_sync_bytes() bytes, ZEROED by the caller before it is set and then
 * owned by the library (every launch leaves it zeroed again; one stream at a
 * time).  With it, kernels whose blocks write partials of a group (the
 * SModel moments' class splits, ...) finish the group's reduction in the
 * group's last block instead of a separate reduce launch.  NULL unsets it. */
size_t pfsgnn_sync_bytes(void);
int pfsgnn_set_sync_buffer(void* buf, size_t bytes);
/* Grid the current edge path launches for a batch (host-only query, for tests
 * and diagnostics): info[0] = KS class splits, [1] = classes per split,
 * [2] = blocks per edge kernel, [3] = 64-fiber groups per graph. */
int pfsgnn_edge_grid(int G, int NF, int NC, int* info);

/* Per-kernel HIP-event timing of the main edge/loss kernels (diagnostics for
 * bench.py; off by default, must stay off while a stream is captured).
 * on = 1: events recorded around each launch; on = 2: the same behind a
 * ~0.1 ms single-wave spin kernel enqueued before the start event, so that
 * the interval holds the kernel alone and not the host's launch latency of
 * an eager step (the GPU reaches the start event only once the kernel is
 * enqueued).  Names: edge_mlp_fwd, source_fwd, target_fwd, target_bwd,
 * source_bwd, edge_bn_sums, edge_mlp_bwd, loss_fwd, loss_bwd.  query()
 * synchronises. */
int pfsgnn_timing_enable(int on);
/* Launch the named main kernel 1 + extra times back to back (0: once, the
 * default).  Diagnostics for bench.py's roofline: the kernel only overwrites
 * its outputs, so a captured step with extra = 1 computes the same results,
 * and the difference between its replay time and the plain step's, per
 * launch, is the kernel's duration inside the replayed step.  Supported:
 * edge_mlp_bwd (complete graphs, MFMA edge paths). */
int pfsgnn_timing_repeat(const char* name, int extra);
int pfsgnn_timing_reset(void);
int pfsgnn_timing_query(const char* name, double* total_ms, long long* count);

/* ---------------------------------------------------------------- node ops
 * The node-level Linear / LeakyReLU(0.1) / BatchNorm1d / RMSNorm pieces of
 * MLP (gnn.py:65), SModel.node_mlp_2 (gnn.py:154), TModel.node_mlp_2
 * (gnn.py:192), GlobalModel (gnn.py:223) and the encoders (gnn.py:297).   */

/* Y[m][n] (+)= sum_k W[m][k] * act(X[k][n]) + bscale*b[m]; act = lrelu if act_in */
int pfsgnn_lin(const float* W, int ldw, int M, int K, const float* X, int N,
               const float* b, float bscale, int act_in, float* Y, int add, void* stream);
/* pfsgnn_lin + per-column gathers in the epilogue:
 * Y[m][n] (+)= (W . act(X))[m][n] + bscale*b[m] + G1[m][idx1[n]] + G2[m][idx2[n]]
 * (G1/G2 [M][ld] node tables or NULL) -- the general-graph path's first
 * per-edge Linear, gnn.py:100/136/188, with its node parts gathered per edge */
int pfsgnn_lin_gather(const float* W, int ldw, int M, int K, const float* X, int N,
                      const float* b, float bscale, int act_in, float* Y, int add,
                      const float* G1, const int* idx1, int ld1, const float* G2, const int* idx2,
                      int ld2, void* stream);
/* out[k][n] (+)= (sum_m W[m][k] dY[m][n]) * (Z ? lrelu'(Z[k][n]) : 1) */
int pfsgnn_lin_t(const float* W, int ldw, int M, int K, const float* dY, int N,
                 const float* Z, float* out, int add, void* stream);
/* dW[m][k] += sum_n dY[m][n] act(X[k][n]);  db[m] += dbscale * sum_n dY[m][n] */
int pfsgnn_wgrad(const float* dY, int M, const float* X, int K, int N, int act_in,
                 float* dW, int lddw, float* db, float dbscale,
                 void* ws, size_t ws_bytes, void* stream);

/* One row block of a virtually concatenated node input: the torch.cat of
 * gnn.py:100 ([x_s[src], x_t[tgt], x_e, u[batch]]), :153 ([x, mean, std,
 * skew, kurt, u[batch]]), :191 and :220, read in place instead of copied.
 * x: `rows` channel-major rows.  per_graph == 0: x is [rows][N].
 * per_graph > 0: x is [rows][N / per_graph] and node n reads column
 * n / per_graph (the u[batch] broadcast; one value for all blocks of a list).
 * col: the weight column that multiplies the block's first row.
 * At most 4 blocks per list.                                                  */
typedef struct {
  const float* x;
  int rows;
  int col;
  int per_graph;
} pfsgnn_seg;

/* pfsgnn_lin over a concatenated input: Y[m][n] (+)= sum over blocks s and
 * their rows r of W[m][col_s + r] * act(x_s[r][n or n/per_graph]) + bscale*b[m] */
int pfsgnn_lin_cat(const float* W, int ldw, int M, const pfsgnn_seg* segs, int nseg, int N,
                   const float* b, float bscale, int act_in, float* Y, int add, void* stream);
/* pfsgnn_wgrad over a concatenated input: dW[m][col_s + r] += sum_n dY[m][n] *
 * act(x_s[r][n or n/per_graph]);  db[m] += dbscale * sum_n dY[m][n]            */
int pfsgnn_wgrad_cat(const float* dY, int M, const pfsgnn_seg* segs, int nseg, int N,
                     int act_in, float* dW, int lddw, float* db, float dbscale,
                     void* ws, size_t ws_bytes, void* stream);

/* Deferred weight gradients.  The node-level weight gradients of a backward
 * pass (autograd's accumulation into .grad, train.py:140) are only read by the
 * optimizer step, so their cross-block reductions can run together, after the
 * backward: pfsgnn_wgrad_cat_part launches the per-block partials into `part`
 * (pfsgnn_wgrad_part_bytes(M, K, N, has_db) bytes, owned by the caller until
 * the reduction has run) and returns up to 5 reduction descriptors in red_out;
 * pfsgnn_reduce_batch finishes any list of them in as few launches as the
 * descriptors' output overlaps allow (fixed order: deterministic).          */
typedef struct {
  const float* part;
  int nb;
  size_t plen;
  int ldp, rows, cols;
  float* out;
  int ldo, add;
  float scale;
} pfsgnn_red;

size_t pfsgnn_wgrad_part_bytes(int M, int K, int N, int has_db);
int pfsgnn_wgrad_cat_part(const float* dY, int M, const pfsgnn_seg* segs, int nseg, int N,
                          int act_in, float* dW, int lddw, float* db, float dbscale,
                          void* part, size_t part_bytes, pfsgnn_red* red_out, int* nred_out,
                          void* stream);
int pfsgnn_reduce_batch(const pfsgnn_red* reds, int n, void* stream);
/* A backward pass's weight gradients in a few launches: each job is one
 * pfsgnn_wgrad_cat (dW[:, col_s..] += dY . act(x_s)^T, db += dbscale * sum dY);
 * jobs of the same kernel shape share a launch, then every reduction runs
 * batched.  Per job the result is bitwise that of pfsgnn_wgrad_cat.  The
 * inputs must be unchanged since the job was formed (the host defers jobs over
 * a backward pass: the gradients of nn.Linear weights in gnn.py:65-71, read by
 * the optimizer only, train.py:140-141).  `part`: a scratch arena of
 * pfsgnn_wgrad_multi_bytes(jobs, n) bytes. */
typedef struct {
  const float* dY;
  int M;
  const pfsgnn_seg* segs;
  int nseg;
  int N;
  int act_in;
  float* dW;
  int lddw;
  float* db;
  float dbscale;
} pfsgnn_wgrad_job;
size_t pfsgnn_wgrad_multi_bytes(const pfsgnn_wgrad_job* jobs, int n);
/* Deferred weight-gradient reductions of the fused edge backward kernels
 * (pfsgnn_target_bwd, _source_bwd, _edge_mlp_bwd): between _begin and _end
 * their per-block weight partials go to `arena` (bump-allocated) and their
 * reductions are queued; _end launches them all, batched.  A kernel whose
 * partials do not fit reduces at once, as with no pass open.
 * pfsgnn_defer_need: the arena bytes the last pass asked for (size the next
 * one).  Results are bitwise those of immediate reductions. */
int pfsgnn_defer_begin(void* arena, size_t bytes);
int pfsgnn_defer_end(void* stream);
size_t pfsgnn_defer_need(void);
int pfsgnn_wgrad_multi(const pfsgnn_wgrad_job* jobs, int n, void* part, size_t part_bytes,
                       void* stream);
/* pfsgnn_defer_end + pfsgnn_wgrad_multi(jobs) as one flush: the jobs' kernels,
 * then the pass's queued edge reductions and the jobs' own in one batch (no
 * job reads a weight gradient, so the order does not change a result). */
int pfsgnn_defer_end_multi(const pfsgnn_wgrad_job* jobs, int n, void* part, size_t part_bytes,
                           void* stream);

/* BatchNorm1d training forward over N rows (biased var for the output,
 * unbiased for the running update; rm/rv may be NULL). */
int pfsgnn_bn_fwd(const float* X, int C, int N, const float* gamma, const float* beta,
                  float* rm, float* rv, float momentum, float eps,
                  float* Y, float* mu, float* var, void* ws, size_t ws_bytes, void* stream);
int pfsgnn_bn_bwd(const float* dY, const float* X, const float* mu, const float* var,
                  const float* gamma, float eps, int C, int N,
                  float* dX, float* dgamma, float* dbeta, void* ws, size_t ws_bytes,
                  void* stream);
/* Fused node MLP (gnn.py:65-71: Linear -> LeakyReLU(0.1) -> Linear) over N
 * nodes, optionally followed by a training-mode BatchNorm1d (SModel gnn.py:154,
 * TModel gnn.py:192):
 *   Z  = W1 . cat(segs) + b1      [H][N] pre-activation (saved for backward; may be NULL)
 *   Yp = W2 . lrelu(Z) + b2       [O][N]
 *   gamma != NULL: Y = BatchNorm1d(Yp) (biased var), mu/var [O] out, running stats
 *                  rm/rv (may be NULL) updated with the unbiased variance.
 * The blocks of `segs` must cover weight columns 0..K in order (col = running
 * row offset).  K, H <= 112; O <= 16.  Two launches with BatchNorm, one without.
 * ws >= pfsgnn_mlp_ws_bytes(N).  Replaces the reference's MLP.forward +
 * BatchNorm1d.forward (gnn.py:69-71, 154, 192, 223, 297-298). */
size_t pfsgnn_mlp_ws_bytes(int N);
int pfsgnn_mlp_fwd(const pfsgnn_seg* segs, int nseg, int N, const float* W1, int ldw1, int H,
                   const float* b1, const float* W2, int O, const float* b2, float* Z, float* Yp,
                   const float* gamma, const float* beta, float* rm, float* rv, float momentum,
                   float eps, float* Y, float* mu, float* var, void* ws, size_t ws_bytes,
                   void* stream);
/* A linear map of a node table written where the table is produced:
 * out[k][n] = sum_o W[k*ldw + col0 + o] * Y[o][n] + b[k] (b may be NULL), k < nk. */
typedef struct {
  const float* W;
  int ldw;
  int col0;
  int nk;
  const float* b;
  float* out;
} pfsgnn_linmap;
/* pfsgnn_mlp_fwd with up to 2 such maps of the normalised output Y (BatchNorm
 * required; nk <= 64) done in the normalising pass: SModel's x_s' feeds TModel's
 * Rs = Wt1[:, :F] x_s' + bt1 (gnn.py:188) and the next block's EdgeModel
 * Ps = W1[:, :F] x_s' (gnn.py:100), which then need no launch of their own. */
int pfsgnn_mlp_fwd_epi(const pfsgnn_seg* segs, int nseg, int N, const float* W1, int ldw1,
                       int H, const float* b1, const float* W2, int O, const float* b2, float* Z,
                       float* Yp, const float* gamma, const float* beta, float* rm, float* rv,
                       float momentum, float eps, float* Y, float* mu, float* var,
                       const pfsgnn_linmap* epi, int nepi, void* ws, size_t ws_bytes, void* stream);
/* The tail of a message-passing block (gnn.py:191-192 + 218-223) in two launches:
 * TModel's node_mlp_2 over the G*NC classes (as pfsgnn_mlp_fwd: Z, Yp, W2 [F][H])
 * and its training BatchNorm1d -> xt [F][G*NC], mu/var [F], running stats rm/rv;
 * then one workgroup per graph applies the norm to its classes and runs the
 * GlobalModel as pfsgnn_global_fwd on the new x_s (xs [F][G*NF]) and x_t:
 * means [2F][G], gZ [gH][G], gV [F][G], unew [F][G] (RMSNorm with weight gw, eps
 * reps, y1/r1/r2 saved; gw NULL: unew = gV); and, with We != NULL, the next
 * block's per-class first-Linear parts from the new x_t and u:
 * Pt = We[:, F:2F] xt + We[:, 3F:4F] unew[g] + be  ([4F][G*NC], EdgeModel, gnn.py:100)
 * Qt = Ws[:, 0:F] xt + bs                          ([2F][G*NC], SModel, gnn.py:136).
 * F <= 16; 3F, gH <= 192; ws >= pfsgnn_mlp_ws_bytes(G*NC). */
int pfsgnn_target_global_fwd(
    const pfsgnn_seg* segs, int nseg, int G, int NC, const float* W1, int ldw1, int H,
    const float* b1, const float* W2, int F, const float* b2, float* Z, float* Yp,
    const float* gamma, const float* beta, float* rm, float* rv, float momentum, float eps,
    float* xt, float* mu, float* var, const float* xs, int NF, const float* u, const float* gW1,
    int gH, const float* gb1, const float* gW2, const float* gb2, const float* gw, float reps,
    float* means, float* gZ, float* gV, float* unew, float* y1, float* r1, float* r2,
    const float* We, const float* be, const float* Ws, const float* bs, float* Pt, float* Qt,
    void* ws, size_t ws_bytes, void* stream);
/* A whole block tail on a COMPLETE batch (gnn.py:188-192 + 218-223) in two
 * launches: TModel's per-edge layer (as pfsgnn_target_fwd: hsum, agg = Wt2 hsum +
 * NF bt2, tmask), then ONE launch for the class side -- the per-class sums of
 * the edge kernel's partials, node_mlp_2 + BatchNorm1d, the GlobalModel and the
 * next block's Pt / Qt -- with every output of pfsgnn_target_global_fwd.  The
 * class launch runs G * ceil(NC / 32) units of 32 classes on at most one
 * workgroup per CU with one device-wide barrier between node_mlp_2 (and its
 * BatchNorm partials) and the norm.  The grid must be co-resident (checked
 * against the occupancy API: an error otherwise); a barrier wait that outlives
 * ~1.5 s -- a workgroup never scheduled because another process holds the
 * CUs -- raises pfsgnn_sync_faults' count and traps, so the launch fails
 * instead of computing with partials that were never handed over.  node_mlp_2's weights: W1 [4F][4F], W2
 * [F][4F] (its input [x_t, agg, u[batch]], gnn.py:191).  Replaces
 * pfsgnn_target_fwd + pfsgnn_target_global_fwd (4 launches) on complete graphs. */
typedef struct {
  int G, NF, NC, F;
  /* TModel per-edge layer (pfsgnn_target_fwd) */
  const float *y, *sc, *sh, *Rs, *Wt1, *Wt2, *bt2;
  unsigned char* tmask;
  float *hsum, *agg;                              /* [2F][G*NC] each */
  /* node_mlp_2 + BatchNorm1d (pfsgnn_target_global_fwd) */
  const float *xt, *u, *W1, *b1, *W2, *b2, *gamma, *beta;
  float *Z, *Yp, *rm, *rv, *xt_new, *mu, *var;
  float momentum, eps;
  /* GlobalModel */
  const float *xs, *gW1, *gb1, *gW2, *gb2, *gw;
  int gH;
  float reps;
  float *means, *gZ, *gV, *unew, *y1, *r1, *r2;
  /* next block's class parts (We NULL: none) */
  const float *We, *be, *Ws, *bs;
  float *Pt, *Qt;
} pfsgnn_block_tail;
int pfsgnn_target_block_fwd(const pfsgnn_block_tail* a, void* ws, size_t ws_bytes, void* stream);
/* sizeof(pfsgnn_block_tail), for bindings to check their struct layout */
size_t pfsgnn_block_tail_bytes(void);
/* The class side of a block's backward on a complete batch (training
 * BatchNorm, gnn.py:191-192 + 218-223 under autograd) in ONE launch, units of
 * 16 classes of one graph around two device-wide barriers:
 *   1. dY = gu_up + the per-graph sums of the pending u[batch] gradients of
 *      the block above (npend tables [F][G*pend_n[i]], pend_n = NF or NC: what
 *      pfsgnn_graph_reduce_multi would add to gu_up).  gu_up is READ ONLY: the
 *      sum feeds step 2 and is not written back;
 *   2. the GlobalModel backward of pfsgnn_global_bwd on that dY (gV, gdZ, dwp
 *      written; gu += its u-input gradient; g_xs += d mean_xs / NF and g_xt +=
 *      d mean_xt / NC broadcast), then TModel's BatchNorm sums on the new g_xt;
 *   3. pfsgnn_mlp_bwd of node_mlp_2 + BatchNorm on dY = g_xt (dYp, dZ written,
 *      dgamma / dbeta accumulated) with dX's rows [0, F) added into gxt_in,
 *      [F, 3F) written to g_agg, [3F, 4F) to gu_t; and g_hsum = Wt2^T g_agg
 *      (TModel's second Linear, gnn.py:188-190).
 * node_mlp_2: W1 [4F][4F], W2 [F][4F]; GlobalModel: gW1 [gH][3F], gW2 [F][gH],
 * RMSNorm weight w (NULL: unnormed, then y1/r1/r2/dwp unused).  Replaces
 * graph_reduce_multi + global_bwd (2 launches) + mlp_bwd (2) + lin_t. */
typedef struct {
  int G, NF, NC, F;
  const float* pend[4];
  int pend_n[4];
  int npend;
  const float *V, *w, *y1, *r1, *r2, *gZ, *gW1, *gW2;
  int gH;
  float *gu_up, *gV, *gdZ, *dwp, *gu, *g_xs, *g_xt;
  const float *Yp, *mu, *var, *gamma, *Z, *W1, *W2, *Wt2;
  float eps;
  float *dgamma, *dbeta, *dYp, *dZ, *gxt_in, *g_agg, *gu_t, *g_hsum;
} pfsgnn_class_bwd;
int pfsgnn_target_class_bwd(const pfsgnn_class_bwd* a, void* ws, size_t ws_bytes, void* stream);
size_t pfsgnn_class_bwd_bytes(void);
/* device-wide barrier time-outs since load (*n = count; 0 in a healthy run --
 * a time-out also traps the launch that hit it) */
int pfsgnn_sync_faults(unsigned* n);
/* the device-wide barrier's form for later launches: 0 (default) the sc1
 * hand-off with relaxed agent-scope counters, 1 acq_rel arrival / acquire poll
 * (an L2 write-back and L1 invalidate per workgroup); bitwise the same results */
int pfsgnn_set_grid_sync_fenced(int fenced);
/* One row block of an input-gradient output: rows `rows` of dX go to x
 * ([rows][N], overwritten, or accumulated when add != 0); x == NULL drops them. */
typedef struct {
  float* x;
  int rows;
  int add;
} pfsgnn_oseg;
/* Its backward (autograd of the same modules, train.py:140), input side:
 *   gamma != NULL: dYp = BatchNorm1d backward of dY (dgamma += sum dY*xhat,
 *                  dbeta += sum dY), written to dYp [O][N];  else dYp := dY;
 *   dZ = (W2^T dYp) * lrelu'(Z)   written to dZ [H][N];
 *   dX = W1^T dZ                  into the `outs` blocks (covering K rows; nout = 0 skips dX).
 * The weight gradients are pfsgnn_wgrad(dYp, Z, act_in=1) and
 * pfsgnn_wgrad_cat(dZ, segs) (deferred-reduction friendly).                   */
int pfsgnn_mlp_bwd(const float* dY, int N, const float* Yp, const float* mu, const float* var,
                   const float* gamma, float eps, float* dgamma, float* dbeta, const float* Z,
                   const float* W1, int ldw1, int H, int K, const float* W2, int O, float* dYp,
                   float* dZ, const pfsgnn_oseg* outs, int nout, void* ws, size_t ws_bytes,
                   void* stream);
/* the same with SModel's node_mlp_2 backward (gnn.py:140-154) folded in:
 *   bn_part != NULL: the BatchNorm sums already made by the producer of dY
 *     (pfsgnn_target_bwd_bn's bn_part, bn_nparts = ceil(N / 64) per-block
 *     partials [n][32]: sum dY in 0..16, sum dY*xhat in 16..32) instead of a
 *     sums launch of its own (gamma required);
 *   coef != NULL: dX rows [mom_k0, mom_k0 + 4 mom_c) -- d loss / d [mean; std;
 *     skew; kurt] of mom_c (16..20) message channels -- are not written; they
 *     become pfsgnn_moment_coef(mom, ., mom_c, N, mom_n)'s coefficients coef
 *     [4][mom_c][N] in the same launch (mom: pfsgnn_source_fwd's [4][mom_c][N];
 *     mom_n: messages per fiber).  The outs entry covering those rows may be
 *     NULL.  Needs the wide form (K or H > 64).
 * Replaces k_bn_sums_part + pfsgnn_mlp_bwd + pfsgnn_moment_coef. */
int pfsgnn_mlp_bwd_pre(const float* dY, int N, const float* Yp, const float* mu,
                       const float* var, const float* gamma, float eps, float* dgamma,
                       float* dbeta, const float* Z, const float* W1, int ldw1, int H, int K,
                       const float* W2, int O, float* dYp, float* dZ, const pfsgnn_oseg* outs,
                       int nout, const float* bn_part, int bn_nparts, const float* mom,
                       float* coef, int mom_k0, int mom_c, int mom_n, void* ws,
                       size_t ws_bytes, void* stream);
/* Several independent small products in one launch: each job is a
 * pfsgnn_lin_cat (trans 0: Y[M][N] (+)= W . act(x_segs) + bscale*b) or a
 * pfsgnn_lin_t (trans 1: Y[M][N] (+)= W^T[M][K] . segs[0] (* lrelu'(Z)), W
 * of K rows).  Jobs must not write the same Y.  K <= 40, M <= 64 (the
 * per-block node parts of gnn.py:100/136/188's first Linear layers and their
 * input gradients). */
typedef struct {
  const float* W;
  int ldw;
  int trans;
  int M;
  int K;
  const pfsgnn_seg* segs;
  int nseg;
  int N;
  const float* b;
  float bscale;
  int act_in;
  const float* Z;
  float* Y;
  int add;
} pfsgnn_gemm_job;
int pfsgnn_gemm_multi(const pfsgnn_gemm_job* jobs, int n, void* stream);

/* ---------------------------------------------------------- graph building
 * edge_index (int64 [2][E], E = G*NF*NC) of G complete bipartite graphs, fiber
 * ids g*NF + f, class ids g*NC + c.  order 0: fiber-major (train.py:94
 * cartesian_prod; graph.py:49's sort by source, ties in construction order);
 * order 1: class-major (graph.py:41-45 construction order).  Replaces
 * to_Graph's host loops (graph.py:40-51). */
int pfsgnn_build_complete(int G, int NF, int NC, int order, long long* edge_index, void* stream);

/* out[c][g] = sum (or mean) over the n nodes of graph g of X[c][g*n + i] */
int pfsgnn_graph_reduce(const float* X, int C, int G, int n, int mean, float* out, void* stream);
/* the same, accumulated: out[c][g] += sum (or mean) ... (u[batch] gradients, gnn.py:100/153/191) */
int pfsgnn_graph_reduce_add(const float* X, int C, int G, int n, int mean, float* out,
                            void* stream);
/* m (1..4) per-graph sums into one accumulator, one launch: out[c][g] +=
 * sum_j sum_i X[j][c][g*n[j] + i] (the u[batch] gradients of gnn.py:100/153/191). */
int pfsgnn_graph_reduce_multi(const float* const* X, const int* n, int m, int C, int G,
                              float* out, void* stream);
/* GlobalModel's two node means (gnn.py:218-219) in one launch:
 * out[c][g] = mean of X1[c][g*n1 ..], out[C + c][g] = mean of X2[c][g*n2 ..] */
int pfsgnn_graph_mean2(const float* X1, int n1, const float* X2, int n2, int C, int G,
                       float* out, void* stream);
/* its backward: out1[c][g*n1 + i] += s1*src[c][g], out2[c][g*n2 + i] += s2*src[C + c][g] */
int pfsgnn_graph_bcast_add2(float* out1, int n1, float s1, float* out2, int n2, float s2, int C,
                            int G, const float* src, void* stream);
/* out[c][g*n + i] += scale * src[c][g] */
int pfsgnn_graph_bcast_add(float* out, int C, int G, int n, const float* src, float scale,
                           void* stream);
/* GlobalModel's RMSNorm, applied twice (gnn.py:223 + the Sequential child),
 * over C features of G rows. y1 [C][G], r1/r2 [G] are saved for backward. */
int pfsgnn_rms2_fwd(const float* X, int C, int G, const float* w, float eps,
                    float* Y, float* y1, float* r1, float* r2, void* stream);
int pfsgnn_rms2_bwd(const float* dY, const float* X, const float* w, const float* y1,
                    const float* r1, const float* r2, int C, int G, float eps,
                    float* dX, float* dw, void* ws, size_t ws_bytes, void* stream);
/* The whole GlobalModel (gnn.py:208-223) in one call (a wide means launch,
 * then a block per graph): means[c][g] / means[F + c][g] = per-graph means of xs / xt
 * (n1 / n2 nodes per graph), Z [H][G] = W1 [u; means] + b1, V [F][G] =
 * W2 lrelu(Z) + b2 (the MLP, W1 [H][3F], W2 [F][H]), Y = RMSNorm applied
 * twice with weight w (y1, r1, r2 saved as pfsgnn_rms2_fwd); w == NULL: Y = V
 * (unnormed).  3F, H <= 192.  Two launches for graph_mean2 + mlp + rms2_fwd. */
int pfsgnn_global_fwd(const float* xs, int n1, const float* xt, int n2, const float* u, int F,
                      int G, const float* W1, int H, const float* b1, const float* W2,
                      const float* b2, const float* w, float eps, float* means, float* Z, float* V,
                      float* Y, float* y1, float* r1, float* r2, void* stream);
/* Its backward (train.py:140's autograd through gnn.py:218-223): gV [F][G] =
 * d loss / d V, dZ [H][G] = d loss / d Z (both kept for the weight gradients),
 * dwp [F][G] the per-graph RMSNorm weight gradient (the caller sums over g),
 * gU [F][G] += d loss / d u, gm [2F][G] = d loss / d means, then
 * gxs[c][g*n1 + i] += s1 * gm[c][g], gxt[c][g*n2 + i] += s2 * gm[F + c][g]
 * (s = 1/n for the mean).  Two launches. */
int pfsgnn_global_bwd(const float* dY, const float* V, const float* w, const float* y1,
                      const float* r1, const float* r2, int F, int G, const float* Z, int H,
                      const float* W1, const float* W2, float* gV, float* dZ, float* dwp,
                      float* gU, float* gm, float* gxs, int n1, float s1, float* gxt, int n2,
                      float s2, void* stream);
/* EdgeModel's BatchNorm applied twice (gnn.py:101): from the batch moments
 * (mu1, var1) of y give xe_new = sc*y + sh; updates running stats twice. */
int pfsgnn_bn2_finalize(const float* mu1, const float* var1, const float* gamma,
                        const float* beta, float* rm, float* rv, int C, long long n,
                        float momentum, float eps, float* sc, float* sh, float* inv1,
                        float* inv2, void* stream);
/* Eval-mode BatchNorm1d (running statistics, none updated) as one per-channel
 * affine sc*y + sh: `times` = 2 for EdgeModel (gnn.py:101 + the Sequential
 * child, replaces nn.BatchNorm1d.forward in eval), 1 for SModel/TModel
 * (gnn.py:154, :192). */
int pfsgnn_bn_eval_coef(const float* gamma, const float* beta, const float* rm,
                        const float* rv, int C, float eps, int times, float* sc, float* sh,
                        void* stream);
/* Its backward (autograd through a model in eval(), gnn.py:101/154/192): inv =
 * 1/sqrt(rv + eps) and scale = d out / d y = (gamma inv)^times per channel; with
 * the input-gradient sums Sg = sum g, Sgx = sum g (y - rm) inv (pfsgnn_rows_bn_sums
 * or pfsgnn_edge_bn_grad_sums with mu = rm and this inv) dgamma / dbeta accumulate
 * the parameter gradients of the `times`-fold application.  Sg NULL: inv and
 * scale only (inv / scale may be NULL when not wanted). */
int pfsgnn_bn_eval_bwd_coef(const float* gamma, const float* beta, const float* rm,
                            const float* rv, int C, float eps, int times, const float* Sg,
                            const float* Sgx, float* inv, float* scale, float* dgamma,
                            float* dbeta, void* stream);
/* Y[c][n] = sc[c]*X[c][n] + sh[c] over a channel-major [C][N] table */
int pfsgnn_affine_rows(const float* X, int C, int N, const float* sc, const float* sh,
                       float* Y, void* stream);
/* its backward: g_y = alpha*g + gam0 + gam1*y from Sg = sum g, Sgx = sum g*xhat */
int pfsgnn_bn2_bwd_coef(const float* Sg, const float* Sgx, const float* mu1, const float* var1,
                        const float* gamma, int C, long long n, float eps, float* alpha,
                        float* gam0, float* gam1, float* dgamma, float* dbeta, void* stream);
/* the same from per-block partials part [nparts][2C] (sum g in 0..C, sum
 * g*xhat in C..2C; pfsgnn_loss_bwd_bn's bn_part), summed in a fixed order */
int pfsgnn_bn2_bwd_coef_part(const float* part, int nparts, int C, const float* gamma,
                             const float* mu1, const float* var1, long long n, float eps,
                             float* alpha, float* gam0, float* gam1, float* dgamma, float* dbeta,
                             void* stream);
/* SModel moment backward (gnn.py:140-153) -> per-fiber coefficients of
 * g_m = C0 + d(C1 + d(C2 + d C3)), d = m - mean.  mom [4][C][NS] =
 * (mean, c2, c3, c4); gst [4C][NS] = dL/d(mean, std, skew, kurt). */
int pfsgnn_moment_coef(const float* mom, const float* gst, int C, int NS, int n,
                       float* coef, void* stream);
/* the same for a general graph: fiber s's count is fib_ptr[s+1] - fib_ptr[s]
 * (clamped at 1, as torch_scatter's mean; gnn.py:140-144) */
int pfsgnn_moment_coef_seg(const float* mom, const float* gst, int C, int NS, const int* fib_ptr,
                           float* coef, void* stream);

/* ------------------------------------------------ general (sparse) bipartite graphs
 * The reference's data model takes any edge_index (gnn.py:7-47; PyG batching
 * gnn.py:32-47) and its scatters reduce over arbitrary src / tgt (gnn.py:140-144
 * per fiber, gnn.py:190 per class).  A batch that is not complete bipartite is
 * laid out once by pfsgnn_sparse_layout; every edge tensor of the step is then
 * channel-major [C][E] in "position" order (edges sorted stably by fiber), and
 * the per-edge MLPs run as node-table gathers + pfsgnn_lin over E columns, the
 * scatters as the deterministic segment kernels below (block per segment,
 * fixed-order trees: bitwise reproducible run to run).  int32 indices: E, G*NF,
 * G*NC < 2^31.  (Replaces torch_scatter.scatter / x[src] / x[tgt] of gnn.py:100,
 * 136-144, 188-190 for such graphs.) */
size_t pfsgnn_sparse_layout_ws_bytes(long long E);
/* edge_index int64 [2][E] (row 0 fiber ids g*NF+f, row 1 class ids g*NC+c).
 * Outputs (device int32): src_p/tgt_p [E] fiber / class of each position,
 * user_of [E] the caller's edge at each position, fib_ptr [G*NF+1] (CSR by
 * fiber over positions), cls_ord [E] positions sorted stably by class and
 * cls_ptr [G*NC+1] (CSR by class over cls_ord).  status[0] != 0 after the call
 * iff some edge is out of range or joins nodes of different graphs (the
 * caller must reject the batch). */
int pfsgnn_sparse_layout(const long long* edge_index, long long E, int G, int NF, int NC,
                         int* src_p, int* tgt_p, int* user_of, int* fib_ptr, int* cls_ord,
                         int* cls_ptr, int* status, void* ws, size_t ws_bytes, void* stream);
/* out[c][e] = X[c][idx[e]] (mode 0), += X[c][idx[e]] (mode 1), or
 * X[c][idx[e]] * lrelu'(Z[c][e]) (mode 2); X is a node table [C][N] */
int pfsgnn_gather_cols(const float* X, int C, int N, const int* idx, long long E, const float* Z,
                       int mode, float* out, void* stream);
/* out[c][s] (+)= sum over the segment's positions p in [ptr[s], ptr[s+1]) of
 * act(X[c][ord ? ord[p] : p]); act = lrelu (0.1) if `act`, identity otherwise;
 * C <= 64 (one wave per segment, every channel in registers) */
int pfsgnn_segment_sum(const float* X, int C, long long E, const int* ord, const int* ptr,
                       int nseg, int act, float* out, int add, void* stream);
/* SModel moments per fiber (gnn.py:140-151), C <= 32: mom [4][C][nseg] = (mean,
 * c2, c3, c4) and the node_mlp_2 inputs hs [4C][nseg] = (mean, std, skew, kurt);
 * an empty fiber gives zeros and std = sqrt(1e-6), as the reference's
 * scatter-mean + nan_to_num do */
int pfsgnn_segment_moments(const float* M, int C, long long E, const int* ptr, int nseg,
                           float* mom, float* hs, void* stream);
/* gm[c][e] = C0 + d(C1 + d(C2 + d C3)), d = M[c][e] - mean[c][seg[e]],
 * coefficients coef [4][C][nseg] from pfsgnn_moment_coef_seg */
int pfsgnn_segment_moment_grad(const float* M, int C, long long E, const int* seg,
                               const float* mean, const float* coef, int nseg, float* gm,
                               void* stream);
/* per-channel batch statistics of a [C][N] table (C <= 256): mean and biased
 * variance (the EdgeModel BatchNorm's, gnn.py:101) */
size_t pfsgnn_rows_ws_bytes(int C, long long N);
int pfsgnn_rows_stats(const float* X, int C, long long N, float* mu, float* var, void* ws,
                      size_t ws_bytes, void* stream);
/* Sg[c] = sum_n g, Sgx[c] = sum_n g (y - mu) inv (the double BatchNorm's gradient sums) */
int pfsgnn_rows_bn_sums(const float* g, const float* y, int C, long long N, const float* mu,
                        const float* inv, float* Sg, float* Sgx, void* ws, size_t ws_bytes,
                        void* stream);
/* out[c][n] = alpha[c] g[c][n] + gam1[c] y[c][n] + gam0[c]; out may alias g or y */
int pfsgnn_rows_axpby(const float* g, const float* y, int C, long long N, const float* alpha,
                      const float* gam1, const float* gam0, float* out, void* stream);

/* ------------------------------------------------ sliced general graphs
 * The FUSED edge kernels for general batches (pfsgnn_sliced.hip): the fiber
 * CSR of pfsgnn_sparse_layout is re-cut into slices of 16 fibers of one graph
 * (each graph's fibers sorted by degree, descending, stable), the k-th edge of
 * slice lane j at position base[s] + 16 k + j for k < len[s] (the slice's
 * largest degree); a fiber with fewer edges leaves padding positions.  Edge
 * tensors are channel-major [C][EP] over these positions and hold 0 at padding.
 * Slices 4 q .. 4 q + 3 are the 4 waves of the blocks of 64-fiber group q =
 * g * ceil(NF/64) + (its group in graph g), each block taking one of KS step
 * splits, so the pfsgnn_sl_* edge ops below run the complete path's grid
 * shape and share its reductions; they take the same arguments and give the
 * same outputs as the complete-graph op of the same name (G, NF, NC: the
 * batch's graphs and per-graph node counts), plus the layout.  NC <= 128
 * classes per graph; Fdim 8, 10, 16; the workspace of pfsgnn_workspace_bytes.
 * (Replaces torch_scatter.scatter, x[src], x[tgt] of gnn.py:100, 136-144,
 * 188-190 for such graphs, fused.) */
typedef struct {
  const int* fib;            /* [G*ceil(NF/64)*4*16] global fiber of each slice lane, -1: none */
  const int* base;           /* [G*ceil(NF/64)*4] first position of each slice */
  const int* len;            /* [G*ceil(NF/64)*4] steps of each slice (its largest degree) */
  const unsigned char* cls;  /* [EP] class within its graph of each position, 0xFF: padding */
  const float* pco;          /* [maxdeg][8] Pebay coefficients (pfsgnn_sliced_fill) */
  long long EP;              /* positions = edge-tensor columns, padding included */
  long long E;               /* edges */
  int maxdeg;                /* largest fiber degree */
} pfsgnn_sliced_t;
/* The most classes per graph (NC) the sliced kernels of the CURRENT edge path
 * take at Fdim F: every kernel's static LDS plus its per-class tables must fit
 * the CU's 160 KB (e.g. 124 at Fdim 16 on the default path), and at most 128.
 * 0: no sliced kernels for this (F, path) -- the bf16 edge-state paths and
 * Fdims other than 8 / 10 / 16.  A batch above the limit runs the composed
 * general-graph ops (pfsgnn.sparse); the pfsgnn_sl_* ops refuse it.
 * (Host-side query; it reads the kernels' attributes from the HIP runtime.) */
int pfsgnn_sliced_max_nc(int F, int* nc);
size_t pfsgnn_sliced_plan_ws_bytes(int G, int NF);
/* From fib_ptr [G*NF+1] (pfsgnn_sparse_layout): the slice lanes `fib`, lengths
 * `len`, first positions `base`, slot_of [G*NF] (the slice lane 16 s + j of
 * each fiber) and, in info (device int64[2]), EP and maxdeg. */
int pfsgnn_sliced_plan(const int* fib_ptr, int G, int NF, int* fib, int* base, int* len,
                       int* slot_of, long long* info, void* ws, size_t ws_bytes, void* stream);
/* From the sparse layout (src_p, tgt_p, user_of, fib_ptr) and the plan: cls [EP]
 * and pos_user [EP] (the caller's edge at each position, -1 at padding), pco
 * [maxdeg*8].  NC < 255. */
int pfsgnn_sliced_fill(const int* src_p, const int* tgt_p, const int* user_of, const int* fib_ptr,
                       long long E, int NF, int NC, const int* slot_of, const int* base,
                       long long EP, int maxdeg, unsigned char* cls, int* pos_user, float* pco,
                       void* stream);
/* caller-order edge rows [E][F] -> a slot tensor [F][EP] (0 at padding), and
 * back (dst [E][F] if rowmajor else [F][E]; with sc/sh the lazy affine first);
 * F = 8, 10 or 16 */
int pfsgnn_edges_to_slots(const float* src, long long E, long long EP, int F, const int* pos_user,
                          float* dst, void* stream);
int pfsgnn_edges_from_slots(const float* y, const float* sc, const float* sh, long long E,
                            long long EP, int F, const int* pos_user, int rowmajor, float* dst,
                            void* stream);

/* ---------------------------------------------------------------- edge ops */

/* EdgeModel per-edge MLP (gnn.py:99-101 with the first Linear split):
 * z1 = Ps[:,f] + Pt[:,c] + W1[:,2F:3F] x ; y = W2 lrelu(z1) + b2, where
 * x = xsc*xe + xsh.  Also the batch moments mu/var (biased) of y. */
int pfsgnn_edge_mlp_fwd(int G, int NF, int NC, int F, const float* xe, const float* xsc,
                        const float* xsh, const float* Ps, const float* Pt, const float* W1,
                        const float* W2, const float* b2, float* y, float* mu, float* var,
                        void* ws, size_t ws_bytes, void* stream);
/* the same + the double BatchNorm's finalize (pfsgnn_bn2_finalize's outputs
 * sc, sh, inv1, inv2 and running-stat updates) in the moments pass: the
 * EdgeModel training forward in one call (gnn.py:99-101) */
int pfsgnn_edge_mlp_fwd_bn(int G, int NF, int NC, int F, const float* xe, const float* xsc,
                           const float* xsh, const float* Ps, const float* Pt, const float* W1,
                           const float* W2, const float* b2, float* y, float* mu, float* var,
                           const float* gamma, const float* beta, float* rm, float* rv,
                           float momentum, float eps, float* sc, float* sh, float* inv1,
                           float* inv2, void* ws, size_t ws_bytes, void* stream);
/* SModel per-edge message + per-fiber centred moments (gnn.py:136-151).
 * mom [4][2F][NS]; hs [8F][NS] receives (mean, std, skew, kurt). */
int pfsgnn_source_fwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                      const float* sh, const float* Qt, const float* Ws1, const float* Ws2,
                      const float* bs2, float* mom, float* hs, void* ws, size_t ws_bytes,
                      void* stream);
/* The SModel message cache (round 6): bytes of the per-edge messages m
 * [2F][E] (gnn.py:136, the output of node_mlp_1) that the current edge path
 * keeps between the forward and the backward -- complete graphs on the
 * PFSGNN_EDGE_MFMA / _MFMA_F32 paths when PFSGNN_MSG=1 is set, 0 otherwise
 * (the backward then recomputes them; the default: the forward's extra
 * 80 B per edge of writes cost more than the recompute).  pfsgnn_source_fwd_msg = pfsgnn_source_fwd + writes the
 * messages to `msg` (this many bytes); pfsgnn_source_bwd(_bn)_msg read them in
 * place of recomputing node_mlp_1's second Linear -- bit for bit the values the
 * forward computed, so results equal the recomputing calls'. */
size_t pfsgnn_msg_bytes(int G, int NF, int NC, int F);
int pfsgnn_source_fwd_msg(int G, int NF, int NC, int F, const float* y, const float* sc,
                          const float* sh, const float* Qt, const float* Ws1, const float* Ws2,
                          const float* bs2, float* mom, float* hs, float* msg, void* ws,
                          size_t ws_bytes, void* stream);
/* TModel per-edge message, summed per class before its second Linear
 * (gnn.py:188-190): hsum[:,c] = sum_f lrelu(Rs[:,f] + Wt1[:,F:2F] x); with Wt2
 * (optional, [2F][2F]) also that Linear in the same call's reduction epilogue:
 * agg[:,c] = Wt2 hsum[:,c] + bscale*bt2. */
int pfsgnn_target_fwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                      const float* sh, const float* Rs, const float* Wt1, float* hsum,
                      const float* Wt2, const float* bt2, float bscale, float* agg,
                      unsigned char* tmask, void* ws, size_t ws_bytes, void* stream);
/* Bytes of the TModel mask the current edge path keeps between the forward
 * and the backward (0: it keeps none, recomputes).  When non-zero and `tmask`
 * (this many bytes) is given to pfsgnn_target_fwd, the forward writes the
 * sign pattern of TModel's per-edge pre-activation (gnn.py:188, the LeakyReLU
 * of node_mlp_1) and pfsgnn_target_bwd / pfsgnn_source_bwd(_bn) given the
 * same buffer read it in place of recomputing that layer. */
size_t pfsgnn_tmask_bytes(int G, int NF, int NC, int F);
/* TModel edge backward: GzT[:,f] = sum_c g_z; dWt1[:,F:2F] += sum g_z x^T;
 * optional gxe = Wt1[:,F:2F]^T g_z (standalone TModel only); optional g_xs
 * += Wt1[:,0:F]^T GzT (the x_s[src] input gradient, in the reduction epilogue). */
int pfsgnn_target_bwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                      const float* sh, const float* Rs, const float* Wt1, const float* g_hsum,
                      float* GzT, float* dWt1, float* gxe, float* g_xs,
                      const unsigned char* tmask, void* ws, size_t ws_bytes, void* stream);
/* the same (complete graphs) where g_xs is final after this call and feeds
 * SModel's node_mlp_2 + BatchNorm backward (gnn.py:153-154): the epilogue
 * that finishes g_xs also writes that BatchNorm's backward sums over its
 * fibers, bn_part [ceil(G*NF / 64)][32] (sum g_xs, sum g_xs*(Yp - mu) /
 * sqrt(var + eps) per channel; bn_Yp [F][G*NF] the pre-norm output, bn_mu /
 * bn_var its batch statistics) for pfsgnn_mlp_bwd_pre. */
int pfsgnn_target_bwd_bn(int G, int NF, int NC, int F, const float* y, const float* sc,
                         const float* sh, const float* Rs, const float* Wt1, const float* g_hsum,
                         float* GzT, float* dWt1, float* gxe, float* g_xs,
                         const unsigned char* tmask, const float* bn_Yp, const float* bn_mu,
                         const float* bn_var, float bn_eps, float* bn_part, void* ws,
                         size_t ws_bytes, void* stream);
/* SModel edge backward fused with TModel's per-edge input gradient, the
 * downstream edge gradient and the edge BatchNorm's two gradient sums:
 * g_tot = Ws1e^T g_zs + [Wt1e^T g_zt] + [g_next]; GzS per class;
 * dWs1[:,F:2F], dWs2, dbs2 accumulated; Sg/Sgx = sums of g_tot, g_tot*xhat
 * (xhat = (y-mu1)*inv1) when mu1 != NULL.  Rs/Wt1/g_hsum may be NULL.
 * Optional g_xt += Ws1[:,0:F]^T GzS (x_t[tgt] input gradient, reduction epilogue). */
int pfsgnn_source_bwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                      const float* sh, const float* Qt, const float* Ws1, const float* Ws2,
                      const float* bs2, const float* mean, const float* coef, const float* Rs,
                      const float* Wt1, const float* g_hsum, const float* g_next,
                      const float* mu1, const float* inv1, float* g_tot, float* GzS,
                      float* dWs1, float* dWs2, float* dbs2, float* Sg, float* Sgx,
                      float* g_xt, const unsigned char* tmask, void* ws, size_t ws_bytes,
                      void* stream);
/* the same with the edge BatchNorm's backward finished in the same call: in
 * place of Sg / Sgx it writes pfsgnn_bn2_bwd_coef's alpha, gam0, gam1 and
 * accumulates dgamma / dbeta (gamma, var1: that BatchNorm's weight and batch
 * variance; n = E) */
int pfsgnn_source_bwd_bn(int G, int NF, int NC, int F, const float* y, const float* sc,
                         const float* sh, const float* Qt, const float* Ws1, const float* Ws2,
                         const float* bs2, const float* mean, const float* coef, const float* Rs,
                         const float* Wt1, const float* g_hsum, const float* g_next,
                         const float* mu1, const float* inv1, const float* var1,
                         const float* gamma, long long n, float eps, float* g_tot, float* GzS,
                         float* dWs1, float* dWs2, float* dbs2, float* alpha, float* gam0,
                         float* gam1, float* dgamma, float* dbeta, float* g_xt,
                         const unsigned char* tmask, void* ws, size_t ws_bytes, void* stream);
/* pfsgnn_source_bwd / _bn with the forward's message cache (pfsgnn_msg_bytes) */
int pfsgnn_source_bwd_msg(int G, int NF, int NC, int F, const float* y, const float* sc,
                          const float* sh, const float* Qt, const float* Ws1, const float* Ws2,
                          const float* bs2, const float* mean, const float* coef,
                          const float* Rs, const float* Wt1, const float* g_hsum,
                          const float* g_next, const float* mu1, const float* inv1,
                          float* g_tot, float* GzS, float* dWs1, float* dWs2, float* dbs2,
                          float* Sg, float* Sgx, float* g_xt, const unsigned char* tmask,
                          const float* msg, void* ws, size_t ws_bytes, void* stream);
int pfsgnn_source_bwd_bn_msg(int G, int NF, int NC, int F, const float* y, const float* sc,
                             const float* sh, const float* Qt, const float* Ws1,
                             const float* Ws2, const float* bs2, const float* mean,
                             const float* coef, const float* Rs, const float* Wt1,
                             const float* g_hsum, const float* g_next, const float* mu1,
                             const float* inv1, const float* var1, const float* gamma,
                             long long n, float eps, float* g_tot, float* GzS, float* dWs1,
                             float* dWs2, float* dbs2, float* alpha, float* gam0, float* gam1,
                             float* dgamma, float* dbeta, float* g_xt,
                             const unsigned char* tmask, const float* msg, void* ws,
                             size_t ws_bytes, void* stream);
/* Sg = sum g, Sgx = sum g*(y-mu1)*inv1 (standalone EdgeModel backward). */
int pfsgnn_edge_bn_grad_sums(int G, int NF, int NC, int F, const float* g, const float* y,
                             const float* mu1, const float* inv1, float* Sg, float* Sgx,
                             void* ws, size_t ws_bytes, void* stream);
/* EdgeModel per-edge MLP backward.  g_y = alpha*g_tot + gam0 + gam1*y;
 * gxe (optional) = W1[:,2F:3F]^T g_z1; GzEs [4F][NS], GzEt [4F][NT] are
 * the per-fiber / per-class sums of g_z1; dW1[:,2F:3F], dW2, db2 accumulated.
 * Optional, in the reductions' epilogues (gnn.py:100's node-input gradients):
 * g_xs += W1[:,0:F]^T GzEs, g_xt += W1[:,F:2F]^T GzEt, Vu [F][NT] =
 * W1[:,3F:4F]^T GzEt (the caller sums it per graph into g_u). */
int pfsgnn_edge_mlp_bwd(int G, int NF, int NC, int F, const float* g_tot, const float* alpha,
                        const float* gam0, const float* gam1, const float* y, const float* xe,
                        const float* xsc, const float* xsh, const float* Ps, const float* Pt,
                        const float* W1, const float* W2, float* dW1, float* dW2, float* db2,
                        float* gxe, float* GzEs, float* GzEt, float* g_xs, float* g_xt,
                        float* Vu, void* ws, size_t ws_bytes, void* stream);

/* The edge ops above on a sliced general batch (pfsgnn_sliced_t): arguments
 * and outputs as the op of the same name; edge tensors are [C][sl->EP]; the
 * EdgeModel BatchNorm counts sl->E edges; `tmask` has pfsgnn_sl_tmask_bytes. */
int pfsgnn_sl_edge_mlp_fwd(const pfsgnn_sliced_t* sl, int G, int NF, int NC, int F,
                           const float* xe, const float* xsc, const float* xsh, const float* Ps,
                           const float* Pt, const float* W1, const float* W2, const float* b2,
                           float* y, float* mu, float* var, void* ws, size_t ws_bytes,
                           void* stream);
int pfsgnn_sl_edge_mlp_fwd_bn(const pfsgnn_sliced_t* sl, int G, int NF, int NC, int F,
                              const float* xe, const float* xsc, const float* xsh,
                              const float* Ps, const float* Pt, const float* W1, const float* W2,
                              const float* b2, float* y, float* mu, float* var,
                              const float* gamma, const float* beta, float* rm, float* rv,
                              float momentum, float eps, float* sc, float* sh, float* inv1,
                              float* inv2, void* ws, size_t ws_bytes, void* stream);
int pfsgnn_sl_source_fwd(const pfsgnn_sliced_t* sl, int G, int NF, int NC, int F, const float* y,
                         const float* sc, const float* sh, const float* Qt, const float* Ws1,
                         const float* Ws2, const float* bs2, float* mom, float* hs, void* ws,
                         size_t ws_bytes, void* stream);
size_t pfsgnn_sl_tmask_bytes(const pfsgnn_sliced_t* sl, int F);
int pfsgnn_sl_target_fwd(const pfsgnn_sliced_t* sl, int G, int NF, int NC, int F, const float* y,
                         const float* sc, const float* sh, const float* Rs, const float* Wt1,
                         float* hsum, const float* Wt2, const float* bt2, float bscale,
                         float* agg, unsigned char* tmask, void* ws, size_t ws_bytes,
                         void* stream);
int pfsgnn_sl_target_bwd(const pfsgnn_sliced_t* sl, int G, int NF, int NC, int F, const float* y,
                         const float* sc, const float* sh, const float* Rs, const float* Wt1,
                         const float* g_hsum, float* GzT, float* dWt1, float* gxe, float* g_xs,
                         const unsigned char* tmask, void* ws, size_t ws_bytes, void* stream);
int pfsgnn_sl_source_bwd(const pfsgnn_sliced_t* sl, int G, int NF, int NC, int F, const float* y,
                         const float* sc, const float* sh, const float* Qt, const float* Ws1,
                         const float* Ws2, const float* bs2, const float* mean,
                         const float* coef, const float* Rs, const float* Wt1,
                         const float* g_hsum, const float* g_next, const float* mu1,
                         const float* inv1, float* g_tot, float* GzS, float* dWs1, float* dWs2,
                         float* dbs2, float* Sg, float* Sgx, float* g_xt,
                         const unsigned char* tmask, void* ws, size_t ws_bytes, void* stream);
int pfsgnn_sl_source_bwd_bn(const pfsgnn_sliced_t* sl, int G, int NF, int NC, int F,
                            const float* y, const float* sc, const float* sh, const float* Qt,
                            const float* Ws1, const float* Ws2, const float* bs2,
                            const float* mean, const float* coef, const float* Rs,
                            const float* Wt1, const float* g_hsum, const float* g_next,
                            const float* mu1, const float* inv1, const float* var1,
                            const float* gamma, long long n, float eps, float* g_tot, float* GzS,
                            float* dWs1, float* dWs2, float* dbs2, float* alpha, float* gam0,
                            float* gam1, float* dgamma, float* dbeta, float* g_xt,
                            const unsigned char* tmask, void* ws, size_t ws_bytes, void* stream);
int pfsgnn_sl_edge_mlp_bwd(const pfsgnn_sliced_t* sl, int G, int NF, int NC, int F,
                           const float* g_tot, const float* alpha, const float* gam0,
                           const float* gam1, const float* y, const float* xe, const float* xsc,
                           const float* xsh, const float* Ps, const float* Pt, const float* W1,
                           const float* W2, float* dW1, float* dW2, float* db2, float* gxe,
                           float* GzEs, float* GzEt, float* g_xs, float* g_xt, float* Vu,
                           void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- loss
 * train.py:29-80: decoder_e (gnn.py:307) + softplus + softfloor (train.py:21)
 * + scatters per class / fiber.  ci = class_info [>=2][NT] (row 0 = T_i,
 * row 1 = N_i).  Noise uniforms come from a counter-based hash of
 * (seed, edge); seed_dev (optional, device uint64) overrides `seed` so a
 * captured graph draws fresh noise per replay.  tt (optional) = per-edge
 * allocated time [E] in train.py's fiber-major order. */
int pfsgnn_loss_fwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                    const float* sh, const float* Wd1, const float* bd1, const float* Wd2,
                    const float* bd2, const float* ci, float scale, float sharpness,
                    float noiselevel, unsigned long long seed,
                    const unsigned long long* seed_dev, float* n_prime,
                    float* fiber_time, float* tmean, float* tvar, float* tt,
                    void* ws, size_t ws_bytes, void* stream);
int pfsgnn_loss_finalize(int G, int NF, int NC, const float* n_prime, const float* fiber_time,
                         const float* tvar, const float* ci, float pclass, float pfiber,
                         float total_time, float nfields, float wutils, float wvar,
                         float* loss, float* utils, float* variance, float* Gn, float* Gf,
                         float* Gv, void* stream);
/* gscale: device scalar (upstream d loss), NULL = 1. gxe = d loss / d xe_final */
int pfsgnn_loss_bwd(int G, int NF, int NC, int F, const float* y, const float* sc,
                    const float* sh, const float* Wd1, const float* bd1, const float* Wd2,
                    const float* bd2, const float* ci, float scale, float sharpness,
                    float noiselevel, unsigned long long seed,
                    const unsigned long long* seed_dev, const float* Gn,
                    const float* Gf, const float* Gv, const float* tmean, const float* gscale,
                    float* dWd1, float* dbd1, float* dWd2, float* dbd2, float* gxe,
                    void* ws, size_t ws_bytes, void* stream);
/* the same, also writing the final EdgeModel BatchNorm's backward sums of gxe
 * (gnn.py:101, the last block's; train.py's objective reads nothing else of
 * it): bn_part [pfsgnn_loss_bn_parts(G, NF, NC)][2F] per-block partials of
 * sum gxe and sum gxe * (y - bn_mu1) * bn_inv1, for pfsgnn_bn2_bwd_coef_part --
 * in place of a pass that reads gxe and y back (pfsgnn_edge_bn_grad_sums) */
int pfsgnn_loss_bn_parts(int G, int NF, int NC);
int pfsgnn_loss_bwd_bn(int G, int NF, int NC, int F, const float* y, const float* sc,
                       const float* sh, const float* Wd1, const float* bd1, const float* Wd2,
                       const float* bd2, const float* ci, float scale, float sharpness,
                       float noiselevel, unsigned long long seed,
                       const unsigned long long* seed_dev, const float* Gn, const float* Gf,
                       const float* Gv, const float* tmean, const float* gscale, float* dWd1,
                       float* dbd1, float* dWd2, float* dbd2, float* gxe, const float* bn_mu1,
                       const float* bn_inv1, float* bn_part, void* ws, size_t ws_bytes,
                       void* stream);

/* ---------------------------------------------------------------- layout
 * The reference takes an arbitrary edge_index [2][E] (int64, gnn.py:7).  A
 * complete bipartite batch in any edge order maps onto the canonical
 * class-major order by a permutation.  pfsgnn_layout_analyze validates
 * edge_index (every (g, f, c) exactly once, src graph == tgt graph) and
 * writes perm[canonical] = caller's edge id; status (device int32[3]):
 * [0] complete, [1] caller order is train.py's fiber-major (g*NF+f)*NC+c
 * (train.py:94), [2] caller order is already canonical.
 * Conversions take mode 0 (perm), 1 (fiber-major, arithmetic), 2 (identity). */
int pfsgnn_layout_analyze(const int64_t* edge_index, long long E, int G, int NF, int NC,
                          int32_t* perm, int32_t* status, void* ws, size_t ws_bytes,
                          void* stream);
/* caller-order row-major edges [E][F] -> channel-major canonical [F][E] */
int pfsgnn_edges_to_canonical(const float* src, int G, int NF, int NC, int F, int mode,
                              const int32_t* perm, float* dst, void* stream);
/* canonical (sc*y+sh) -> caller order, row-major [E][F] (rowmajor = 1) or
 * channel-major [F][E] (rowmajor = 0) */
int pfsgnn_edges_from_canonical(const float* y, const float* sc, const float* sh, int G, int NF,
                                int NC, int F, int mode, const int32_t* perm, int rowmajor,
                                float* dst, void* stream);

/* ---------------------------------------------------------------- optimiser
 * torch.optim.Adam (amsgrad=False, maximize=False) over one flat buffer
 * (replaces optimizer.step(), train.py:111/141).  step_dev (optional, device
 * float) overrides `step` (capturable form).  live (optional, device byte
 * per element): elements with live[i] == 0 belong to parameters whose .grad
 * the reference leaves None (unused by the loss); torch.optim.Adam skips
 * those, so they are left untouched (matters when weight_decay != 0).
 * The hyper-parameters are the Python floats (doubles) torch's Adam holds:
 * its scalars 1 - beta1, 1 - beta2 and lr / (1 - beta1^t) are formed in
 * double and rounded to fp32 once, as torch's capturable=False Adam does
 * (torch/optim/adam.py _multi_tensor_adam / _single_tensor_adam), so the
 * update is that one's bit for bit up to the order of the last division
 * (CUDA's addcdiv: value * (m / denom)).  With step_dev the same double
 * scalars are formed from the device count (once per block): still the
 * capturable=False update at that step, not torch's capturable=True one,
 * whose corrections come from fp32 step tensors. */
int pfsgnn_adam(float* p, const float* g, float* m, float* v, long long n, int step,
                const float* step_dev, double lr, double beta1, double beta2, double eps,
                double weight_decay, const unsigned char* live, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PFSGNN_H */
