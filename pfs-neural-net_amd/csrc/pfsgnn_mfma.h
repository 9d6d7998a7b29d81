// pfsgnn_mfma.h -- host launchers of the MFMA edge kernels (pfsgnn_mfma.hip).
//
// Same inputs, outputs and per-block partial formats as the fp32 VALU kernels
// of pfsgnn_edge.hip, so the entry points in pfsgnn_edge.hip pick one or the
// other per call (pfsgnn_set_edge_path) and share every finishing reduction.
// Per-class node tables (Pt, Qt, g_hsum) are passed channel-major [D][NT] as
// the node ops produce them; each block stages its class rows in LDS.
#pragma once
#include "pfsgnn_common.h"

namespace pfm {

// grid of the MFMA kernels: 4 waves x 16 fibers per block (64 fibers, as the
// fp32 kernels), KS class splits to about this many blocks.  `prec`: 0 exact
// fp32 contractions, 1 bf16x3 gradient chains in the backward kernels, 2 single
// bf16 everywhere (pfsgnn_mfma.hip, PREC); `bfy`: round the edge state y to
// bf16 at its store (bf16 edge-state numerics)
static constexpr int TARGET_BLOCKS = 2048;
// classes per block at most (the block's class-table rows are staged in LDS)
static constexpr int MAX_CPS = 64;

int edge_mlp_fwd(const EdgeGeo& geo, int F, const float* xe, const float* xsc, const float* xsh,
                 const float* Ps, const float* PtS, const float* W1, const float* W2,
                 const float* b2, float* y, float* part, const MomFin& fin, int prec, int bfy,
                 hipStream_t st);
int source_fwd(const EdgeGeo& geo, int F, const float* y, const float* sc, const float* sh,
               const float* QtS, const float* Ws1, const float* Ws2, const float* bs2,
               float* partS, int prec, hipStream_t st);
// the fiber-tile form (pfsgnn_mfma.hip km_source_fwd_ft): moments straight to
// mom / hs, no partials; NC <= 256.  NC <= wave_nc (capped at 64): one wave
// per 16 fibers over all classes (no in-block merge)
int source_fwd_tiles(const EdgeGeo& geo, int F, const float* y, const float* sc,
                     const float* sh, const float* QtS, const float* Ws1, const float* Ws2,
                     const float* bs2, float* mom, float* hs, float* msg, int prec, int wave_nc,
                     hipStream_t st);
// TModel's LeakyReLU mask (pfsgnn_mfma.hip mask_bits): target_fwd writes it
// when `tmask` is non-null (4 bytes per edge), target_bwd / source_bwd read
// it in place of recomputing that layer when non-null
int target_fwd(const EdgeGeo& geo, int F, const float* y, const float* sc, const float* sh,
               const float* Rs, const float* Wt1, float* part, uint8_t* tmask, int prec,
               hipStream_t st);
int target_bwd(const EdgeGeo& geo, int F, const float* y, const float* sc, const float* sh,
               const float* Rs, const float* Wt1, const float* ghS, float* gz, float* gxe,
               float* part, const uint8_t* tmask, int prec, hipStream_t st);
// msg (optional): the SModel message cache [2F][E] written by source_fwd_tiles
// (mfma / mfma32 paths): read in place of recomputing the message's second layer
int source_bwd(const EdgeGeo& geo, int F, const float* msg, const float* y, const float* sc,
               const float* sh, const float* QtS, const float* Ws1, const float* Ws2,
               const float* bs2, const float* mean, const float* coef, const float* Rs,
               const float* Wt1, const float* ghS, const float* g_next, const float* mu1,
               const float* inv1, float* g_tot, float* pW2, float* pW1, float* pCol, float* pBN,
               const uint8_t* tmask, int prec, hipStream_t st);
int edge_mlp_bwd(const EdgeGeo& geo, int F, const float* g_tot, const float* alpha,
                 const float* gam0, const float* gam1, const float* y, const float* xe,
                 const float* xsc, const float* xsh, const float* Ps, const float* PtS,
                 const float* W1, const float* W2, float* gxe, float* gs, float* pW2, float* pW1,
                 float* pCol, int prec, hipStream_t st);

// ------------------------------------------------------------ sliced general graphs
// A general (non-complete) batch laid out in slices (pfsgnn_sliced.hip,
// include/pfsgnn.h pfsgnn_sliced_t): slice s = 16 fibers of one graph, the k-th
// edge of lane j at position base[s] + 16 k + j for k < len[s]; cls[p] the class
// within its graph of position p (0xFF: padding).  The kernels take the
// complete path's EdgeGeo with NFG = ceil(NF / 64) 4-slice groups per graph,
// KS step splits per slice (sl_geo) and E = EP (edge-tensor columns), and write
// the same per-block partials (class partials: one row per split), so every
// finishing reduction is shared.
struct SlGeo {
  const int* fib;        // [nslices * 16] global fiber of each lane, -1: none
  const int* base;       // [nslices]
  const int* len;        // [nslices]
  const uint8_t* cls;    // [EP]
  const float* pco;      // [maxdeg][8] Pebay coefficients of counts 1..maxdeg
  long long EP, E;       // positions (padding included), real edges
  int maxdeg;
};
static constexpr int SL_MAX_NC = 128;   // classes per graph (LDS class rows + accumulators)
// the most classes per graph that every sliced kernel of (F, prec) fits in the
// LDS (static + dynamic <= 160 KB), <= SL_MAX_NC; 0: (F, prec) not built
int sl_max_nc(int F, int prec);
EdgeGeo sl_geo(int G, int NF, int NC, const SlGeo& sl);
int sl_edge_mlp_fwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* xe, const float* xsc,
                    const float* xsh, const float* Ps, const float* PtS, const float* W1,
                    const float* W2, const float* b2, float* y, float* part, float* tabs,
                    int prec, hipStream_t st);
// moments straight to mom / hs (per-fiber counts: the fiber degrees)
int sl_source_fwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* y, const float* sc,
                  const float* sh, const float* QtS, const float* Ws1, const float* Ws2,
                  const float* bs2, float* mom, float* hs, float* tabs, int prec,
                  hipStream_t st);
int sl_target_fwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* y, const float* sc,
                  const float* sh, const float* Rs, const float* Wt1, float* part, uint8_t* tmask,
                  int prec, hipStream_t st);
int sl_target_bwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* y, const float* sc,
                  const float* sh, const float* Rs, const float* Wt1, const float* ghS, float* gz,
                  float* gxe, float* part, const uint8_t* tmask, float* tabs, int prec,
                  hipStream_t st);
int sl_source_bwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* y, const float* sc,
                  const float* sh, const float* QtS, const float* Ws1, const float* Ws2,
                  const float* bs2, const float* mean, const float* coef, const float* Rs,
                  const float* Wt1, const float* ghS, const float* g_next, const float* mu1,
                  const float* inv1, float* g_tot, float* pW2, float* pW1, float* pCol,
                  float* pBN, const uint8_t* tmask, float* tabs, int prec, hipStream_t st);
// (tabs: workspace for the class tables in global memory, sl_tab_floats
// floats: source_bwd's two C-wide ones, or one H-wide one)
static inline long long sl_tab_floats(const EdgeGeo& geo, int F) {
  const long long c = 16 * ((((2 * F + 3) / 4) + 3) / 4), h = 16 * ((((4 * F + 3) / 4) + 3) / 4);
  return geo.NT * (2 * c > h ? 2 * c : h);
}
int sl_edge_mlp_bwd(const EdgeGeo& geo, const SlGeo& sl, int F, const float* g_tot,
                    const float* alpha, const float* gam0, const float* gam1, const float* y,
                    const float* xe, const float* xsc, const float* xsh, const float* Ps,
                    const float* PtS, const float* W1, const float* W2, float* gxe, float* gs,
                    float* pW2, float* pW1, float* pCol, float* tabs, int prec, hipStream_t st);

}  // namespace pfm
