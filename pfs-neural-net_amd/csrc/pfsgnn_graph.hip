// pfsgnn_graph.hip -- graph construction on the device (src/graph.py:14-67
// to_Graph, src/train.py:88-104): the edge_index of a batch of complete
// bipartite fiber -> class graphs, written straight into HBM instead of the
// reference's Python loops + torch.argsort on the host.
#include "pfsgnn_common.h"
#include "../../include/pfsgnn.h"

#include <algorithm>

namespace {

// one thread per edge; ORDER 0: fiber-major e = (g*NF + f)*NC + c (train.py:94's
// cartesian_prod order, and graph.py:49's sort by source with ties kept in
// construction order); ORDER 1: class-major e = (g*NC + c)*NF + f (graph.py:41-45)
__global__ __launch_bounds__(256) void k_build_complete(int G, int NF, int NC, int order,
                                                        long long* __restrict__ ei) {
  const long long E = (long long)G * NF * NC;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < E;
       e += (long long)gridDim.x * 256) {
    long long g, f, c;
    if (order == 0) {
      c = e % NC;
      const long long gf = e / NC;
      f = gf % NF;
      g = gf / NF;
    } else {
      f = e % NF;
      const long long gc = e / NF;
      c = gc % NC;
      g = gc / NC;
    }
    ei[e] = g * NF + f;
    ei[E + e] = g * NC + c;
  }
}

}  // namespace

extern "C" int pfsgnn_build_complete(int G, int NF, int NC, int order, long long* edge_index,
                                     void* stream) {
  PF_REQUIRE(G > 0 && NF > 0 && NC > 0 && (order == 0 || order == 1) && edge_index,
             "pfsgnn_build_complete", "bad arguments");
  const long long E = (long long)G * NF * NC;
  const unsigned blocks = (unsigned)std::min<long long>((E + 255) / 256, 65536);
  hipLaunchKernelGGL(k_build_complete, dim3(blocks), dim3(256), 0, as_stream(stream), G, NF, NC,
                     order, edge_index);
  return pf::check_launch("pfsgnn_build_complete");
}
