# general-graph throughput table on the final tree (tools/sparse_bench.py defaults: densities 1.0, 0.999, 0.3, 0.05; median of 5 graph-replayed runs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/sparse_bench.py > gpurun_out/r06ae_sparse.txt 2>&1 || exit 2
