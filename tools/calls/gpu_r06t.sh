# sliced (general-graph) kernels without the MF_SRC_KEEP tie: 30 % dense batch, both arms twice
set -o pipefail
mkdir -p gpurun_out
for v in "" slk0 "" slk0; do
  echo "== ${v:-default}" >> gpurun_out/r06t_sparse.txt
  PFSGNN_LIB_VARIANT=$v SPARSE_RUNS=3 SPARSE_DENSITIES=1.0,0.3 timeout -k 10 300 python tools/sparse_bench.py >> gpurun_out/r06t_sparse.txt 2>&1 || exit 2
done
