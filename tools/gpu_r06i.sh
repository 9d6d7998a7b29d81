set -o pipefail
mkdir -p gpurun_out
for v in "" nob6s ""; do
  PFSGNN_EDGE_PATH=bf16x6 PFSGNN_LIB_VARIANT=$v timeout -k 10 180 python tools/step_digest.py 16 2394 128 8 2>&1 | tail -1 | sed "s/^/bf16x6 ${v:-default} /" >> gpurun_out/r06i_digest.txt || exit 2
done
for v in nob6s ""; do
  echo "== ${v:-default}" >> gpurun_out/r06i_g16.log
  PFSGNN_G16_PATHS=bf16x6 PFSGNN_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_geometry.py -m gpu -x -q --timeout 240 --timeout-method thread >> gpurun_out/r06i_g16.log 2>&1 || echo "rc=$? ${v:-default}" >> gpurun_out/r06i_g16.log
done
