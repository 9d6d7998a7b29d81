set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/probes/mfma_war 4096 64 1 > gpurun_out/r06d_mfma_seq.txt 2>&1 || exit 5
for v in "" nopack nowg4; do
  PFSGNN_LIB_VARIANT=$v PFSGNN_TOL_REPORT=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k graph0 -x -q -s --timeout 180 --timeout-method thread -m gpu 2>&1 | grep -E "TOLREPORT.*(t_model.node_mlp_2.2.bias|x_e)|passed|failed" | sed "s/^/${v:-default} /" >> gpurun_out/r06d_graph0.txt || exit 1
done
for p in mfma mfma32; do
  for v in "" nowg4; do
    PFSGNN_EDGE_PATH=$p PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/step_digest.py 2 2394 128 8 2>/dev/null | sed "s/^/$p ${v:-default} /" >> gpurun_out/r06d_digest.txt || exit 2
  done
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06d_tests.log 2>&1 || exit 3
timeout -k 10 400 bash tools/variant_ab.sh nopack nowg4 > gpurun_out/r06d_ab.txt 2>&1 || exit 4
timeout -k 10 400 bash tools/variant_ab.sh nopack nowg4 >> gpurun_out/r06d_ab.txt 2>&1 || exit 4
timeout -k 10 300 bash -c 'AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths , --edge-path bf16x6" bash tools/env_ab.sh ""' > gpurun_out/r06d_bf16x6_kernels.txt 2>&1 || exit 6
