set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/probes/mfma_war 4096 64 > gpurun_out/r06c_mfma_war.txt 2>&1 || exit 1
for p in mfma mfma32 bf16x6; do
  for v in "" nopack; do
    PFSGNN_EDGE_PATH=$p PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/step_digest.py 2 2394 128 8 2>/dev/null | sed "s/^/$p ${v:-pack} /" >> gpurun_out/r06c_digest.txt || exit 2
    PFSGNN_EDGE_PATH=$p PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/step_digest.py 2 24 16 2 2>/dev/null | sed "s/^/$p ${v:-pack} /" >> gpurun_out/r06c_digest.txt || exit 2
  done
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1 || exit 3
timeout -k 10 300 bash tools/variant_ab.sh nopack > gpurun_out/r06c_ab.txt 2>&1 || exit 4
timeout -k 10 300 bash tools/variant_ab.sh nopack >> gpurun_out/r06c_ab.txt 2>&1 || exit 4
