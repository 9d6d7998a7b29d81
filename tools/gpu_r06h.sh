set -o pipefail
mkdir -p gpurun_out
for p in bf16x6 mfma; do
  for v in "" nob6s; do
    PFSGNN_EDGE_PATH=$p PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/step_digest.py 2 2394 128 8 2>/dev/null | sed "s/^/$p ${v:-default} /" >> gpurun_out/r06h_digest.txt || exit 2
  done
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06h_tests.log 2>&1 || exit 3
for r in 1 2; do
  AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 300 bash tools/env_ab.sh "" "PFSGNN_LIB_VARIANT=nob6s" >> gpurun_out/r06h_ab.txt 2>&1 || exit 4
done
