set -o pipefail
mkdir -p gpurun_out
for p in bf16x6; do
  for v in "" nopipe6; do
    PFSGNN_EDGE_PATH=$p PFSGNN_LIB_VARIANT=$v timeout -k 10 180 python tools/step_digest.py 2 2394 128 8 2>&1 | tail -1 | sed "s/^/$p ${v:-default} /" >> gpurun_out/r06p_digest.txt || exit 2
  done
done
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 400 bash tools/env_ab.sh "" "PFSGNN_LIB_VARIANT=nopipe6" "" "PFSGNN_LIB_VARIANT=nopipe6" > gpurun_out/r06p_ab.txt 2>&1 || exit 4
