set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/op_det_where.py 16 2394 128 bf16x6 6 > gpurun_out/r06k_where.txt 2>&1 || exit 2
for v in "" nob6s sft1 sft2 nokeep pin; do
  PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/op_det_probe.py 16 2394 128 bf16x6 5 2>&1 | grep source_fwd | sed "s/^/${v:-default} /" >> gpurun_out/r06k_opdet.txt || exit 3
done
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 300 bash tools/env_ab.sh "" "PFSGNN_LIB_VARIANT=nob6s" "" "PFSGNN_LIB_VARIANT=nob6s" > gpurun_out/r06k_ab.txt 2>&1 || exit 4
