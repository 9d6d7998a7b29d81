set -o pipefail
mkdir -p gpurun_out
PFSGNN_LIB_VARIANT=nokeep timeout -k 10 120 python tools/op_det_where.py 16 2394 128 bf16x6 3 > gpurun_out/r06l_where_nokeep.txt 2>&1 || exit 2
for v in vf0 nop nopnokeep; do
  PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/op_det_probe.py 16 2394 128 bf16x6 5 2>&1 | grep source_fwd | sed "s/^/$v /" >> gpurun_out/r06l_opdet.txt || exit 3
done
