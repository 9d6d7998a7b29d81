set -o pipefail
mkdir -p gpurun_out
for v in "" nob6s; do
  PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/op_det_probe.py 16 2394 128 bf16x6,mfma 4 2>&1 | sed "s/^/${v:-default} /" >> gpurun_out/r06j_opdet.txt || exit 2
done
for v in nob6s nob6s "" ""; do
  PFSGNN_EDGE_PATH=bf16x6 PFSGNN_LIB_VARIANT=$v timeout -k 10 180 python tools/step_digest.py 16 2394 128 8 2>&1 | tail -1 | sed "s/^/bf16x6 ${v:-default} /" >> gpurun_out/r06j_digest.txt || exit 3
done
for v in "" ""; do
  PFSGNN_EDGE_PATH=mfma PFSGNN_LIB_VARIANT=$v timeout -k 10 180 python tools/step_digest.py 16 2394 128 8 2>&1 | tail -1 | sed "s/^/mfma ${v:-default} /" >> gpurun_out/r06j_digest.txt || exit 4
done
