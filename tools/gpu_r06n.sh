set -o pipefail
mkdir -p gpurun_out
for p in bf16x6 mfma; do
  PFSGNN_EDGE_PATH=$p timeout -k 10 180 python tools/step_digest.py 16 2394 128 8 2>&1 | tail -1 | sed "s/^/$p default /" >> gpurun_out/r06n_digest.txt || exit 2
done
for v in "" keep0 b6s keep0b6s; do
  PFSGNN_LIB_VARIANT=$v timeout -k 10 150 python tools/op_det_probe.py 16 2394 128 bf16x6,bf16x3,mfma 5 2>&1 | grep -v amdgpu.ids | sed "s/^/${v:-default} /" >> gpurun_out/r06n_opdet.txt || exit 3
done
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 400 bash tools/env_ab.sh "" "PFSGNN_LIB_VARIANT=keep0" "PFSGNN_LIB_VARIANT=b6s" "" "PFSGNN_LIB_VARIANT=keep0" "PFSGNN_LIB_VARIANT=b6s" > gpurun_out/r06n_ab.txt 2>&1 || exit 4
