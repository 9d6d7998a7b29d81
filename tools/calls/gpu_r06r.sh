set -o pipefail
mkdir -p gpurun_out
for p in bf16x6 mfma; do
  for v in "" keepall; do
    PFSGNN_EDGE_PATH=$p PFSGNN_LIB_VARIANT=$v timeout -k 10 180 python tools/step_digest.py 16 2394 128 8 2>&1 | tail -1 | sed "s/^/$p ${v:-default} /" >> gpurun_out/r06r_digest.txt || exit 2
  done
done
timeout -k 10 150 python tools/op_det_probe.py 16 2394 128 bf16x6,bf16x3,mfma,mfma32 4 2>&1 | grep -v amdgpu.ids > gpurun_out/r06r_opdet.txt || exit 3
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 400 bash tools/env_ab.sh "" "PFSGNN_LIB_VARIANT=keepall" "" "PFSGNN_LIB_VARIANT=keepall" > gpurun_out/r06r_ab.txt 2>&1 || exit 4
