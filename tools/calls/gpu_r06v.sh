# the sliced kernels without the MF_SRC_KEEP tie (slk0): bitwise reproducibility at 30 % / 99.9 % density
set -o pipefail
mkdir -p gpurun_out
for v in "" slk0; do
  for d in 0.3 0.999; do
    PFSGNN_LIB_VARIANT=$v timeout -k 10 240 python tools/sparse_det.py $d 3 2>&1 | grep density | sed "s/^/${v:-default} /" >> gpurun_out/r06v_sparse_det.txt || exit 2
  done
done
