# race mechanism probe: the LDS-table build with each fold's coefficient rows checked against c_peb (printf on mismatch)
set -o pipefail
mkdir -p gpurun_out
for v in lds diag; do
  PFSGNN_LIB_VARIANT=$v timeout -k 10 150 python tools/op_det_probe.py 16 2394 128 bf16x6 5 > gpurun_out/r06aa_$v.txt 2>&1 || exit 2
done
PFSGNN_LIB_VARIANT=diag timeout -k 10 150 python tools/op_det_where.py 16 2394 128 bf16x6 3 > gpurun_out/r06aa_diag_where.txt 2>&1 || exit 3
