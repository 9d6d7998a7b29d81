#!/bin/bash
# Parity error report of the bf16x3 edge path per model mask (PFSGNN_X3_MASK:
# bit 0 EdgeModel, bit 1 SModel/TModel run bf16x3 forward contractions).
export PFSGNN_TOL_REPORT=1 PFSGNN_PARITY_PATHS=bf16x3
for m in 1 2 3; do
  echo "=== mask $m"
  PFSGNN_X3_MASK=$m timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s \
    -k "training_step or eval" --timeout 120 --timeout-method thread 2>&1 | \
    awk '/TOLREPORT/ {split($0,a,"err/bound "); if (a[2]+0 > 0.5) print}' || exit 1
done
