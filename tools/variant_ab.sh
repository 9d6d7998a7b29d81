#!/bin/bash
# A/B of tuning builds (tools/variants.sh) on the bench step: ms/step and the
# edge kernels' per-step times (roofline.kernel_ms_per_step), default first.
#   bash tools/variant_ab.sh name1 [name2 ...]
a="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ,"
for v in "" "$@"; do
  PFSGNN_LIB_VARIANT=$v python bench.py $a 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('${v:-default}', round(d['ms_per_step'],3), {k: v for k, v in d['roofline']['kernel_ms_per_step'].items()})"
done
