#!/bin/bash
# A/B of environment knobs on the bench step: ms/step and the edge kernels'
# per-step times (roofline.kernel_ms_per_step), one bench process per setting.
#   bash tools/env_ab.sh "" "PFSGNN_XCD_ORDER=0" ...      ("" = defaults)
a=${AB_ARGS:-"--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ,"}
for v in "$@"; do
  env $v python bench.py $a 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('${v:-default}', round(d['ms_per_step'],3), {k: v for k, v in d['roofline']['kernel_ms_per_step'].items()}, flush=True)"
done
