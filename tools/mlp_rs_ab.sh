#!/bin/bash
# Node-MLP micro-benchmark under the RS A/B knobs (GPU box, repo root)
for v in "X=0" "PFSGNN_MLP_FWD_RS=1" "PFSGNN_MLP_BWD_RS=0"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 tools/mlp_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
