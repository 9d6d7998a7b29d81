#!/bin/bash
# A/B of the register-staged wide node MLPs (pfsgnn_mlp.hip RS) on the bench step
a="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ,"
for v in "" "PFSGNN_MLP_FWD_RS=0" "PFSGNN_MLP_BWD_RS=0"; do
  env $v python bench.py $a 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/${v:-default} /"
done
