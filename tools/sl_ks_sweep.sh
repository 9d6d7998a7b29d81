#!/bin/bash
# step-split count of the sliced kernels (PFSGNN_SL_KS) on tools/sparse_bench.py
for ks in 1 2 3 4; do
  for d in 0.3 0.999; do
    PFSGNN_SL_KS=$ks SPARSE_DENSITIES=$d python tools/sparse_bench.py 2>/dev/null | sed "s/^/KS=$ks /"
  done
done
