#!/bin/bash
# A/B of sliced-kernel builds on tools/sparse_bench.py, one process per run:
#   bash tools/sl_ab.sh <densities> variant1 [variant2 ...]   ("" = default build)
dens=$1; shift
for v in "" "$@"; do
  for d in ${dens//,/ }; do
    PFSGNN_LIB_VARIANT=$v SPARSE_DENSITIES=$d python tools/sparse_bench.py 2>/dev/null | sed "s/^/${v:-default} /"
  done
done
