#!/bin/bash
# rocprofv3 kernel trace + stats of tools/sparse_bench.py (on the GPU box, from
# the repo root):  bash tools/prof_sparse.sh <outdir> <tag> <densities> [bench args]
out=$1; tag=$2; dens=$3; shift 3
root=$(pwd)
mkdir -p "$root/$out"
cd /tmp && export TMPDIR=/tmp
SPARSE_DENSITIES=$dens timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$root/$out/${tag}_trace" -o run -- python3 "$root/tools/sparse_bench.py" "$@" \
  > "$root/$out/${tag}_trace.log" 2>&1 || { echo "[trace] failed"; exit 1; }
echo "[trace] ok"
