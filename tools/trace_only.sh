#!/bin/bash
# rocprofv3 --kernel-trace --stats of a short bench run (on the GPU box, from
# the repo root):  bash tools/trace_only.sh <outdir> <tag> [bench args]
# Summarise the per-step kernels with tools/step_trace.py <dir>/run_kernel_trace.csv.
out=$1; tag=$2; shift 2
args=${@:-"--steps 20 --warmup 5 --no-cpu-baseline --alt-paths ,"}
root=$(pwd)
mkdir -p "$root/$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/${tag}_trace" -o run -- \
  python3 "$root/bench.py" $args > "$root/$out/${tag}_trace.log" 2>&1 || { echo "[trace] failed"; exit 1; }
echo "[trace] ok"
