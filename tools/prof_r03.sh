#!/bin/bash
# Round-3 profile set (on the GPU box, from the repo root):
#   bash tools/prof_r03.sh <outdir> <tag> [bench args]
# 1. rocprofv3 --kernel-trace --stats of a short bench run (kernel stats + the
#    per-step trace: tools/step_trace.py);
# 2. separate PMC passes: SQ issue/wait counters, FETCH_SIZE, WRITE_SIZE.
# Every step has its own time limit; the script stops at the first failure.
out=$1; tag=$2; shift 2
args=${@:-"--steps 20 --warmup 5 --no-cpu-baseline"}
root=$(pwd)
mkdir -p "$root/$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/${tag}_trace" -o run -- \
  python3 "$root/bench.py" $args > "$root/$out/${tag}_trace.log" 2>&1 || { echo "[trace] failed"; exit 1; }
echo "[trace] ok"
pmc() {
  name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$root/$out/${tag}_$name" -o run -- \
    python3 "$root/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${args#--steps 20 --warmup 5 --no-cpu-baseline} \
    > "$root/$out/${tag}_$name.log" 2>&1
  rc=$?; echo "[pmc $name] rc=$rc"; return $rc
}
pmc sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS &&
pmc fetch FETCH_SIZE &&
pmc write WRITE_SIZE
