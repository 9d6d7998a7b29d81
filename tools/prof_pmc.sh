#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 process per counter group).
# Usage (on the GPU box, from the repo root): bash tools/prof_pmc.sh <outdir> [bench args]
out=$1; shift
args=${@:-"--steps 3 --warmup 1 --no-cpu-baseline --alt-paths ,"}
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$root/$out/$name" -o run -- \
    python3 "$root/bench.py" $args > "$root/$out/$name.log" 2>&1
  rc=$?; echo "[pmc $name] rc=$rc"; return $rc
}
mkdir -p "$root/$out"
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE
