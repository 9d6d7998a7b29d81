#!/bin/bash
# Pipe-utilisation PMC passes over a short bench run.
# Usage (GPU box, repo root): bash tools/prof_pmc2.sh <outdir>
out=$1; shift
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$root/$out/$name" -o run -- \
    python3 "$root/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$root/$out/$name.log" 2>&1
  rc=$?; echo "[pmc $name] rc=$rc"; return $rc
}
mkdir -p "$root/$out"
run pipe SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT &&
run wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
