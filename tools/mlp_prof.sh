#!/bin/bash
# Node-MLP micro-benchmark with its kernel stats and two SQ PMC passes.
# Usage (GPU box, repo root): bash tools/mlp_prof.sh <outdir>
out=$1; shift
root=$(pwd)
mkdir -p "$root/$out"
timeout -k 10 120 python3 tools/mlp_bench.py > "$root/$out/times.txt" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/kt" -o run -- \
  python3 "$root/tools/mlp_bench.py" 38304 5 > "$root/$out/kt.log" 2>&1 || exit 1
run() {
  name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d "$root/$out/$name" -o run -- \
    python3 "$root/tools/mlp_bench.py" 38304 5 > "$root/$out/$name.log" 2>&1
  rc=$?; echo "[pmc $name] rc=$rc"; return $rc
}
run pipe SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT &&
run wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
