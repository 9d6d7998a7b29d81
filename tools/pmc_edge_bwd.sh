#!/bin/bash
# SQ counter passes over the two backward edge kernels (tools/pcs_driver.py),
# one rocprofv3 process per pass (<= 8 SQ counters each).  On the GPU box,
# from the repo root:  bash tools/pmc_edge_bwd.sh <outdir> [path]
out=$1; path=${2:-mfma}
root=$(pwd)
mkdir -p "$root/$out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
  "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
  "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$root/$out/p$i" -o run -- \
    python3 "$root/tools/pcs_driver.py" 8 "$path" > "$root/$out/p$i.log" 2>&1
  rc=$?; echo "[pmc p$i] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 "$root/tools/pmc_summary.py" "$root/$out/p$i/run_counter_collection.csv" edge_mlp_bwd source_bwd \
    >> "$root/$out/summary.txt" || exit 1
done
