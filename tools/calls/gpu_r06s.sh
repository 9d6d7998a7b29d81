# Round-6 closing measurements (after the race fix) on the bench default (bf16x6, configs[4]):
# GPU tests, bench, rocprofv3 trace, PMC traffic + SQ counters, bench again
# (its roofline.traffic then reads this round's PMC pass).
set -o pipefail
mkdir -p gpurun_out
T=r06s
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 2
bash tools/trace_only.sh gpurun_out $T || exit 3
python tools/step_trace.py gpurun_out/${T}_trace/run_kernel_trace.csv > gpurun_out/${T}_step_trace.txt 2>&1 || true
cp gpurun_out/${T}_trace/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv 2>/dev/null || true
rm -rf gpurun_out/${T}_trace
bash tools/prof_pmc.sh gpurun_out/${T}_pmc || exit 4
PFSGNN_PMC_PREC=4 python tools/pmc_traffic.py gpurun_out/${T}_pmc $T > gpurun_out/${T}_traffic.log 2>&1 || exit 5
cp profiles/${T}_traffic.json gpurun_out/ || true
python tools/pmc_summary.py gpurun_out/${T}_pmc/sq/run_counter_collection.csv > gpurun_out/${T}_pmc_sq.txt 2>&1 || true
rm -rf gpurun_out/${T}_pmc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.err || exit 6
