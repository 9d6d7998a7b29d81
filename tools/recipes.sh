#!/bin/bash
# Named GPU-box recipes over tools/gpu_run.sh (each step under its own time
# limit, the first failure stops the call).  Run from the repo root on the box:
#   bash tools/recipes.sh <tag> <recipe> [<recipe> ...]
# Outputs land in gpurun_out/<tag>_<recipe>*.  Recipes:
#   tests      the whole -m gpu suite
#   det        the bench-geometry reproducibility tests
#   bench      bench.py (headline line, CPU baseline included)
#   bench16    configs[2]: 256 graphs of 2394x16
#   trace      rocprofv3 --kernel-trace --stats of a short bench run
#   pmc        SQ / FETCH_SIZE / WRITE_SIZE passes (tools/prof_pmc.sh)
#   pmcbwd     SQ passes over the two backward edge kernels (tools/pmc_edge_bwd.sh)
#   precision  the edge paths' precision table at configs[4]'s shape
#   bias       the BatchNorm-cancelled bias gradients vs random fp32 orders
#   sparse     general-graph throughput (tools/sparse_bench.py)
#   dist1      the data-parallel step with RCCL captured, one rank (torchrun)
#   rank2      two ranks on the box's one GPU over gloo (rehearsal)
#   ab         env / library-variant A/B: AB="'' PFSGNN_LIB_VARIANT=x ..." bash tools/recipes.sh t ab
tag=$1; shift
specs=()
for r in "$@"; do
  case $r in
    tests) specs+=("${tag}_tests:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread") ;;
    det) specs+=("${tag}_det:300:python -u -m pytest tests/test_gpu_determinism.py -x -q --timeout 200 --timeout-method thread") ;;
    bench) specs+=("${tag}_bench:300:python bench.py > gpurun_out/${tag}_bench.json") ;;
    bench16) specs+=("${tag}_bench16:300:python bench.py --classes 16 --graphs 256 --steps 50 --alt-paths , --no-cpu-baseline > gpurun_out/${tag}_bench16.json") ;;
    trace) specs+=("${tag}_trace:360:bash tools/trace_only.sh gpurun_out ${tag}") ;;
    pmc) specs+=("${tag}_pmc:600:bash tools/prof_pmc.sh gpurun_out/${tag}_pmc")
         specs+=("${tag}_pmcsum:120:python tools/pmc_traffic.py gpurun_out/${tag}_pmc ${tag} > gpurun_out/${tag}_traffic.log && cp profiles/${tag}_traffic.json gpurun_out/ && python tools/pmc_summary.py gpurun_out/${tag}_pmc/sq/run_counter_collection.csv > gpurun_out/${tag}_pmc_sq.txt && rm -rf gpurun_out/${tag}_pmc") ;;
    pmcbwd) specs+=("${tag}_pmcbwd:400:bash tools/pmc_edge_bwd.sh gpurun_out/${tag}_pmcbwd && rm -rf gpurun_out/${tag}_pmcbwd/p1 gpurun_out/${tag}_pmcbwd/p2 gpurun_out/${tag}_pmcbwd/p3") ;;
    precision) specs+=("${tag}_precision:700:PFSGNN_TOL_OUT=gpurun_out/${tag}_precision.json python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_precision_table.py -m gpu") ;;
    bias) specs+=("${tag}_bias:400:PFSGNN_BIAS_OUT=gpurun_out/${tag}_bias.json python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_bias_noise.py -m gpu") ;;
    sparse) specs+=("${tag}_sparse:400:SPARSE_DENSITIES=1.0,0.3 python tools/sparse_bench.py > gpurun_out/${tag}_sparse.txt") ;;
    dist1) specs+=("${tag}_dist1:240:PFSGNN_DIST_FORCE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 30 --warmup 3 --alt-paths , --no-cpu-baseline > gpurun_out/${tag}_dist1.json") ;;
    rank2) specs+=("${tag}_rank2:300:PFSGNN_BENCH_SAME_DEVICE=1 PFSGNN_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --steps 10 --warmup 2 --alt-paths , --no-cpu-baseline > gpurun_out/${tag}_rank2.json") ;;
    ab) specs+=("${tag}_ab:700:bash tools/env_ab.sh ${AB} > gpurun_out/${tag}_ab.txt") ;;
    *) echo "unknown recipe $r"; exit 2 ;;
  esac
done
bash tools/gpu_run.sh "${specs[@]}"
exit $?
