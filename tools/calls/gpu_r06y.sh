# per-kernel times of the bf16x6 and mfma paths, same call, alternating x2
set -o pipefail
mkdir -p gpurun_out
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 600 bash tools/env_ab.sh "PFSGNN_EDGE_PATH=bf16x6" "PFSGNN_EDGE_PATH=mfma" "PFSGNN_EDGE_PATH=bf16x6" "PFSGNN_EDGE_PATH=mfma" > gpurun_out/r06y_paths.txt 2>&1 || exit 2
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 600 bash tools/env_ab.sh "PFSGNN_LIB_VARIANT=ctl" "PFSGNN_LIB_VARIANT=recf32" "PFSGNN_LIB_VARIANT=ctl" "PFSGNN_LIB_VARIANT=recf32" > gpurun_out/r06y_recf32.txt 2>&1 || exit 3
