set -o pipefail
mkdir -p gpurun_out
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 600 bash tools/env_ab.sh "" "PFSGNN_LIB_VARIANT=minb4" "PFSGNN_LIB_VARIANT=depth4" "PFSGNN_LIB_VARIANT=pairs4" "PFSGNN_LIB_VARIANT=sbldsw" "" "PFSGNN_LIB_VARIANT=minb4" "PFSGNN_LIB_VARIANT=depth4" "PFSGNN_LIB_VARIANT=pairs4" "PFSGNN_LIB_VARIANT=sbldsw" > gpurun_out/r06q_ab.txt 2>&1 || exit 4
