# edge grid (class splits) on the bf16x6 bench: KS 5 (default, 3040 blocks) vs 4 (2432) vs 6 (3648), alternating x2
set -o pipefail
mkdir -p gpurun_out
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 600 bash tools/env_ab.sh "" "PFSGNN_MFMA_BLOCKS=2432" "PFSGNN_MFMA_BLOCKS=3648" "" "PFSGNN_MFMA_BLOCKS=2432" "PFSGNN_MFMA_BLOCKS=3648" > gpurun_out/r06x_grid_ab.txt 2>&1 || exit 2
