# the mfma path's edge_mlp_bwd without the class pipeline (nopipe) vs with (ctl), single-object builds, alternating x2
set -o pipefail
mkdir -p gpurun_out
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths , --edge-path mfma" timeout -k 10 600 bash tools/env_ab.sh "PFSGNN_LIB_VARIANT=ctl" "PFSGNN_LIB_VARIANT=nopipe" "PFSGNN_LIB_VARIANT=ctl" "PFSGNN_LIB_VARIANT=nopipe" > gpurun_out/r06z_mfma_pipe.txt 2>&1 || exit 2
