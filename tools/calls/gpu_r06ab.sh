# bf16x6: the round-6 backward operand knobs re-checked on the headline path (single-object builds vs ctl), alternating x2
set -o pipefail
mkdir -p gpurun_out
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 700 bash tools/env_ab.sh "PFSGNN_LIB_VARIANT=ctl" "PFSGNN_LIB_VARIANT=nowg4" "PFSGNN_LIB_VARIANT=nopack" "PFSGNN_LIB_VARIANT=noearly" "PFSGNN_LIB_VARIANT=ctl" "PFSGNN_LIB_VARIANT=nowg4" "PFSGNN_LIB_VARIANT=nopack" "PFSGNN_LIB_VARIANT=noearly" > gpurun_out/r06ab_bwd_knobs.txt 2>&1 || exit 2
