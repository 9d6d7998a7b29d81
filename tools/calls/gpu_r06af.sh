# bf16x6 edge_mlp_fwd at six waves per SIMD (MF_EFWD_MINB6=6: 80 VGPRs, 5 dwords spilled) vs five, single-object keep-0 builds, alternating x2
set -o pipefail
mkdir -p gpurun_out
AB_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --alt-paths ," timeout -k 10 600 bash tools/env_ab.sh "PFSGNN_LIB_VARIANT=ctl0" "PFSGNN_LIB_VARIANT=minb66" "PFSGNN_LIB_VARIANT=ctl0" "PFSGNN_LIB_VARIANT=minb66" > gpurun_out/r06af_minb66.txt 2>&1 || exit 2
