set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 600 bash tools/env_ab.sh "" "PFSGNN_LIB_VARIANT=ldsw" "PFSGNN_LIB_VARIANT=depth3" "PFSGNN_MFMA_BLOCKS=2432" >> gpurun_out/r06f_ab.txt 2>&1 || exit 4
done
