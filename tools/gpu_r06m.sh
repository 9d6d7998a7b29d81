set -o pipefail
mkdir -p gpurun_out
for v in pcoreg mssep nokeeppco nokeep; do
  PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/op_det_probe.py 16 2394 128 bf16x6 5 2>&1 | grep source_fwd | sed "s/^/$v /" >> gpurun_out/r06m_opdet.txt || exit 3
done
for v in noslp; do
  PFSGNN_LIB_VARIANT=$v timeout -k 10 120 python tools/op_det_probe.py 16 2394 128 bf16x6,mfma 5 2>&1 | grep source_fwd | sed "s/^/$v /" >> gpurun_out/r06m_opdet.txt || exit 4
done
