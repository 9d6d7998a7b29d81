set -o pipefail
mkdir -p gpurun_out
for p in mfma mfma32; do
  for m in 1 0; do
    PFSGNN_EDGE_PATH=$p PFSGNN_MSG=$m timeout -k 10 120 python tools/step_digest.py 2 2394 128 8 2>/dev/null | sed "s/^/$p msg=$m /" >> gpurun_out/r06e_digest.txt || exit 2
    PFSGNN_EDGE_PATH=$p PFSGNN_MSG=$m timeout -k 10 120 python tools/step_digest.py 2 24 16 2 2>/dev/null | sed "s/^/$p msg=$m /" >> gpurun_out/r06e_digest.txt || exit 2
  done
done
timeout -k 10 400 bash tools/env_ab.sh "" "PFSGNN_MSG=0" > gpurun_out/r06e_ab.txt 2>&1 || exit 4
timeout -k 10 400 bash tools/env_ab.sh "" "PFSGNN_MSG=0" >> gpurun_out/r06e_ab.txt 2>&1 || exit 4
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06e_tests.log 2>&1 || exit 3
