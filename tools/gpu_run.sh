#!/bin/bash
# Run a list of GPU steps on the gpurun box, each under its own time limit.
# Usage: tools/gpu_run.sh "name:seconds:command" ...
# Stops at the first step that fails in any way (a failing GPU test may have
# left the device faulted: nothing more runs on it in this call).
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "[$name] failed rc=$rc: stopping"; exit $rc; fi
done
exit 0
