# round-4 close: the whole GPU suite on the final tree (the driver's command)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ap_gputests.log 2>&1
