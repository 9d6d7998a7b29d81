# round-4 close: precision table of the edge paths on the final tree (node-level bf16x3 included)
PFSGNN_TOL_OUT=gpurun_out/r04ak_precision.json timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_precision_table.py -m gpu > gpurun_out/r04ak_precision_table.log 2>&1
