# round-4: node-level precision policy pinned (mfma32 fp32, mfma bf16x3)
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu -k "node_x3_policy or mlp_fused" > gpurun_out/r04ao_tests.log 2>&1
