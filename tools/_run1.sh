bash tools/gpu_run.sh \
 "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k 'epilogues or global_fused'"
