bash tools/gpu_run.sh \
 "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k 'ops or parity or baseline'" \
 "bench:300:python bench.py --no-cpu-baseline"
