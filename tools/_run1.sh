bash tools/gpu_run.sh \
 "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py --no-cpu-baseline"
