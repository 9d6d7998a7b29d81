bash tools/gpu_run.sh \
 "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py" \
 "ktrace:300:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/kt -o run -- python3 $PWD/bench.py --steps 10 --warmup 3 --no-cpu-baseline"
