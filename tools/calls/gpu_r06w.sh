# final-tree check: GPU tests, smoke(), bench (default flags, as the driver runs it)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06w_gputests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06w_smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/r06w_bench.json 2> gpurun_out/r06w_bench.err || exit 3
