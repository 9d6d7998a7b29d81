set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06o_gputests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/r06o_bench.json 2> gpurun_out/r06o_bench.err || exit 3
timeout -k 10 150 python tools/op_det_probe.py 16 2394 128 bf16x6,bf16x3,mfma,mfma32 5 2>&1 | grep -v amdgpu.ids > gpurun_out/r06o_opdet.txt || exit 4
