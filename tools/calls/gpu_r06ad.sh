# configs[2] (256 graphs of 2394x16) on the final tree, bf16x6 headline and the other paths beside it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --classes 16 --graphs 256 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r06ad_bench16.json 2> gpurun_out/r06ad_bench16.err || exit 2
