# round-4 closing measurements, part B: kernel traces (both shapes) and PMC passes
bash tools/trace_only.sh gpurun_out/r04g bench && bash tools/trace_only.sh gpurun_out/r04g bench16 --classes 16 --graphs 256 --steps 10 --warmup 3 --no-cpu-baseline --alt-paths , && bash tools/prof_pmc.sh gpurun_out/r04g_pmc
