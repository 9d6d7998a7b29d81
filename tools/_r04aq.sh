# round-4 close: configs[2] trace and PMC passes (guide for the node level)
bash tools/trace_only.sh gpurun_out/r04aq bench16 --classes 16 --graphs 256 --steps 10 --warmup 3 --no-cpu-baseline --alt-paths , && bash tools/prof_pmc.sh gpurun_out/r04aq_pmc --classes 16 --graphs 256 --steps 2 --warmup 1 --no-cpu-baseline --alt-paths ,
