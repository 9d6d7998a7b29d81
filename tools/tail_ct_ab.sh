for ct in 8 16 32; do echo "== CT $ct"; PFSGNN_TAIL_CT=$ct PFSGNN_LIB_VARIANT=stamps timeout -k 10 200 python tools/tail_stamps.py 2>&1 | grep -v amdgpu.ids | head -9 || exit 1; done
for ct in 8 32; do echo "== bench CT $ct"; PFSGNN_TAIL_CT=$ct timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --alt-paths , 2>&1 | grep -o '"ms_per_step": [0-9.]*' || exit 1; done
