for wb in 256 128 64 32; do
  PFSGNN_WG_BLOCKS=$wb timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/wb$wb.log 2>&1 || exit 1
  echo "wb=$wb $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wb$wb.log)"
done
