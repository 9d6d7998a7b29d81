# round-4 close: general graphs on the final tree (median of 5 runs)
SPARSE_DENSITIES=1.0,0.3 timeout -k 10 400 python tools/sparse_bench.py > gpurun_out/r04ar_sparse.txt 2>&1
