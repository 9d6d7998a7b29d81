for ks in 1 2 4; do PFSGNN_SL_KS=$ks SPARSE_DENSITIES=0.3,0.999 python tools/sparse_bench.py 2>&1 | grep edges | sed "s/^/KS=$ks /"; done
