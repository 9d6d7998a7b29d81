set -e
for v in base slnoacc slnoacclds slgtab slgtabnoacc; do
  echo "== $v"
  if [ $v = base ]; then unset PFSGNN_LIB_VARIANT; else export PFSGNN_LIB_VARIANT=$v; fi
  SPARSE_DENSITIES=0.3 SPARSE_RUNS=3 timeout -k 10 200 python -u tools/sparse_bench.py 2>&1 | grep -v amdgpu.ids
done
