#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 process each) of a short bench
# run under an environment setting:  bash tools/fetch_ab.sh <outdir> <tag> [VAR=val ...]
out=$1; tag=$2; shift 2
root=$(pwd)
mkdir -p "$root/$out"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  env "$@" timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d "$root/$out/${tag}_$c" -o run -- \
    python3 "$root/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --alt-paths , \
    > "$root/$out/${tag}_$c.log" 2>&1 || { echo "[fetch_ab $tag $c] failed"; exit 1; }
  echo "[fetch_ab $tag $c] ok"
done
