#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over tools/fetch_calib (known byte counts).
# Usage (GPU box, repo root): bash tools/calib_pmc.sh <outdir>
out=$1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
mkdir -p "$root/$out"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d "$root/$out/$c" -o run -- \
    "$root/tools/fetch_calib" > "$root/$out/$c.log" 2>&1
  rc=$?; echo "[calib $c] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
