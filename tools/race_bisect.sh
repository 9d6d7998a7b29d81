#!/bin/bash
# Round 6's bisection of the km_source_fwd_ft run-to-run race
# (profiles/r06m_race_bisect.txt, DESIGN.md "The km_source_fwd_ft race, found").
#   bash tools/race_bisect.sh build   # here: the variant libraries (tools/variants.sh)
#   bash tools/race_bisect.sh run     # on the GPU box: op determinism per variant
# The bisection ran on the tree BEFORE the fix, where the Pebay coefficients were
# a per-block LDS table; on the fixed tree MF_PEB_CONST=0 restores that table, so
# every variant below adds it to reproduce the race (the LDS weight tuples on:
# MF_EFWD_B6S=1 MF_SFT_B6S=3, the library default).
#   lds      the old table (reproduces: M3 / M4 of channels 15 and 17 differ)
#   nob6s    the old table, register weight tuples (no race seen)
#   sft1     the old table, only L1's tuples in LDS (races)
#   nokeep   the old table, MF_SRC_KEEP=0 (about 20x more)
#   pin      the old table, MF_SRC_PIN=3 (no race seen)
#   noslp    the old table, -fno-slp-vectorize: no packed-fp32 FMAs (no race)
#   diag     the old table, every fold's rows compared in-kernel with c_peb
#            (MF_PEB_DIAG: a printf per mismatch; none, while the race stays)
# and the fixed tree's default (c_peb, scalar loads), with and without the tie.
set -o pipefail
cd "$(dirname "$0")/.."
case "$1" in
build)
  P="-DMF_PEB_CONST=0 -DMF_SRC_KEEP=1"
  # (four at a time: each pair of hipcc processes takes a few GB)
  bash tools/variants.sh lds "$P" nob6s "$P -DMF_EFWD_B6S=0 -DMF_SFT_B6S=0" \
    sft1 "$P -DMF_SFT_B6S=1" nokeep "-DMF_PEB_CONST=0 -DMF_SRC_KEEP=0" || exit 1
  bash tools/variants.sh pin "$P -DMF_SRC_PIN=3" noslp "$P -fno-slp-vectorize" \
    fixed "-DMF_SRC_KEEP=1" fixednokeep "-DMF_SRC_KEEP=0" || exit 1
  bash tools/variants.sh diag "$P -DMF_PEB_DIAG" || exit 1
  ;;
run)
  mkdir -p gpurun_out
  for v in lds nob6s sft1 nokeep pin noslp fixed fixednokeep diag; do
    PFSGNN_LIB_VARIANT=$v timeout -k 10 150 python tools/op_det_probe.py 16 2394 128 bf16x6 5 2>&1 |
      grep -e source_fwd -e PEBDIAG | sed "s/^/$v /" >> gpurun_out/race_bisect.txt || exit 2
  done
  PFSGNN_LIB_VARIANT=lds timeout -k 10 150 python tools/op_det_where.py 16 2394 128 bf16x6 4 \
    > gpurun_out/race_where.txt 2>&1 || exit 3
  ;;
*) echo "usage: $0 build|run" >&2; exit 1 ;;
esac
