#!/bin/bash
# Spilling pass at 7,000 groups (1B rows, C4 shape) for kept shares of 4/8..7/8 of the compact
# table (QE_SPILL_LOAD), kernel trace per run:  bash tools/exp_spill_load.sh OUTDIR
set -o pipefail
export TMPDIR=/tmp
OUT=$1
mkdir -p "$OUT"
for L in 4 5 6 7; do
  QE_SPILL_LOAD=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/l$L" -o run -- python3 tools/bench_groups.py 1000000000 7000 > "$OUT/l$L.log" 2>&1 || exit 1
done
