#!/bin/bash
# C2 (10M rows) select-project knob A/B on one box: tools/bench_configs.py C2 per variant
# (CFG=C2L: the same kernel at 1B rows).
set -o pipefail
OUT=$1
shift
mkdir -p "$OUT"
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  echo "== $v" >> "$OUT/c2.txt"
  env $e timeout -k 10 120 python3 tools/bench_configs.py ${CFG:-C2} >> "$OUT/c2.txt" 2>> "$OUT/c2.err" || exit 1
done
