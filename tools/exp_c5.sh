#!/bin/bash
# C5 workgroup shape A/B on one box: tools/bench_configs.py C5 per variant (ENV=.. words, "-" = defaults).
set -o pipefail
OUT=$1
shift
mkdir -p "$OUT"
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  echo "== $v" >> "$OUT/c5.txt"
  env $e timeout -k 10 120 python3 tools/bench_configs.py C5 >> "$OUT/c5.txt" 2>> "$OUT/c5.err" || exit 1
done
