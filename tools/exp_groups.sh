#!/bin/bash
# GROUP BY cardinality A/B on one box: tools/bench_groups.py ROWS G... per variant.
#   bash tools/exp_groups.sh OUTDIR ROWS "G G G" VARIANT...   (VARIANT: ENV=.. words, "-" = defaults)
set -o pipefail
OUT=$1; ROWS=$2; GS=$3
shift 3
mkdir -p "$OUT"
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  echo "== $v" >> "$OUT/groups.txt"
  env $e timeout -k 10 200 python3 tools/bench_groups.py $ROWS $GS >> "$OUT/groups.txt" 2>> "$OUT/groups.err" || exit 1
done
