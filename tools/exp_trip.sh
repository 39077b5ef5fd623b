#!/bin/bash
# tripdata (K:1336) A/B on one box: tools/bench_tripdata.py per variant (ENV=.. words, "-" = defaults).
set -o pipefail
OUT=$1
shift
mkdir -p "$OUT"
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  echo "== $v" >> "$OUT/trip.txt"
  env $e timeout -k 10 200 python3 tools/bench_tripdata.py >> "$OUT/trip.txt" 2>> "$OUT/trip.err" || exit 1
done
