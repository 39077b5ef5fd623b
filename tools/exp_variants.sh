#!/bin/bash
# A/B of fused-kernel environment knobs on one box: bench.py --no-cpu once per variant.
#   bash tools/exp_variants.sh OUTDIR "ENV=.. ENV=.." "ENV=.." ...   ("-" = defaults)
set -o pipefail
export TMPDIR=/tmp
OUT=$1
shift
mkdir -p "$OUT"
i=0
for v in "$@"; do
  i=$((i + 1))
  if [ "$v" = "-" ]; then v=""; fi
  echo "variant $i: $v" >> "$OUT/variants.txt"
  env $v timeout -k 10 240 python3 bench.py --no-cpu --steps ${STEPS:-20} --warmup 3 > "$OUT/v$i.json" 2> "$OUT/v$i.err" || exit 1
done
