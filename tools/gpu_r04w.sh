#!/bin/bash
# Round 4: how full the one-pass compact table may run (QE_COMPACT_LOAD percent); 1B rows.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04w
mkdir -p $OUT
for L in 80 88 92; do
  QE_COMPACT_LOAD=$L timeout -k 10 200 python3 tools/bench_groups.py 1000000000 5000 5400 5700 > $OUT/load$L.jsonl 2> $OUT/load$L.err || exit 1
done
