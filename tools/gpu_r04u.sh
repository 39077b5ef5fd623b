#!/bin/bash
# Round 4: kept share of the compact spill (QE_SPILL_LOAD eighths) and aggregation slices per CU
# for the fast pass; 1B rows, one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04u
mkdir -p $OUT
for L in 5 6 7; do
  QE_SPILL_LOAD=$L timeout -k 10 200 python3 tools/bench_groups.py 1000000000 5500 6500 > $OUT/load$L.jsonl 2> $OUT/load$L.err || exit 1
done
for S in 4 8 16; do
  QE_PAGG_SLICES_PER_CU=$S timeout -k 10 200 python3 tools/bench_groups.py 1000000000 65536 1048576 > $OUT/slices$S.jsonl 2> $OUT/slices$S.err || exit 1
done
