#!/bin/bash
# GROUP BY just past the compact table (C4 shape, 1B rows): the spilling pass's reach
# (QE_SPILL_MAXPCT: spilled groups' share of the aggregation table) against the partitioned path.
# Output: gpurun_out/spill/.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/spill
mkdir -p "$OUT"
G="6000 7000 8192 9000"
timeout -k 10 300 python3 tools/bench_groups.py 1000000000 $G > "$OUT/base.jsonl" 2> "$OUT/base.err" || exit 1
for p in 60 70 80; do
  QE_SPILL_MAXPCT=$p timeout -k 10 300 python3 tools/bench_groups.py 1000000000 $G > "$OUT/p$p.jsonl" 2> "$OUT/p$p.err" || exit 1
done
