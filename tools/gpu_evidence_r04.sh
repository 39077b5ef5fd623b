#!/bin/bash
# Round-4 evidence on one GPU. Mode A: bench.py (default N=1 line), the bench's kernel trace + PMC
# passes (profiles/run_profile.sh), the C2 call's trace + FETCH/WRITE/SQ passes. Mode B: the
# partitioned GROUP BY at 1B rows: kernel trace at 64K / 1M groups, FETCH / WRITE / SQ at 64K.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ev_r04
mkdir -p $OUT
if [ "$1" = "A" ]; then
  timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
  STEPS=3 timeout -k 10 900 bash profiles/run_profile.sh > $OUT/run_profile.log 2>&1 || exit 1
  CFG=C2 timeout -k 10 600 bash tools/prof_c2.sh > $OUT/prof_c2.log 2>&1 || exit 1
else
  timeout -k 10 1000 bash tools/prof_groups_narrow.sh > $OUT/groups.log 2>&1 || exit 1
fi
