#!/bin/bash
# Kernel trace of the partitioned GROUP BY at 1B rows for the given group counts (per-kernel split).
#   bash tools/prof_groups_trace.sh OUTDIR "65536 1048576"
set -o pipefail
export TMPDIR=/tmp
OUT=$1
mkdir -p "$OUT"
for G in $2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g$G -o run -- python3 tools/bench_groups.py 1000000000 $G > $OUT/g$G.log 2>&1 || exit 1
done
