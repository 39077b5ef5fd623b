#!/bin/bash
# Round-4 final tree: GROUP BY cardinality sweep at 1B rows (C4 shape) under a kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sweep_r04
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 tools/bench_groups.py 1000000000 1024 2048 2500 3500 4096 5000 8192 65536 262144 1048576 4194304 \
  > $OUT/sweep.jsonl 2> $OUT/sweep.err || exit 1
