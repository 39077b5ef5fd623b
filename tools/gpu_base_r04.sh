#!/bin/bash
# Round-4 baseline on the unchanged round-3 tree: GROUP BY sweep at the VERDICT's regimes and the
# per-kernel split (rocprofv3 kernel trace) at 64K and 1M groups.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/base_r04
mkdir -p $OUT
timeout -k 10 300 python3 tools/bench_groups.py 1000000000 1024 4096 5000 65536 1048576 > $OUT/groups.jsonl 2> $OUT/groups.err || exit 1
bash tools/prof_groups_trace.sh $OUT/trace "65536 1048576" || exit 1
