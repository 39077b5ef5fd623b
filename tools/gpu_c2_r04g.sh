#!/bin/bash
# Round 4: host floor of a synchronous call (empty launches + event/stream/spin waits), then the
# C2 configs under a kernel trace (warm, cold and back-to-back calls).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c2_r04g
mkdir -p $OUT
timeout -k 10 120 ./tools/_build/exp_sync_latency > $OUT/sync.jsonl 2> $OUT/sync.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 tools/bench_configs.py C2 > $OUT/c2.jsonl 2> $OUT/c2.err || exit 1
