#!/bin/bash
# Round 4: where the fast aggregation pass loses at 1M groups (walk only / no flush / general
# pass), plus the host floor of a synchronous call and the C2 configs under a kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pagg_r04h
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 262144 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err
}
run def QE_X=1 || exit 1
run walk QE_PAGG_EXP=1 || exit 1
run noflush QE_PAGG_EXP=3 || exit 1
run gen QE_PAGG_FAST=0 || exit 1
run d4 QE_PAGG_FAST_DEPTH=4 || exit 1
C2=gpurun_out/c2_r04g
mkdir -p $C2
timeout -k 10 120 ./tools/_build/exp_sync_latency > $C2/sync.jsonl 2> $C2/sync.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $C2/trace -o run -- \
  python3 tools/bench_configs.py C2 > $C2/c2.jsonl 2> $C2/c2.err || exit 1
