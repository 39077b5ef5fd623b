#!/bin/bash
# Round 4: the fast aggregation pass for 32-bit chunked records. Partitioned parity tests, then
# 1B rows at 64K / 1M groups under a kernel trace: general pass (QE_PAGG_FAST=0) against the fast
# pass with 2 and 4 rotating record buffers.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pagg_r04${1:-}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "partition or narrow or multipass or spill or adapts" > $OUT/tests.txt 2>&1 || exit 1
for cfg in "QE_PAGG_FAST=0" "QE_PAGG_FAST_DEPTH=2" "QE_PAGG_FAST_DEPTH=4"; do
  export $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${cfg} -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 1048576 > $OUT/${cfg}.jsonl 2> $OUT/${cfg}.err || exit 1
  unset QE_PAGG_FAST QE_PAGG_FAST_DEPTH
done
