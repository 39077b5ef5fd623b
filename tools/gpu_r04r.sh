#!/bin/bash
# Round 4: compact two-pass (~6.75K-10K groups): parity, then 1B rows with it on / off.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04r
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "compact or multipass or spill or speculation" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_groups.py 1000000000 5500 6500 7000 8192 9500 10500 > $OUT/on.jsonl 2> $OUT/on.err || exit 1
QE_COMPACT_SPILL=0 timeout -k 10 300 python3 tools/bench_groups.py 1000000000 5500 6500 7000 8192 9500 10500 > $OUT/off.jsonl 2> $OUT/off.err || exit 1
