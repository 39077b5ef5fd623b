#!/bin/bash
# Round 4 last check: compact-table tests with the one-pass table filled to 92 %.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04x
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "compact or speculation or multipass or spill or adapts" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_groups.py 1000000000 5000 5500 5800 6000 6500 > $OUT/groups.jsonl 2> $OUT/groups.err || exit 1
