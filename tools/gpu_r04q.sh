#!/bin/bash
# Round 4: compact-spill range capped: parity, then 1B rows around the cap.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "compact or multipass or spill or speculation" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_groups.py 1000000000 5500 6500 6700 7000 8192 > $OUT/groups.jsonl 2> $OUT/groups.err || exit 1
