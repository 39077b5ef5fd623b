#!/bin/bash
# Round 4: resident select-project with the done word published after the last prefix: parity,
# then C2 and C3 twice (box-to-box and run-to-run spread of the synchronous calls).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04o
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_selproj.py \
  -k "resident or c2_shape or async" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py C2 C3 > $OUT/configs1.jsonl 2> $OUT/configs1.err || exit 1
timeout -k 10 300 python3 tools/bench_configs.py C2 C3 > $OUT/configs2.jsonl 2> $OUT/configs2.err || exit 1
