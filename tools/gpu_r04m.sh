#!/bin/bash
# Round 4: the resident select-project walking rounds of tiles: parity, then C2 (10M) and the C2
# shape at 1B rows with rounds off (look-back single pass) and on, under kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04m
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_selproj.py \
  -k "resident or c2_shape" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/off -o run -- \
  python3 tools/bench_configs.py C2L > $OUT/off.jsonl 2> $OUT/off.err || exit 1
QE_SELPROJ_RESIDENT_ROUNDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/on -o run -- \
  python3 tools/bench_configs.py C2L > $OUT/on.jsonl 2> $OUT/on.err || exit 1
