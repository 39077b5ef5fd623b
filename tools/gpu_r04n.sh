#!/bin/bash
# Round 4: polled global aggregate: its parity tests, then every config (C2 C2L C2LN C3 C4 C5).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_global_partial.py \
  tests/test_config_sizes.py tests/test_gpu_parity.py -k "global or c3 or C3 or config" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 600 python3 tools/bench_configs.py C2 C2L C2LN C3 C4 C5 > $OUT/configs.jsonl 2> $OUT/configs.err || exit 1
