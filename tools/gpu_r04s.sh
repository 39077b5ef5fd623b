#!/bin/bash
# Round 4 final: compact-table tests after the two-pass became opt-in.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04s
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "compact or speculation or multipass or spill" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_global_partial.py \
  tests/test_config_sizes.py tests/test_arrow_io.py > $OUT/tests2.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_configs.py C3 > $OUT/c3.jsonl 2> $OUT/c3.err || exit 1
