#!/bin/bash
# C2 (10M rows) call anatomy: kernel trace of tools/bench_configs.py C2 (two-pass default and the
# look-back single pass), so the cold calls' kernels and the gaps between them can be read off.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c2_r04${1:-}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/twopass -o run -- \
  python3 tools/bench_configs.py C2 > $OUT/twopass.jsonl 2> $OUT/twopass.err || exit 1
QE_SELPROJ_TWOPASS=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/lookback -o run -- \
  python3 tools/bench_configs.py C2 > $OUT/lookback.jsonl 2> $OUT/lookback.err || exit 1
