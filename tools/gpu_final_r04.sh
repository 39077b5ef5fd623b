#!/bin/bash
# Round-4 final tree: bench line and every config on one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final_r04
mkdir -p $OUT
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 600 python3 tools/bench_configs.py C2 C2L C2LN C3 C4 C5 > $OUT/configs.jsonl 2> $OUT/configs.err || exit 1
