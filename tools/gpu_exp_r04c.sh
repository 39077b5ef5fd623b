#!/bin/bash
# Round 4 experiments: aggregation pass reading each slice's chunks as one contiguous range
# (QE_PAGG_EXP=2, timing only) and without its flush (3); the C2 call anatomy.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/exp_r04c
mkdir -p $OUT
for e in 2 3; do
  QE_PAGG_EXP=$e timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/exp$e -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 1048576 > $OUT/exp$e.jsonl 2> $OUT/exp$e.err || exit 1
done
bash tools/prof_c2_r04.sh || exit 1
