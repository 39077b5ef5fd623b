#!/bin/bash
# Round 4: compact one-pass LDS table for groups just past the regular table (parity + 1B-row
# timings against the spilling two-bucket path), and aggregation-pass walk experiments.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/compact_r04d
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "compact or multipass or one_pass or spill" tests/test_fused_property.py > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_groups.py 1000000000 2500 3500 4096 5000 > $OUT/compact.jsonl 2> $OUT/compact.err || exit 1
QE_LDS_COMPACT=0 timeout -k 10 200 python3 tools/bench_groups.py 1000000000 2500 3500 4096 5000 > $OUT/spill.jsonl 2> $OUT/spill.err || exit 1
for e in 1 4; do
  QE_PAGG_EXP=$e timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/exp$e -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 > $OUT/exp$e.jsonl 2> $OUT/exp$e.err || exit 1
done
QE_PAGG_EXP=1 QE_PAGG_FAST_DEPTH=4 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/exp1d4 -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 > $OUT/exp1d4.jsonl 2> $OUT/exp1d4.err || exit 1
