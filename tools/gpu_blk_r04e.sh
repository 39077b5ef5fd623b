#!/bin/bash
# Round 4: blocks-of-64 record layout (fast scatter + fast aggregation pass, bucketized 32-bit key
# tables) and the compact fused table with 4-slot buckets: parity, then 1B-row sweeps against the
# record-major layout (QE_PSCATTER_FAST=0) and the spilling path (QE_LDS_COMPACT=0).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/blk_r04e
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "partition or narrow or multipass or spill or adapts or compact or one_pass" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/def -o run -- \
  python3 tools/bench_groups.py 1000000000 3500 4096 5000 65536 1048576 > $OUT/def.jsonl 2> $OUT/def.err || exit 1
QE_PSCATTER_FAST=0 QE_LDS_COMPACT=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/old -o run -- \
  python3 tools/bench_groups.py 1000000000 3500 4096 5000 65536 1048576 > $OUT/old.jsonl 2> $OUT/old.err || exit 1
