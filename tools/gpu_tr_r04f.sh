#!/bin/bash
# Round 4: fast aggregation pass with LDS-regrouped contiguous loads, branch-free bucketized key
# tables, compact fused table: parity, then same-box A/B at 1B rows.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/tr_r04f
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "partition or narrow or multipass or spill or adapts or compact or one_pass" > $OUT/tests.txt 2>&1 || exit 1
run() {  # name, env..., groups
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 tools/bench_groups.py 1000000000 3500 4096 5000 65536 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err
}
run def QE_X=1 || exit 1
run notr QE_PAGG_TRANSPOSE=0 || exit 1
run r03 QE_PAGG_FAST=0 QE_PSCATTER_FAST=0 QE_LDS_COMPACT=0 || exit 1
