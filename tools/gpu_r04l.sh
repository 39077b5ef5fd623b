#!/bin/bash
# Round 4: parity of the parallel multi-row probe (fast aggregation pass, compact table), then at
# 1B rows: defaults, fuller fast tables (QE_PART_FAST_FILL=68), 4096-row scatter tiles (1024 threads).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04l
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "partition or narrow or adapts or knobs or compact" > $OUT/tests.txt 2>&1 || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 tools/bench_groups.py 1000000000 5000 65536 262144 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err
}
run def QE_X=1 || exit 1
run fill68 QE_PART_FAST_FILL=68 || exit 1
run b1024 QE_PSCATTER_BLOCK=1024 || exit 1
run b1024f68 QE_PSCATTER_BLOCK=1024 QE_PART_FAST_FILL=68 || exit 1
