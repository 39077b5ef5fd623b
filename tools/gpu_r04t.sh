#!/bin/bash
# Round 4: step-interleaved walk of the fast aggregation pass: parity, then 1B rows on / off.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04t
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "knobs" > $OUT/tests.txt 2>&1 || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 262144 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err
}
run off QE_X=1 || exit 1
run on QE_PAGG_INTERLEAVE=1 || exit 1
run off2 QE_X=1 || exit 1
run on2 QE_PAGG_INTERLEAVE=1 || exit 1
