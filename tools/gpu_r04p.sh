#!/bin/bash
# Round 4: spilling pass over the compact kept table (~5K-9.5K groups): parity, then 1B rows with
# it on and off (QE_COMPACT_SPILL=0: the 8-bucket partitioned path), kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04p
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "compact or multipass or spill" > $OUT/tests.txt 2>&1 || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 tools/bench_groups.py 1000000000 5000 5500 6500 8192 9000 > $OUT/$name.jsonl 2> $OUT/$name.err
}
run on QE_X=1 || exit 1
run off QE_COMPACT_SPILL=0 || exit 1
