#!/bin/bash
# Round 4: chain-hop latency far vs XCD-local; parity of the sized fast aggregation table and the
# register-resident select-project; group sweep (fast vs general aggregation pass, same box) and
# the C2 configs under kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 120 ./tools/_build/exp_xcd_chain > $OUT/chain.jsonl 2> $OUT/chain.err || exit 1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_selproj.py \
  tests/test_gpu_parity.py -k "c2 or nullable or async or persistent or partition or narrow or adapts or knobs" \
  > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c2 -o run -- \
  python3 tools/bench_configs.py C2 > $OUT/c2.jsonl 2> $OUT/c2.err || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 262144 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err
}
run def QE_X=1 || exit 1
run gen QE_PAGG_FAST=0 || exit 1
