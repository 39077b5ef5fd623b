#!/bin/bash
# Round 4: two-bucket hit window (fast aggregation pass, compact table), polled select-project
# completion: parity subsets, then the group sweep and C2 under kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_selproj.py \
  -k "partition or narrow or multipass or spill or adapts or compact or one_pass or knobs or select" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/groups -o run -- \
  python3 tools/bench_groups.py 1000000000 3500 4096 5000 65536 262144 1048576 > $OUT/groups.jsonl 2> $OUT/groups.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c2 -o run -- \
  python3 tools/bench_configs.py C2 > $OUT/c2.jsonl 2> $OUT/c2.err || exit 1
