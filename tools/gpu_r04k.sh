#!/bin/bash
# Round 4: bucket count for the fast aggregation pass's own table (QE_PART_FAST_FILL), its 3-bucket
# hit window, and scatter workgroups per CU; 1B rows, same box, kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 262144 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err
}
run def QE_X=1 || exit 1
run fill50 QE_PART_FAST_FILL=50 || exit 1
run fill68 QE_PART_FAST_FILL=68 || exit 1
run fill68w3 QE_PART_FAST_FILL=68 QE_PAGG_WINDOW=3 || exit 1
run fill80w3 QE_PART_FAST_FILL=80 QE_PAGG_WINDOW=3 || exit 1
run wg3 QE_PART_WG_PER_CU=3 || exit 1
run wg4 QE_PART_WG_PER_CU=4 || exit 1
QE_HOST_PROFILE=1 timeout -k 10 200 python3 tools/bench_configs.py C2 > $OUT/c2_hostprof.jsonl 2> $OUT/c2_hostprof.err || exit 1
