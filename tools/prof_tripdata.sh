#!/bin/bash
# Kernel trace of tools/bench_tripdata.py (CSV scan -> CAST -> string-keyed GROUP BY), on the GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/proftrip
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_tripdata.py ${ROWS:-4000000} > $OUT/trace.log 2>&1
