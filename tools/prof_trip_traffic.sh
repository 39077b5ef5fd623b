#!/bin/bash
# HBM traffic of the tripdata kernels (K:1336 query, tools/bench_tripdata.py): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes (TCC counters do not fit one pass), on the GPU box.
# Output: gpurun_out/triptraffic/{fetch,write}/ ; summarise with tools/trip_traffic.py.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/triptraffic
mkdir -p $OUT
B="python3 tools/bench_tripdata.py ${ROWS:-4000000}"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit 1
