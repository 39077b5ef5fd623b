#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/profc2
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_configs.py C2 > $OUT/log 2>&1
