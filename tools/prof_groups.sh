#!/bin/bash
# Kernel trace of tools/bench_groups.py (partitioned GROUP BY kernels), on the GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pgrp
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_groups.py ${ROWS:-200000000} ${GROUPS_LIST:-65536 262144 1048576} > $OUT/log 2>&1
