#!/bin/bash
# Kernel trace of tools/step_breakdown.py (finalize / small-kernel timeline), on the GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/profstep
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/step_breakdown.py ${ROWS:-100000000} > $OUT/trace.log 2>&1
