#!/bin/bash
# Kernel trace + HBM bytes + SQ counters over the C3 configuration (tools/bench_configs.py C3:
# 100M fp64 global SUM/MIN/MAX/COUNT/AVG), on the GPU box; one rocprofv3 pass per counter group.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c3_pmc
rm -rf $OUT && mkdir -p $OUT
B="python3 tools/bench_configs.py C3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || exit 1
# the counters this box offers (for the TA pass below), then TA activity of the same kernels
rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
timeout -s KILL 200 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum --output-format csv -d $OUT/ta -o run -- $B > $OUT/ta.log 2>&1 || exit 1
