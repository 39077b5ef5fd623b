#!/bin/bash
# Kernel trace + PMC passes over the select-project configuration (tools/bench_configs.py C2 C2L:
# 10M rows and the same kernel at 1B rows), on the GPU box. One rocprofv3 run per counter pass.
#   bash tools/prof_c2.sh            -> gpurun_out/profc2/{trace,fetch,write,sq}
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/profc2
rm -rf $OUT && mkdir -p $OUT
B="python3 tools/bench_configs.py ${CFG:-C2 C2L}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || exit 1
