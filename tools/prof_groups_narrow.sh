#!/bin/bash
# Partitioned GROUP BY with 32-bit records at 1B rows: per-kernel trace at 64K / 1M groups and the
# HBM bytes of the 64K case (FETCH_SIZE, WRITE_SIZE in separate passes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/gnarrow
mkdir -p $OUT
bash tools/prof_groups_trace.sh $OUT "65536 1048576" || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/g65536_fetch -o run -- python3 tools/bench_groups.py 1000000000 65536 > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/g65536_write -o run -- python3 tools/bench_groups.py 1000000000 65536 > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/g65536_sq -o run -- python3 tools/bench_groups.py 1000000000 65536 > $OUT/sq.log 2>&1 || exit 1
