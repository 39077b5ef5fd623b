#!/bin/bash
# C5 fused kernel: kernel trace + SQ / LDS counter passes per fp64 SUM mode (tools/exp_fp64_sum.py), on
# the GPU box. Output: gpurun_out/fp64_pmc/<mode>_{trace,sq,lds}/
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/fp64_pmc
rm -rf $OUT && mkdir -p $OUT
for MODE in ${MODES:-exact fast}; do
  B="python3 tools/exp_fp64_sum.py C5 --rounds 1 --mode $MODE"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${MODE}_trace -o run -- $B > $OUT/${MODE}_trace.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/${MODE}_sq -o run -- $B > $OUT/${MODE}_sq.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d $OUT/${MODE}_lds -o run -- $B > $OUT/${MODE}_lds.log 2>&1 || exit 1
done
