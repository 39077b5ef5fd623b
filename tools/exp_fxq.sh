#!/bin/bash
# A/B of the exact-SUM fused kernel's code shape on C5 (exact vs fast per variant), on the GPU box.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/fxq
mkdir -p $OUT
for v in "QE_FX_QUEUE=0 QE_FX_INLINE=0" "QE_FX_QUEUE=0 QE_FX_INLINE=1" "QE_FXQ_ROLL=1 QE_FX_INLINE=0" "QE_FXQ_ROLL=0 QE_FX_INLINE=0" "QE_FXQ_ROLL=1 QE_FX_INLINE=1" "QE_FXQ_ROLL=0 QE_FX_INLINE=1"; do
  echo "== $v" >> $OUT/ab.txt
  env $v timeout -k 10 120 python3 -u tools/exp_fp64_sum.py C5 --rounds 2 | grep summary >> $OUT/ab.txt || exit 1
done
