#!/bin/bash
# Host-overhead A/B on one box: blocking vs polled stream waits (bench step vs fused kernel).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/sync
mkdir -p $OUT
for rep in 1 2; do
for v in block spin; do
  QE_SYNC=$v timeout -k 10 120 python3 tools/step_breakdown.py > $OUT/step_${v}_$rep.json 2>/dev/null || exit 1
  echo "$v $rep $(tail -1 $OUT/step_${v}_$rep.json)"
done
done
