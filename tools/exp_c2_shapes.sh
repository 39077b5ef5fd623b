#!/bin/bash
# Select-project launch-shape sweep at 1B rows (tools/bench_configs.py C2L) on the GPU box:
# rows per thread x resident workgroups per CU x tile order. One process per setting.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c2shapes
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 tools/bench_configs.py C2L > $OUT/$name.json 2> $OUT/$name.err || return 1
  echo "$name $(cat $OUT/$name.json)"
}
run lb1024 QE_SELPROJ_LB_BLOCK=1024 && \
run lb1024_w2 QE_SELPROJ_LB_BLOCK=1024 QE_SELPROJ_LBW=2 && \
run lb1024_w4 QE_SELPROJ_LB_BLOCK=1024 QE_SELPROJ_LBW=4 && \
run lb256_w4 QE_SELPROJ_LBW=4 && \
run lb512_w4 QE_SELPROJ_LB_BLOCK=512 QE_SELPROJ_LBW=4
