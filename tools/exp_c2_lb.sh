#!/bin/bash
# C2 at 1B rows: look-back workgroup size A/B (1 x 1024 threads vs 2 x 512 resident per CU).
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c2lb
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 tools/bench_configs.py C2L > $OUT/$name.json 2> $OUT/$name.err || return 1
  echo "$name $(python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(round(d['ms'],3), round(d['frac'],3))")"
}
run lb1024_a QE_SELPROJ_LB_BLOCK=1024 && \
run lb512 QE_SELPROJ_LB_BLOCK=512 && \
run lb1024_b QE_SELPROJ_LB_BLOCK=1024 && \
run lb512_b QE_SELPROJ_LB_BLOCK=512 && \
run lb512_r8 QE_SELPROJ_LB_BLOCK=512 QE_SELPROJ_ROWS=8
