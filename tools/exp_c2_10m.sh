#!/bin/bash
# C2 at 10M rows: two-pass (default) against the single look-back pass, per call and back to back.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c2_10m
mkdir -p $OUT
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 tools/bench_configs.py C2 > $OUT/$name.jsonl 2> $OUT/$name.err || return 1
}
run twopass && run lookback QE_SELPROJ_TWOPASS=0 && run lookback256 QE_SELPROJ_TWOPASS=0 QE_SELPROJ_LB_BLOCK=256
