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
run pipe && \
run pipe_wg6 QE_SELPROJ_WG_PER_CU=6 QE_SELPROJ_OCC_MARGIN=0 && \
run pipe_wg8 QE_SELPROJ_WG_PER_CU=8 QE_SELPROJ_OCC_MARGIN=0 && \
run pipe_wave QE_SELPROJ_MAP=wave && \
run pipe_r16 QE_SELPROJ_ROWS=16 && \
run nopipe_wg6 QE_SELPROJ_PIPE=0 QE_SELPROJ_WG_PER_CU=6 QE_SELPROJ_OCC_MARGIN=0 && \
run nopipe QE_SELPROJ_PIPE=0
