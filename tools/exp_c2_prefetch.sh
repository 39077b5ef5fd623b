#!/bin/bash
# Select-project next-tile prefetch (QE_SELPROJ_PREFETCH) on/off and its launch shape: parity
# tests, then C2 at 1B rows (the look-back path), alternating settings on one box.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c2pf
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_selproj.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # name, config, env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 tools/bench_configs.py $cfg > $OUT/$name.json 2> $OUT/$name.err || return 1
  echo "$name $(python3 -c "import json; d=json.load(open('$OUT/$name.json')); print(round(d['ms'],4), round(d['frac'],3))")"
}
run pf C2L QE_SELPROJ_PREFETCH=1 && run nopf C2L QE_SELPROJ_PREFETCH=0 && \
run pf_lb512 C2L QE_SELPROJ_LB_BLOCK=512 && run pf_lbw2 C2L QE_SELPROJ_LBW=2 && \
run pf_r8 C2L QE_SELPROJ_ROWS=8 && run pf_b C2L QE_SELPROJ_PREFETCH=1
