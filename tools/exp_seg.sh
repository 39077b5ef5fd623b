#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/seg
mkdir -p $OUT
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 tools/bench_configs.py C2L > $OUT/$tag.jsonl 2> $OUT/$tag.err || return 1
  python3 -c "import json; d=json.loads(open('$OUT/$tag.jsonl').readline()); print('$tag', round(d['ms'],4), round(d['frac'],3))"
}
QE_SELPROJ_AHEAD=2 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_selproj.py > $OUT/pytest.log 2>&1 || exit 1
run a2 QE_SELPROJ_SEG=1 QE_SELPROJ_OCC_MARGIN=0 QE_SELPROJ_AHEAD=2 && \
run a3 QE_SELPROJ_SEG=1 QE_SELPROJ_OCC_MARGIN=0 QE_SELPROJ_AHEAD=3 && \
run a2r8 QE_SELPROJ_SEG=1 QE_SELPROJ_OCC_MARGIN=0 QE_SELPROJ_AHEAD=2 QE_SELPROJ_ROWS=8 && \
run a4 QE_SELPROJ_SEG=1 QE_SELPROJ_OCC_MARGIN=0 QE_SELPROJ_AHEAD=4 && \
run lbm0 QE_SELPROJ_SEG=0 QE_SELPROJ_OCC_MARGIN=0
