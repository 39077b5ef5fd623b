#!/bin/bash
# Select-project full-tile loads: buffer descriptor (QE_SELPROJ_BUFLD=1) vs 64-bit addresses (0):
# parity tests with the look-back and two-pass modes, then C2 at 1B rows and the 10M calls.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c2b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_selproj.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # name, config, env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 tools/bench_configs.py $cfg > $OUT/$name.jsonl 2> $OUT/$name.err || return 1
  python3 - $OUT/$name.jsonl $name <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    print(sys.argv[2], round(d["ms"] * 1e3, 1), "us", round(d["frac"], 3), d["config"][:60])
PY
}
run b1 C2L QE_SELPROJ_BUFLD=1 && run b0 C2L QE_SELPROJ_BUFLD=0 && run b1b C2L QE_SELPROJ_BUFLD=1 && run b0b C2L QE_SELPROJ_BUFLD=0 && \
run b1_10m C2 QE_SELPROJ_BUFLD=1 && run b0_10m C2 QE_SELPROJ_BUFLD=0
