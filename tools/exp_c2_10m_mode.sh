#!/bin/bash
# C2 at 10M rows: auto (two-pass) against the look-back pass with next-tile prefetch.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c2m
mkdir -p $OUT
for v in auto 0 auto 0; do
  if [ $v = auto ]; then e=""; else e="QE_SELPROJ_TWOPASS=$v"; fi
  env $e timeout -k 10 120 python3 tools/bench_configs.py C2 > $OUT/c2_$v.jsonl 2> $OUT/c2_$v.err || exit 1
  python3 - $OUT/c2_$v.jsonl $v <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    print(sys.argv[2], round(d["ms"] * 1e3, 1), "us", d.get("call_ms") and round(d["call_ms"] * 1e3, 1), d["config"][:70])
PY
done
