#!/bin/bash
# C3 (100M fp64 global aggregate) launch-shape A/B: QE_AG_PER_CU workgroups per CU, one process
# each (the knob is read once), then a kernel trace of the default shape. Output: gpurun_out/c3/.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c3
mkdir -p "$OUT"
for v in 4 5 8; do
  QE_AG_PER_CU=$v timeout -k 10 120 python3 tools/bench_configs.py C3 > "$OUT/c3_$v.json" 2>/dev/null || exit 1
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o c3 -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" C3 > "$OUT/trace.log" 2>&1
