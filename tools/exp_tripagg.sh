#!/bin/bash
# Tripdata aggregate (3 groups, 4M rows): fused-kernel time against the fused grid size
# (QE_FUSED_MAX_WG), kernel trace per setting. Output: gpurun_out/tripagg/.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/tripagg
mkdir -p "$OUT"
for g in 0 32 64 128; do
  QE_FUSED_MAX_WG=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/g$g" -o run -- python3 tools/bench_tripdata.py 4000000 > "$OUT/g$g.log" 2>&1 || exit 1
done
