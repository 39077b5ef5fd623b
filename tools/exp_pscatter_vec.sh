#!/bin/bash
# Staged scatter: per-workgroup chunk id ranges (QE_PART_STATIC), reload after the scan
# (QE_PSCATTER_RELOAD), 16-byte vector prefetch buffers loaded unconditionally (QE_PSCATTER_VEC=2),
# double-buffered aggregation pass (QE_PAGG_WALK=2), each against the previous form, at prefetch depths 1-3 (1B rows, 64K and 1M groups), one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/vec
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "partitioned or multipass or narrow or spill or tiny or adapts" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 python3 tools/bench_groups.py 1000000000 8192 65536 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err || return 1
  python3 -c "import json,sys; print('$name', [(d['groups'], round(d['update_ms'],2)) for d in map(json.loads, open('$OUT/$name.jsonl'))])"
}
run new QE_X=0 || exit 1
run walk1 QE_PAGG_WALK=1 || exit 1
run static0 QE_PART_STATIC=0 || exit 1
run reload0 QE_PART_STATIC=0 QE_PSCATTER_RELOAD=0 || exit 1
run old QE_PART_STATIC=0 QE_PSCATTER_RELOAD=0 QE_PSCATTER_VEC=0 QE_PAGG_WALK=1 || exit 1
run new_d1 QE_PSCATTER_DEPTH=1 || exit 1
run new2 QE_X=0 || exit 1
