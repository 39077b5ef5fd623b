#!/bin/bash
# Partitioned GROUP BY with 32-bit records: the partitioned / two-bucket parity tests, then a knob
# sweep (1B rows, 64K and 1M groups, plus 4096 for the two-bucket path), one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/knobs
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "narrow or multipass or partitioned or spill or adapts or growth" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 python3 tools/bench_groups.py 1000000000 4096 65536 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err || return 1
  python3 -c "import json,sys; print('$name', [(d['groups'], round(d['update_ms'],2)) for d in map(json.loads, open('$OUT/$name.jsonl'))])"
}
run default QE_X=0 || exit 1
run walk0 QE_PAGG_WALK=0 || exit 1
run sdepth1 QE_PSCATTER_DEPTH=1 || exit 1
run sdepth3 QE_PSCATTER_DEPTH=3 || exit 1
run wg1 QE_PART_WG_PER_CU=1 || exit 1
run sblk1024 QE_PSCATTER_BLOCK=1024 || exit 1
run fill1 QE_PART_FILL_SHIFT=1 || exit 1
run default2 QE_X=0 || exit 1
run walk0b QE_PAGG_WALK=0 || exit 1
