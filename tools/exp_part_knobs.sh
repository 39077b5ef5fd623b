#!/bin/bash
# Partitioned GROUP BY knob sweep with 32-bit records (1B rows, 64K and 1M groups), one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/knobs
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 python3 tools/bench_groups.py 1000000000 65536 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err || return 1
  python3 -c "import json,sys; print('$name', [(d['groups'], round(d['update_ms'],2)) for d in map(json.loads, open('$OUT/$name.jsonl'))])"
}
run default QE_X=0 || exit 1
run sdepth1 QE_PSCATTER_DEPTH=1 || exit 1
run sdepth3 QE_PSCATTER_DEPTH=3 || exit 1
run wg1 QE_PART_WG_PER_CU=1 || exit 1
run wg4 QE_PART_WG_PER_CU=4 || exit 1
run sblk256 QE_PSCATTER_BLOCK=256 || exit 1
run sblk1024 QE_PSCATTER_BLOCK=1024 || exit 1
run pdepth2 QE_PAGG_DEPTH=2 || exit 1
run fill1 QE_PART_FILL_SHIFT=1 || exit 1
run pblk512 QE_PAGG_BLOCK=512 || exit 1
run default2 QE_X=0 || exit 1
