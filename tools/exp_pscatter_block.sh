#!/bin/bash
# Staged scatter workgroup size and prefetch depth with 32-bit records (1B rows), one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sblock
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 python3 tools/bench_groups.py 1000000000 8192 65536 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err || return 1
  python3 -c "import json,sys; print('$name', [(d['groups'], round(d['update_ms'],2), d['out_groups'] == d['groups']) for d in map(json.loads, open('$OUT/$name.jsonl'))])"
}
run b512 QE_X=0 || exit 1
run b256 QE_PSCATTER_BLOCK=256 || exit 1
run b256_wg4 QE_PSCATTER_BLOCK=256 QE_PART_WG_PER_CU=4 || exit 1
run b512_d1 QE_PSCATTER_DEPTH=1 || exit 1
run b256_d1_wg4 QE_PSCATTER_BLOCK=256 QE_PSCATTER_DEPTH=1 QE_PART_WG_PER_CU=4 || exit 1
run b512b QE_X=0 || exit 1
