#!/bin/bash
# Partitioned GROUP BY aggregation slices per CU (QE_PAGG_SLICES_PER_CU), 1B rows, one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/slices
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 python3 tools/bench_groups.py 1000000000 8192 65536 262144 1048576 > $OUT/$name.jsonl 2> $OUT/$name.err || return 1
  python3 -c "import json,sys; print('$name', [(d['groups'], round(d['update_ms'],2), d['out_groups'] == d['groups']) for d in map(json.loads, open('$OUT/$name.jsonl'))])"
}
run spc8 QE_X=0 || exit 1
run spc4 QE_PAGG_SLICES_PER_CU=4 || exit 1
run spc2 QE_PAGG_SLICES_PER_CU=2 || exit 1
run spc1 QE_PAGG_SLICES_PER_CU=1 || exit 1
run spc16 QE_PAGG_SLICES_PER_CU=16 || exit 1
run spc8b QE_X=0 || exit 1
