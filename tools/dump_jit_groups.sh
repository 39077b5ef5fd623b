#!/bin/bash
# JIT kernel sources of the GROUP BY paths at the given group counts (1B rows, C4 shape), for
# offline ISA inspection:  bash tools/dump_jit_groups.sh OUTDIR "5800 7000"
set -o pipefail
export TMPDIR=/tmp
OUT=$1
mkdir -p "$OUT/src"
export QE_JIT_DUMP=$OUT/src
timeout -k 10 200 python3 tools/bench_groups.py 1000000000 $2 > "$OUT/groups.jsonl" 2> "$OUT/groups.err"
