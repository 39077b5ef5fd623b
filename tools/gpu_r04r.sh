#!/bin/bash
# Round 4 final tree: full GPU suite + smoke, then 1B rows around the compact-table ranges with the
# compact spill / two-pass on and off.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04r
mkdir -p $OUT
timeout -k 10 800 python3 -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_groups.py 1000000000 5500 6500 7000 8192 9500 10500 > $OUT/on.jsonl 2> $OUT/on.err || exit 1
QE_COMPACT_SPILL=0 timeout -k 10 200 python3 tools/bench_groups.py 1000000000 5500 6500 7000 8192 9500 10500 > $OUT/off.jsonl 2> $OUT/off.err || exit 1
