#!/bin/bash
# Full GPU test suite (pytest -m gpu) with a per-test timeout, then smoke(); output under gpurun_out/$1.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tests_r04}
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit 1
