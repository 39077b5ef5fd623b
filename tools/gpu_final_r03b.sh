#!/bin/bash
# Round-3 (second session) final check on one box: the full GPU suite, smoke(), the bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final_b
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_b/gputests.log 2>&1 || { tail -40 gpurun_out/final_b/gputests.log; exit 1; }
tail -2 gpurun_out/final_b/gputests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_b/smoke.log 2>&1 || { tail -20 gpurun_out/final_b/smoke.log; exit 1; }
tail -1 gpurun_out/final_b/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/final_b/bench.json 2> gpurun_out/final_b/bench.err || exit 1
cat gpurun_out/final_b/bench.json
