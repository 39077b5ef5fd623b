#!/bin/bash
# Round-3 narrow partition records: the GPU suite (incl. the 32-bit record tests), the bench line,
# then the GROUP BY sweep at 1B rows with 32-bit records (default) and with QE_PART_NARROW=0.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/narrow
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/narrow/gputests.log 2>&1 || { tail -40 gpurun_out/narrow/gputests.log; exit 1; }
tail -3 gpurun_out/narrow/gputests.log
timeout -k 10 300 python3 bench.py > gpurun_out/narrow/bench.json 2> gpurun_out/narrow/bench.err || exit 1
cat gpurun_out/narrow/bench.json
timeout -k 10 300 python3 tools/bench_groups.py 1000000000 8192 65536 262144 1048576 4194304 > gpurun_out/narrow/groups_n32.jsonl 2> gpurun_out/narrow/groups_n32.err || exit 1
QE_PART_NARROW=0 timeout -k 10 300 python3 tools/bench_groups.py 1000000000 8192 65536 262144 1048576 4194304 > gpurun_out/narrow/groups_wide.jsonl 2> gpurun_out/narrow/groups_wide.err || exit 1
cat gpurun_out/narrow/groups_n32.jsonl gpurun_out/narrow/groups_wide.jsonl
