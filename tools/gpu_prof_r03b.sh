#!/bin/bash
# Round-3 (second session): the 32-bit record tests (partitioned + spilling GROUP BY), the
# two-bucket A/B (32-bit vs 64-bit spill records), the headline's rocprofv3 trace + PMC passes
# (profiles/run_profile.sh, refreshes traffic.json for the current fused-kernel signature), then the
# 32-bit partitioned GROUP BY trace and counters (tools/prof_groups_narrow.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "narrow or multipass or partitioned or spill" > gpurun_out/r3b/tests.log 2>&1 || { tail -40 gpurun_out/r3b/tests.log; exit 1; }
tail -2 gpurun_out/r3b/tests.log
timeout -k 10 200 python3 tools/bench_groups.py 1000000000 4096 5000 > gpurun_out/r3b/mp_n32.jsonl 2> gpurun_out/r3b/mp_n32.err || exit 1
QE_PART_NARROW=0 timeout -k 10 200 python3 tools/bench_groups.py 1000000000 4096 5000 > gpurun_out/r3b/mp_wide.jsonl 2> gpurun_out/r3b/mp_wide.err || exit 1
cat gpurun_out/r3b/mp_n32.jsonl gpurun_out/r3b/mp_wide.jsonl
bash profiles/run_profile.sh || exit 1
bash tools/prof_groups_narrow.sh || exit 1
