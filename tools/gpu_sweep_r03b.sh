#!/bin/bash
# Round-3 (second session) sweep on the final tree: every BASELINE config (tools/bench_configs.py) and
# the GROUP BY cardinality sweep at 1B rows.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep_b
timeout -k 10 400 python3 tools/bench_configs.py C2 C2L C2LN C3 C4 C5 > gpurun_out/sweep_b/configs.jsonl 2> gpurun_out/sweep_b/configs.err || exit 1
timeout -k 10 600 python3 tools/bench_groups.py 1000000000 1024 2048 2500 4096 5000 8192 65536 262144 1048576 4194304 > gpurun_out/sweep_b/groups.jsonl 2> gpurun_out/sweep_b/groups.err || exit 1
python3 -c "import json; [print(d.get('config', d.get('groups')), {k: v for k, v in d.items() if k in ('update_ms', 'ms', 'call_ms', 'kernel_ms', 'frac')}) for d in map(json.loads, open('gpurun_out/sweep_b/groups.jsonl'))]"
