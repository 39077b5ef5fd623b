#!/bin/bash
# Round-3 final measurements on one box: the bench line (N=1), every BASELINE config
# (tools/bench_configs.py), the GROUP BY cardinality sweep.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
cd gpurun_out/final && rm -f *.json *.jsonl *.err && cd ../..
timeout -k 10 400 python3 bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit 1
timeout -k 10 400 python3 tools/bench_configs.py C2 C2L C2LN C3 C4 C5 > gpurun_out/final/configs.jsonl 2> gpurun_out/final/configs.err || exit 1
timeout -k 10 600 python3 tools/bench_groups.py 1000000000 1024 2048 2500 4096 5000 8192 65536 262144 1048576 4194304 > gpurun_out/final/groups.jsonl 2> gpurun_out/final/groups.err || exit 1
