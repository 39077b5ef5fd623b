#!/bin/bash
# Round-3 GPU check: full GPU suite, then the C4 bench with the exchange leg on one rank (torch
# all-to-all and the native RCCL communicator).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 300 python3 bench.py --exchange --no-cpu --steps 20 --warmup 3 > gpurun_out/exch.json 2> gpurun_out/exch.err || exit 1
timeout -k 10 300 python3 bench.py --exchange --exchange-impl native --no-cpu --steps 20 --warmup 3 > gpurun_out/exch_native.json 2> gpurun_out/exch_native.err || exit 1
for f in exch exch_native; do grep '^{' gpurun_out/$f.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', d['ms_per_step'], d['kernel_ms'], d['exchange_ms'])"; done
