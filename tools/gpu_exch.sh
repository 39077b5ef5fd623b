#!/bin/bash
# Hash-aggregate parity tests, then a kernel trace of the N > 1 step (exchange leg on one GPU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ex2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "hashagg or fused or export or exchange or c4 or c5 or strkeys or tuple or determinism or import or global" > gpurun_out/ex2/pytest.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu --steps 10 > gpurun_out/ex2/bench.json 2> gpurun_out/ex2/bench.err && \
timeout -k 10 300 python3 bench.py --no-cpu --steps 10 --exchange > gpurun_out/ex2/bench_x.json 2> gpurun_out/ex2/bench_x.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ex2/trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --exchange > gpurun_out/ex2/trace.log 2>&1
