#!/bin/bash
# Round measurement on the GPU box: the bench line, the rocprofv3 recipe (kernel trace + PMC
# passes; profiles/run_profile.sh) and a kernel trace of the N > 1 step (exchange leg on one GPU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
bash profiles/run_profile.sh && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/exch -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --exchange > gpurun_out/exch.json 2> gpurun_out/exch.err
