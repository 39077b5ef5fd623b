set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "hashagg or fused or export or exchange or c4 or c5 or strkeys or tuple or determinism" > gpurun_out/r02b/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r02b/bench.json 2> gpurun_out/r02b/bench.err && \
timeout -k 10 120 python3 tools/step_breakdown.py > gpurun_out/r02b/step.json 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02b/trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r02b/trace.log 2>&1 && \
true
