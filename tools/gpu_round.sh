set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_trace.log 2>&1
