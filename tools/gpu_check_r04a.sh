#!/bin/bash
# Round-4 correctness changes on the GPU: deterministic-mode status word, generic-kernel LDS
# budget, JNI harness (Utf8 MAX, chunked CSV scan), pipelined select-project drain, bench N>1 default check.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/check_r04a
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_determinism.py tests/test_gpu_parity.py::test_generic_kernel_lds_budget tests/test_jni_shim.py \
  tests/test_selproj.py tests/test_bench_dist.py > gpurun_out/check_r04a/tests.txt 2>&1
