#!/bin/bash
# Fused C4 kernel variants (QE_FUSED_PF / QE_FUSED_BLOCK) at 1B rows, on the GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/expf
mkdir -p $OUT/src
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 150 python3 bench.py --no-cpu --steps 10 --warmup 2 > $OUT/$tag.json 2> $OUT/$tag.err || return 1
  python3 -c "import json,sys; d=json.load(open('$OUT/$tag.json')); r=d['roofline']; print('$tag', round(r['avg_kernel_ms'],4), round(d['ms_per_step'],4), round(r['frac'],4))"
}
run base QE_JIT_DUMP=$OUT/src QE_FUSED_PF=0 && \
run pf QE_FUSED_PF=1 && \
run b1024 QE_FUSED_BLOCK=1024 && \
run pf_b1024 QE_FUSED_PF=1 QE_FUSED_BLOCK=1024 && \
run b256 QE_FUSED_BLOCK=256 && \
run base2 QE_FUSED_PF=0 && \
QE_JIT_DUMP=$OUT/src QE_FUSED_PF=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_property.py tests/test_gpu_parity.py -k "fused or random or hashagg or c5" > $OUT/pytest_pf.log 2>&1 && \
QE_FUSED_BLOCK=1024 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_property.py > $OUT/pytest_b1024.log 2>&1 && \
timeout -k 10 120 python3 tools/step_breakdown.py > $OUT/step.json 2>&1
