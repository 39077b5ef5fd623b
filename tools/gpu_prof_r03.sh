#!/bin/bash
# Round-3 profiling call on the GPU box: the headline's rocprofv3 recipe (kernel trace + FETCH /
# WRITE / SQ / LDS passes, profiles/run_profile.sh) and the C5 kernel's SQ / LDS counters.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 bash profiles/run_profile.sh > gpurun_out/prof.log 2>&1 || exit 1
timeout -k 10 400 bash tools/prof_c5_pmc.sh > gpurun_out/c5pmc.log 2>&1 || exit 1
