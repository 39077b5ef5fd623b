#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sx
for v in "-" "QE_MP_SPILL=0"; do
  e=$v; [ "$e" = "-" ] && e=""
  echo "== $v" >> gpurun_out/sx/k.txt
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sx/t -o run -- python3 tools/bench_groups.py 1000000000 4096 5000 > gpurun_out/sx/log.txt 2>&1 || exit 1
  cut -c1-100 gpurun_out/sx/log.txt | grep groups >> gpurun_out/sx/k.txt; cut -d, -f1-4 gpurun_out/sx/t/run_kernel_stats.csv | grep -E "qe_fused|qe_pagg" >> gpurun_out/sx/k.txt
done
