#!/bin/bash
# Round 4: fast staged scatter (LDS records before the scan, index permutation, 2 workgroups/CU)
# and fast aggregation pass. Parity subset, kernel traces (scatter fast on/off), then PMC passes at
# 64K groups for the fast kernels and the general aggregation pass.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/part_r04b
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "partition or narrow or multipass or spill or adapts" > $OUT/tests.txt 2>&1 || exit 1
for cfg in "QE_PSCATTER_FAST=0" "QE_PSCATTER_FAST=1"; do
  export $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${cfg} -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 1048576 > $OUT/${cfg}.jsonl 2> $OUT/${cfg}.err || exit 1
  unset QE_PSCATTER_FAST
done
QE_PAGG_EXP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/exp1 -o run -- \
    python3 tools/bench_groups.py 1000000000 65536 1048576 > $OUT/exp1.jsonl 2> $OUT/exp1.err || exit 1
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM"
for tag in fast gen; do
  if [ $tag = gen ]; then export QE_PAGG_FAST=0; fi
  i=0
  for set in FETCH_SIZE WRITE_SIZE "$SQ1" "$SQ2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_${tag}_$i -o run -- \
      python3 tools/bench_groups.py 1000000000 65536 > $OUT/pmc_${tag}_$i.log 2>&1 || exit 1
  done
  unset QE_PAGG_FAST
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit 1
