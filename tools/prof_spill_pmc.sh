#!/bin/bash
# Counters of the one-pass compact GROUP BY (5,800 groups) against the spilling pass (7,000 groups),
# 1B rows, C4 shape: SQ instruction / wait counters, then HBM bytes, in separate rocprofv3 passes.
#   bash tools/prof_spill_pmc.sh OUTDIR
set -o pipefail
export TMPDIR=/tmp
OUT=$1
mkdir -p "$OUT"
G=${G:-"1000000000 5800 7000"}
run() {  # name, counters...
  local n=$1
  shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$n" -o run -- python3 tools/bench_groups.py $G > "$OUT/$n.log" 2>&1
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD
