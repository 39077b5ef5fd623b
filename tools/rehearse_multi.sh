#!/bin/bash
# N > 1 rehearsal of bench.py on ONE GPU: 2 and 4 ranks sharing the device over gloo (RCCL refuses
# two ranks on one GPU). Checks the multi-rank step (rank-offset rows, export -> all-to-all ->
# import, the cross-rank result checks, max-over-ranks timing); the numbers mean nothing.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/multi
mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 3 --warmup 1 --rows 100000000 --dist-backend gloo \
    > $OUT/n$n.json 2> $OUT/n$n.err || exit 1
done
