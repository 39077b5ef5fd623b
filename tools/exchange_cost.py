#!/usr/bin/env python3
"""Cost of the multi-GPU step's exchange leg, measured on ONE GPU with a world-1 RCCL group:
export -> all-to-all (RCCL) -> import -> finalize, after the headline's fused partial aggregate.
With one rank the all-to-all is a local copy, so this isolates the host calls, syncs and small
kernels the exchange adds per step (what the 8-GPU efficiency loses besides xGMI latency).

    python tools/exchange_cost.py [rows]
"""
import json
import os
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kquery import native as N  # noqa: E402
from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.columnar import Context  # noqa: E402
from kquery.datasource import C4_COLUMNS, generate_column  # noqa: E402
from kquery.exchange import exchange_partials  # noqa: E402
from kquery.workloads import C4_AGGS, c4_spec  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ctx = Context.get(0)
    cols = [generate_column(s, rows, 0, 42, ctx) for s in C4_COLUMNS]
    partial = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024)
    owner = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024)
    spec = c4_spec()
    t = {k: [] for k in ("update", "exchange", "finalize", "step")}
    for it in range(30):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        partial.reset()
        partial.update_fused(cols, spec)
        t1 = time.perf_counter()
        owner.reset()
        exchange_partials(partial, owner)
        t2 = time.perf_counter()
        owner.finalize()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if it >= 5:
            t["update"].append((t1 - t0) * 1e3)
            t["exchange"].append((t2 - t1) * 1e3)
            t["finalize"].append((t3 - t2) * 1e3)
            t["step"].append((t3 - t0) * 1e3)
    print(json.dumps({k: round(statistics.median(v), 4) for k, v in t.items()} | {"rows": rows}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
