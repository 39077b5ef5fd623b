#!/usr/bin/env python3
"""Host-side time of each call of bench.py's exchange step (world-1 RCCL group on one GPU):
median wall µs per call over 30 steps. Where the host spends the time that the GPU waits for.

    python tools/exchange_host_profile.py [rows]
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
from kquery.exchange import all_to_all_slots  # noqa: E402
from kquery.workloads import C4_AGGS, c4_spec  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    ctx = Context.get(0)
    cols = [generate_column(s, rows, 0, 42, ctx) for s in C4_COLUMNS]
    ctx.synchronize()
    partial = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024, async_update=True)
    owner = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024)
    spec = c4_spec()
    t = {k: [] for k in ("reset", "update", "owner_reset", "export_slots", "all_to_all", "prepare_output",
                         "import_slots", "finalize", "kernel_time", "step")}
    for it in range(40):
        marks = [time.perf_counter()]
        partial.reset()
        partial.set_row_base(0)
        marks.append(time.perf_counter())
        partial.update_fused(cols, spec)
        marks.append(time.perf_counter())
        owner.reset()
        marks.append(time.perf_counter())
        send = partial.export_slots(1, 1024)
        marks.append(time.perf_counter())
        recv = all_to_all_slots(send)
        marks.append(time.perf_counter())
        owner.prepare_output()
        marks.append(time.perf_counter())
        n = owner.import_slots(recv, 1, 1024)
        marks.append(time.perf_counter())
        owner.finalize()
        marks.append(time.perf_counter())
        partial.last_kernel_time()
        marks.append(time.perf_counter())
        assert n is not None
        if it >= 10:
            for k, a, b in zip(list(t)[:-1], marks, marks[1:]):
                t[k].append((b - a) * 1e6)
            t["step"].append((marks[-1] - marks[0]) * 1e6)
    print(json.dumps({k: round(statistics.median(v), 1) for k, v in t.items()}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
