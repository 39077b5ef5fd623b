#!/usr/bin/env python3
"""Where a bench.py step's wall time goes beyond the fused kernel (host calls, syncs, finalize).

    python tools/step_breakdown.py [rows]

Prints one JSON line: median wall ms of each host call of the step, the fused kernel's event time
and the step total."""
import json
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import torch  # noqa: E402

from kquery import native as N  # noqa: E402
from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.columnar import Context  # noqa: E402
from kquery.datasource import C4_COLUMNS, generate_column  # noqa: E402
from kquery.workloads import C4_AGGS, c4_spec  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    ctx = Context.get(0)
    cols = [generate_column(s, rows, 0, 42, ctx) for s in C4_COLUMNS]
    ctx.synchronize()
    st = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024)
    spec = c4_spec()
    parts = {k: [] for k in ("reset", "update_fused", "kernel_event", "finalize", "step")}
    for it in range(25):
        t0 = time.perf_counter()
        st.reset()
        st.set_row_base(0)
        t1 = time.perf_counter()
        st.update_fused(cols, spec)
        t2 = time.perf_counter()
        ms, _ = st.last_kernel_time()
        st.last_kernel_kind()
        t3 = time.perf_counter()
        st.finalize()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        if it >= 5:
            parts["reset"].append((t1 - t0) * 1e3)
            parts["update_fused"].append((t2 - t1) * 1e3)
            parts["kernel_event"].append(ms)
            parts["finalize"].append((t4 - t3) * 1e3)
            parts["step"].append((t4 - t0) * 1e3)
    print(json.dumps({k: round(statistics.median(v), 4) for k, v in parts.items()} | {"rows": rows}))


if __name__ == "__main__":
    main()
