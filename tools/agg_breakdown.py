#!/usr/bin/env python3
"""Host-side breakdown of a string-keyed aggregate (the K:1336 tripdata shape on synthetic device
columns): HashAggregateState create / update / finalize / close, wall time per phase with a device
sync after each, median of 20.

  python tools/agg_breakdown.py [rows] [--profile]   (--profile: cProfile of 20 iterations, top calls)
"""
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from kquery import native as N  # noqa: E402
from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.columnar import Context, DeviceColumn  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rows = int(args[0]) if args else 4_000_000
    ctx = Context.get(0)
    rng = np.random.default_rng(1)
    keys = np.array(["1", "2", "4"], dtype=object)[rng.integers(0, 3, rows)]
    vendor = DeviceColumn.from_strings(list(keys), ctx=ctx)
    fare = DeviceColumn.from_numpy(N.TYPE_FLOAT64, rng.random(rows) * 100, None, ctx=ctx)
    ctx.synchronize()
    phases = {"create": [], "update": [], "finalize": [], "close": [], "total": []}
    for it in range(22):
        t0 = time.perf_counter()
        st = HashAggregateState(ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64)], 16)
        ctx.synchronize()
        t1 = time.perf_counter()
        st.update([vendor], [fare])
        ctx.synchronize()
        t2 = time.perf_counter()
        k, v = st.finalize()
        ctx.synchronize()
        t3 = time.perf_counter()
        st.close()
        ctx.synchronize()
        t4 = time.perf_counter()
        if it >= 2:
            for name, dt in (("create", t1 - t0), ("update", t2 - t1), ("finalize", t3 - t2), ("close", t4 - t3),
                             ("total", t4 - t0)):
                phases[name].append(dt * 1e3)
    print({k: round(statistics.median(v), 4) for k, v in phases.items()})
    if "--profile" in sys.argv:
        import cProfile
        import pstats

        def run():
            for _ in range(20):
                st = HashAggregateState(ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64)], 16, async_update=True)
                st.update([vendor], [fare])
                st.finalize()
                st.close()
            ctx.synchronize()

        pr = cProfile.Profile()
        pr.runcall(run)
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
