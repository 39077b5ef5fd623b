#!/usr/bin/env python3
"""Host latency of each C-ABI call of the K:1336 aggregate stage (string key, MAX of fp64) on
synthetic device columns: wall time of the call itself (no device sync around it), median of 50,
next to the same calls with a device sync after each. Shows which calls block or spend host time.

  python tools/agg_host_calls.py [rows]
"""
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import numpy as np  # noqa: E402

from kquery import native as N  # noqa: E402
from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.columnar import Context, DeviceColumn  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    ctx = Context.get(0)
    rng = np.random.default_rng(1)
    vendor = DeviceColumn.from_strings(list(np.array(["1", "2", "4"], dtype=object)[rng.integers(0, 3, rows)]), ctx=ctx)
    vendor.max_len = 1  # as qe_csv_column reports it for the tripdata column
    fare = DeviceColumn.from_numpy(N.TYPE_FLOAT64, rng.random(rows) * 100, None, ctx=ctx)
    ctx.synchronize()
    t = {k: [] for k in ("create", "update", "finalize_sizes", "finalize", "close", "py_update", "py_finalize")}
    for it in range(60):
        t0 = time.perf_counter()
        st = HashAggregateState(ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64)], 16, async_update=True)
        t1 = time.perf_counter()
        kc = (N.QeColumn * 1)(vendor.as_c())
        ic = (N.QeColumn * 1)(fare.as_c())
        t2 = time.perf_counter()
        N.check(N.lib().qe_hashagg_update(st.handle, kc, ic, None))
        t3 = time.perf_counter()
        g = N.C.c_int64()
        kb = (N.C.c_int64 * 1)()
        N.check(N.lib().qe_hashagg_finalize_sizes(st.handle, N.C.byref(g), kb))
        t4 = time.perf_counter()
        keys, vals = st.finalize()
        t5 = time.perf_counter()
        ctx.synchronize()
        t6 = time.perf_counter()
        st.close()
        t7 = time.perf_counter()
        if it >= 10:
            t["create"].append(t1 - t0)
            t["update"].append(t3 - t2)
            t["finalize_sizes"].append(t4 - t3)
            t["finalize"].append(t5 - t4)
            t["close"].append(t7 - t6)
        # the Python wrappers alone (update through HashAggregateState)
        st = HashAggregateState(ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64)], 16, async_update=True)
        a = time.perf_counter()
        st.update([vendor], [fare])
        b = time.perf_counter()
        st.finalize()
        c = time.perf_counter()
        ctx.synchronize()
        st.close()
        if it >= 10:
            t["py_update"].append(b - a)
            t["py_finalize"].append(c - b)
    print({k: round(statistics.median(v) * 1e6, 1) for k, v in t.items()}, "(us, host wall per call, median of 50)")


if __name__ == "__main__":
    main()
