#!/usr/bin/env python3
"""Per-call host overhead of the hot entry points on tiny inputs (1000 rows): wall time per call
with a device sync, median of 200. Covers qe_hashagg create/update/update_fused/finalize/destroy,
qe_select_project, qe_agg_global, qe_cast_utf8_to_f64 and the string-dictionary encode.

  python tools/overhead.py
"""
import json
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
from kquery.datasource import C4_COLUMNS, generate_column  # noqa: E402
from kquery.workloads import C4_AGGS, c4_spec  # noqa: E402


def med(fn, ctx, reps=200):
    fn()
    ctx.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ctx.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    return round(statistics.median(ts), 1)


def main():
    ctx = Context.get(0)
    n = 1000
    cols = [generate_column(s, n, 0, 42, ctx) for s in C4_COLUMNS]
    spec = c4_spec()
    rng = np.random.default_rng(0)
    strs = DeviceColumn.from_strings([str(x) for x in rng.integers(0, 3, n)], ctx=ctx)
    fare = DeviceColumn.from_numpy(N.TYPE_FLOAT64, rng.random(n), None, ctx=ctx)
    out = {}
    st = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024)
    out["sync_only"] = med(lambda: None, ctx)
    out["hashagg_create_destroy"] = med(lambda: HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024).close(), ctx)
    out["hashagg_reset"] = med(st.reset, ctx)
    out["hashagg_update_fused"] = med(lambda: (st.reset(), st.update_fused(cols, spec)), ctx)
    out["hashagg_update"] = med(lambda: (st.reset(), st.update([cols[0]], [cols[1], None, cols[1], cols[2]])), ctx)
    st.reset()
    st.update_fused(cols, spec)
    out["hashagg_finalize"] = med(st.finalize, ctx)
    s2 = HashAggregateState(ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64)], 16)
    out["strkey_update"] = med(lambda: (s2.reset(), s2.update([strs], [fare])), ctx)
    out["strkey_finalize"] = med(s2.finalize, ctx)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
