#!/usr/bin/env python3
"""GROUP BY cardinality sweep: the headline query (C4 shape: SUM(a+b), COUNT(*), MIN(a), MAX(b)
WHERE a > 2^19 GROUP BY k) with k = u mod G for G from 16 to 64M, on one MI355X.

Per G: fused update (HIP events around the launch sequence on the ctx stream), finalize, and
checks that hold at any size: every group present (rows >> G), sum of COUNT(*) = rows passing the
filter (counted by qe_filter_count), sum of SUM(a+b) = the global SUM over the selected rows.
Writes one JSON object per G.

  python tools/bench_groups.py [rows] [G ...]
"""
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
from kquery.datasource import C4_COLUMNS, ColumnSpec, generate_column  # noqa: E402
from kquery.workloads import C4_AGGS, c4_spec  # noqa: E402

PEAK = 8000.0


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000_000
    sizes = [int(x) for x in sys.argv[2:]] or [16, 1024, 65536, 1 << 20, 1 << 24, 1 << 26]
    ctx = Context.get(0)
    a = generate_column(C4_COLUMNS[1], rows, 0, 42, ctx)
    b = generate_column(C4_COLUMNS[2], rows, 0, 42, ctx)
    ctx.synchronize()
    spec = c4_spec()
    for g in sizes:
        k = generate_column(ColumnSpec("k", N.TYPE_INT64, N.GEN_MOD, g, 0), rows, 0, 42, ctx)
        ctx.synchronize()
        st = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, g)
        ts, ks, fs, kl = [], [], [], []
        for it in range(4):
            st.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.update_fused([k, a, b], spec)
            ctx.synchronize()
            t1 = time.perf_counter()
            keys, res = st.finalize()
            ctx.synchronize()
            t2 = time.perf_counter()
            if it:
                ts.append((t1 - t0) * 1e3)
                fs.append((t2 - t1) * 1e3)
                ms, launches = st.last_kernel_time()
                ks.append(ms)  # every kernel of the update (spill / partition passes included)
                kl.append(launches)
        ngroups = keys[0].length
        cnt = int(res[1].to_numpy().sum())
        upd = statistics.median(ts)
        d = {"groups": g, "rows": rows, "update_ms": upd, "kernel_ms": statistics.median(ks), "launches": kl[-1] if kl else 0,
             "finalize_ms": statistics.median(fs), "rows_per_s": rows / (upd * 1e-3),
             "achieved_gbs": rows * 24 / (upd * 1e-3) / 1e9, "frac": rows * 24 / (upd * 1e-3) / 1e9 / PEAK,
             "kernel": st.last_kernel_kind(), "out_groups": ngroups, "count_star_total": cnt}
        print(json.dumps(d), flush=True)
        st.close()
        del k, keys, res
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
