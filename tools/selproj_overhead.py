#!/usr/bin/env python3
"""Host overhead of one qe_select_project call: the C2 plan on a 1-row input (kernels trivial),
median wall time per call, both tile-base schemes.

  python tools/selproj_overhead.py
"""
import os
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd"), str(ROOT / "tests")]

from kquery import native as N  # noqa: E402
from kquery.columnar import Context, DeviceColumn  # noqa: E402
from kquery.datasource import C2_COLUMNS, generate_column  # noqa: E402
from test_selproj import _spec  # noqa: E402


def main():
    ctx = Context.get(0)
    for tp in ("1", "0"):
        os.environ["QE_SELPROJ_TWOPASS"] = tp
        for n in (1, 10_000_000):
            cols = [generate_column(s, n, 0, 42, ctx) for s in C2_COLUMNS]
            spec = _spec(N, [(0, N.OP_GT, -1, 1 << 19)], [[(N.TOK_COL, 0, None), (N.TOK_COL, 1, None), (N.TOK_ADD, 0, None)]])
            out = DeviceColumn.empty(N.TYPE_INT64, n, False, ctx=ctx)
            cc = (N.QeColumn * 2)(*[c.as_c() for c in cols])
            oc = (N.QeColumn * 1)(out.as_c())
            cnt = N.C.c_int64()
            ts = []
            for i in range(60):
                oc[0].length = n
                t0 = time.perf_counter()
                N.check(N.lib().qe_select_project(ctx.handle, cc, 2, N.C.byref(spec), oc, N.C.byref(cnt)))
                ts.append((time.perf_counter() - t0) * 1e6)
            print(f"twopass={tp} n={n}: median {statistics.median(ts[10:]):.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
