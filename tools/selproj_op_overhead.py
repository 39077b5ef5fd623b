#!/usr/bin/env python3
"""Host-side cost of FusedSelectProjectExec.run_batch over the C2 batch (10M rows): the operator
call against the bare qe_select_project call, and the pieces in between (output allocation with
and without a validity bitmap, ctypes marshalling). Median wall time per call, torch stream synced
after each call.

  python tools/selproj_op_overhead.py
"""
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import torch  # noqa: E402

from kquery import native as N  # noqa: E402
from kquery.columnar import Context, DeviceColumn, Field, RecordBatch, Schema  # noqa: E402
from kquery.datasource import C2_COLUMNS, InMemoryDataSource, generate_column  # noqa: E402
from kquery.expressions import AddExpression, ColumnExpression, GtExpression, LiteralLongExpression  # noqa: E402
from kquery.operators import ProjectionExec, ScanExec, SelectionExec, fuse  # noqa: E402


def med(fn, reps=60):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(ts[10:])


def main():
    ctx = Context.get(0)
    n = 10_000_000
    cols = [generate_column(s, n, 0, 42, ctx) for s in C2_COLUMNS]
    schema = Schema([s.field() for s in C2_COLUMNS])
    batch = RecordBatch(schema, cols)
    scan = ScanExec(InMemoryDataSource(schema, [batch]), ["a", "b"])
    sel = SelectionExec(scan, GtExpression(ColumnExpression(0), LiteralLongExpression(1 << 19)))
    proj = ProjectionExec(sel, Schema([Field("ab", N.TYPE_INT64)]), [AddExpression(ColumnExpression(0), ColumnExpression(1))])
    fused = fuse(proj)
    print("plan:", fused)
    print("operator execute   %.1f us" % med(lambda: next(fused.execute())))
    print("run_batch          %.1f us" % med(lambda: fused.run_batch(batch)))
    print("empty nullable     %.1f us" % med(lambda: DeviceColumn.empty(N.TYPE_INT64, n, True, ctx=ctx)))
    print("empty non-null     %.1f us" % med(lambda: DeviceColumn.empty(N.TYPE_INT64, n, False, ctx=ctx)))
    out = DeviceColumn.empty(N.TYPE_INT64, n, True, ctx=ctx)
    cc = (N.QeColumn * 2)(*[c.as_c() for c in cols])
    cnt = N.C.c_int64()

    def call(o):
        oc = (N.QeColumn * 1)(o.as_c())
        N.check(N.lib().qe_select_project(ctx.handle, cc, 2, N.C.byref(fused.spec), oc, N.C.byref(cnt)))

    print("call, validity     %.1f us" % med(lambda: call(out)))
    out2 = DeviceColumn.empty(N.TYPE_INT64, n, False, ctx=ctx)
    print("call, no validity  %.1f us" % med(lambda: call(out2)))
    print("marshal cols       %.1f us" % med(lambda: (N.QeColumn * 2)(*[c.as_c() for c in cols])))


if __name__ == "__main__":
    main()
