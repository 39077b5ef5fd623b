#!/usr/bin/env python3
"""Per-configuration measurements (BASELINE.json configs[1..4] on one MI355X), next to the headline
bench.py line. Each config: device-resident synthetic input, warmup, then the median of N timed
runs (HIP events on the stream the kernels run on), reported as rows/s and as algorithmic
HBM bytes / time against the 8 TB/s peak. Writes one JSON object per config to stdout.

  C2  10M int64:  SelectionExec(a > 2^19) -> ProjectionExec(a + b)        per-family operators
  C3  100M fp64:  SUM/MIN/MAX/COUNT/AVG global aggregate                   qe_agg_global
  C4  1B int64:   fused filter+project+GROUP BY (the headline)              qe_hashagg_update_fused
  C5  1.25B rows (10B / 8 GPUs) lineitem-shaped Q1-like, 2 keys, 3 predicates  fused
"""
import json
import pathlib
import statistics
import time
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import torch  # noqa: E402

from kquery import native as N  # noqa: E402
from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.columnar import Context, DeviceColumn, Field, RecordBatch, Schema  # noqa: E402
from kquery.datasource import (C2_COLUMNS, C3_COLUMNS, C4_COLUMNS, C5_COLUMNS, ColumnSpec,  # noqa: E402
                               InMemoryDataSource, generate_column)
from kquery.expressions import (AddExpression, ColumnExpression, GtExpression,  # noqa: E402
                                LiteralLongExpression)
from kquery.operators import ProjectionExec, ScanExec, SelectionExec, fuse  # noqa: E402
from kquery.workloads import C4_AGGS, C5_AGGS, C5_KEY_TYPES, c4_spec, c5_spec  # noqa: E402

PEAK = 8000.0


def timed(fn, reps=10, warmup=3):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def report(cfg, rows, bytes_per_row, ms, **extra):
    gbs = rows * bytes_per_row / (ms * 1e-3) / 1e9
    d = {"config": cfg, "rows": rows, "ms": ms, "rows_per_s": rows / (ms * 1e-3), "alg_bytes_per_row": bytes_per_row,
         "achieved_gbs": gbs, "peak_gbs": PEAK, "frac": gbs / PEAK}
    d.update(extra)
    print(json.dumps(d), flush=True)


def main():
    ctx = Context.get(0)
    which = sys.argv[1:] or ["C2", "C3", "C4", "C5"]
    if "C2" in which:
        n = 10_000_000
        cols = [generate_column(s, n, 0, 42, ctx) for s in C2_COLUMNS]
        schema = Schema([s.field() for s in C2_COLUMNS])
        scan = ScanExec(InMemoryDataSource(schema, [RecordBatch(schema, cols)]), ["a", "b"])
        sel = SelectionExec(scan, GtExpression(ColumnExpression(0), LiteralLongExpression(1 << 19)))
        proj = ProjectionExec(sel, Schema([Field("ab", N.TYPE_INT64)]),
                              [AddExpression(ColumnExpression(0), ColumnExpression(1))])
        out = {}

        def run():  # the selected-row count comes back once, at the end of the chain
            out["b"] = next(proj.execute())
            out["n"] = out["b"].rowCount()

        ms = timed(run)
        sel_rows = out["n"]
        # algorithmic: read a, b (16 B) + write a+b for the selected rows
        report("C2 filter(a>2^19)+project(a+b), 10M int64 (160 MB: fits the 256 MB MALL)", n,
               16 + 8 * sel_rows / n, ms, selected=sel_rows, path="per-family operators (cmp, compact, arith)")
        from kquery import operators as ops  # the same chain with the count / scan / gather compaction
        ops.SELECTION_COMPACTION = "gather"
        ms_b = timed(run)
        ops.SELECTION_COMPACTION = "select_project"
        report("C2 per-family, compaction by count + scan + gather (qe_filter_apply_async)", n,
               16 + 8 * sel_rows / n, ms_b, selected=out["n"], path="per-family operators (cmp, count, gather, arith)")
        fused = fuse(proj)
        assert type(fused).__name__ == "FusedSelectProjectExec"

        def run_fused():
            out["f"] = next(fused.execute())

        ms_f = timed(run_fused)
        assert out["f"].rowCount() == sel_rows
        # kernel-only time (HIP events on the ctx stream around the one launch)
        c = [x.as_c() for x in cols]
        cc = (N.QeColumn * 2)(*c)
        o = DeviceColumn.empty(N.TYPE_INT64, n, False, ctx=ctx)
        oc = (N.QeColumn * 1)(o.as_c())
        cnt = N.C.c_int64()

        def run_kernel():
            oc[0].length = n  # the call sets it to the selected count
            N.check(N.lib().qe_select_project(ctx.handle, cc, 2, N.C.byref(fused.spec), oc, N.C.byref(cnt)))

        ms_k = timed(run_kernel)

        def wall(fn, reps=30, warmup=5, before=None):
            """Host wall time of a synchronous call (what a caller waits), median; `before` runs
            untimed ahead of each call, followed by a stream synchronisation."""
            ts = []
            for it in range(warmup + reps):
                if before is not None:
                    before(it)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                t1 = time.perf_counter()
                if it >= warmup:
                    ts.append((t1 - t0) * 1e3)
            torch.cuda.synchronize()
            return statistics.median(ts)

        ms_wall = wall(run_kernel)  # synchronous call: returns once the kernels have completed
        # host split of one stream-ordered call: enqueue (qe_select_project_async) and the time to
        # the row count (qe_select_pending_wait; the kernel's last stores may still be in flight)
        enq, wt = [], []
        for it in range(35):
            torch.cuda.synchronize()
            oc[0].length = n
            pend = N.C.c_void_p()
            t0 = time.perf_counter()
            N.check(N.lib().qe_select_project_async(ctx.handle, cc, 2, N.C.byref(fused.spec), oc, N.C.byref(pend)))
            t1 = time.perf_counter()
            N.check(N.lib().qe_select_pending_wait(pend, N.C.byref(cnt)))
            t2 = time.perf_counter()
            if it >= 5:
                enq.append((t1 - t0) * 1e3)
                wt.append((t2 - t1) * 1e3)
        ms_enq, ms_wait = statistics.median(enq), statistics.median(wt)
        # the same call with the input evicted from the 256 MB MALL first (a 1 GiB write between
        # calls, outside the timed region): what one 10M batch costs from HBM. The write leaves the
        # MALL full of dirty lines, so the call's reads also pay their write-back; "clean" evicts
        # with a 1 GiB READ instead (MALL holding clean lines of another buffer)
        flush = torch.empty(1 << 30, dtype=torch.uint8, device=ctx.torch_device)
        cold = []
        for it in range(13):
            flush.fill_(it & 0xFF)
            s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_ev.record()
            run_kernel()
            e_ev.record()
            e_ev.synchronize()
            if it >= 3:
                cold.append(s_ev.elapsed_time(e_ev))
        ms_cold = statistics.median(cold)
        ms_cold_wall = wall(run_kernel, reps=10, warmup=3, before=lambda it: flush.fill_(it & 0xFF))
        fl64 = flush.view(torch.int64)
        fl64.fill_(1)
        ms_clean_wall = wall(run_kernel, reps=10, warmup=3, before=lambda it: fl64.max())
        del flush, fl64
        report("C2 fused select+project (qe_select_project), 10M int64", n, 16 + 8 * sel_rows / n, ms_f,
               selected=sel_rows, call_ms=ms_k, call_gbs=n * (16 + 8 * sel_rows / n) / (ms_k * 1e-3) / 1e9,
               call_cold_ms=ms_cold, call_cold_gbs=n * (16 + 8 * sel_rows / n) / (ms_cold * 1e-3) / 1e9,
               call_wall_ms=ms_wall, call_wall_gbs=n * (16 + 8 * sel_rows / n) / (ms_wall * 1e-3) / 1e9,
               call_enqueue_ms=ms_enq, call_time_to_count_ms=ms_wait,
               call_cold_wall_ms=ms_cold_wall, call_cold_clean_wall_ms=ms_clean_wall,
               call_cold_clean_frac=n * (16 + 8 * sel_rows / n) / (ms_clean_wall * 1e-3) / 8e12,
               path="one hipRTC-specialised kernel: predicate, look-back compaction, projection")
        # stream-ordered calls (qe_select_project_async): call i+1 is queued before call i's count
        # is read back, as the pipelined FusedSelectProjectExec does batch to batch
        def run_pipelined(k=20):
            prev = None
            for _ in range(k):
                oc[0].length = n
                pend = N.C.c_void_p()
                N.check(N.lib().qe_select_project_async(ctx.handle, cc, 2, N.C.byref(fused.spec), oc, N.C.byref(pend)))
                if prev is not None:
                    N.check(N.lib().qe_select_pending_wait(prev, N.C.byref(cnt)))
                prev = pend
            N.check(N.lib().qe_select_pending_wait(prev, N.C.byref(cnt)))

        ms_p = timed(run_pipelined, reps=5, warmup=1) / 20
        report("C2 fused select+project, stream-ordered calls back to back (qe_select_project_async), 10M int64", n,
               16 + 8 * sel_rows / n, ms_p, selected=sel_rows, path="20 async calls, each count read while the next runs")
        # the pipelined operator over a Sequence of 8 batches of 10M rows
        batches = [RecordBatch(schema, [generate_column(s, n, i * n, 42, ctx) for s in C2_COLUMNS]) for i in range(8)]
        fused8 = fuse(ProjectionExec(SelectionExec(ScanExec(InMemoryDataSource(schema, batches), ["a", "b"]),
                                                   GtExpression(ColumnExpression(0), LiteralLongExpression(1 << 19))),
                                     Schema([Field("ab", N.TYPE_INT64)]),
                                     [AddExpression(ColumnExpression(0), ColumnExpression(1))]))

        def run_op8():
            out["n8"] = sum(b.rowCount() for b in fused8.execute())

        ms_o = timed(run_op8, reps=5, warmup=1) / 8
        report("C2 pipelined FusedSelectProjectExec over 8 batches of 10M rows (per batch)", n,
               16 + 8 * (out["n8"] / 8) / n, ms_o, selected=out["n8"])
        del batches, fused8
        for sel_k in (1 << 13, (1 << 20) - (1 << 13)):  # ~1 % / ~99 % selectivity sweep
            spec2 = N.QeSelectSpec.from_buffer_copy(fused.spec)
            spec2.terms[0].lit = N.scalar(sel_k, N.TYPE_INT64)

            def run_sweep():
                oc[0].length = n
                N.check(N.lib().qe_select_project(ctx.handle, cc, 2, N.C.byref(spec2), oc, N.C.byref(cnt)))

            ms_s = timed(run_sweep)
            report(f"C2 fused, a > {sel_k}", n, 16 + 8 * cnt.value / n, ms_s, selected=cnt.value)
        del cols, out
    if "C2L" in which:  # the C2 kernel at 1B rows: its bandwidth once launch latency is amortised
        n = 1_000_000_000
        cols = [generate_column(s, n, 0, 42, ctx) for s in C2_COLUMNS]
        schema = Schema([s.field() for s in C2_COLUMNS])
        scan = ScanExec(InMemoryDataSource(schema, [RecordBatch(schema, cols)]), ["a", "b"])
        sel = SelectionExec(scan, GtExpression(ColumnExpression(0), LiteralLongExpression(1 << 19)))
        proj = ProjectionExec(sel, Schema([Field("ab", N.TYPE_INT64)]),
                              [AddExpression(ColumnExpression(0), ColumnExpression(1))])
        fused = fuse(proj)
        cc = (N.QeColumn * 2)(*[x.as_c() for x in cols])
        o = DeviceColumn.empty(N.TYPE_INT64, n, False, ctx=ctx)
        oc = (N.QeColumn * 1)(o.as_c())
        cnt = N.C.c_int64()

        def run_large():
            oc[0].length = n
            N.check(N.lib().qe_select_project(ctx.handle, cc, 2, N.C.byref(fused.spec), oc, N.C.byref(cnt)))

        ms_l = timed(run_large)
        report("C2 shape at 1B rows: fused select+project (qe_select_project call)", n, 16 + 8 * cnt.value / n, ms_l,
               selected=cnt.value)
        del cols, o
    if "C2LN" in which:  # the C2 shape at 1B rows with 1 % nulls in b: a nullable output (a + b)
        n = 1_000_000_000
        specs = [C2_COLUMNS[0], ColumnSpec("b", N.TYPE_INT64, N.GEN_RAW, 0, 2, null_permille=10)]
        cols = [generate_column(s, n, 0, 42, ctx) for s in specs]
        schema = Schema([s.field() for s in specs])
        scan = ScanExec(InMemoryDataSource(schema, [RecordBatch(schema, cols)]), ["a", "b"])
        sel = SelectionExec(scan, GtExpression(ColumnExpression(0), LiteralLongExpression(1 << 19)))
        proj = ProjectionExec(sel, Schema([Field("ab", N.TYPE_INT64)]),
                              [AddExpression(ColumnExpression(0), ColumnExpression(1))])
        fused = fuse(proj)
        cc = (N.QeColumn * 2)(*[x.as_c() for x in cols])
        o = DeviceColumn.empty(N.TYPE_INT64, n, True, ctx=ctx)
        oc = (N.QeColumn * 1)(o.as_c())
        cnt = N.C.c_int64()

        def run_nullable():
            oc[0].length = n
            N.check(N.lib().qe_select_project(ctx.handle, cc, 2, N.C.byref(fused.spec), oc, N.C.byref(cnt)))

        ms_n = timed(run_nullable)
        # a, b, b's validity bits in; a+b and its validity bits out for the selected rows
        report("C2 shape at 1B rows, b 1 % null (nullable output)", n, 16 + 1 / 8 + (8 + 1 / 8) * cnt.value / n, ms_n,
               selected=cnt.value)
        del cols, o
    if "C3" in which:
        n = 100_000_000
        col = generate_column(C3_COLUMNS[0], n, 0, 42, ctx)
        c = col.as_c()
        r = N.QeGlobalAgg()

        def run():
            N.check(N.lib().qe_agg_global(ctx.handle, N.C.byref(c), None, N.C.byref(r)))

        ms = timed(run)
        # host wall of the synchronous call (the result is polled from pinned memory)
        ws = []
        for it in range(35):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run()
            if it >= 5:
                ws.append((time.perf_counter() - t0) * 1e3)
        ms_wall = statistics.median(ws)
        cc = (N.QeColumn * 1)(col.as_c())
        sms = N.C.c_double()
        shape = N.C.create_string_buffer(128)
        N.check(N.lib().qe_stream_read_best(ctx.handle, cc, 1, 5, N.C.byref(sms), shape, 128))
        report("C3 SUM/MIN/MAX/COUNT/AVG global aggregate, 100M fp64", n, 8, ms, path="k_agg_global + final", call_wall_ms=ms_wall, call_wall_frac=n * 8 / (ms_wall * 1e-3) / 8e12,
               stream_read_ceiling_gbs=n * 8 / (sms.value * 1e-3) / 1e9, stream_read_shape=shape.value.decode())
        del col
    for cfg, specs, rows, aggs, keys, spec, bpr, ng in (
            ("C4", C4_COLUMNS, 1_000_000_000, C4_AGGS, [N.TYPE_INT64], c4_spec(), 24, 1024),
            ("C5", C5_COLUMNS, 1_250_000_000, C5_AGGS, C5_KEY_TYPES, c5_spec(), 38, 16)):
        if cfg not in which:
            continue
        cols = [generate_column(s, rows, 0, 42, ctx) for s in specs]
        st = HashAggregateState(ctx, keys, aggs, ng)
        kms = []

        def run():
            st.reset()
            st.update_fused(cols, spec)
            kms.append(st.last_kernel_time()[0])
            st.finalize()

        ms = timed(run)
        kind = st.last_kernel_kind()
        kmed = statistics.median(kms[-10:])
        name = ("C4 SELECT k,SUM(a+b),COUNT(*),MIN(a),MAX(b) WHERE a>2^19 GROUP BY k, 1B int64" if cfg == "C4" else
                "C5 lineitem Q1-like (3 predicates, GROUP BY returnflag,linestatus, 4 SUM+AVG+COUNT), 1.25B rows/GPU")
        # streaming-read ceiling over the same columns (best launch shape, qe_stream_read_best)
        cc = (N.QeColumn * len(cols))(*[c.as_c() for c in cols])
        sms = N.C.c_double()
        shape = N.C.create_string_buffer(128)
        N.check(N.lib().qe_stream_read_best(ctx.handle, cc, len(cols), 5, N.C.byref(sms), shape, 128))
        report(name, rows, bpr, ms, kernel_ms=kmed, kernel_gbs=rows * bpr / (kmed * 1e-3) / 1e9,
               specialised=kind[0], note=kind[1], groups=st.num_groups(),
               stream_read_ceiling_gbs=rows * bpr / (sms.value * 1e-3) / 1e9, stream_read_shape=shape.value.decode())
        del cols, st


if __name__ == "__main__":
    main()
