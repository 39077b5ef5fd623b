"""Re-entrancy (SURVEY §8b Threading): the reference runs its per-month partial queries
concurrently, one ExecutionContext per coroutine (Main.kt:1309-1313, :1333). Here several host
threads, each with its own HIP stream and qe_ctx, run the same device pipeline at once — GPU CSV
scan -> CAST(fare_amount AS double) -> string-keyed MAX aggregate, plus a fused numeric
aggregate — and every result must equal the oracle's. ctypes releases the GIL around each
library call, so the native code really runs concurrently."""
import random
import threading

import pytest

from oracle import cast_ref as R
from oracle import csv_ref as CR
from oracle import semantics as S

pytestmark = pytest.mark.gpu


def _month_csv(path, seed, rows):
    rng = random.Random(seed)
    lines = ["VendorID,passenger_count,fare_amount"]
    for _ in range(rows):
        lines.append(f"{rng.choice(['1', '2', '4', 'VTS'])},{rng.randint(1, 6)},{rng.uniform(-5, 300):.2f}")
    path.write_text("\n".join(lines) + "\n")


def _expected(path):
    names, _, rows = CR.parse(path.read_bytes())
    vend, fare = CR.project(rows, [0, 2])
    want = S.hash_aggregate_rows([vend], [[R.parse_java_double(f) for f in fare]], [S.AGG_MAX], [True])
    return {k[0]: v[0] for k, v in want.items()}


def _partial_query(path, ctx):
    from kquery import native as N
    from kquery.columnar import Field, Schema
    from kquery.csv_source import CsvDataSource
    from kquery.expressions import CastExpression, ColumnExpression, MaxExpression
    from kquery.operators import HashAggregateExec, ScanExec

    agg = HashAggregateExec(ScanExec(CsvDataSource(str(path), True, 0, ctx=ctx), ["VendorID", "fare_amount"]),
                            [ColumnExpression(0)], [MaxExpression(CastExpression(ColumnExpression(1), N.TYPE_FLOAT64))],
                            Schema([Field("VendorID", N.TYPE_UTF8), Field("max_amount", N.TYPE_FLOAT64)]))
    out = next(agg.execute())
    ctx.synchronize()
    return dict(zip(out.field(0).to_pylist(), out.field(1).to_pylist()))


def _fused_c4(ctx, rows, row0):
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.datasource import C4_COLUMNS, generate_column
    from kquery.workloads import C4_AGGS, c4_spec

    cols = [generate_column(s, rows, row0, 42, ctx) for s in C4_COLUMNS]
    st = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024)
    st.set_row_base(row0)
    st.update_fused(cols, c4_spec())
    keys, aggs = st.finalize()
    ctx.synchronize()
    return sorted(zip(keys[0].to_pylist(), *[a.to_pylist() for a in aggs]))


def test_concurrent_contexts(tmp_path):
    import torch

    from kquery.columnar import Context

    months = []
    for m in range(1, 9):
        p = tmp_path / f"yc-{m:02d}.csv"
        _month_csv(p, m, 20_000 + 1000 * m)
        months.append(p)
    expected = [_expected(p) for p in months]
    sequential_c4 = _fused_c4(Context.get(0), 2_000_000, 0)

    results, errors = {}, []

    def worker(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                ctx = Context.get(0)  # one qe_ctx per (device, stream)
                for m in range(t, len(months), 4):
                    results[m] = _partial_query(months[m], ctx)
                results[("c4", t)] = _fused_c4(ctx, 2_000_000, 0)
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors
    for m in range(len(months)):
        assert results[m] == expected[m], m
    for t in range(4):
        assert results[("c4", t)] == sequential_c4
