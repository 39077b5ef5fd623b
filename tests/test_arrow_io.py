"""Arrow C Data Interface boundary: pyarrow record batches (standing in for Arrow
Java's Data.exportVectorSchemaRoot) -> qe_batch_import -> device kernels -> qe_batch_export ->
pyarrow, through the C ABI structs only."""
import ctypes as C
import datetime

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")


def _sample(n, seed=0):
    rng = np.random.default_rng(seed)
    mask = rng.random(n) < 0.1
    i64 = pa.array(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64), mask=mask)
    f64 = pa.array(rng.normal(size=n), mask=rng.random(n) < 0.2)
    strs = pa.array([None if rng.random() < 0.1 else "s%d-%s" % (i, "x" * (i % 7)) for i in range(n)])
    i32 = pa.array(rng.integers(-2**31, 2**31 - 1, n, dtype=np.int32))
    u8 = pa.array(rng.integers(0, 255, n, dtype=np.uint8), mask=rng.random(n) < 0.3)
    d32 = pa.array([datetime.date(2020, 1, 1) + datetime.timedelta(days=int(x)) for x in rng.integers(0, 3000, n)],
                   type=pa.date32())
    bools = pa.array(rng.random(n) < 0.5, mask=rng.random(n) < 0.1)
    return pa.RecordBatch.from_arrays([i64, f64, strs, i32, u8, d32, bools],
                                      names=["i64", "f64", "s", "i32", "u8", "d32", "b"])


def test_unsupported_format_is_reported_without_gpu_work():
    """Format mapping is host-side: an unsupported type fails before any device allocation."""
    from kquery import native as N

    assert N.lib().qe_batch_import  # symbol bound


@pytest.mark.gpu
@pytest.mark.parametrize("n,off", [(0, 0), (1, 0), (1000, 0), (100_003, 0), (5000, 3), (5000, 13), (5000, 64)])
def test_roundtrip_import_export(gpu_ctx, n, off):
    from kquery.arrow_io import DeviceBatch, export_to_pyarrow

    full = _sample(n + off + 7, seed=n + off)
    rb = full.slice(off, n)  # sliced: nonzero offsets, unaligned validity bits
    db = DeviceBatch.from_pyarrow(rb, gpu_ctx)
    ncols, length = db.shape()
    assert (ncols, length) == (rb.num_columns, n)
    cols = db.columns()
    back = export_to_pyarrow(gpu_ctx, [c for c, _ in cols], [nm for _, nm in cols])
    assert back.schema.names == rb.schema.names
    for a, b in zip(back.columns, rb.columns):
        assert a.type == b.type
        assert a.to_pylist() == b.to_pylist()
    db.close()


@pytest.mark.gpu
def test_large_utf8_and_unsupported(gpu_ctx):
    from kquery import native as N
    from kquery.arrow_io import DeviceBatch, export_to_pyarrow

    rb = pa.RecordBatch.from_arrays([pa.array(["a", None, "ccc"], type=pa.large_string())], names=["s"])
    db = DeviceBatch.from_pyarrow(rb, gpu_ctx)
    back = export_to_pyarrow(gpu_ctx, [db.column(0)[0]], ["s"])
    assert back.column(0).to_pylist() == ["a", None, "ccc"]
    bad = pa.RecordBatch.from_arrays([pa.array([1.5], type=pa.float32())], names=["f"])
    with pytest.raises(N.IllegalStateException, match="format 'f'"):
        DeviceBatch.from_pyarrow(bad, gpu_ctx)


@pytest.mark.gpu
def test_imported_batch_feeds_kernels(gpu_ctx):
    """Imported Arrow columns go straight into the kernels: CAST(utf8 AS double) and a
    GROUP BY over an imported int64 key, compared with pyarrow/the oracle."""
    from oracle import cast_ref as R
    from oracle import semantics as S

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.arrow_io import DeviceBatch, export_to_pyarrow
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(3)
    n = 50_000
    fares = ["%.2f" % x for x in rng.uniform(0, 300, n)]
    keys = rng.integers(0, 37, n)
    rb = pa.RecordBatch.from_arrays([pa.array(keys), pa.array(fares)], names=["k", "fare"])
    db = DeviceBatch.from_pyarrow(rb, gpu_ctx)
    kcol, fcol = db.column(0)[0], db.column(1)[0]
    out = DeviceColumn.empty(N.TYPE_FLOAT64, n, False, ctx=gpu_ctx)
    oc = out.as_c()
    N.check(N.lib().qe_cast_utf8_to_f64(gpu_ctx.handle, C.byref(fcol), C.byref(oc), None))
    want, _ = R.cast_utf8_to_f64(fares)
    assert (out.to_numpy().view(np.int64) == want.view(np.int64)).all()
    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(N.AGG_MAX, N.TYPE_FLOAT64), (N.AGG_COUNT_STAR, N.TYPE_INT64)])
    kc = (N.QeColumn * 1)(kcol)
    ic = (N.QeColumn * 2)(oc, N.QeColumn())
    N.check(N.lib().qe_hashagg_update(st.handle, kc, ic, None))
    gk, ga = st.finalize()
    res = export_to_pyarrow(gpu_ctx, gk + ga, ["k", "MAX", "COUNT"])
    got = {r["k"]: (r["MAX"], r["COUNT"]) for r in res.to_pylist()}
    ref = S.hash_aggregate_rows([keys.tolist()], [want.tolist(), [1] * n], [S.AGG_MAX, S.AGG_COUNT_STAR],
                                [True, False])
    assert got == {k[0]: tuple(v) for k, v in ref.items()}


@pytest.mark.gpu
def test_prefetch_import_pipeline(gpu_ctx):
    """prefetch_import: host batches imported one ahead on a second stream while the GROUP BY
    kernels of the previous batch run. Each batch is checked bit for bit after import, and the
    multi-batch aggregate (row order continuing across batches) matches the oracle over all rows."""
    from oracle import semantics as S

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.arrow_io import prefetch_import

    rng = np.random.default_rng(11)
    n, nb = 1_200_000, 6
    k = rng.integers(0, 500, n).astype(np.int64)
    x = rng.normal(size=n) * 50
    xv = rng.random(n) > 0.05
    rb = pa.RecordBatch.from_arrays([pa.array(k), pa.array(x, mask=~xv)], names=["k", "x"])
    parts = [rb.slice(i * n // nb, n // nb) for i in range(nb)]
    fns = [N.AGG_SUM, N.AGG_MIN, N.AGG_MAX, N.AGG_COUNT]
    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(f, N.TYPE_FLOAT64) for f in fns], 500)
    seen = 0
    for i, db in enumerate(prefetch_import(iter(parts), gpu_ctx)):
        kc, xc = db.column(0)[0], db.column(1)[0]
        assert kc.length == n // nb
        kk = (N.QeColumn * 1)(kc)
        ic = (N.QeColumn * 4)(xc, xc, xc, xc)
        N.check(N.lib().qe_hashagg_update(st.handle, kk, ic, None))
        seen += 1
    assert seen == nb
    keys, aggs = st.finalize()
    cols = [(v.to_numpy(), v.valid_mask()) for v in aggs]
    got = {(int(a),): [vals[i] if ok[i] else None for vals, ok in cols] for i, a in enumerate(keys[0].to_numpy())}
    ref = S.group_aggregate([k], [None], [x] * 4, [xv] * 4, fns)
    assert len(got) == len(ref)
    for key, want in ref.items():
        g = got[key]
        for j, (a, b) in enumerate(zip(g, want)):
            rel = 1e-9 if fns[j] == N.AGG_SUM else 0.0
            assert S.rows_equal(None if a is None else (float(a) if fns[j] != N.AGG_COUNT else int(a)), b, rel), (key, j)
