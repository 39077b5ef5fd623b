"""SelectionExec -> ProjectionExec on device. SelectionExec compacts
non-nullable int64 / fp64 columns with one select-project pass (the mask column as the selection),
and every other fixed-width batch stream-ordered: qe_filter_apply_async leaves the selected-row
count in HBM, qe_eval_arith_dlen computes only the rows below it, and the count comes back once, when
a consumer reads a length. Both forms are checked per row against numpy on the same seeded inputs
(bit-exact: int64 wraps, fp64 IEEE, nulls propagate), for empty, full and partial selections,
nullable inputs, and against qe_filter_apply's synchronous result."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _plan(N, cols, threshold, op_cls, out_type):
    from kquery.columnar import Field, RecordBatch, Schema
    from kquery.datasource import InMemoryDataSource
    from kquery.expressions import ColumnExpression, GtExpression, LiteralLongExpression
    from kquery.operators import ProjectionExec, ScanExec, SelectionExec

    schema = Schema([Field("a", cols[0].type), Field("b", cols[1].type)])
    scan = ScanExec(InMemoryDataSource(schema, [RecordBatch(schema, cols)]), ["a", "b"])
    sel = SelectionExec(scan, GtExpression(ColumnExpression(0), LiteralLongExpression(threshold)))
    return sel, ProjectionExec(sel, Schema([Field("ab", out_type)]), [op_cls(ColumnExpression(0), ColumnExpression(1))])


@pytest.fixture(params=["select_project", "gather"])
def compaction(request, monkeypatch):
    from kquery import operators as ops

    monkeypatch.setattr(ops, "SELECTION_COMPACTION", request.param)
    return request.param


@pytest.mark.parametrize("threshold", [-(1 << 62), 1 << 19, 1 << 62])
@pytest.mark.parametrize("nulls", [False, True])
def test_select_then_add_int64(gpu_ctx, threshold, nulls, compaction):
    """Both compactions SelectionExec takes for fixed-width columns (select-project pass, or the
    stream-ordered gather; nullable columns always gather)."""
    from kquery import native as N
    from kquery.columnar import DeviceColumn
    from kquery.expressions import AddExpression

    rng = np.random.default_rng(5)
    n = 1_000_003
    a = rng.integers(-(1 << 20), 1 << 20, n).astype(np.int64)
    b = rng.integers(-(1 << 62), 1 << 62, n).astype(np.int64)
    bv = rng.random(n) > 0.1 if nulls else None
    cols = [DeviceColumn.from_numpy(N.TYPE_INT64, a, None, ctx=gpu_ctx),
            DeviceColumn.from_numpy(N.TYPE_INT64, b, bv, ctx=gpu_ctx)]
    _, proj = _plan(N, cols, threshold, AddExpression, N.TYPE_INT64)
    out = next(proj.execute())
    col = out.field(0)
    if compaction == "gather" or nulls:
        assert col.pending is not None  # nothing read back yet
    keep = a > threshold
    assert out.rowCount() == int(keep.sum())
    with np.errstate(over="ignore"):
        want = a[keep] + b[keep]
    got = col.to_numpy()
    if nulls:
        vm = col.valid_mask()
        assert np.array_equal(vm, bv[keep])
        assert np.array_equal(got[vm], want[vm])
    else:
        assert np.array_equal(got, want)


def test_select_then_multiply_f64(gpu_ctx, compaction):
    from kquery import native as N
    from kquery.columnar import DeviceColumn
    from kquery.expressions import MultiplyExpression

    rng = np.random.default_rng(6)
    n = 300_001
    a = rng.integers(0, 1000, n).astype(np.int64)
    b = rng.normal(size=n)
    b[::97] = np.nan
    cols = [DeviceColumn.from_numpy(N.TYPE_INT64, a, None, ctx=gpu_ctx),
            DeviceColumn.from_numpy(N.TYPE_FLOAT64, b, None, ctx=gpu_ctx)]
    _, proj = _plan(N, cols, 500, MultiplyExpression, N.TYPE_FLOAT64)
    out = next(proj.execute())
    keep = a > 500
    want = a[keep].astype(np.float64) * b[keep]
    got = out.field(0).to_numpy()
    assert got.tobytes() == want.tobytes()


def test_async_count_matches_sync_filter(gpu_ctx):
    import torch

    from kquery import native as N
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(7)
    n = 777_777
    m = rng.random(n) > 0.37
    mv = rng.random(n) > 0.05
    x = rng.integers(-5, 5, n).astype(np.int32)
    mask = DeviceColumn.from_numpy(N.TYPE_BOOL, m, mv, ctx=gpu_ctx)
    xc = DeviceColumn.from_numpy(N.TYPE_INT32, x, None, ctx=gpu_ctx)
    out = DeviceColumn.empty(N.TYPE_INT32, n, False, ctx=gpu_ctx)
    cnt = torch.zeros(1, dtype=torch.int64, device=gpu_ctx.torch_device)
    mc, ic, oc = mask.as_c(), xc.as_c(), out.as_c()
    N.check(N.lib().qe_filter_apply_async(gpu_ctx.handle, N.C.byref(mc), N.C.byref(ic), 1, N.C.byref(oc),
                                          N.C.c_void_p(cnt.data_ptr())))
    gpu_ctx.synchronize()
    k = int(cnt.cpu().item())
    sel = m & mv
    assert k == int(sel.sum())
    assert np.array_equal(out.values[:k].cpu().numpy(), x[sel])
    # a UTF8 column is refused (its outputs need the count): qe_filter_apply handles it
    s = DeviceColumn.from_strings(["x"] * n, ctx=gpu_ctx)
    sc = s.as_c()
    st = N.lib().qe_filter_apply_async(gpu_ctx.handle, N.C.byref(mc), N.C.byref(sc), 1, N.C.byref(sc),
                                       N.C.c_void_p(cnt.data_ptr()))
    assert st == N.QE_ERR_UNSUPPORTED
