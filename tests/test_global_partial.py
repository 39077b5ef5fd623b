"""Global aggregate over a column split into pieces (batches, or rank shards — SURVEY §8e):
qe_agg_global_partial per piece with its global row base, then qe_agg_global_merge, must equal
the oracle over the whole column (MaxAccumulator K:538-561 order rules across piece boundaries:
a NaN seed in a later piece, ±0.0 ties between pieces, all-null and empty pieces), and every
merge order of the same partials gives the same bits."""
import numpy as np
import pytest

from oracle import semantics as S

pytestmark = pytest.mark.gpu
REL = 1e-9


def _partials(ctx, N, DeviceColumn, pieces, t):
    import torch

    parts, cols = [], []
    base = 0
    for x, xv in pieces:
        p = torch.empty(N.GLOBAL_PARTIAL_BYTES, dtype=torch.uint8, device=ctx.torch_device)
        cols.append(DeviceColumn.from_numpy(t, x, xv, ctx=ctx))  # held until the kernels are done
        c = cols[-1].as_c()
        N.check(N.lib().qe_agg_global_partial(ctx.handle, N.C.byref(c), None, base, N.C.c_void_p(p.data_ptr())))
        parts.append(p)
        base += len(x)
    ctx.synchronize()
    return parts


def _merge(ctx, N, parts, t):
    import torch

    buf = torch.cat(parts)
    out = N.QeGlobalAgg()
    N.check(N.lib().qe_agg_global_merge(ctx.handle, t, N.C.c_void_p(buf.data_ptr()), len(parts), N.C.byref(out)))
    return out


def _check(r, ref, is_f):
    from kquery.columnar import f64_from_bits

    assert r.rows == ref["rows"] and r.count == ref["count"]
    if ref["count"] == 0:
        assert r.valid == 0
        return
    if is_f:
        assert S.rows_equal(f64_from_bits(r.sum), ref["sum"], REL)
        assert S.rows_equal(f64_from_bits(r.min), ref["min"]) and S.rows_equal(f64_from_bits(r.max), ref["max"])
    else:
        assert (r.sum, r.min, r.max) == (ref["sum"], ref["min"], ref["max"])
    assert S.rows_equal(r.avg, ref["avg"], REL)


CASES = {
    "nan_seed_in_second_piece": [([], []), ([np.nan, 3.0], [1, 1]), ([7.0], [1])],
    "nan_after_seed": [([1.0], [1]), ([np.nan, 9.0], [1, 1])],
    "zero_ties": [([-1.0, -0.0], [1, 1]), ([0.0, -2.0], [1, 1])],
    "pos_zero_first": [([0.0], [1]), ([-0.0], [1])],
    "all_null_pieces": [([5.0, 6.0], [0, 0]), ([np.nan, -0.0, 4.0], [0, 1, 1])],
    "all_null": [([1.0], [0]), ([2.0], [0])],
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_piece_boundaries(gpu_ctx, case):
    from kquery import native as N
    from kquery.columnar import DeviceColumn

    pieces = [(np.array(x, dtype=np.float64), np.array(v, dtype=bool)) for x, v in CASES[case]]
    x = np.concatenate([p[0] for p in pieces])
    xv = np.concatenate([p[1] for p in pieces])
    ref = S.global_aggregate(x, xv)
    parts = _partials(gpu_ctx, N, DeviceColumn, pieces, N.TYPE_FLOAT64)
    r = _merge(gpu_ctx, N, parts, N.TYPE_FLOAT64)
    _check(r, ref, True)
    r2 = _merge(gpu_ctx, N, parts[::-1], N.TYPE_FLOAT64)  # partial order does not matter
    assert (r2.sum, r2.min, r2.max, r2.count, r2.rows) == (r.sum, r.min, r.max, r.count, r.rows)


@pytest.mark.parametrize("kind", ["f64", "i64"])
def test_random_pieces_match_whole_column(gpu_ctx, kind):
    from kquery import native as N
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(11)
    n = 3_000_001
    if kind == "i64":
        x = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
        xv = rng.random(n) > 0.1
        t = N.TYPE_INT64
    else:
        x = rng.normal(size=n) * 1e3
        x[rng.random(n) < 0.01] = np.nan
        x[rng.random(n) < 0.01] = -0.0
        xv = rng.random(n) > 0.1
        t = N.TYPE_FLOAT64
    cuts = sorted(rng.choice(np.arange(1, n), 6, replace=False).tolist())
    bounds = [0] + cuts + [n]
    pieces = [(x[a:b], xv[a:b]) for a, b in zip(bounds[:-1], bounds[1:])]
    r = _merge(gpu_ctx, N, _partials(gpu_ctx, N, DeviceColumn, pieces, t), t)
    _check(r, S.global_aggregate(x, xv), t == N.TYPE_FLOAT64)
