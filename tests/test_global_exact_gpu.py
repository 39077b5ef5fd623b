"""Global (no GROUP BY) fp64 SUM / AVG: the correctly rounded exact sum, math.fsum's value bit for
bit over the whole fp64 range (SURVEY §8a A9 asks for 1e-9; the same contract as the GROUP BY sums
of tests/test_fp64_sum_gpu.py).

qe_agg_global sums with Neumaier-compensated partials and bounds their error at the end
(qe_agg_global.hip sum_certified): when every value within the bound rounds to the same double, that
double is the answer; otherwise — cancellation, a sum near a rounding boundary, finite inputs whose
running sum overflowed — the column is summed again exactly (k_agg_global_fx: 256-bit fixed point
plus full-range words for inputs of 2^126 or more and bits below 2^-128). qe_agg_global_merge of
shard partials returns QE_NEED_EXACT in that case, and the exact round (qe_agg_global_exact_partial
per shard, qe_agg_global_merge_exact) gives the exact sum over all shards."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _global(ctx, x, valid=None, mask=None):
    from kquery import native as N
    from kquery.columnar import DeviceColumn

    r = N.QeGlobalAgg()
    col = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, valid, ctx=ctx)  # (held: the C views borrow its memory)
    mcol = DeviceColumn.from_numpy(N.TYPE_BOOL, mask, None, ctx=ctx) if mask is not None else None
    c = col.as_c()
    m = mcol.as_c() if mcol is not None else None
    N.check(N.lib().qe_agg_global(ctx.handle, N.C.byref(c), N.C.byref(m) if m is not None else None, N.C.byref(r)))
    ctx.synchronize()
    return r


def _bits(v):
    return np.float64(v).view(np.int64)


def _cancelling(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.choice([1.0, 0.5, 0.1, -0.25, 3.0], n)
    k = n // 100
    x[:k] = 2.0 ** 60
    x[-k:] = -(2.0 ** 60)
    return x[rng.permutation(n)]


@pytest.mark.parametrize("form", ["dense", "nulls", "mask"])
def test_cancellation_is_exact(gpu_ctx, form):
    from kquery.columnar import f64_from_bits

    n = 2_000_003
    x = _cancelling(n, 5)
    rng = np.random.default_rng(6)
    valid = rng.random(n) > 0.1 if form == "nulls" else None
    mask = rng.random(n) > 0.3 if form == "mask" else None
    sel = np.ones(n, dtype=bool)
    if valid is not None:
        sel &= valid
    if mask is not None:
        sel &= mask
    want = math.fsum(x[sel].tolist())
    r = _global(gpu_ctx, x, valid, mask)
    assert r.count == int(sel.sum())
    assert f64_from_bits(r.sum) == want, (f64_from_bits(r.sum), want)
    assert _bits(r.avg) == _bits(want / r.count)


def test_well_conditioned_is_fsum(gpu_ctx):
    from kquery.columnar import f64_from_bits

    for seed in range(3):
        x = np.random.default_rng(3 + seed).normal(size=3_000_000) * 1e3 + 5.0
        want = math.fsum(x.tolist())
        r = _global(gpu_ctx, x)
        assert _bits(f64_from_bits(r.sum)) == _bits(want)


def _fsum(xs):
    """math.fsum; on its intermediate-overflow error the exact sum (fractions, ties to even)."""
    from fractions import Fraction

    try:
        return math.fsum(xs)
    except OverflowError:
        q = sum((Fraction(float(v)) for v in xs), Fraction(0))
        try:
            return float(q)
        except OverflowError:
            return math.inf if q > 0 else -math.inf


FULL_RANGE = [[1e-40] * 5000, [1e300] + [1.0] * 3000 + [-1e300], [5e-324] * 4097, [1e308, 1e308, -1e308],
              [1e308, 1e308], [-1e-320, 3e-322, 2.2250738585072014e-308, -5e-324], [2.0 ** 200, 1.0, -(2.0 ** 200)]]


@pytest.mark.parametrize("case", range(len(FULL_RANGE)))
@pytest.mark.parametrize("form", ["dense", "mask"])
def test_full_range_is_fsum(gpu_ctx, case, form):
    from kquery.columnar import f64_from_bits

    x = np.random.default_rng(case).permutation(np.array(FULL_RANGE[case]))
    mask = np.ones(len(x), dtype=bool) if form == "mask" else None
    r = _global(gpu_ctx, x, None, mask)
    assert _bits(f64_from_bits(r.sum)) == _bits(_fsum(x.tolist())), (f64_from_bits(r.sum), _fsum(x.tolist()))


@pytest.mark.parametrize("vals,want", [([math.inf, 1.0, 2.0], math.inf), ([math.inf, -math.inf, 1.0], math.nan),
                                       ([1.0, math.nan, -math.inf], math.nan),
                                       ([-0.0, -0.0], 0.0),  # an exact zero sum is +0.0, as in GROUP BY
                                       ([2.0 ** 100, 1.0, -(2.0 ** 100)], 1.0)])
def test_specials(gpu_ctx, vals, want):
    from kquery.columnar import f64_from_bits

    r = _global(gpu_ctx, np.array(vals))
    got = f64_from_bits(r.sum)
    if math.isnan(want):
        assert math.isnan(got)
    else:
        assert _bits(got) == _bits(want), (got, want)


def _merge(gpu_ctx, pieces):
    """qe_agg_global_partial per piece, qe_agg_global_merge, and the exact round when it asks."""
    import torch

    from kquery import native as N
    from kquery.columnar import DeviceColumn

    parts, words, cols = [], [], []
    base = 0
    for x in pieces:
        p = torch.empty(N.GLOBAL_PARTIAL_BYTES, dtype=torch.uint8, device=gpu_ctx.torch_device)
        c = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=gpu_ctx)
        cols.append(c)
        cc = c.as_c()
        N.check(N.lib().qe_agg_global_partial(gpu_ctx.handle, N.C.byref(cc), None, base, N.C.c_void_p(p.data_ptr())))
        parts.append(p)
        base += len(x)
    buf = torch.cat(parts)
    out = N.QeGlobalAgg()
    st = N.lib().qe_agg_global_merge(gpu_ctx.handle, N.TYPE_FLOAT64, N.C.c_void_p(buf.data_ptr()), len(pieces),
                                     N.C.byref(out))
    if st == N.QE_NEED_EXACT:
        for c in cols:
            w = torch.empty(N.GLOBAL_EXACT_BYTES, dtype=torch.uint8, device=gpu_ctx.torch_device)
            cc = c.as_c()
            N.check(N.lib().qe_agg_global_exact_partial(gpu_ctx.handle, N.C.byref(cc), None, N.C.c_void_p(w.data_ptr())))
            words.append(w)
        allw = torch.cat(words)
        st = N.lib().qe_agg_global_merge_exact(gpu_ctx.handle, N.C.c_void_p(allw.data_ptr()), len(pieces),
                                               N.C.byref(out))
    N.check(st)
    return out, bool(words)


def test_merge_of_cancelling_shards_is_exact(gpu_ctx):
    from kquery.columnar import f64_from_bits

    pieces = [np.array([2.0 ** 100] + [1.0] * 1000), np.array([-(2.0 ** 100)] + [0.5] * 1000)]
    out, second = _merge(gpu_ctx, pieces)
    assert second and f64_from_bits(out.sum) == 1500.0 and out.count == 2002
    assert out.avg == 1500.0 / 2002
    # the whole column through qe_agg_global: the same
    r = _global(gpu_ctx, np.concatenate(pieces))
    assert f64_from_bits(r.sum) == 1500.0


def test_merge_of_zero_sum_shards(gpu_ctx):
    """Shards whose sums cancel to exactly zero (an uncertifiable bound: zero has no relative
    error) take the exact round and give +0.0; full-range shards give math.fsum's value."""
    from kquery.columnar import f64_from_bits

    out, second = _merge(gpu_ctx, [np.array([3.5, -1.25]), np.array([-2.25, 0.0])])
    assert second and _bits(f64_from_bits(out.sum)) == _bits(0.0)
    pieces = [np.array([1e308, 5e-324]), np.array([1e308, -1e-300]), np.array([-1e308, 1e-300])]
    out, _ = _merge(gpu_ctx, pieces)
    assert _bits(f64_from_bits(out.sum)) == _bits(_fsum(np.concatenate(pieces).tolist()))
    out, second = _merge(gpu_ctx, [np.arange(1000, dtype=np.float64), np.arange(1000, dtype=np.float64)])
    assert not second and f64_from_bits(out.sum) == 999000.0
