"""Global (no GROUP BY) fp64 SUM / AVG within 1e-9 of the exact sum, or a loud failure (SURVEY §8a
A9, the same contract as the GROUP BY sums of tests/test_fp64_sum_gpu.py).

qe_agg_global sums with Neumaier-compensated partials and bounds their error at the end
(qe_agg_global.hip sum_certified); a column whose sum the bound cannot place within 1e-9 — heavy
cancellation, or finite inputs whose running sum overflowed — is summed again exactly in fixed point
(k_agg_global_fx), so the result is then math.fsum's bit for bit. qe_agg_global_merge has no rows to
go back to: an uncertifiable merge of shard partials fails with QE_ERR_UNSUPPORTED instead."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _global(ctx, x, valid=None, mask=None):
    from kquery import native as N
    from kquery.columnar import DeviceColumn

    r = N.QeGlobalAgg()
    c = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, valid, ctx=ctx).as_c()
    m = DeviceColumn.from_numpy(N.TYPE_BOOL, mask, None, ctx=ctx).as_c() if mask is not None else None
    N.check(N.lib().qe_agg_global(ctx.handle, N.C.byref(c), N.C.byref(m) if m is not None else None, N.C.byref(r)))
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


def test_well_conditioned_stays_within_bound(gpu_ctx):
    from kquery.columnar import f64_from_bits

    x = np.random.default_rng(3).normal(size=3_000_000) * 1e3 + 5.0
    want = math.fsum(x.tolist())
    r = _global(gpu_ctx, x)
    assert abs(f64_from_bits(r.sum) - want) <= 1e-9 * abs(want)


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


def test_overflowing_finite_inputs_fail_loudly(gpu_ctx):
    """1e308 + 1e308 - 1e308: the running sum overflows and 1e308 is beyond the exact range, so
    no sum within 1e-9 can be given: an error, never a silent Inf."""
    with pytest.raises(Exception, match="not exact to 1e-9"):
        _global(gpu_ctx, np.array([1e308, 1e308, -1e308]))


def test_merge_of_cancelling_shards_fails_loudly(gpu_ctx):
    import torch

    from kquery import native as N
    from kquery.columnar import DeviceColumn, f64_from_bits

    pieces = [np.array([2.0 ** 100] + [1.0] * 1000), np.array([-(2.0 ** 100)] + [0.5] * 1000)]
    parts = []
    base = 0
    for x in pieces:
        p = torch.empty(N.GLOBAL_PARTIAL_BYTES, dtype=torch.uint8, device=gpu_ctx.torch_device)
        c = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=gpu_ctx).as_c()
        N.check(N.lib().qe_agg_global_partial(gpu_ctx.handle, N.C.byref(c), None, base, N.C.c_void_p(p.data_ptr())))
        parts.append(p)
        base += len(x)
    buf = torch.cat(parts)
    out = N.QeGlobalAgg()
    with pytest.raises(Exception, match="cannot be certified"):
        N.check(N.lib().qe_agg_global_merge(gpu_ctx.handle, N.TYPE_FLOAT64, N.C.c_void_p(buf.data_ptr()), 2,
                                            N.C.byref(out)))
    # the whole column through qe_agg_global is exact
    r = _global(gpu_ctx, np.concatenate(pieces))
    assert f64_from_bits(r.sum) == 1500.0
