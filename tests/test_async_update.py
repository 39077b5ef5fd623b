"""Stream-ordered hash-aggregate updates (qe_hashagg_set_async): an update returns once its
kernel is queued, and the next call on the state reads its counters back — including the growth
and retry pass when the global table overflowed, which re-reads the (still live) input columns.
Results must equal the synchronous path's and the oracle's (HashAggregateExec, Main.kt:615-651)."""
import numpy as np
import pytest

from kquery import native as N
from kquery.aggregate import HashAggregateState
from oracle import gen
from oracle import semantics as S

from test_gpu_parity import ALL_FNS, C4_AGGS, C4_FNS, _c4_spec, assert_groups_equal, dcol, result_dict

pytestmark = pytest.mark.gpu


def _c4_ref(n, row0=0):
    k, _ = gen.generate(gen.GEN_MOD, 1024, 42, 0, row0, n)
    a, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 1, row0, n)
    b, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 2, row0, n)
    return S.group_aggregate([k], [None], [a + b, None, a, b], [None] * 4, C4_FNS, a > (1 << 19))


def test_async_fused_c4_equals_oracle(gpu_ctx):
    from kquery.datasource import C4_COLUMNS, generate_column

    n = 2_000_003
    cols = [generate_column(s, n, 0, 42, gpu_ctx) for s in C4_COLUMNS]
    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], C4_AGGS, 1024, async_update=True)
    ref = _c4_ref(n)
    for _ in range(3):  # reset -> update -> finalize, as bench.py's step
        st.reset()
        st.update_fused(cols, _c4_spec())
        kk, aa = st.finalize()
        assert_groups_equal(result_dict(kk, aa), ref, C4_FNS)
        ms, launches = st.last_kernel_time()
        assert ms > 0 and launches == 1


def test_async_overflow_retry_at_finalize(gpu_ctx):
    """Far more groups than expected: the global table overflows, rows are deferred, and the
    growth + retry pass run when finalize settles the update."""
    rng = np.random.default_rng(3)
    n = 300_000
    k = rng.integers(0, 60_000, n).astype(np.int64) * 31 + 7
    x = rng.integers(-2**40, 2**40, n).astype(np.int64)
    xv = rng.random(n) > 0.1
    K, X = dcol(gpu_ctx, N.TYPE_INT64, k), dcol(gpu_ctx, N.TYPE_INT64, x, xv)
    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(f, N.TYPE_INT64) for f in ALL_FNS], 16, async_update=True)
    st.update([K], [X] * len(ALL_FNS))
    keys, aggs = st.finalize()
    _, launches = st.last_kernel_time()
    assert launches >= 2, "expected the retry pass of deferred rows"
    ref = S.group_aggregate([k], [None], [x] * 6, [xv] * 6, ALL_FNS)
    assert_groups_equal(result_dict(keys, aggs), ref, ALL_FNS)


def test_async_multibatch_and_num_groups(gpu_ctx):
    """Several async updates in a row (each settles the one before), MIN/MAX row order across
    batches, then num_groups and finalize."""
    rng = np.random.default_rng(9)
    n = 120_000
    k = rng.choice(np.array([np.nan, 0.0, -0.0, 1.5, -2.25]), n)
    x = rng.choice(np.array([0.0, -0.0, -1.0, np.nan, 4.0]), n)
    xv = rng.random(n) > 0.2
    fns = [N.AGG_MAX, N.AGG_MIN, N.AGG_COUNT, N.AGG_SUM]
    st = HashAggregateState(gpu_ctx, [N.TYPE_FLOAT64], [(f, N.TYPE_FLOAT64) for f in fns], 16, async_update=True)
    batches = []
    for s in range(0, n, 25_000):
        e = min(n, s + 25_000)
        b = (dcol(gpu_ctx, N.TYPE_FLOAT64, k[s:e]), dcol(gpu_ctx, N.TYPE_FLOAT64, x[s:e], xv[s:e]))
        batches.append(b)  # inputs stay alive until the state settles
        st.update([b[0]], [b[1]] * 4)
    ref = S.group_aggregate([k], [None], [x] * 4, [xv] * 4, fns)
    assert st.num_groups() == len(ref)
    keys, aggs = st.finalize()
    assert_groups_equal(result_dict(keys, aggs), ref, fns)


def test_async_reset_discards_and_sync_toggle(gpu_ctx):
    rng = np.random.default_rng(4)
    n = 50_000
    k = rng.integers(0, 100, n).astype(np.int64)
    x = rng.integers(0, 1000, n).astype(np.int64)
    K, X = dcol(gpu_ctx, N.TYPE_INT64, k), dcol(gpu_ctx, N.TYPE_INT64, x)
    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(N.AGG_SUM, N.TYPE_INT64)], 128, async_update=True)
    st.update([K], [X])
    st.reset()  # the pending update is dropped with the table
    assert st.num_groups() == 0
    st.update([K], [X])
    N.check(N.lib().qe_hashagg_set_async(st.handle, 0))  # settles the pending update
    st.update([K], [X])  # synchronous from here on
    keys, aggs = st.finalize()
    ref = S.group_aggregate([k], [None], [x * 2], [None], [N.AGG_SUM])
    assert_groups_equal(result_dict(keys, aggs), ref, [N.AGG_SUM])


def test_finalize_output_resizes(gpu_ctx):
    """finalize carves its outputs at the previous result's size; a larger result carves again."""
    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(N.AGG_COUNT_STAR, N.TYPE_INT64)], 4)
    for groups in (3, 5000, 7, 0):
        k = np.arange(groups * 3, dtype=np.int64) % max(groups, 1)
        st.reset()
        if groups:
            st.update([dcol(gpu_ctx, N.TYPE_INT64, k)], [dcol(gpu_ctx, N.TYPE_INT64, k)])
        keys, aggs = st.finalize()
        assert keys[0].length == groups and aggs[0].length == groups
        if groups:
            assert sorted(keys[0].to_numpy().tolist()) == list(range(groups))
            assert set(aggs[0].to_numpy().tolist()) == {3}
