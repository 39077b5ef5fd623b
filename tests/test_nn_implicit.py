"""Implicit non-null counts in the hash-aggregate table: while an aggregate's inputs have been
non-nullable, its per-group non-null count equals COUNT(*), the table does not store it and the
fused kernel's flush skips those atomics. Nullable batches, table growth, exports and imports must
still give the oracle's COUNT(x) / AVG / all-null results (MaxAccumulator null rules, Main.kt:538-561;
HashAggregateExec, Main.kt:615-651)."""
import numpy as np
import pytest

from kquery import native as N
from kquery.aggregate import HashAggregateState
from oracle import semantics as S

from test_gpu_parity import ALL_FNS, agg_ctx, assert_groups_equal, dcol, result_dict  # noqa: F401

pytestmark = pytest.mark.gpu


def _batches(seed, n, ngroups, nullable_pattern):
    rng = np.random.default_rng(seed)
    out = []
    for nullable in nullable_pattern:
        k = rng.integers(0, ngroups, n).astype(np.int64) * 13 - 5
        x = rng.integers(-1000, 1000, n).astype(np.int64)
        xv = (rng.random(n) > 0.3) if nullable else None
        out.append((k, x, xv))
    return out


def _ref(batches):
    k = np.concatenate([b[0] for b in batches])
    x = np.concatenate([b[1] for b in batches])
    xv = np.concatenate([b[2] if b[2] is not None else np.ones(len(b[0]), bool) for b in batches])
    return S.group_aggregate([k], [None], [x] * 6, [xv] * 6, ALL_FNS)


@pytest.mark.parametrize("pattern", [(False, True, False), (False, False), (True, False), (False,)])
def test_nullable_batch_after_implicit_counts(agg_ctx, pattern):
    batches = _batches(len(pattern) * 7 + sum(pattern), 60_000, 300, pattern)
    st = HashAggregateState(agg_ctx, [N.TYPE_INT64], [(f, N.TYPE_INT64) for f in ALL_FNS], 512)
    for k, x, xv in batches:
        st.update([dcol(agg_ctx, N.TYPE_INT64, k)], [dcol(agg_ctx, N.TYPE_INT64, x, xv)] * 6)
    keys, aggs = st.finalize()
    assert_groups_equal(result_dict(keys, aggs), _ref(batches), ALL_FNS)


def test_growth_export_import_keep_counts(agg_ctx):
    """Many more groups than expected (table growth while counts are implicit), then the partial's
    records (exported COUNT(x) = COUNT(*)) merged into a second state that also saw nulls."""
    b1 = _batches(3, 200_000, 40_000, (False,))
    b2 = _batches(4, 50_000, 40_000, (True,))
    a = HashAggregateState(agg_ctx, [N.TYPE_INT64], [(f, N.TYPE_INT64) for f in ALL_FNS], 16)
    for k, x, xv in b1:
        a.update([dcol(agg_ctx, N.TYPE_INT64, k)], [dcol(agg_ctx, N.TYPE_INT64, x, xv)] * 6)
    b = HashAggregateState(agg_ctx, [N.TYPE_INT64], [(f, N.TYPE_INT64) for f in ALL_FNS], 16)
    for k, x, xv in b2:
        b.update([dcol(agg_ctx, N.TYPE_INT64, k)], [dcol(agg_ctx, N.TYPE_INT64, x, xv)] * 6)
    recs, counts = a.export(1)
    b.import_records(recs, counts[0])
    keys, aggs = b.finalize()
    assert_groups_equal(result_dict(keys, aggs), _ref(b1 + b2), ALL_FNS)
    # the exporter itself still finalises from its implicit counts
    keys, aggs = a.finalize()
    assert_groups_equal(result_dict(keys, aggs), _ref(b1), ALL_FNS)
