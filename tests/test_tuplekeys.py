"""Composite GROUP BY keys (K:621-626: the row key is a List of key values, compared with
List.equals) beyond what packs into 63 bits: every distinct key tuple gets a dictionary code
(qe_strdict_encode_tuple) and the hash aggregate groups by the code. Checked against the oracle's
literal HashAggregateExec loop: nulls are a key value, fp64 keys follow Double.equals (all NaNs
equal, +0.0 != -0.0), UTF-8 members compare by content."""
import math

import numpy as np
import pytest

from oracle import semantics as S


def test_packable_rule():
    from kquery import native as N
    from kquery.aggregate import packable

    assert packable([]) and packable([N.TYPE_INT64]) and packable([N.TYPE_FLOAT64])
    assert packable([N.TYPE_INT32, N.TYPE_UINT8]) and packable([N.TYPE_UINT8] * 4)
    assert not packable([N.TYPE_INT64, N.TYPE_INT64]) and not packable([N.TYPE_INT32, N.TYPE_INT32])
    assert not packable([N.TYPE_BOOL]) and not packable([N.TYPE_FLOAT64, N.TYPE_UINT8])


def _col(ctx, t, vals, valid):
    from kquery.columnar import DeviceColumn

    return DeviceColumn.from_numpy(t, vals, valid, ctx=ctx)


def _py(t, vals, valid):
    out = []
    for v, ok in zip(vals, valid if valid is not None else [True] * len(vals)):
        if not ok:
            out.append(None)
        elif t == "f64":
            out.append(float(v))
        elif t == "bool":
            out.append(bool(v))
        else:
            out.append(int(v))
    return out


def _gen(rng, t, n, distinct):
    if t == "i64":
        pool = rng.integers(-2**63, 2**63 - 1, distinct, dtype=np.int64, endpoint=True)
        return pool[rng.integers(0, distinct, n)], rng.random(n) > 0.05
    if t == "i32":
        pool = rng.integers(-2**31, 2**31 - 1, distinct).astype(np.int32)
        return pool[rng.integers(0, distinct, n)], rng.random(n) > 0.05
    if t == "f64":
        pool = np.array([0.0, -0.0, np.nan, -np.nan, 1.5, -2.25, np.inf, 1e300][:max(2, min(distinct, 8))])
        return pool[rng.integers(0, len(pool), n)], rng.random(n) > 0.05
    if t == "u8":
        return rng.integers(0, min(distinct, 256), n).astype(np.uint8), rng.random(n) > 0.05
    return rng.random(n) < 0.5, rng.random(n) > 0.05  # bool


TYPES = {"i64": 1, "f64": 2, "bool": 3, "i32": 5, "u8": 6}


@pytest.mark.gpu
@pytest.mark.parametrize("kinds,distinct,n", [
    (("i64", "i64"), 50, 100_000),
    (("f64", "i64"), 8, 80_000),
    (("i32", "i32", "i32"), 20, 120_000),
    (("bool",), 2, 10_000),
    (("u8", "i64", "bool", "f64"), 6, 150_000),
    (("i64", "i32"), 100_000, 300_000),  # many distinct tuples: growth past the initial capacity
])
def test_tuple_group_by(gpu_ctx, kinds, distinct, n):
    from kquery import native as N
    from kquery.aggregate import HashAggregateState

    rng = np.random.default_rng(n + distinct)
    keys = [_gen(rng, t, n, distinct) for t in kinds]
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    types = [TYPES[t] for t in kinds]
    aggs = [(N.AGG_SUM, N.TYPE_INT64), (N.AGG_COUNT_STAR, N.TYPE_INT64), (N.AGG_MAX, N.TYPE_INT64)]
    st = HashAggregateState(gpu_ctx, types, aggs, 64)
    assert st.key_layout == 2  # key-tuple codes
    # two batches: the dictionary keeps codes across update calls
    h = n // 2
    for a, b in ((0, h), (h, n)):
        st.update([_col(gpu_ctx, ty, kv[a:b], kvv[a:b]) for ty, (kv, kvv) in zip(types, keys)],
                  [_col(gpu_ctx, N.TYPE_INT64, v[a:b], None), None, _col(gpu_ctx, N.TYPE_INT64, v[a:b], None)])
    kout, aout = st.finalize()
    got = {}
    cols = [c.to_pylist() for c in kout] + [c.to_pylist() for c in aout]
    for row in zip(*cols):
        got[tuple(S.canon(x) for x in row[:len(kinds)])] = list(row[len(kinds):])
    want = S.hash_aggregate_rows([_py(t, kv, kvv) for t, (kv, kvv) in zip(kinds, keys)],
                                 [v.tolist(), [1] * n, v.tolist()], [S.AGG_SUM, S.AGG_COUNT_STAR, S.AGG_MAX],
                                 [False, False, False])
    assert len(got) == len(want)
    for k, w in want.items():
        assert got[k] == w, (k, got.get(k), w)


@pytest.mark.gpu
def test_utf8_and_int64_keys(gpu_ctx):
    """GROUP BY (Utf8, int64): the UTF-8 member is dictionary-encoded first, then the tuple."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(4)
    n = 60_000
    words = ["", "a", "VendorID", "Pärsson", "x" * 50]
    s = [None if rng.random() < 0.03 else words[i] for i in rng.integers(0, len(words), n)]
    k = rng.integers(-3, 3, n).astype(np.int64) * (2**40)
    kv = rng.random(n) > 0.05
    f = rng.normal(size=n)
    st = HashAggregateState(gpu_ctx, [N.TYPE_UTF8, N.TYPE_INT64], [(N.AGG_MAX, N.TYPE_FLOAT64),
                                                                  (N.AGG_COUNT, N.TYPE_FLOAT64)], 16)
    st.update([DeviceColumn.from_strings(s, ctx=gpu_ctx), DeviceColumn.from_numpy(N.TYPE_INT64, k, kv, ctx=gpu_ctx)],
              [DeviceColumn.from_numpy(N.TYPE_FLOAT64, f, ctx=gpu_ctx)] * 2)
    kout, aout = st.finalize()
    cols = [c.to_pylist() for c in kout] + [c.to_pylist() for c in aout]
    got = {(r[0], r[1]): [r[2], r[3]] for r in zip(*cols)}
    want = S.hash_aggregate_rows([s, _py("i64", k, kv)], [f.tolist()] * 2, [S.AGG_MAX, S.AGG_COUNT], [True, True])
    assert len(got) == len(want)
    for key, w in want.items():
        g = got[key]
        assert g[1] == w[1] and (g[0] == w[0] or (math.isnan(g[0]) and math.isnan(w[0])))
