"""Dictionary-keyed partials merged and exchanged by key CONTENT through the C ABI (VERDICT r05 #1;
the reference's partial -> final merge, Main.kt:1309-1325, over its Utf8-keyed query, K:1336).

A UTF-8 GROUP BY key (or a key list that does not pack into 63 bits) is grouped by dictionary codes
the C state owns; codes mean nothing to another state, so:
* qe_hashagg_merge of two states whose dictionaries number the same strings differently (keys
  longer than 7 bytes, inserted in different orders) gives the oracle's groups;
* the same for key-tuple codes, for codes a caller encoded with its own dictionary
  (qe_hashagg_bind_key_dict), and for a lone UTF-8 key mixing packed (<= 7 bytes) and long keys;
* the raw record calls refuse a dictionary-keyed state;
* qe_hashagg_exchange of dictionary-keyed partials across two ranks (in-process loopback
  communicator: the C ABI's own exchange, no torch on the data path) for K:1336's shape — Utf8
  VendorID, MAX(CAST(fare_amount AS double)) — and for a tuple-keyed SUM / COUNT / MIN state.
Every result is compared per group with oracle/semantics.py."""
import random
import threading

import numpy as np
import pytest

from oracle import cast_ref as R
from oracle import semantics as S

pytestmark = pytest.mark.gpu

WORDS = ["1", "2", "VTS", "", "Pärsson", "x" * 45, "long-key-alpha-1", "beta-long-key-2", "gamma-key-3"]


def _rows(seed, n, nulls=0.03):
    rng = np.random.default_rng(seed)
    s = [None if rng.random() < nulls else WORDS[i] for i in rng.integers(0, len(WORDS), n)]
    k = rng.integers(-3, 4, n).astype(np.int64) * (2 ** 40)
    kv = rng.random(n) > 0.05
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    return s, k, kv, v


def _groups(keys, aggs):
    rows = [c.to_pylist() for c in keys] + [c.to_pylist() for c in aggs]
    return {tuple(r[: len(keys)]): list(r[len(keys):]) for r in zip(*rows)}


def _aggs(N):
    return [(N.AGG_SUM, N.TYPE_INT64), (N.AGG_COUNT_STAR, N.TYPE_INT64), (N.AGG_MIN, N.TYPE_INT64)]


def _update(st, ctx, mode, s, k, kv, v):
    from kquery import native as N
    from kquery.columnar import DeviceColumn

    keys = [DeviceColumn.from_strings(s, ctx=ctx)]
    if mode == "tuple":
        keys.append(DeviceColumn.from_numpy(N.TYPE_INT64, k, kv, ctx=ctx))
    vc = DeviceColumn.from_numpy(N.TYPE_INT64, v, ctx=ctx)
    st.update(keys, [vc, None, vc])


def _want(mode, parts):
    ks, kk, vs = [], [], []
    for s, k, kv, v in parts:
        ks += s
        kk += [int(x) if ok else None for x, ok in zip(k, kv)]
        vs += v.tolist()
    kcols = [ks] if mode == "utf8" else [ks, kk]
    return S.hash_aggregate_rows(kcols, [vs, [1] * len(vs), vs], [S.AGG_SUM, S.AGG_COUNT_STAR, S.AGG_MIN],
                                 [False] * 3)


@pytest.mark.parametrize("mode", ["utf8", "tuple"])
def test_merge_by_content(gpu_ctx, mode):
    from kquery import native as N
    from kquery.aggregate import HashAggregateState

    types = [N.TYPE_UTF8] if mode == "utf8" else [N.TYPE_UTF8, N.TYPE_INT64]
    parts = [_rows(11, 20_000), _rows(12, 17_000)]
    # the second partition sees the strings in reverse first-occurrence order: different codes
    parts[1] = (list(reversed(parts[1][0])), parts[1][1], parts[1][2], parts[1][3])
    states = []
    for p in parts:
        st = HashAggregateState(gpu_ctx, types, _aggs(N), 64)
        _update(st, gpu_ctx, mode, *p)
        states.append(st)
    assert states[0].key_layout == (1 if mode == "utf8" else 2)
    owner = HashAggregateState(gpu_ctx, types, _aggs(N), 8)
    owner.merge(states[1])
    owner.merge(states[0])
    assert _groups(*owner.finalize()) == _want(mode, parts)
    # partition 0's groups merged straight into partition 1's state (the other dictionary)
    states[1].merge(states[0])
    assert _groups(*states[1].finalize()) == _want(mode, parts)


def test_raw_record_calls_refuse_dictionary_keys(gpu_ctx):
    from kquery import native as N
    from kquery.aggregate import HashAggregateState

    st = HashAggregateState(gpu_ctx, [N.TYPE_UTF8], _aggs(N), 16)
    _update(st, gpu_ctx, "utf8", *_rows(3, 1000))
    with pytest.raises(N.IllegalStateException):
        st.export(2)
    with pytest.raises(N.IllegalStateException):
        st.export_slots(2, 64)
    other = HashAggregateState(gpu_ctx, [N.TYPE_INT64], _aggs(N), 16)
    with pytest.raises(N.IllegalArgumentException):  # different key types: no merge
        other.merge(st)


def test_bound_external_dictionaries_merge_by_content(gpu_ctx):
    """Codes a caller encodes with its own dictionary (two partitions, two dictionaries): binding
    the dictionary (qe_hashagg_bind_key_dict) makes finalize decode and merges go by content."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn
    from kquery.strdict import StringDictionary

    parts = [_rows(21, 9000), _rows(22, 7000)]
    parts[1] = (list(reversed(parts[1][0])), parts[1][1], parts[1][2], parts[1][3])
    states, dicts = [], []
    for p in parts:
        d = StringDictionary(gpu_ctx, 64)
        st = HashAggregateState(gpu_ctx, [N.TYPE_INT32], _aggs(N), 64)
        st.bind_key_dict(0, d)
        codes = d.encode(DeviceColumn.from_strings(p[0], ctx=gpu_ctx))
        vc = DeviceColumn.from_numpy(N.TYPE_INT64, p[3], ctx=gpu_ctx)
        st.update([codes], [vc, None, vc])
        states.append(st)
        dicts.append(d)
    states[1].merge(states[0])
    assert _groups(*states[1].finalize()) == _want("utf8", parts)


def test_wide_keys_packed_and_long_merge(gpu_ctx):
    """A lone UTF-8 key: values of <= 7 bytes are their own wide codes (no dictionary; a CSV-style
    length bound skips even the dictionary pass), longer ones get dictionary codes; a merge of a
    packed-only partial into a state that holds long keys, and the reverse, by content."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    short = ["1", "2", "4", "VTS", "CMT"]
    rng = random.Random(5)
    s0 = [rng.choice(short) for _ in range(5000)]
    s1 = [rng.choice(short + ["a-much-longer-vendor-name"]) for _ in range(4000)]
    v0 = np.arange(5000, dtype=np.int64)
    v1 = np.arange(4000, dtype=np.int64) * 3
    a = HashAggregateState(gpu_ctx, [N.TYPE_UTF8], _aggs(N), 16)
    c0 = DeviceColumn.from_strings(s0, ctx=gpu_ctx)
    c0.max_len = 3  # the producer's bound: packed codes straight from the bytes
    a.update([c0], [DeviceColumn.from_numpy(N.TYPE_INT64, v0, ctx=gpu_ctx), None,
                    DeviceColumn.from_numpy(N.TYPE_INT64, v0, ctx=gpu_ctx)])
    b = HashAggregateState(gpu_ctx, [N.TYPE_UTF8], _aggs(N), 16)
    vb = DeviceColumn.from_numpy(N.TYPE_INT64, v1, ctx=gpu_ctx)
    b.update([DeviceColumn.from_strings(s1, ctx=gpu_ctx)], [vb, None, vb])
    want = S.hash_aggregate_rows([s0 + s1], [v0.tolist() + v1.tolist(), [1] * 9000, v0.tolist() + v1.tolist()],
                                 [S.AGG_SUM, S.AGG_COUNT_STAR, S.AGG_MIN], [False] * 3)
    owner = HashAggregateState(gpu_ctx, [N.TYPE_UTF8], _aggs(N), 16)
    owner.merge(a)
    owner.merge(b)
    assert _groups(*owner.finalize()) == want
    b.merge(a)
    assert _groups(*b.finalize()) == want


def test_max_len_bound_is_checked(gpu_ctx):
    """A wrong length bound fails the aggregate loudly instead of grouping two strings as one."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    st = HashAggregateState(gpu_ctx, [N.TYPE_UTF8], _aggs(N), 16)
    c = DeviceColumn.from_strings(["short", "much-longer-than-seven"], ctx=gpu_ctx)
    c.max_len = 5
    v = DeviceColumn.from_numpy(N.TYPE_INT64, np.array([1, 2], dtype=np.int64), ctx=gpu_ctx)
    with pytest.raises(N.IllegalArgumentException, match="max_len"):  # at the update's read-back or at finalize
        st.update([c], [v, None, v])
        st.finalize()


def test_keyed_blocks_numeric_keys(gpu_ctx):
    """qe_hashagg_export_keyed / import_keyed work for every state: numeric keys by content give
    the raw merge's groups (4 partitions exported, imported in reverse order)."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(9)
    n = 30_000
    k = rng.integers(0, 3000, n).astype(np.int64)
    kv = rng.random(n) > 0.02
    x = rng.normal(size=n)
    aggs = [(N.AGG_SUM, N.TYPE_FLOAT64), (N.AGG_MAX, N.TYPE_FLOAT64), (N.AGG_COUNT_STAR, N.TYPE_INT64)]
    src = HashAggregateState(gpu_ctx, [N.TYPE_INT64], aggs, 4096)
    kc = DeviceColumn.from_numpy(N.TYPE_INT64, k, kv, ctx=gpu_ctx)
    xc = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, ctx=gpu_ctx)
    src.update([kc], [xc, xc, None])
    blocks, sizes = src.export_keyed(4)
    assert len(sizes) == 4 and sum(sizes) == blocks.numel()
    dst = HashAggregateState(gpu_ctx, [N.TYPE_INT64], aggs, 64)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    got_recs = 0
    for p in reversed(range(4)):
        got_recs += dst.import_keyed(blocks[int(offs[p]): int(offs[p + 1])], [sizes[p]])
    want = S.hash_aggregate_rows([[int(a) if ok else None for a, ok in zip(k, kv)]], [x.tolist(), x.tolist(), [1] * n],
                                 [S.AGG_SUM, S.AGG_MAX, S.AGG_COUNT_STAR], [True, True, False])
    assert got_recs == len(want)
    assert _groups(*dst.finalize()) == want


def _loopback(world, rank_main):
    from kquery import native as N

    hub = N.C.c_void_p()
    N.check(N.lib().qe_comm_loopback_hub_create(world, N.C.byref(hub)))
    out, errors = [None] * world, []

    def run(r):
        try:
            out[r] = rank_main(r, hub)
        except Exception as e:  # reported by the main thread
            errors.append(repr(e))

    threads = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(100)
    N.lib().qe_comm_loopback_hub_destroy(hub)
    assert not errors, errors
    assert all(o is not None for o in out)
    return out


def test_exchange_k1336_shape_two_ranks(gpu_ctx):
    """Main.kt:1336 across two ranks through qe_hashagg_exchange: each rank CASTs its fare strings,
    aggregates MAX by Utf8 VendorID (long and short vendor strings, nulls), and the exchange moves
    each group to the rank owning its content hash, where it is re-encoded and merged."""
    import torch

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import Context, DeviceColumn
    from kquery.exchange import exchange_partials_native

    vendors = ["1", "2", "4", "Creative Mobile Technologies", "VeriFone Inc.", None]
    data = []
    for r in range(2):
        rng = random.Random(1336 + r)
        n = 30_000 + 5000 * r
        vend = [rng.choice(vendors) for _ in range(n)]
        fare = [repr(round(rng.uniform(-5, 300), 2)) for _ in range(n)]
        data.append((vend, fare))

    class Comm:  # what exchange_partials_native reads of a NativeComm
        pass

    def rank_main(r, hub):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            ctx = Context.get(0)
            vend, fare = data[r]
            fc = DeviceColumn.from_strings(fare, ctx=ctx)
            fd = DeviceColumn.empty(N.TYPE_FLOAT64, fc.length, False, ctx=ctx)
            fcc, fdc = fc.as_c(), fd.as_c()
            N.check(N.lib().qe_cast_utf8_to_f64(ctx.handle, N.C.byref(fcc), N.C.byref(fdc), None))
            partial = HashAggregateState(ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64)], 16)
            owner = HashAggregateState(ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64)], 16)
            partial.update([DeviceColumn.from_strings(vend, ctx=ctx)], [fd])
            h = N.C.c_void_p()
            N.check(N.lib().qe_comm_create_loopback(ctx.handle, 2, r, hub, N.C.byref(h)))
            comm = Comm()
            comm.handle = h
            try:
                n = exchange_partials_native(partial, owner, comm, 0)
            finally:
                N.lib().qe_comm_destroy(h)
            g = _groups(*owner.finalize())
            ctx.synchronize()
            assert n >= len(g)  # (a group both senders hold arrives twice)
            return g

    out = _loopback(2, rank_main)
    assert not (set(out[0]) & set(out[1])), "a group owned by both ranks"
    got = {**out[0], **out[1]}
    allv = data[0][0] + data[1][0]
    allf = [R.parse_java_double(f) for f in data[0][1] + data[1][1]]
    want = S.hash_aggregate_rows([allv], [allf], [S.AGG_MAX], [True])
    assert got == want


def test_exchange_tuple_keys_two_ranks(gpu_ctx):
    import torch

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import Context
    from kquery.exchange import exchange_partials_native

    parts = [_rows(31, 25_000), _rows(32, 21_000)]
    types = [N.TYPE_UTF8, N.TYPE_INT64]

    class Comm:
        pass

    def rank_main(r, hub):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            ctx = Context.get(0)
            partial = HashAggregateState(ctx, types, _aggs(N), 64)
            owner = HashAggregateState(ctx, types, _aggs(N), 64)
            _update(partial, ctx, "tuple", *parts[r])
            h = N.C.c_void_p()
            N.check(N.lib().qe_comm_create_loopback(ctx.handle, 2, r, hub, N.C.byref(h)))
            comm = Comm()
            comm.handle = h
            try:
                exchange_partials_native(partial, owner, comm, 0)
            finally:
                N.lib().qe_comm_destroy(h)
            g = _groups(*owner.finalize())
            ctx.synchronize()
            return g

    out = _loopback(2, rank_main)
    assert not (set(out[0]) & set(out[1])), "a group owned by both ranks"
    assert {**out[0], **out[1]} == _want("tuple", parts)
