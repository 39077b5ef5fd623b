"""Exact fp64 SUM / AVG of the hash aggregate on MI355X (within 1e-9 relative of the
exact sum; here: the correctly rounded exact sum, bit for bit) on adversarial groups, on every
aggregation path: the plan-specialised fused kernel (per-wave fx queue), the LDS table through
qe_hashagg_update, the generic kernel, the two-bucket (spilling) pass and the radix-partitioned
pass, in the default state and with QE_HASHAGG_DETERMINISTIC (the same accumulator).

Each group holds +2^60 in the first rows of the batch and -2^60 in the last rows (different
workgroups), unit terms and other small values between them, -0.0, and — in some groups — inputs
outside the per-workgroup LDS window ([2^-44, 2^62): 1e-30 and 3e19, which take the global
accumulator), inputs for the full-range words E (1e-40, subnormals, 2^190, a +-1e300 pair), NaN or
+Inf. fp64 atomics in arrival order lose the unit terms next to 2^60 (its ulp is 256); the exact
accumulator must equal math.fsum of each group. The oracle is math.fsum over the same rows
(Python's exact, correctly rounded sum). test_full_range_exchange carries E through every partial
form: export / import records, fixed-capacity slots, keyed blocks and qe_hashagg_merge."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(groups, n, seed):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, groups, n).astype(np.int64)
    x = rng.choice([1.0, 1.0, 1.0, 0.5, 0.1, -0.25, 3.0, -0.0], n)
    m = rng.random(n) < 0.2
    x[m] = rng.normal(size=int(m.sum())) * 100
    perm = rng.permutation(groups)
    k[:groups] = perm
    x[:groups] = 2.0 ** 60
    k[n - groups:] = rng.permutation(groups)
    x[n - groups:] = -(2.0 ** 60)
    # inputs outside the LDS window in a tenth of the groups, NaN / +Inf in two groups
    odd = rng.choice(np.arange(groups // 2, n - groups), size=max(16, groups // 5), replace=False)
    x[odd[0::8]] = 1e-30
    x[odd[1::8]] = 3e19
    x[odd[2::8]] = 1e-40
    x[odd[3::8]] = 5e-324 * 77
    x[odd[4::8]] = 2.0 ** 190
    x[odd[5::8]] = 1e300
    x[odd[6::8]] = -1e300
    sp = rng.choice(np.arange(groups, n - groups), size=2, replace=False)
    x[sp[0]] = np.nan
    x[sp[1]] = np.inf
    return k, x


def _expected(k, x, groups):
    order = np.argsort(k, kind="stable")
    ks, xs = k[order], x[order]
    b = np.searchsorted(ks, np.arange(groups + 1))
    out = {}
    for g in range(groups):
        v = xs[b[g]:b[g + 1]]
        if len(v) == 0:
            continue
        s = float("nan") if np.isnan(v).any() else (math.inf if np.isinf(v).any() else math.fsum(v.tolist()))
        out[g] = (s, len(v))
    return out


def _same(a, b):
    return (math.isnan(a) and math.isnan(b)) or np.float64(a).tobytes() == np.float64(b).tobytes()


@pytest.mark.parametrize("deterministic", [False, True], ids=["default", "deterministic"])
@pytest.mark.parametrize("groups,expected,path", [(1024, 1024, "lds"), (300, 64, "generic"), (4500, 4500, "two-bucket"),
                                                  (65536, 65536, "partitioned"), (6, 16, "fused")])
def test_fp64_sum_adversarial(gpu_ctx, groups, expected, path, deterministic):
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    n = max(3_000_000, groups * 40)
    k, x = _data(groups, n, groups + 17)
    want = _expected(k, x, groups)
    aggs = [(N.AGG_SUM, N.TYPE_FLOAT64), (N.AGG_AVG, N.TYPE_FLOAT64), (N.AGG_COUNT_STAR, N.TYPE_INT64)]
    if path == "generic":
        N.check(N.lib().qe_ctx_set_jit(gpu_ctx.handle, 0))
    try:
        st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], aggs, expected, deterministic=deterministic)
        kc = DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=gpu_ctx)
        xc = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=gpu_ctx)
        if path == "fused":
            spec = N.QeFusedSpec()
            spec.mask_col = -1
            spec.nterms = 0
            spec.key_cols[0] = 0
            for j in (0, 1):
                spec.inputs[j].ntokens = 1
                spec.inputs[j].tokens[0] = N.QeToken(N.TOK_COL, 1, N.QeScalar())
            st.update_fused([kc, xc], spec)
            kind = st.last_kernel_kind()
            assert kind[0], kind
        else:
            st.update([kc], [xc, xc, None])
        keys, vals = st.finalize()
        gpu_ctx.synchronize()
    finally:
        N.check(N.lib().qe_ctx_set_jit(gpu_ctx.handle, 1))
    kv = keys[0].to_numpy()
    sv, av, cv = (v.to_numpy() for v in vals)
    assert len(kv) == len(want)
    for i in range(len(kv)):
        s, c = want[int(kv[i])]
        assert int(cv[i]) == c
        assert _same(sv[i], s), (int(kv[i]), sv[i], s)
        assert _same(av[i], s / c), (int(kv[i]), av[i], s / c)


def _full_range_batch(rng, n, groups):
    k = rng.integers(0, groups, n).astype(np.int64)
    x = rng.normal(size=n)
    sel = rng.random(n)
    x[sel < 0.05] = 1e-40 * (1 + rng.random(int((sel < 0.05).sum())))
    x[(sel >= 0.05) & (sel < 0.08)] = 5e-324
    x[(sel >= 0.08) & (sel < 0.09)] = 1e300
    x[(sel >= 0.09) & (sel < 0.10)] = -1e300
    x[(sel >= 0.10) & (sel < 0.11)] = 2.0 ** 190
    return k, x


@pytest.mark.parametrize("form", ["records", "slots", "keyed", "merge", "utf8-merge"])
def test_full_range_exchange(gpu_ctx, form):
    """Two partial states with full-range inputs combined through one partial form, then finalized:
    every group's sum is math.fsum's over both batches (E travels as CHUNK records)."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(11)
    groups = 500
    batches = [_full_range_batch(rng, 200_000, groups) for _ in range(2)]
    utf8 = form == "utf8-merge"
    ktype = N.TYPE_UTF8 if utf8 else N.TYPE_INT64

    def keycol(k):
        if utf8:
            return DeviceColumn.from_strings([f"key-{int(v):05d}-long-enough-not-to-pack" for v in k], ctx=gpu_ctx)
        return DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=gpu_ctx)

    aggs = [(N.AGG_SUM, N.TYPE_FLOAT64), (N.AGG_COUNT_STAR, N.TYPE_INT64)]
    parts = []
    for k, x in batches:
        st = HashAggregateState(gpu_ctx, [ktype], aggs, 1024)
        st.update([keycol(k)], [DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=gpu_ctx), None])
        parts.append(st)
    final = HashAggregateState(gpu_ctx, [ktype], aggs, 1024)
    for p in parts:
        if form == "records":
            recs, counts = p.export(3)
            assert sum(counts) > p.num_groups()  # chunk records of the groups with E
            final.import_records(recs, sum(counts))
        elif form == "slots":
            cap = max(p.export_counts(2))
            slots = p.export_slots(2, cap)
            assert final.import_slots(slots, 2, cap) is not None
        elif form == "keyed":
            blocks, sizes = p.export_keyed(2)
            final.import_keyed(blocks, sizes)
        else:
            final.merge(p)
    keys, vals = final.finalize()
    gpu_ctx.synchronize()
    k = np.concatenate([b[0] for b in batches])
    x = np.concatenate([b[1] for b in batches])
    kv = keys[0].to_pylist()
    sv = vals[0].to_numpy()
    cv = vals[1].to_numpy()
    assert len(kv) == len(np.unique(k))
    for i, key in enumerate(kv):
        g = int(key.split("-")[1]) if utf8 else int(key)
        sel = k == g
        assert int(cv[i]) == int(sel.sum())
        assert sv[i] == math.fsum(x[sel].tolist()), (g, sv[i], math.fsum(x[sel].tolist()))


def test_fp64_sum_reset_clears_full_range_words(gpu_ctx):
    """Inputs for the full-range words (2^200, 1e-40) are summed exactly (they used to fail
    finalize); a reset clears the words the groups used, so the next query starts from zero."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(N.AGG_SUM, N.TYPE_FLOAT64)], 16)
    k = np.arange(1000, dtype=np.int64) % 7
    x = np.ones(1000)
    x[500] = 2.0 ** 200
    x[501] = 1e-40
    st.update([DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=gpu_ctx)],
              [DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=gpu_ctx)])
    keys, vals = st.finalize()
    got = dict(zip(keys[0].to_pylist(), vals[0].to_pylist()))
    for g in range(7):
        assert got[g] == math.fsum(x[k == g].tolist())
    st.reset()
    st.update([DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=gpu_ctx)],
              [DeviceColumn.from_numpy(N.TYPE_FLOAT64, np.full(1000, 0.1), None, ctx=gpu_ctx)])
    keys, vals = st.finalize()
    got = dict(zip(keys[0].to_pylist(), vals[0].to_pylist()))
    for g in range(7):
        assert got[g] == math.fsum([0.1] * int(np.sum(k == g)))

