"""Run-to-run determinism on the GPU (SURVEY §5 "Race detection / sanitizers": the device side's
race check). Every device path runs several times over the same inputs, on the default stream and
on a second context (own HIP stream); results must be identical bit for bit, except where the
design documents otherwise:

* compaction (filter, select-project), CAST, CSV scan, global aggregate (per-block partials and a
  fixed-order final pass), and every integer / MIN / MAX / COUNT group result: bit-identical;
* hash-aggregate fp64 SUM / AVG: exact fixed point by default (qe_dev.hpp fx_*): bit-identical
  across runs, streams, batchings and kernel paths, and equal to math.fsum of each group;
* with QE_HASHAGG_FAST_FP64 (opt-in fp64 atomics) the per-group sums combine in arrival order:
  run to run they agree within 1e-13 × Σ|x| of the group (a condition-aware bound; this mode does
  not promise the 1e-9 contract for groups whose terms cancel — DESIGN.md "fp64 SUM").
Group ORDER is unspecified (HashMap iteration order, K:639), so groups are compared as maps."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
RUNS = 4


def _runs(gpu_ctx):
    """Yields the context of each run: the default context three times, then a second context on
    its own HIP stream; each run allocates and launches under that context's stream."""
    import torch

    from kquery.columnar import Context

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        other = Context.get(0)
    for ctx, stream in [(gpu_ctx, torch.cuda.current_stream())] * (RUNS - 1) + [(other, s)]:
        with torch.cuda.stream(stream):
            yield ctx
            ctx.synchronize()


def _bits(c):
    from kquery import native as N

    if c.type == N.TYPE_UTF8:
        return c.offsets[: c.length + 1].cpu().numpy().tobytes(), c.to_numpy().tolist(), c.valid_mask().tobytes()
    return c.to_numpy().view(np.uint8).tobytes(), c.valid_mask().tobytes()


def test_filter_and_select_project(gpu_ctx):
    from kquery import native as N
    from kquery.columnar import DeviceColumn, RecordBatch, Schema
    from kquery.operators import filter_batch
    from test_selproj import _run, _spec

    rng = np.random.default_rng(3)
    n = 6_000_001
    a = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
    f = rng.normal(size=n)
    m = rng.random(n) < 0.5
    av = rng.random(n) > 0.1
    outs = []
    for ctx in _runs(gpu_ctx):
        cols = [DeviceColumn.from_numpy(N.TYPE_INT64, a, av, ctx=ctx),
                DeviceColumn.from_numpy(N.TYPE_FLOAT64, f, None, ctx=ctx)]
        fb = filter_batch(RecordBatch(Schema([]), cols), DeviceColumn.from_numpy(N.TYPE_BOOL, m, None, ctx=ctx))
        spec = _spec(N, [(1, N.OP_GT, -1, 0.25)], [[(N.TOK_COL, 0, None), (N.TOK_COL, 1, None), (N.TOK_MUL, 0, None)],
                                                  [(N.TOK_COL, 0, None)]])
        cnt, sp = _run(ctx, cols, spec, [N.TYPE_FLOAT64, N.TYPE_INT64])
        ctx.synchronize()
        outs.append([_bits(c) for c in fb.fields] + [cnt] + [_bits(c) for c in sp])
    assert all(o == outs[0] for o in outs[1:])


def test_global_aggregate_f64(gpu_ctx):
    from kquery import native as N
    from kquery.columnar import DeviceColumn
    from test_gpu_parity import _global

    rng = np.random.default_rng(5)
    n = 40_000_003
    x = rng.normal(size=n) * np.exp(rng.normal(size=n) * 8)  # wide dynamic range: order-sensitive
    res = []
    for ctx in _runs(gpu_ctx):
        r = _global(ctx, DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=ctx))
        res.append((r.sum, r.min, r.max, r.count, r.avg))
    assert all(r == res[0] for r in res[1:]), res


def test_hash_aggregate(gpu_ctx):
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(9)
    n = 8_000_000
    k = rng.integers(0, 5000, n).astype(np.int64)  # beyond one LDS table: global merge path too
    x = rng.normal(size=n) * 1e3
    y = rng.integers(-2**40, 2**40, n).astype(np.int64)
    aggs = [(N.AGG_SUM, N.TYPE_FLOAT64), (N.AGG_AVG, N.TYPE_FLOAT64), (N.AGG_MIN, N.TYPE_FLOAT64),
            (N.AGG_MAX, N.TYPE_FLOAT64), (N.AGG_SUM, N.TYPE_INT64), (N.AGG_COUNT, N.TYPE_INT64),
            (N.AGG_MIN, N.TYPE_INT64)]
    yv = rng.random(n) > 0.2
    for fast in (False, True):
        runs = []
        for ctx in _runs(gpu_ctx):
            kc = DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=ctx)
            xc = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=ctx)
            yc = DeviceColumn.from_numpy(N.TYPE_INT64, y, yv, ctx=ctx)
            st = HashAggregateState(ctx, [N.TYPE_INT64], aggs, 1024, fast_fp64=fast)
            st.update([kc], [xc, xc, xc, xc, yc, yc, yc])
            keys, vals = st.finalize()
            ctx.synchronize()
            cols = [v.to_pylist() for v in vals]
            runs.append({kk: [c[i] for c in cols] for i, kk in enumerate(keys[0].to_pylist())})
        absum = np.bincount(k, weights=np.abs(x))
        cnt = np.bincount(k)
        base = runs[0]
        for r in runs[1:]:
            assert r.keys() == base.keys()
            for kk, v in r.items():
                b = base[kk]
                if not fast:
                    assert v == b, kk  # exact fp64 sums too: bit-identical
                    continue
                assert v[2:] == b[2:], kk  # MIN/MAX fp64 and every integer result: bit-identical
                bound = 1e-13 * absum[kk]  # fast fp64 SUM / AVG: atomic arrival order
                assert abs(v[0] - b[0]) <= bound, (kk, v[0], b[0])
                assert abs(v[1] - b[1]) <= bound / cnt[kk], (kk, v[1], b[1])


def test_csv_cast_string_keys(gpu_ctx, tmp_path):
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn
    from kquery.csv_source import CsvDataSource

    rng = np.random.default_rng(1)
    rows = 300_000
    vend = rng.choice(["1", "2", "VTS", "CMT", '"q,x"'], rows)
    fare = rng.uniform(-5, 500, rows)
    p = tmp_path / "t.csv"
    p.write_text("VendorID,fare_amount\n" + "".join(f"{v},{x:.3f}\n" for v, x in zip(vend, fare)))
    outs = []
    for ctx in _runs(gpu_ctx):
        b = next(CsvDataSource(str(p), True, 0, ctx=ctx).scan(["VendorID", "fare_amount"]))
        fs = b.field(1)
        out = DeviceColumn.empty(N.TYPE_FLOAT64, fs.length, False, ctx=ctx)
        ic, oc = fs.as_c(), out.as_c()
        N.check(N.lib().qe_cast_utf8_to_f64(ctx.handle, N.C.byref(ic), N.C.byref(oc), None))
        st = HashAggregateState(ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64), (N.AGG_COUNT, N.TYPE_FLOAT64)], 16)
        st.update([b.field(0)], [out, out])
        keys, vals = st.finalize()
        ctx.synchronize()
        groups = dict(zip(keys[0].to_pylist(), zip(*[v.to_pylist() for v in vals])))
        outs.append((_bits(b.field(0)), _bits(fs), _bits(out), groups))
    assert all(o == outs[0] for o in outs[1:])


@pytest.mark.parametrize("groups,expected,path", [(37, 64, "lds"), (4500, 4500, "two-bucket"),
                                                   (50_000, 50_000, "partitioned"), (300, 64, "generic")])
def test_deterministic_fp64_group_sums(gpu_ctx, groups, expected, path):
    """fp64 SUM / AVG in exact fixed point (the default; QE_HASHAGG_DETERMINISTIC names it). Every
    run — default stream, second context, two batches instead of one — gives the same bits, and
    they equal the correctly rounded exact sum (math.fsum) of each group, as the reference's
    ordered row loop would give with exact arithmetic. Values span 2^-80 .. 2^30: some take the LDS
    window, some (below 2^-44) the global table's full accumulator."""
    import math

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(groups)
    n = 3_000_000
    k = rng.integers(0, groups, n).astype(np.int64)
    x = rng.normal(size=n) * np.exp2(rng.integers(-80, 30, n))  # wide range: fp64 atomics would wobble
    xv = rng.random(n) > 0.05
    aggs = [(N.AGG_SUM, N.TYPE_FLOAT64), (N.AGG_AVG, N.TYPE_FLOAT64), (N.AGG_COUNT_STAR, N.TYPE_INT64)]
    runs = []
    for i, ctx in enumerate(_runs(gpu_ctx)):
        if path == "generic":
            N.check(N.lib().qe_ctx_set_jit(ctx.handle, 0))
        try:
            st = HashAggregateState(ctx, [N.TYPE_INT64], aggs, expected, deterministic=True)
            cuts = [0, n] if i % 2 == 0 else [0, n // 3, n]  # one batch, or two
            for lo, hi in zip(cuts[:-1], cuts[1:]):
                kc = DeviceColumn.from_numpy(N.TYPE_INT64, k[lo:hi], None, ctx=ctx)
                xc = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x[lo:hi], xv[lo:hi], ctx=ctx)
                st.update([kc], [xc, xc, None])
            keys, vals = st.finalize()
            ctx.synchronize()
        finally:
            N.check(N.lib().qe_ctx_set_jit(ctx.handle, 1))
        cols = [v.to_numpy() for v in vals]
        kv = keys[0].to_numpy()
        runs.append({int(kv[g]): (cols[0][g].tobytes(), cols[1][g].tobytes(), int(cols[2][g])) for g in range(len(kv))})
    assert all(r == runs[0] for r in runs[1:])
    order = np.argsort(k, kind="stable")
    ks, xs, vs = k[order], x[order], xv[order]
    bounds = np.searchsorted(ks, np.arange(groups + 1))
    for g in range(groups):
        lo, hi = bounds[g], bounds[g + 1]
        vals_g = xs[lo:hi][vs[lo:hi]]
        want = math.fsum(vals_g.tolist())
        got_sum, got_avg, cstar = runs[0][g]
        assert cstar == hi - lo
        assert np.frombuffer(got_sum, np.float64)[0] == want, g
        assert np.frombuffer(got_avg, np.float64)[0] == want / len(vals_g), g


@pytest.mark.parametrize("expected", [16, 4500, 50_000])
def test_exact_sum_specials(gpu_ctx, expected):
    """IEEE specials and large inputs on the LDS, two-bucket and radix-partitioned paths: NaN and
    +-Inf give the IEEE result of the sum in their group only; 2^70 and 2^150 (outside the LDS
    window, in the global words) and 2^190, 1e308 and -1e308 twice (the full-range words E; the
    last overflows to -Inf) are summed exactly: math.fsum's value."""
    import math

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    n = 200_000
    ng = max(7, expected)
    kv = np.arange(n, dtype=np.int64) % ng
    for bad, want in ((np.nan, math.nan), (np.inf, math.inf), (-np.inf, -math.inf), (2.0 ** 70, None),
                      (2.0 ** 150, None), (2.0 ** 190, None), (1e308, None), ((-1e308, -1e308), -math.inf)):
        x = np.ones(n)
        x[n // 2] = bad if not isinstance(bad, tuple) else bad[0]
        if isinstance(bad, tuple):
            x[n // 2 + ng] = bad[1]  # the same group
        st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(N.AGG_SUM, N.TYPE_FLOAT64)], expected)
        st.update([DeviceColumn.from_numpy(N.TYPE_INT64, kv, None, ctx=gpu_ctx)],
                  [DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=gpu_ctx)])
        keys, vals = st.finalize()
        got = dict(zip(keys[0].to_pylist(), vals[0].to_pylist()))
        g = int(kv[n // 2])
        for kk, v in got.items():
            ref = math.fsum(x[kv == kk].tolist()) if kk != g or want is None else want
            assert (math.isnan(v) and math.isnan(ref)) or v == ref, (bad, kk, v, ref)


def test_exact_sum_tiny_inputs(gpu_ctx):
    """Values with bits below 2^-128 go unrounded to the group's full-range words: every group's
    sum is math.fsum's bit for bit, deterministic run to run — values around 1e-25 alone, values
    that cancel exactly (exactly 0; ADVICE r04: {3.7e-5, -3.7e-5}), groups of 1e-40 values and
    subnormals (these used to fail finalize)."""
    import math

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    rng = np.random.default_rng(3)
    n = 100_000
    k = rng.integers(0, 50, n).astype(np.int64)
    x = rng.random(n) * 10.0 + rng.random(n) * 1e-4  # low bits well below 2^-64 on the small terms
    x[::7] = 3.7e-5  # full-mantissa values under 2^-11
    x[k == 3] = 1e-40 * (1 + rng.random(int((k == 3).sum())))
    x[k == 4] = 5e-324 * rng.integers(1, 1000, int((k == 4).sum()))
    outs = []
    for ctx in _runs(gpu_ctx):
        st = HashAggregateState(ctx, [N.TYPE_INT64], [(N.AGG_SUM, N.TYPE_FLOAT64)], 64)
        st.update([DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=ctx)],
                  [DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=ctx)])
        keys, vals = st.finalize()
        ctx.synchronize()
        kv, sv = keys[0].to_numpy(), vals[0].to_numpy()
        outs.append({int(kv[i]): sv[i].tobytes() for i in range(len(kv))})
    assert all(o == outs[0] for o in outs[1:])
    for g, b in outs[0].items():
        want = math.fsum(x[k == g].tolist())
        assert np.frombuffer(b, np.float64)[0] == want, (g, np.frombuffer(b, np.float64)[0], want)
    k2 = np.array([0, 1, 1, 1, 0, 2, 2], dtype=np.int64)
    x2 = np.array([1.0, 1.1e-25, 0.9e-25, 1.3e-25, 2.0, 3.7e-5, -3.7e-5])
    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(N.AGG_SUM, N.TYPE_FLOAT64)], 16)
    st.update([DeviceColumn.from_numpy(N.TYPE_INT64, k2, None, ctx=gpu_ctx)],
              [DeviceColumn.from_numpy(N.TYPE_FLOAT64, x2, None, ctx=gpu_ctx)])
    keys, vals = st.finalize()
    got = dict(zip(keys[0].to_pylist(), vals[0].to_pylist()))
    assert got[0] == 3.0 and got[2] == 0.0 and got[1] == math.fsum(x2[1:4].tolist())
