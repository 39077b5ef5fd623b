"""Randomised plans through the operator layer: ScanExec -> SelectionExec ->
ProjectionExec -> HashAggregateExec with random column types and null rates, random predicate
terms (column vs literal / column), random projection arithmetic and aggregate functions. Each
plan runs fused (operators.fuse: one hipRTC-specialised kernel, or the dictionary / unfused path
when the plan is outside it) and unfused, and both must equal the oracle: integer results exactly,
fp64 SUM/AVG within 1e-9 relative. Covers empty inputs, selectivity 0 % and 100 %, one group,
many groups, null keys, NaN/±0.0 keys, int64 wrap, narrow (int32/uint8) aggregate inputs,
COUNT(*) with no input column, UTF-8 keys and key sets wider than 63 bits (the dictionary-keyed
fused path)."""
import random

import numpy as np
import pytest

from oracle import semantics as S

pytestmark = pytest.mark.gpu
REL = 1e-9

TYPES = ["i64", "f64", "i32", "u8"]


def _column(rng, t, n, card):
    if t == "i64":
        v = rng.choice([rng.integers(-card, card, n), rng.integers(-2**62, 2**62, n)]).astype(np.int64)
    elif t == "f64":
        # (1e25: beyond the exact SUM's LDS window, and its products stay inside the exact range,
        # |x| < 2^182; larger inputs make finalize report the group instead)
        pool = np.array([0.0, -0.0, np.nan, 1.5, -2.5, 1e25, -np.inf, 3.25])
        v = np.where(rng.random(n) < 0.5, pool[rng.integers(0, len(pool), n)], rng.normal(size=n) * 100)
    elif t == "i32":
        v = rng.integers(-card, card, n).astype(np.int32)
    else:
        v = rng.integers(0, min(card, 255) + 1, n).astype(np.uint8)
    valid = (rng.random(n) > 0.1) if rng.random() < 0.5 else None
    return v, valid


def _qe_type(N, t):
    return {"i64": N.TYPE_INT64, "f64": N.TYPE_FLOAT64, "i32": N.TYPE_INT32, "u8": N.TYPE_UINT8}[t]


def _plan(seed):
    rng = random.Random(seed)
    nrng = np.random.default_rng(seed)
    n = rng.choice([0, 1, 777, 4096, 50_000, 200_003])
    card = rng.choice([1, 3, 100, 10_000])
    types = [rng.choice(TYPES) for _ in range(5)]
    cols = [_column(nrng, t, n, card) for t in types]
    # column 5: UTF-8 key "k<v>" over an int column v (the oracle groups by v)
    sv = nrng.integers(-card, card, n)
    cols.append((sv, (nrng.random(n) > 0.1) if rng.random() < 0.5 else None))
    nkeys = rng.choice([0, 1, 1, 2])
    keys = rng.sample(range(6), nkeys)
    terms = []
    for _ in range(rng.choice([0, 1, 2])):
        c = rng.randrange(5)
        op = rng.choice([10, 11, 12, 13, 14, 15])
        if rng.random() < 0.3:
            terms.append((c, op, rng.randrange(5), None))
        else:
            lit = rng.choice([0, 1, -1, 7, 100]) if types[c] != "f64" else rng.choice([0.0, 1.5, -2.5])
            if rng.random() < 0.2:
                lit = rng.choice([2**31, -2**31])
            terms.append((c, op, None, lit))
    aggs = []
    for _ in range(rng.choice([1, 2, 4])):
        fn = rng.choice([1, 2, 3, 4, 5, 6])
        shape = rng.choice(["col", "add", "mul", "sub_lit"])
        a, b = rng.randrange(5), rng.randrange(5)
        aggs.append((fn, shape, a, b))
    return n, types, cols, keys, terms, aggs


def _oracle_expr(shape, a, b, cols, types):
    va, vva = cols[a]
    vb, vvb = cols[b]
    if shape == "col":
        return va if types[a] in ("i64", "f64") else va.astype(np.int64), vva
    if shape == "add":
        return S.arith(S.OP_ADD, va.astype(np.float64 if types[a] == "f64" else np.int64), vva,
                       vb.astype(np.float64 if types[b] == "f64" else np.int64), vvb)
    if shape == "mul":
        return S.arith(S.OP_MUL, va.astype(np.float64 if types[a] == "f64" else np.int64), vva,
                       vb.astype(np.float64 if types[b] == "f64" else np.int64), vvb)
    return S.arith(S.OP_SUB, va.astype(np.float64 if types[a] == "f64" else np.int64), vva, 3, None)


def _expr(E, shape, a, b):
    if shape == "col":
        return E.ColumnExpression(a)
    if shape == "add":
        return E.AddExpression(E.ColumnExpression(a), E.ColumnExpression(b))
    if shape == "mul":
        return E.MultiplyExpression(E.ColumnExpression(a), E.ColumnExpression(b))
    return E.SubtractExpression(E.ColumnExpression(a), E.LiteralLongExpression(3))


@pytest.mark.parametrize("seed", range(60))
def test_random_plan(gpu_ctx, seed):
    from kquery import expressions as E
    from kquery import native as N
    from kquery.columnar import DeviceColumn, Field, RecordBatch, Schema
    from kquery.datasource import InMemoryDataSource
    from kquery.operators import (FusedHashAggregateExec, HashAggregateExec, ProjectionExec, ScanExec,
                                  SelectionExec, fuse)

    n, types, cols, keys, terms, aggs = _plan(seed)
    if not keys and not aggs:
        pytest.skip("empty plan")
    qtypes = [_qe_type(N, t) for t in types] + [N.TYPE_UTF8]
    schema = Schema([Field(f"c{i}", qtypes[i]) for i in range(6)])
    sv, svv = cols[5]
    strs = [None if svv is not None and not svv[r] else f"k{v}" for r, v in enumerate(sv.tolist())]
    batch = RecordBatch(schema, [DeviceColumn.from_numpy(qtypes[i], cols[i][0], cols[i][1], ctx=gpu_ctx)
                                 for i in range(5)] + [DeviceColumn.from_strings(strs, ctx=gpu_ctx)])
    scan = ScanExec(InMemoryDataSource(schema, [batch]), [f"c{i}" for i in range(6)])
    cmp_cls = {10: E.EqExpression, 11: E.NeqExpression, 12: E.LtExpression, 13: E.LtEqExpression,
               14: E.GtExpression, 15: E.GtEqExpression}
    pred = None
    sel = np.ones(n, dtype=bool)
    for c, op, rc, lit in terms:
        rhs = E.ColumnExpression(rc) if rc is not None else (
            E.LiteralDoubleExpression(lit) if isinstance(lit, float) else E.LiteralLongExpression(lit))
        t = cmp_cls[op](E.ColumnExpression(c), rhs)
        pred = t if pred is None else E.AndExpression(pred, t)
        a = cols[c][0].astype(np.float64 if types[c] == "f64" else np.int64)
        if rc is not None:
            b, bv = cols[rc][0].astype(np.float64 if types[rc] == "f64" else np.int64), cols[rc][1]
        else:
            b, bv = lit, None
        m, mv = S.cmp(op, a, cols[c][1], b, bv)
        sel &= S.select_mask(m, mv)
    node = SelectionExec(scan, pred) if pred is not None else scan
    proj_exprs = [E.ColumnExpression(k) for k in keys] + [_expr(E, sh, a, b) for _, sh, a, b in aggs]
    in_types = []
    for fn, sh, a, b in aggs:
        is_f = types[a] == "f64" or (sh in ("add", "mul") and types[b] == "f64")
        in_types.append(N.TYPE_FLOAT64 if is_f else N.TYPE_INT64)
    pschema = Schema([Field(f"k{i}", qtypes[k]) for i, k in enumerate(keys)] +
                     [Field(f"x{j}", t) for j, t in enumerate(in_types)])
    proj = ProjectionExec(node, pschema, proj_exprs)
    agg_exprs = []
    cls = {1: E.SumExpression, 2: E.MinExpression, 3: E.MaxExpression, 4: E.CountExpression, 6: E.AvgExpression}
    for j, (fn, _, _, _) in enumerate(aggs):
        agg_exprs.append(E.CountStarExpression() if fn == 5 else cls[fn](E.ColumnExpression(len(keys) + j)))
    out_fields = [Field(f"k{i}", qtypes[k]) for i, k in enumerate(keys)]
    for (fn, _, _, _), t in zip(aggs, in_types):
        out_fields.append(Field("agg", N.TYPE_INT64 if fn in (4, 5) else (N.TYPE_FLOAT64 if fn == 6 else t)))
    plan = HashAggregateExec(proj, [E.ColumnExpression(i) for i in range(len(keys))], agg_exprs,
                             Schema(out_fields), expected_groups=64)
    # oracle
    okeys = [cols[k][0] for k in keys]
    okv = [cols[k][1] for k in keys]
    ins, insv = [], []
    for fn, sh, a, b in aggs:
        v, vv = _oracle_expr(sh, a, b, cols, types)
        ins.append(v)
        insv.append(vv)
    fns = [fn for fn, _, _, _ in aggs]
    want = S.group_aggregate(okeys, okv, ins, insv, fns, sel) if keys else None
    if not keys:
        want = S.group_aggregate([np.zeros(n, dtype=np.int64)], [None], ins, insv, fns, sel)
        want = {(): v for v in want.values()}
    fused = fuse(plan)
    if keys or terms or any(fn != 5 for fn in fns):  # every generated shape is in the fused kernel
        assert isinstance(fused, FusedHashAggregateExec), fused
    for p in (fused, plan):
        out = list(p.execute())
        assert len(out) == 1
        b = out[0]
        got = {}
        cl = [b.field(i).to_pylist() for i in range(len(b.fields))]
        for r in zip(*cl):
            kk = [int(x[1:]) if k == 5 and x is not None else x for k, x in zip(keys, r[:len(keys)])]
            got[tuple(S.canon(x) for x in kk)] = list(r[len(keys):])
        assert len(got) == len(want), (type(p).__name__, len(got), len(want))
        for k, w in want.items():
            ck = tuple(S.canon(x) for x in k)
            assert ck in got, (type(p).__name__, k)
            for j, (g, x) in enumerate(zip(got[ck], w)):
                rel = REL if fns[j] in (1, 6) and isinstance(x, float) else 0.0
                assert S.rows_equal(g, x, rel), (type(p).__name__, seed, k, j, g, x)


@pytest.mark.parametrize("seed", range(60))
def test_random_select_project(gpu_ctx, monkeypatch, seed):
    """Random Projection(Selection(Scan)) plans (the same random columns, predicates and projection
    arithmetic): the fused select-project kernel (tile-base mode by seed: two passes, look-back,
    scanned; nullable and narrow outputs, staged validity words) and the unfused operators must
    both return the oracle's rows, in input order."""
    from kquery import expressions as E
    from kquery import native as N
    from kquery.columnar import DeviceColumn, Field, RecordBatch, Schema
    from kquery.datasource import InMemoryDataSource
    from kquery.operators import ProjectionExec, ScanExec, SelectionExec, fuse

    monkeypatch.setenv("QE_SELPROJ_TWOPASS", ("1", "0", "2")[seed % 3])
    n, types, cols, keys, terms, aggs = _plan(seed + 1000)
    keys = [k for k in keys if k < 5]  # fixed-width outputs (UTF-8 projections take the unfused path)
    qtypes = [_qe_type(N, t) for t in types]
    schema = Schema([Field(f"c{i}", qtypes[i]) for i in range(5)])
    batch = RecordBatch(schema, [DeviceColumn.from_numpy(qtypes[i], cols[i][0], cols[i][1], ctx=gpu_ctx)
                                 for i in range(5)])
    scan = ScanExec(InMemoryDataSource(schema, [batch]), [f"c{i}" for i in range(5)])
    cmp_cls = {10: E.EqExpression, 11: E.NeqExpression, 12: E.LtExpression, 13: E.LtEqExpression,
               14: E.GtExpression, 15: E.GtEqExpression}
    pred = None
    sel = np.ones(n, dtype=bool)
    for c, op, rc, lit in terms:
        rhs = E.ColumnExpression(rc) if rc is not None else (
            E.LiteralDoubleExpression(lit) if isinstance(lit, float) else E.LiteralLongExpression(lit))
        t = cmp_cls[op](E.ColumnExpression(c), rhs)
        pred = t if pred is None else E.AndExpression(pred, t)
        a = cols[c][0].astype(np.float64 if types[c] == "f64" else np.int64)
        if rc is not None:
            b, bv = cols[rc][0].astype(np.float64 if types[rc] == "f64" else np.int64), cols[rc][1]
        else:
            b, bv = lit, None
        m, mv = S.cmp(op, a, cols[c][1], b, bv)
        sel &= S.select_mask(m, mv)
    if pred is None:
        pred = E.GtEqExpression(E.ColumnExpression(0), E.LiteralLongExpression(-2**62))
        m, mv = S.cmp(15, cols[0][0].astype(np.float64 if types[0] == "f64" else np.int64), cols[0][1], -2**62, None)
        sel &= S.select_mask(m, mv)
    exprs = [E.ColumnExpression(k) for k in keys] + [_expr(E, sh, a, b) for _, sh, a, b in aggs]
    want = [(cols[k][0], cols[k][1]) for k in keys] + [_oracle_expr(sh, a, b, cols, types) for _, sh, a, b in aggs]
    out_types = [qtypes[k] for k in keys]
    for _, sh, a, b in aggs:
        is_f = types[a] == "f64" or (sh in ("add", "mul") and types[b] == "f64")
        out_types.append(N.TYPE_FLOAT64 if is_f else (qtypes[a] if sh == "col" else N.TYPE_INT64))
    plan = ProjectionExec(SelectionExec(scan, pred), Schema([Field(f"o{j}", t) for j, t in enumerate(out_types)]),
                          exprs)
    fused = fuse(plan)
    assert type(fused).__name__ == "FusedSelectProjectExec", fused
    for p in (fused, plan):
        rows = [b for b in p.execute()]
        got = [[] for _ in exprs]
        for b in rows:
            for j in range(len(exprs)):
                got[j].extend(b.field(j).to_pylist())
        for j, (v, vv) in enumerate(want):
            exp = [None if vv is not None and not vv[i] else v[i].item() for i in np.nonzero(sel)[0]]
            assert len(got[j]) == len(exp), (type(p).__name__, seed, j, len(got[j]), len(exp))
            for g, x in zip(got[j], exp):
                assert S.rows_equal(g, x, 0.0), (type(p).__name__, seed, j, g, x)
