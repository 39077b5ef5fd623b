"""Every BASELINE.json configuration at the size it names, on one GPU (VERDICT r02 "exercise every
BASELINE config at its size"):

* C2 — 10M int64 rows, filter(a > 2^19) + project(a + b) on the default (auto) select-project
  path: bit-exact against the oracle's restatement over all 10M rows;
* C3 — 100M fp64 rows (UNIT53 generator: every value a multiple of 2^-42, so the exact sum is an
  integer sum of the u53 words): COUNT / MIN / MAX bit-exact, SUM within 1e-9 of the exact sum;
* C4 — 1B int64 rows, 1024 groups: EVERY group's SUM / COUNT / MIN / MAX against the C oracle
  (oracle/cpu_baseline.c, pinned to oracle/semantics.py by tests/test_oracle.py) over the same
  1B rows;
* C5 — one GPU's 1.25B-row slice of the 10B lineitem config: COUNT(*) against the filter count of
  the four predicates, int64 SUM(l_quantity) exactly against qe_agg_global over the selected rows,
  fp64 SUMs / AVG within 1e-9 of the compensated global SUM, 6 groups.

Semantics restated: Main.kt:538-561 (MAX), 615-651 (HashAggregateExec), 589-594 (ProjectionExec),
build-defined SelectionExec / SUM / MIN / COUNT."""
import ctypes as C
import os
import pathlib
from fractions import Fraction

import numpy as np
import pytest

from oracle import gen
from oracle import semantics as S

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

from kquery import native as N  # noqa: E402
from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.columnar import DeviceColumn, f64_from_bits  # noqa: E402

REL = 1e-9
ROOT = pathlib.Path(__file__).resolve().parents[1]


def _eval(ctx, fn_name, op, lhs, rhs, out):
    keep = []

    def operand(x):
        if isinstance(x, DeviceColumn):
            c = x.as_c()
            keep.append(c)
            return N.QeOperand(N.C.pointer(c), N.QeScalar())
        return N.QeOperand(None, N.scalar(x))

    a, b = operand(lhs), operand(rhs)
    oc = out.as_c()
    N.check(getattr(N.lib(), fn_name)(ctx.handle, op, N.C.byref(a), N.C.byref(b), N.C.byref(oc)))
    return out


def _global(ctx, col, mask=None):
    r = N.QeGlobalAgg()
    c = col.as_c()
    mc = mask.as_c() if mask is not None else None
    N.check(N.lib().qe_agg_global(ctx.handle, N.C.byref(c), N.C.byref(mc) if mc is not None else None, N.C.byref(r)))
    return r


def _count(ctx, mask):
    cnt = N.C.c_int64()
    mc = mask.as_c()
    N.check(N.lib().qe_filter_count(ctx.handle, N.C.byref(mc), N.C.byref(cnt)))
    return cnt.value


def test_c2_full_size_default_path(gpu_ctx, monkeypatch):
    """C2 exactly as configured: 10M rows through the default (auto) qe_select_project path."""
    from kquery.datasource import C2_COLUMNS, generate_column

    monkeypatch.delenv("QE_SELPROJ_TWOPASS", raising=False)
    n, k = 10_000_000, 1 << 19
    cols = [generate_column(s, n, 0, 42, gpu_ctx) for s in C2_COLUMNS]
    spec = N.QeSelectSpec()
    spec.mask_col = -1
    spec.nterms = 1
    spec.terms[0].col, spec.terms[0].op, spec.terms[0].rhs_col = 0, N.OP_GT, -1
    spec.terms[0].lit = N.scalar(k)
    spec.nout = 1
    prog = [(N.TOK_COL, 0), (N.TOK_COL, 1), (N.TOK_ADD, 0)]
    spec.outputs[0].ntokens = len(prog)
    for j, (op, arg) in enumerate(prog):
        spec.outputs[0].tokens[j] = N.QeToken(op, arg, N.QeScalar())
    out = DeviceColumn.empty(N.TYPE_INT64, n, True, ctx=gpu_ctx)
    cc = (N.QeColumn * 2)(*[c.as_c() for c in cols])
    oc = (N.QeColumn * 1)(out.as_c())
    cnt = N.C.c_int64()
    N.check(N.lib().qe_select_project(gpu_ctx.handle, cc, 2, N.C.byref(spec), oc, N.C.byref(cnt)))
    a, _ = gen.generate(C2_COLUMNS[0].dist, C2_COLUMNS[0].param, 42, C2_COLUMNS[0].col_id, 0, n)
    b, _ = gen.generate(C2_COLUMNS[1].dist, C2_COLUMNS[1].param, 42, C2_COLUMNS[1].col_id, 0, n)
    m, mv = S.cmp(S.OP_GT, a, None, k, None)
    fa, fb = S.filter_columns(m, mv, [a, b])
    want, _ = S.arith(S.OP_ADD, fa, None, fb, None)
    assert cnt.value == len(fa)
    out.length = cnt.value
    assert np.array_equal(out.to_numpy(), want)


def test_c3_full_size_exact(gpu_ctx):
    """C3: 100M fp64 rows, global SUM / MIN / MAX / COUNT (K4a; MaxAccumulator K:538-561)."""
    from kquery.datasource import C3_COLUMNS, generate_column

    n = 100_000_000
    spec = C3_COLUMNS[0]
    x = generate_column(spec, n, 0, 42, gpu_ctx)
    r = _global(gpu_ctx, x)
    # exact sum: x = u53 * 2^-42 - 1024, so SUM = (sum of u53) * 2^-42 - 1024 n exactly
    su53, mn, mx = 0, None, None
    step = 10_000_000
    for r0 in range(0, n, step):
        rows = np.arange(r0, min(n, r0 + step), dtype=np.uint64)
        u53 = gen.gen_u64(42, spec.col_id, rows) >> np.uint64(11)
        su53 += int((u53 >> np.uint64(32)).sum(dtype=np.uint64)) << 32
        su53 += int((u53 & np.uint64(0xFFFFFFFF)).sum(dtype=np.uint64))
        v = u53.astype(np.float64) * 2.0 ** -42 - 1024.0
        mn = v.min() if mn is None else min(mn, v.min())
        mx = v.max() if mx is None else max(mx, v.max())
    exact = Fraction(su53, 1 << 42) - 1024 * n
    assert r.rows == n and r.count == n and r.valid == 1
    assert f64_from_bits(r.min) == mn and f64_from_bits(r.max) == mx
    got = Fraction(f64_from_bits(r.sum))
    assert abs(got - exact) <= Fraction(REL) * abs(exact), (float(got), float(exact))
    assert abs(Fraction(r.avg) - exact / n) <= Fraction(REL) * abs(exact / n)


def test_c4_full_size_every_group(gpu_ctx):
    """C4 at 1B rows: every one of the 1024 groups equals the C oracle over the same rows."""
    from kquery.datasource import C4_COLUMNS, generate_column
    from kquery.workloads import C4_AGGS, c4_spec

    n = 1_000_000_000
    cols = [generate_column(s, n, 0, 42, gpu_ctx) for s in C4_COLUMNS]
    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], C4_AGGS, 1024, async_update=True)
    st.update_fused(cols, c4_spec())
    kk, aa = st.finalize()
    kv = kk[0].to_numpy()
    av = [a.to_numpy() for a in aa]
    got = {int(kv[i]): tuple(int(a[i]) for a in av) for i in range(kk[0].length)}
    del cols

    class G(C.Structure):
        _fields_ = [(f, C.c_int64) for f in ("key", "sum", "count", "min", "max")]

    lib = C.CDLL(str(ROOT / "oracle" / "build" / "libqe_oracle.so"))
    lib.qe_cpu_c4_fast.restype = C.c_double
    lib.qe_cpu_c4_fast.argtypes = [C.c_int64, C.c_int64, C.c_uint64, C.c_int, C.c_int64, C.c_int64,
                                   C.POINTER(G), C.c_int64, C.POINTER(C.c_int64)]
    out = (G * 2048)()
    ng = C.c_int64()
    threads = min(64, len(os.sched_getaffinity(0)))
    assert lib.qe_cpu_c4_fast(0, n, 42, threads, 1 << 19, 1024, out, 2048, C.byref(ng)) >= 0
    want = {int(g.key): (int(g.sum), int(g.count), int(g.min), int(g.max)) for g in out[: ng.value]}
    assert len(got) == 1024 and got == want


def test_c5_full_size_slice(gpu_ctx):
    """C5: one GPU's 1.25B-row slice (of 10B over 8 GPUs) of the lineitem-shaped Q1 query."""
    from kquery.datasource import C5_COLUMNS, generate_column
    from kquery.workloads import C5_AGGS, C5_KEY_TYPES, c5_spec

    n = 1_250_000_000
    row0 = 3 * n  # rank 3's slice
    cols = {s.name: generate_column(s, n, row0, 42, gpu_ctx) for s in C5_COLUMNS}
    st = HashAggregateState(gpu_ctx, C5_KEY_TYPES, C5_AGGS, 16)
    st.update_fused([cols[s.name] for s in C5_COLUMNS], c5_spec())
    kk, aa = st.finalize()
    assert kk[0].length == 6
    sq, sp, sdp, sdpt, avg, cstar = (a.to_numpy() for a in aa)
    # the predicate, per family: four comparisons and three ANDs
    ms = []
    for col, op, lit in (("l_shipdate", N.OP_LE, 2400), ("l_discount", N.OP_GE, 0.05),
                         ("l_discount", N.OP_LE, 0.07), ("l_quantity", N.OP_LT, 24)):
        ms.append(_eval(gpu_ctx, "qe_eval_cmp", op, cols[col], lit, DeviceColumn.empty(N.TYPE_BOOL, n, False, ctx=gpu_ctx)))
    mask = ms[0]
    for m in ms[1:]:
        out = DeviceColumn.empty(N.TYPE_BOOL, n, False, ctx=gpu_ctx)
        ac, bc, oc = mask.as_c(), m.as_c(), out.as_c()
        N.check(N.lib().qe_eval_bool(gpu_ctx.handle, N.OP_AND, N.C.byref(ac), N.C.byref(bc), N.C.byref(oc)))
        mask = out
    del ms
    sel = _count(gpu_ctx, mask)
    assert int(cstar.sum()) == sel
    gq = _global(gpu_ctx, cols["l_quantity"], mask)
    assert gq.count == sel and int(sq.astype(np.uint64).sum(dtype=np.uint64).view(np.int64)) == gq.sum

    def close(group_sum, g):
        want = f64_from_bits(g.sum)
        return abs(group_sum - want) <= REL * abs(want), (group_sum, want)

    gp = _global(gpu_ctx, cols["l_extendedprice"], mask)
    ok, why = close(float(np.sum(sp)), gp)
    assert ok, why
    ok, why = close(float(np.sum(avg * cstar.astype(np.float64))), gp)
    assert ok, why
    one_minus = _eval(gpu_ctx, "qe_eval_arith", N.OP_SUB, 1.0, cols["l_discount"],
                      DeviceColumn.empty(N.TYPE_FLOAT64, n, False, ctx=gpu_ctx))
    dp = _eval(gpu_ctx, "qe_eval_arith", N.OP_MUL, cols["l_extendedprice"], one_minus,
               DeviceColumn.empty(N.TYPE_FLOAT64, n, False, ctx=gpu_ctx))
    del one_minus
    ok, why = close(float(np.sum(sdp)), _global(gpu_ctx, dp, mask))
    assert ok, why
    one_plus = _eval(gpu_ctx, "qe_eval_arith", N.OP_ADD, 1.0, cols["l_tax"],
                     DeviceColumn.empty(N.TYPE_FLOAT64, n, False, ctx=gpu_ctx))
    dpt = _eval(gpu_ctx, "qe_eval_arith", N.OP_MUL, dp, one_plus, DeviceColumn.empty(N.TYPE_FLOAT64, n, False, ctx=gpu_ctx))
    ok, why = close(float(np.sum(sdpt)), _global(gpu_ctx, dpt, mask))
    assert ok, why
