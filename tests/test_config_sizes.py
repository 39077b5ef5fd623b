"""Every BASELINE.json configuration at the size it names, on one GPU (VERDICT r02 "exercise every
BASELINE config at its size"):

* C2 — 10M int64 rows, filter(a > 2^19) + project(a + b) on the default (auto) select-project
  path: bit-exact against the oracle's restatement over all 10M rows;
* C3 — 100M fp64 rows (UNIT53 generator: every value a multiple of 2^-42, so the exact sum is an
  integer sum of the u53 words): COUNT / MIN / MAX bit-exact, SUM within 1e-9 of the exact sum;
* C4 — 1B int64 rows, 1024 groups: EVERY group's SUM / COUNT / MIN / MAX against the C oracle
  (oracle/cpu_baseline.c, pinned to oracle/semantics.py by tests/test_oracle.py) over the same
  1B rows;
* C5 — one GPU's 1.25B-row slice of the 10B lineitem config: every one of the 6 groups against the
  C oracle over the same rows (oracle/cpu_baseline.c qe_cpu_c5_exact, exact fp64 sums): COUNT(*)
  and SUM(l_quantity) exact, the fp64 SUMs and AVG bit for bit (the correctly rounded exact sums).

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


def test_c5_full_size_every_group(gpu_ctx):
    """C5: one GPU's 1.25B-row slice (of 10B over 8 GPUs) of the lineitem-shaped Q1 query, every
    group against the C oracle over the same rows (oracle/cpu_baseline.c qe_cpu_c5_exact: the rows
    regenerated bit for bit, fp64 sums accumulated exactly). COUNT(*) and SUM(quantity) exact; the
    three fp64 SUMs equal the correctly rounded exact sums and AVG their quotient by the count, bit
    for bit — the default exact accumulation is held to more than the 1e-9 contract here."""
    from kquery.datasource import C5_COLUMNS, generate_column
    from kquery.workloads import C5_AGGS, C5_KEY_TYPES, c5_spec

    n = 1_250_000_000
    row0 = 3 * n  # rank 3's slice
    cols = [generate_column(s, n, row0, 42, gpu_ctx) for s in C5_COLUMNS]
    st = HashAggregateState(gpu_ctx, C5_KEY_TYPES, C5_AGGS, 16)
    st.update_fused(cols, c5_spec())
    kk, aa = st.finalize()
    del cols
    assert kk[0].length == 6
    flags, stats = kk[0].to_numpy(), kk[1].to_numpy()
    vals = [a.to_numpy() for a in aa]

    lib = C.CDLL(str(ROOT / "oracle" / "build" / "libqe_oracle.so"))
    lib.qe_cpu_c5_exact.restype = C.c_double
    lib.qe_cpu_c5_exact.argtypes = [C.c_int64, C.c_int64, C.c_uint64, C.c_int, C.POINTER(C.c_int64)]
    out = (C.c_int64 * 48)()
    threads = min(64, len(os.sched_getaffinity(0)))
    assert lib.qe_cpu_c5_exact(row0, n, 42, threads, out) >= 0, "a value was not a multiple of 2^-80"

    def exact(hi, lo):
        return Fraction((hi << 64) + (lo & ((1 << 64) - 1)), 1 << 80)

    for i in range(6):
        g = int(flags[i]) * 2 + int(stats[i])
        o = list(out[g * 8:(g + 1) * 8])
        sq, sp, sdp, sdpt, avg, cstar = (v[i] for v in vals)
        assert int(cstar) == o[0] and int(sq) == o[1], (g, int(cstar), o[0], int(sq), o[1])
        want = [float(exact(o[2 + 2 * k], o[3 + 2 * k])) for k in range(3)]
        got = [float(sp), float(sdp), float(sdpt)]
        assert got == want, (g, got, want)
        assert float(avg) == want[0] / o[0], (g, float(avg), want[0] / o[0])
