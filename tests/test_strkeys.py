"""UTF-8 group keys (K:620-627: HashMap keyed by String(bytes)) through the device string
dictionary, and the reference's own workloads that need them:

* config 1 aggregate: employee.csv GROUP BY state, MAX(CAST(salary AS double)) against the
  fixture's known answer (tests/golden/employee_kat.json);
* main()'s two-phase query (K:1307-1336): per-month partial
  ``SELECT VendorID, MAX(CAST(fare_amount AS double)) AS max_amount FROM tripdata GROUP BY VendorID``
  over CSV files, then ``SELECT VendorID, MAX(max_amount) ... GROUP BY VendorID`` over the collected
  partial batches — synthetic trip CSVs of that shape, checked against the oracle's literal
  HashAggregateExec loop.
"""
import json
import math
import pathlib
import random

import numpy as np
import pytest

from oracle import cast_ref as R
from oracle import semantics as S

GOLD = pathlib.Path(__file__).resolve().parent / "golden"


def _random_strings(rng, n, distinct):
    pool = set()
    alphabet = "abcXYZ019 _-åäö€"
    while len(pool) < distinct:
        ln = rng.choice([0, 1, 2, 7, 8, 9, 15, 16, 17, 40, 100])
        pool.add("".join(rng.choice(alphabet) for _ in range(ln)))
    pool = sorted(pool)
    # near-duplicates: same prefix, differ in the last byte
    pool += [p[:-1] + "#" for p in pool[:10] if p]
    return [rng.choice(pool) for _ in range(n)], pool


def test_oracle_groups_strings_by_content():
    g = S.hash_aggregate_rows([["a", "b", "a", None, "a"]], [[1.0, 2.0, 5.0, 7.0, None]], [S.AGG_MAX], [True])
    assert g == {("a",): [5.0], ("b",): [2.0], (None,): [7.0]}


@pytest.mark.gpu
@pytest.mark.parametrize("n,distinct,expected", [(1, 1, 16), (1000, 3, 16), (100_003, 500, 16),
                                                 (300_000, 120_000, 16), (200_000, 50, 100_000)])
def test_strdict_roundtrip(gpu_ctx, n, distinct, expected):
    from kquery.columnar import DeviceColumn
    from kquery.strdict import StringDictionary

    rng = random.Random(n + distinct)
    strings, pool = _random_strings(rng, n, distinct)
    strings = [None if rng.random() < 0.03 else s for s in strings]
    d = StringDictionary(gpu_ctx, expected)
    col = DeviceColumn.from_strings(strings, ctx=gpu_ctx)
    codes = d.encode(col)
    c = codes.to_numpy()
    valid = codes.valid_mask()
    assert valid.tolist() == [s is not None for s in strings]
    seen = {}
    for s, code, v in zip(strings, c, valid):
        if not v:
            continue
        assert seen.setdefault(s, int(code)) == int(code)  # same string -> same code
    assert len(set(seen.values())) == len(seen)  # distinct strings -> distinct codes
    assert d.size() == len(seen)
    assert sorted(seen.values()) == list(range(len(seen)))  # dense codes
    assert d.decode(codes).to_pylist() == strings
    # a second batch keeps the first batch's codes and extends them
    more = [rng.choice(pool) for _ in range(5000)] + ["brand-new-%d" % i for i in range(100)]
    c2 = d.encode(DeviceColumn.from_strings(more, ctx=gpu_ctx)).to_numpy()
    for s, code in zip(more, c2):
        if s in seen:
            assert int(code) == seen[s]
    assert d.size() == len(seen | {s: 0 for s in more})


@pytest.mark.gpu
@pytest.mark.parametrize("n,distinct", [(1, 1), (1000, 3), (100_003, 500), (300_000, 120_000)])
def test_strdict_wide_codes_roundtrip(gpu_ctx, n, distinct):
    """Wide (INT64) codes: keys of at most 7 bytes are their own code (bytes + length, no
    dictionary entry), longer keys 2^62 | a dense dictionary code. Same string -> same code,
    different strings -> different codes (incl. 'a' vs 'a\\0', 7 vs 8 bytes, ''), decode restores."""
    from kquery import native as N
    from kquery.columnar import DeviceColumn
    from kquery.strdict import StringDictionary

    rng = random.Random(n * 7 + distinct)
    strings, pool = _random_strings(rng, n, distinct)
    edge = ["", "a", "a\0", "\0", "abcdefg", "abcdefgh", "åäö", "1", "2", "4"]
    strings = edge + [None if rng.random() < 0.03 else s for s in strings]
    d = StringDictionary(gpu_ctx, 16, wide=True)
    codes = d.encode(DeviceColumn.from_strings(strings, ctx=gpu_ctx))
    assert codes.type == N.TYPE_INT64
    c = codes.to_numpy()
    valid = codes.valid_mask()
    assert valid.tolist() == [s is not None for s in strings]
    seen = {}
    for s, code, v in zip(strings, c, valid):
        if not v:
            continue
        b = s.encode()
        assert seen.setdefault(s, int(code)) == int(code)
        if len(b) <= 7:  # packed: bytes little-endian, length in bits 56..58
            assert int(code) == int.from_bytes(b, "little") | (len(b) << 56)
        else:
            assert int(code) >> 62 == 1
    assert len(set(seen.values())) == len(seen)
    long_keys = {s for s in seen if len(s.encode()) > 7}
    assert d.size() == len(long_keys)  # only long keys enter the dictionary
    assert sorted(seen[s] & ((1 << 62) - 1) for s in long_keys) == list(range(len(long_keys)))
    assert d.decode(codes).to_pylist() == strings


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 777, 70_000, 300_001])
def test_strdict_packed_codes_match_dictionary(gpu_ctx, n):
    """qe_strdict_encode_packed (a column known to hold values of at most 7 bytes, e.g. from the
    CSV scan's max length) gives exactly qe_strdict_encode's wide codes, without a dictionary;
    qe_strdict_decode_packed (one-block path up to 65536 rows, the general one above) restores
    the strings, nulls included."""
    from kquery.columnar import DeviceColumn
    from kquery.strdict import StringDictionary

    rng = random.Random(n)
    alphabet = "abcxyz0129åé,\"\0 "
    strings = ["", "a", "\0", "abcdefg", "åäö", "1234567"][: n] + [
        None if rng.random() < 0.05 else "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 3)))
        for _ in range(max(0, n - 6))]
    strings = [s if s is None or len(s.encode()) <= 7 else s[:2] for s in strings]
    col = DeviceColumn.from_strings(strings, ctx=gpu_ctx)
    ref = StringDictionary(gpu_ctx, 16, wide=True)
    want = ref.encode(col)  # max_len unknown: the dictionary kernel
    col.max_len = 7
    d = StringDictionary(gpu_ctx, 16, wide=True)
    got = d.encode(col)
    assert d._handle is None  # no device dictionary was needed
    gv, wv = got.valid_mask(), want.valid_mask()
    assert gv.tolist() == wv.tolist() == [s is not None for s in strings]
    assert (got.to_numpy()[gv] == want.to_numpy()[wv]).all()
    assert d.decode(got, trusted=True).to_pylist() == strings
    assert ref.decode(want).to_pylist() == strings


@pytest.mark.gpu
def test_group_by_lone_utf8_key_wide_codes(gpu_ctx):
    """A lone UTF-8 group key takes wide codes: short and long keys, nulls and empty strings
    group by content against the oracle's HashAggregateExec loop."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    rng = random.Random(5)
    keys = [rng.choice(["", "1", "2", "4", "abcdefg", "abcdefgh", "a-much-longer-vendor-id", None]) for _ in range(50_000)]
    vals = [rng.random() * 100 for _ in keys]
    st = HashAggregateState(gpu_ctx, [N.TYPE_UTF8], [(N.AGG_MAX, N.TYPE_FLOAT64), (N.AGG_COUNT_STAR, N.TYPE_INT64)], 16)
    assert st.device_key_types == [N.TYPE_INT64]
    for a, b in ((0, 20_000), (20_000, 50_000)):  # two batches: codes stable across updates
        st.update([DeviceColumn.from_strings(keys[a:b], ctx=gpu_ctx)],
                  [DeviceColumn.from_numpy(N.TYPE_FLOAT64, np.array(vals[a:b]), ctx=gpu_ctx), None])
    k, v = st.finalize()
    got = {kk: (m, c) for kk, m, c in zip(k[0].to_pylist(), v[0].to_pylist(), v[1].to_pylist())}
    want = S.hash_aggregate_rows([keys], [vals, [1.0] * len(keys)], [S.AGG_MAX, S.AGG_COUNT_STAR], [True, True])
    assert {kk[0]: (w[0], w[1]) for kk, w in want.items()} == got


@pytest.mark.gpu
def test_strdict_rejects_foreign_codes(gpu_ctx):
    from kquery import native as N
    from kquery.columnar import DeviceColumn
    from kquery.strdict import StringDictionary

    d = StringDictionary(gpu_ctx, 16)
    d.encode(DeviceColumn.from_strings(["x", "y"], ctx=gpu_ctx))
    with pytest.raises(N.IllegalArgumentException):
        d.decode(DeviceColumn.from_numpy(N.TYPE_INT32, np.array([0, 5], dtype=np.int32), ctx=gpu_ctx))


@pytest.mark.gpu
def test_config1_group_by_state_max_salary(gpu_ctx):
    """BASELINE config 1 aggregate on the device: GROUP BY state (UTF-8 key),
    MAX(CAST(salary AS double)) — against the reference fixture's known answer."""
    from kquery import native as N
    from kquery.columnar import Field, Schema
    from kquery.csv_source import CsvDataSource
    from kquery.expressions import CastExpression, ColumnExpression, MaxExpression
    from kquery.operators import HashAggregateExec, ScanExec

    kat = json.loads((GOLD / "employee_kat.json").read_text())["group_state_max_salary"]
    ds = CsvDataSource(str(GOLD / "employee.csv"), True, 1000, ctx=gpu_ctx)
    scan = ScanExec(ds, ["state", "salary"])
    agg = HashAggregateExec(scan, [ColumnExpression(0)],
                            [MaxExpression(CastExpression(ColumnExpression(1), N.TYPE_FLOAT64))],
                            Schema([Field("state", N.TYPE_UTF8), Field("MAX", N.TYPE_FLOAT64)]))
    out = list(agg.execute())
    assert len(out) == 1
    got = dict(zip(out[0].field(0).to_pylist(), out[0].field(1).to_pylist()))
    assert got == kat


def _write_trip_csv(path, rng, rows, vendors):
    lines = ["VendorID,tpep_pickup_datetime,passenger_count,fare_amount"]
    for i in range(rows):
        v = rng.choice(vendors)
        fare = rng.choice(["%.2f" % rng.uniform(-50, 500), "%d" % rng.randint(0, 900), "%.1f" % rng.uniform(0, 99),
                           "1e2", "0.30000000000000004", " 12.5 "])
        if rng.random() < 0.01:
            fare = ""  # empty field: "".toDouble() throws (test_empty_fare_throws_number_format)
        lines.append(f"{v},2024-01-{1 + i % 28:02d} 10:00:00,{rng.randint(1, 6)},{fare}")
    path.write_text("\n".join(lines) + "\n")


@pytest.mark.gpu
def test_main_two_phase_vendor_max_fare(gpu_ctx, tmp_path):
    """K:1307-1336: 12 per-month partial aggregates over CSV -> collected batches -> final
    GROUP BY VendorID, MAX(max_amount)."""
    from kquery import native as N
    from kquery.columnar import Field, Schema
    from kquery.csv_source import CsvDataSource
    from kquery.datasource import InMemoryDataSource
    from kquery.expressions import CastExpression, ColumnExpression, MaxExpression
    from kquery.operators import HashAggregateExec, ScanExec

    rng = random.Random(2024)
    vendors = ["1", "2", "6", "7"]
    results = []
    all_vendor, all_fare = [], []
    for month in range(1, 13):
        p = tmp_path / f"yc-{month:02d}.csv"
        _write_trip_csv(p, rng, 3000 + 97 * month, vendors[: 2 + month % 3])
        # drop the rows with empty fares (they make toDouble throw in the reference)
        text = [ln for ln in p.read_text().splitlines() if not ln.endswith(",")]
        p.write_text("\n".join(text) + "\n")
        for ln in text[1:]:
            f = ln.split(",")
            all_vendor.append(f[0].strip())
            all_fare.append(f[3].strip())
        ds = CsvDataSource(str(p), True, 1000, ctx=gpu_ctx)
        part = HashAggregateExec(ScanExec(ds, ["VendorID", "fare_amount"]), [ColumnExpression(0)],
                                 [MaxExpression(CastExpression(ColumnExpression(1), N.TYPE_FLOAT64))],
                                 Schema([Field("VendorID", N.TYPE_UTF8), Field("max_amount", N.TYPE_FLOAT64)]))
        results.extend(part.execute())
    schema = results[0].schema
    final = HashAggregateExec(ScanExec(InMemoryDataSource(schema, results), ["VendorID", "max_amount"]),
                              [ColumnExpression(0)], [MaxExpression(ColumnExpression(1))],
                              Schema([Field("VendorID", N.TYPE_UTF8), Field("MAX", N.TYPE_FLOAT64)]))
    out = list(final.execute())[0]
    got = dict(zip(out.field(0).to_pylist(), out.field(1).to_pylist()))
    fares = [R.parse_java_double(f) for f in all_fare]
    want = S.hash_aggregate_rows([all_vendor], [fares], [S.AGG_MAX], [True])
    assert got == {k[0]: v[0] for k, v in want.items()}


@pytest.mark.gpu
def test_group_by_utf8_with_nulls_and_many_groups(gpu_ctx):
    """Unfused HashAggregateExec with a UTF-8 key plus a UINT8 key: SUM/COUNT/MIN/MAX/AVG vs the
    oracle's literal loop; null strings form their own group; 20k distinct strings force growth."""
    from kquery import native as N
    from kquery.columnar import DeviceColumn, Field, RecordBatch, Schema
    from kquery.datasource import InMemoryDataSource
    from kquery.expressions import (AvgExpression, ColumnExpression, CountExpression, MaxExpression,
                                    MinExpression, SumExpression)
    from kquery.operators import HashAggregateExec, ScanExec

    rng = random.Random(99)
    batches, ks, ts, vs = [], [], [], []
    # multi-key groups pack into 63 bits: the UTF-8 code (32+1) with a UINT8 key (8+1)
    schema = Schema([Field("s", N.TYPE_UTF8), Field("t", N.TYPE_UINT8), Field("v", N.TYPE_INT64)])
    for b in range(3):
        n = 40_000
        strings, _ = _random_strings(rng, n, 20_000 if b == 1 else 30)
        strings = [None if rng.random() < 0.02 else s for s in strings]
        t = np.array([rng.randint(0, 2) for _ in range(n)], dtype=np.uint8)
        v = np.array([rng.randint(-10**6, 10**6) for _ in range(n)], dtype=np.int64)
        batches.append(RecordBatch(schema, [DeviceColumn.from_strings(strings, ctx=gpu_ctx),
                                            DeviceColumn.from_numpy(N.TYPE_UINT8, t, ctx=gpu_ctx),
                                            DeviceColumn.from_numpy(N.TYPE_INT64, v, ctx=gpu_ctx)]))
        ks += strings
        ts += t.tolist()
        vs += v.tolist()
    aggs = [SumExpression(ColumnExpression(2)), CountExpression(ColumnExpression(2)),
            MinExpression(ColumnExpression(2)), MaxExpression(ColumnExpression(2)), AvgExpression(ColumnExpression(2))]
    out_schema = Schema([Field("s", N.TYPE_UTF8), Field("t", N.TYPE_UINT8)] +
                        [Field(a.name, N.TYPE_INT64) for a in aggs])
    plan = HashAggregateExec(ScanExec(InMemoryDataSource(schema, batches), ["s", "t", "v"]),
                             [ColumnExpression(0), ColumnExpression(1)], aggs, out_schema, expected_groups=64)
    out = list(plan.execute())[0]
    cols = [out.field(i).to_pylist() for i in range(2 + len(aggs))]
    got = {(r[0], r[1]): list(r[2:]) for r in zip(*cols)}
    fns = [S.AGG_SUM, S.AGG_COUNT, S.AGG_MIN, S.AGG_MAX, S.AGG_AVG]
    want = S.hash_aggregate_rows([ks, ts], [vs] * 5, fns, [False] * 5)
    assert len(got) == len(want)
    for k, w in want.items():
        g = got[k]
        assert g[:4] == w[:4], k
        assert math.isclose(g[4], w[4], rel_tol=1e-12), k


@pytest.mark.gpu
def test_empty_fare_throws_number_format(gpu_ctx, tmp_path):
    """An empty CSV field reads as "" (K:263) and "".toDouble() throws NumberFormatException."""
    from kquery import native as N
    from kquery.columnar import Field, Schema
    from kquery.csv_source import CsvDataSource
    from kquery.expressions import CastExpression, ColumnExpression, MaxExpression
    from kquery.operators import HashAggregateExec, ScanExec

    p = tmp_path / "yc-01.csv"
    p.write_text("VendorID,fare_amount\n1,2.5\n2,\n1,3\n")
    agg = HashAggregateExec(ScanExec(CsvDataSource(str(p), True, 1000, ctx=gpu_ctx), ["VendorID", "fare_amount"]),
                            [ColumnExpression(0)], [MaxExpression(CastExpression(ColumnExpression(1), N.TYPE_FLOAT64))],
                            Schema([Field("VendorID", N.TYPE_UTF8), Field("max_amount", N.TYPE_FLOAT64)]))
    with pytest.raises(N.NumberFormatException):
        list(agg.execute())
