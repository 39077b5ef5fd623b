"""CAST(utf8 AS double) — CastExpression, Main.kt:772-805 (K:791 String.toDouble()).

CPU: the oracle (oracle/cast_ref.py) against the hand-written JDK known answers
(tests/golden/cast_kat.json) and against exact rational rounding on random inputs.
GPU: qe_cast_utf8_to_f64 bit-exact against the oracle over a corpus that drives both the fast
path and the big-integer exact path (halfway cases, >800-digit strings, subnormals, overflow
boundaries, hex floats), plus nulls, whitespace, error rows and the CastExpression operator."""
import json
import math
import pathlib
import random
import struct
from decimal import Decimal
from fractions import Fraction

import numpy as np
import pytest

from oracle import cast_ref as R

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden" / "cast_kat.json"
KAT = json.loads(GOLDEN.read_text())


def _bits(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", x))[0]


def _f(b: int) -> float:
    return struct.unpack("<d", struct.pack("<q", b))[0]


def _hexbits(v: float) -> str:
    return "NaN" if math.isnan(v) else "%016x" % (_bits(v) & (2**64 - 1))


def exact_round(fr: Fraction) -> float:
    """Nearest double to a non-negative rational, ties to even — by bisection over bit patterns
    (independent of float()/strtod)."""
    inf = 0x7FF0000000000000
    lo, hi = 0, inf
    while hi - lo > 1:
        m = (lo + hi) // 2
        if Fraction(_f(m)) <= fr:
            lo = m
        else:
            hi = m
    if Fraction(_f(lo)) == fr:
        return _f(lo)
    # overflow: beyond DBL_MAX + half ulp (the value 2^1024 acts as the successor)
    up = Fraction(2) ** 1024 if hi == inf else Fraction(_f(hi))
    a, b = fr - Fraction(_f(lo)), up - fr
    pick = lo if (a < b or (a == b and lo % 2 == 0)) else hi
    return math.inf if pick == inf else _f(pick)


# ---- corpus -----------------------------------------------------------------------------------
def _midpoint_str(x: float, up: bool = True) -> str:
    """Exact decimal expansion of the midpoint between x (> 0) and its neighbour."""
    b = _bits(x)
    y = _f(b + 1) if up else _f(b - 1)
    m = (Fraction(x) + Fraction(y)) / 2
    return format(Decimal(m.numerator) / Decimal(m.denominator), "f") if m.denominator == 1 else \
        _exact_decimal(m)


def _exact_decimal(m: Fraction) -> str:
    # denominator is a power of two: m = n / 2^k = n * 5^k / 10^k
    k = m.denominator.bit_length() - 1
    assert m.denominator == 1 << k
    digits = str(m.numerator * 5**k)
    if k == 0:
        return digits
    digits = digits.rjust(k + 1, "0")
    return digits[:-k] + "." + digits[-k:]


def corpus(seed: int = 7, n_random: int = 3000):
    rng = random.Random(seed)
    out = [e["in"] for e in KAT if e["out"] != "NFE"]
    # random finite doubles, shortest repr / 17 digits / fixed / scientific with many digits
    for _ in range(n_random):
        b = rng.getrandbits(63)
        if (b >> 52) == 0x7FF:
            continue
        x = _f(b)
        out.append(repr(x))
        out.append("%.17g" % x)
        out.append("%.25e" % x)
        out.append("-" + repr(x))
    # typical CSV numbers (fast path): prices, ints, small exponents
    for _ in range(n_random):
        out.append("%.2f" % rng.uniform(-1000, 100000))
        out.append(str(rng.randint(-10**15, 10**15)))
        out.append("%de%d" % (rng.randint(1, 10**6), rng.randint(-30, 30)))
    # random digit strings with random exponents (many digits -> exact path)
    for _ in range(n_random // 2):
        nd = rng.choice([1, 5, 16, 17, 18, 19, 20, 25, 40, 100])
        d = "".join(rng.choice("0123456789") for _ in range(nd))
        e = rng.randint(-360, 320)
        s = (d[:1] + "." + d[1:] if rng.random() < 0.5 else d) + "e" + str(e)
        out.append(s)
    # halfway cases (exact midpoints; ties to even) and midpoints +- a tiny tail
    for _ in range(300):
        b = rng.choice([rng.randint(1, 2**20), rng.randint(2**52 - 5, 2**52 + 5),
                        rng.randint(1, 0x7FEFFFFFFFFFFFFF)])
        x = _f(b)
        m = _midpoint_str(x, up=True)
        out.append(m)
        out.append(m + "000000001" if "." in m else m + ".000000001")
        if b > 1:
            m2 = _midpoint_str(x, up=False)
            out.append(m2)
    # > 800 significant digits (sticky tail) around a midpoint
    x = 1.0
    m = _midpoint_str(x, up=True)  # 1 + 2^-53
    out.append(m + "0" * 900)
    out.append(m + "0" * 900 + "1")
    out.append("9" * 1000)
    out.append("0." + "0" * 300 + "1" * 900 + "e300")
    # hex floats
    for _ in range(500):
        b = rng.getrandbits(63)
        if (b >> 52) == 0x7FF:
            continue
        out.append(_f(b).hex())
        out.append("0x" + "%x" % rng.getrandbits(rng.choice([8, 60, 64, 80])) + "p" + str(rng.randint(-1150, 1000)))
        out.append("0X" + "%X" % rng.getrandbits(24) + "." + "%x" % rng.getrandbits(90) + "P-" +
                   str(rng.randint(0, 1100)) + rng.choice(["", "d", "F"]))
    # whitespace, signs, suffixes
    for s in list(out[:500]):
        sfx = "" if s[-1] in "fFdDNy" or s.strip(R._TRIM) != s else rng.choice(["", "d", "D", "f", "F"])
        out.append(" \t" + s + sfx + "\n ")
    return out


# ---- CPU: the oracle ---------------------------------------------------------------------------
def test_oracle_matches_jdk_known_answers():
    for e in KAT:
        s, want = e["in"], e["out"]
        try:
            got = _hexbits(R.parse_java_double(s))
        except R.NumberFormatException:
            got = "NFE"
        assert got == want, (s, want, got)


def test_oracle_matches_exact_rounding():
    rng = random.Random(11)
    cases = corpus(seed=3, n_random=120)
    for s in cases:
        t = s.strip(R._TRIM)
        body = t.lstrip("+-")
        if body in ("NaN", "Infinity"):
            continue
        if body[-1] in "fFdD":
            body = body[:-1]
        if body[:2].lower() == "0x":
            mant, _, ex = body[2:].partition("p") if "p" in body else body[2:].partition("P")
            ip, _, fp = mant.partition(".")
            fr = Fraction(int((ip + fp) or "0", 16)) * Fraction(2) ** (int(ex) - 4 * len(fp))
        else:
            fr = Fraction(Decimal(body)) if abs(int(Decimal(body).adjusted())) < 5000 else None
            if fr is None:
                continue
        want = exact_round(abs(fr))
        got = abs(R.parse_java_double(s))
        assert _bits(got) == _bits(want), (s[:80], got, want)
    assert rng  # deterministic


def test_oracle_error_row_and_nulls():
    vals, valid = R.cast_utf8_to_f64(["1.5", None, " -2 ", "NaN"])
    assert valid.tolist() == [True, False, True, True]
    assert vals[0] == 1.5 and vals[2] == -2.0 and math.isnan(vals[3])
    with pytest.raises(R.NumberFormatException, match="row 2"):
        R.cast_utf8_to_f64(["1", None, "1e", "x"])


# ---- CPU: the device parser compiled for the host (algorithm check without a GPU) --------------
@pytest.fixture(scope="module")
def host_parser():
    import ctypes
    import subprocess

    d = pathlib.Path(__file__).resolve().parent / "native"
    r = subprocess.run(["make", "-s", "-C", str(d)], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("hipcc host build unavailable: " + r.stderr[-300:])
    lib = ctypes.CDLL(str(d / "_build" / "libqe_cast_host.so"))
    fn = lib.qe_cast_host
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]

    def parse(s: str):
        b = s.encode()
        out, slow = ctypes.c_double(), ctypes.c_int()
        st = fn(b, len(b), ctypes.byref(out), ctypes.byref(slow))
        return (None if st else out.value), bool(slow.value)

    return parse


def test_device_parser_on_host_matches_oracle(host_parser):
    strings = corpus()
    nslow = 0
    bad = []
    for s in strings:
        v, slow = host_parser(s)
        nslow += slow
        want = R.parse_java_double(s)
        if v is None or not R.same_f64(v, want):
            bad.append((s[:70], v, want))
    assert not bad, (len(bad), bad[:10])
    assert nslow > 1000  # the corpus exercises the exact (big-integer) path
    for e in KAT:
        v, _ = host_parser(e["in"])
        assert (v is None) == (e["out"] == "NFE"), e["in"]


# ---- GPU ---------------------------------------------------------------------------------------
def _dev_cast(ctx, strings):
    from kquery import native as N
    from kquery.columnar import DeviceColumn

    col = DeviceColumn.from_strings(strings, ctx=ctx)
    out = DeviceColumn.empty(N.TYPE_FLOAT64, len(strings), col.nullable, ctx=ctx)
    ic, oc = col.as_c(), out.as_c()
    row = N.C.c_int64(-7)
    st = N.lib().qe_cast_utf8_to_f64(ctx.handle, N.C.byref(ic), N.C.byref(oc), N.C.byref(row))
    return st, row.value, out


@pytest.mark.gpu
def test_cast_kernel_matches_oracle(gpu_ctx):
    from kquery import native as N

    strings = corpus()
    rng = random.Random(5)
    with_nulls = [None if rng.random() < 0.05 else s for s in strings]
    for data in (strings, with_nulls):
        st, row, out = _dev_cast(gpu_ctx, data)
        assert st == N.QE_OK, N.lib().qe_last_error()
        assert row == -1
        want, wvalid = R.cast_utf8_to_f64(data)
        got, gvalid = out.to_numpy(), out.valid_mask()
        assert (gvalid == wvalid).all()
        bad = [(data[i][:60], _hexbits(got[i]), _hexbits(want[i])) for i in range(len(data))
               if wvalid[i] and not R.same_f64(float(got[i]), float(want[i]))]
        assert not bad, (len(bad), bad[:10])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 8193, 200_001])
def test_cast_sizes(gpu_ctx, n):
    from kquery import native as N

    rng = np.random.default_rng(n)
    vals = rng.uniform(-1e6, 1e6, n)
    strings = ["%.2f" % v if i % 11 else None for i, v in enumerate(vals)]
    st, row, out = _dev_cast(gpu_ctx, strings)
    assert st == N.QE_OK and row == -1
    want, wvalid = R.cast_utf8_to_f64(strings)
    assert (out.valid_mask() == wvalid).all()
    got = out.to_numpy()
    assert (got[wvalid].view(np.int64) == want[wvalid].view(np.int64)).all()


@pytest.mark.gpu
def test_cast_number_format_errors(gpu_ctx):
    from kquery import native as N

    bad = [e["in"] for e in KAT if e["out"] == "NFE"]
    for s in bad:
        st, row, _ = _dev_cast(gpu_ctx, ["1.0", None, s, "2", s])
        assert st == N.QE_ERR_INVALID_ARG, repr(s)
        assert row == 2, repr(s)
        assert "NumberFormatException" in N.lib().qe_last_error().decode()
    # first offending row over a large column
    strings = ["%d.5" % i for i in range(300_000)]
    strings[123_457] = "12x"
    strings[250_000] = ""
    st, row, _ = _dev_cast(gpu_ctx, strings)
    assert st == N.QE_ERR_INVALID_ARG and row == 123_457


@pytest.mark.gpu
def test_cast_expression_operator(gpu_ctx):
    from kquery import native as N
    from kquery.columnar import DeviceColumn, Field, RecordBatch, Schema
    from kquery.expressions import CastExpression, ColumnExpression

    strings = ["7.25", None, "1e3", " -0 ", "0x1p-2"]
    batch = RecordBatch(Schema([Field("s", N.TYPE_UTF8)]), [DeviceColumn.from_strings(strings, ctx=gpu_ctx)])
    out = CastExpression(ColumnExpression(0), N.TYPE_FLOAT64).evaluate(batch)
    assert out.to_pylist() == [7.25, None, 1000.0, -0.0, 0.25]
    assert math.copysign(1, out.to_pylist()[3]) == -1
    with pytest.raises(N.NumberFormatException):
        bb = RecordBatch(batch.schema, [DeviceColumn.from_strings(["1", "one"], ctx=gpu_ctx)])
        CastExpression(ColumnExpression(0), N.TYPE_FLOAT64).evaluate(bb)
    # K:792: non-String values throw; K:799: other targets throw
    ints = RecordBatch(Schema([Field("i", N.TYPE_INT64)]),
                       [DeviceColumn.from_numpy(N.TYPE_INT64, np.array([5, 6]), np.array([False, True]), ctx=gpu_ctx)])
    with pytest.raises(N.IllegalStateException, match="Cannot cast value to Double: 6"):
        CastExpression(ColumnExpression(0), N.TYPE_FLOAT64).evaluate(ints)
    nulls = RecordBatch(ints.schema, [DeviceColumn.from_numpy(N.TYPE_INT64, np.array([5, 6]),
                                                              np.array([False, False]), ctx=gpu_ctx)])
    assert CastExpression(ColumnExpression(0), N.TYPE_FLOAT64).evaluate(nulls).to_pylist() == [None, None]
    with pytest.raises(N.IllegalStateException, match="not supported"):
        CastExpression(ColumnExpression(0), N.TYPE_INT64).evaluate(batch)


def test_register_fast_path_on_host(host_parser):
    """The CAST kernel's register fast path (qe_cast_parse.hpp fast_decimal: [+-]digits[.digits],
    at most 15 digits, one exact division) returns exactly what the full parser returns wherever it
    applies, declines everything else, and agrees with every JDK known answer it takes."""
    import ctypes
    import random

    d = pathlib.Path(__file__).resolve().parent / "native"
    fast = ctypes.CDLL(str(d / "_build" / "libqe_cast_host.so")).qe_cast_host_fast
    fast.restype = ctypes.c_int
    fast.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]

    def f(s):
        out = ctypes.c_double()
        return out.value if fast(s.encode(), len(s.encode()), ctypes.byref(out)) else None

    rng = random.Random(5)
    taken = 0
    for _ in range(20000):
        a = "".join(rng.choice("0123456789") for _ in range(rng.randint(0, 9)))
        b = "".join(rng.choice("0123456789") for _ in range(rng.randint(0, 8)))
        dot = rng.random() < 0.7
        s = rng.choice(["", "-", "+"]) + a + (("." + b) if dot else "")
        digits = a + (b if dot else "")
        v = f(s)
        if v is not None:
            taken += 1
            want = R.parse_java_double(s)
            assert R.same_f64(v, want), (s, v, want)
            assert R.same_f64(v, host_parser(s)[0]), s
        elif digits:
            assert len(digits) > 15 or len(s) > 16, s  # declined only beyond its range
    assert taken > 15000
    for s in ["", ".", "-", "+", "1e5", " 1", "1 ", "NaN", "0x1p3", "1d", "1.2.3", "12345678901234567", "1_0"]:
        assert f(s) is None, s
    for e in KAT:
        v = f(e["in"])
        if v is not None:
            assert e["out"] != "NFE" and np.float64(v).view(np.uint64) == int(e["out"], 16), e["in"]
