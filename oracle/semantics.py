"""ORACLE (test infrastructure only — never imported by the product path).

CPU restatement of the kquerydiy hot path (folkol/query-engines kquerydiy/src/Main.kt, "K:"),
the checker for every HIP kernel in query-engines_amd/csrc. Two forms per function:

* literal row-at-a-time restatements (pure Python) that follow the reference line by line —
  ``MaxAccumulator`` K:538-561, ``HashAggregateExec.execute`` K:615-651 — used on small inputs;
* numpy-vectorised equivalents for sizes where the loops are too slow, cross-checked against the
  literal forms in tests/test_oracle.py.

PARITY PINNING. The reference is Kotlin/JVM and cannot run in this container (no JVM/kotlinc,
SURVEY §8c); it has no tests. The only reference fixture is kquerydiy/employee.csv, whose known
answers (tests/golden/employee_kat.json) pin the CSV/filter/group-by/MAX restatement. Everything
the reference does not define (int64 columns, arithmetic, comparisons, boolean logic, filter,
SUM/MIN/COUNT/AVG — SURVEY §0 / §8a A5, A9) is build-defined: those semantics are "parity
unpinned by reference" and documented in include/qe_hip.h and DESIGN.md.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

# op codes (include/qe_hip.h)
OP_ADD, OP_SUB, OP_MUL, OP_DIV = 1, 2, 3, 4
OP_EQ, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE = 10, 11, 12, 13, 14, 15
OP_AND, OP_OR, OP_NOT, OP_IS_NULL, OP_IS_NOT_NULL = 20, 21, 22, 23, 24
AGG_SUM, AGG_MIN, AGG_MAX, AGG_COUNT, AGG_COUNT_STAR, AGG_AVG = 1, 2, 3, 4, 5, 6

I64_MIN = -(1 << 63)


def _valid(v: Optional[np.ndarray], n: int) -> np.ndarray:
    return np.ones(n, dtype=bool) if v is None else np.asarray(v, dtype=bool)


# ---- K1 arithmetic (build-defined: JVM Long wrap, truncating division, x/0 -> null) ---------------
def arith(op: int, a, av, b, bv) -> Tuple[np.ndarray, np.ndarray]:
    """a/b: ndarray or python scalar (literal). Returns (values, valid)."""
    n = len(a) if isinstance(a, np.ndarray) else len(b)
    is_f = (np.asarray(a).dtype == np.float64) or (np.asarray(b).dtype == np.float64) \
        or isinstance(a, float) or isinstance(b, float)
    valid = _valid(av, n) & _valid(bv, n)
    if is_f:
        x = np.broadcast_to(np.asarray(a, dtype=np.float64), (n,))
        y = np.broadcast_to(np.asarray(b, dtype=np.float64), (n,))
        with np.errstate(all="ignore"):
            r = {OP_ADD: x + y, OP_SUB: x - y, OP_MUL: x * y, OP_DIV: x / y}[op]
        return r.astype(np.float64), valid
    x = np.broadcast_to(np.asarray(a, dtype=np.int64), (n,))
    y = np.broadcast_to(np.asarray(b, dtype=np.int64), (n,))
    with np.errstate(all="ignore"):
        if op == OP_ADD:
            r = (x.astype(np.uint64) + y.astype(np.uint64)).view(np.int64)
        elif op == OP_SUB:
            r = (x.astype(np.uint64) - y.astype(np.uint64)).view(np.int64)
        elif op == OP_MUL:
            r = (x.astype(np.uint64) * y.astype(np.uint64)).view(np.int64)
        else:
            r = np.zeros(n, dtype=np.int64)
            nz = y != 0
            m1 = y == -1
            r[m1] = (np.uint64(0) - x[m1].astype(np.uint64)).view(np.int64)
            ok = nz & ~m1
            q = np.abs(x[ok].astype(object)) // np.abs(y[ok].astype(object))  # exact, truncation
            sgn = np.sign(x[ok]) * np.sign(y[ok])
            r[ok] = np.array([int(s) * int(v) for s, v in zip(sgn, q)], dtype=np.int64) if ok.any() else []
            valid = valid & nz
    return r, valid


# ---- K2 comparison (IEEE fp64: NaN -> only NE true; signed int64; UTF-8 byte equality) -----------
def cmp(op: int, a, av, b, bv) -> Tuple[np.ndarray, np.ndarray]:
    n = len(a) if isinstance(a, np.ndarray) else len(b)
    valid = _valid(av, n) & _valid(bv, n)
    is_f = (np.asarray(a).dtype == np.float64) or (np.asarray(b).dtype == np.float64) \
        or isinstance(a, float) or isinstance(b, float)
    dt = np.float64 if is_f else np.int64
    x = np.broadcast_to(np.asarray(a, dtype=dt), (n,))
    y = np.broadcast_to(np.asarray(b, dtype=dt), (n,))
    with np.errstate(invalid="ignore"):
        r = {OP_EQ: x == y, OP_NE: x != y, OP_LT: x < y, OP_LE: x <= y, OP_GT: x > y, OP_GE: x >= y}[op]
    return r & valid, valid


def cmp_utf8(op: int, strings: Sequence[Optional[str]], lit: str) -> Tuple[np.ndarray, np.ndarray]:
    valid = np.array([s is not None for s in strings], dtype=bool)
    eq = np.array([s is not None and s.encode() == lit.encode() for s in strings], dtype=bool)
    r = eq if op == OP_EQ else (~eq & valid)
    return r, valid


# ---- K3a boolean (SQL three-valued logic) --------------------------------------------------------
def bool3(op: int, a, av, b=None, bv=None) -> Tuple[np.ndarray, np.ndarray]:
    n = len(a)
    a = np.asarray(a, dtype=bool)
    la = _valid(av, n)
    if op == OP_NOT:
        return ~a & la, la
    if op == OP_IS_NULL:
        return ~la, np.ones(n, dtype=bool)
    if op == OP_IS_NOT_NULL:
        return la.copy(), np.ones(n, dtype=bool)
    b = np.asarray(b, dtype=bool)
    lb = _valid(bv, n)
    a_t, a_f = a & la, ~a & la
    b_t, b_f = b & lb, ~b & lb
    if op == OP_AND:
        valid = (la & lb) | a_f | b_f
        return a_t & b_t, valid
    valid = (la & lb) | a_t | b_t
    return (a_t | b_t), valid


# ---- K3b selection: keep rows whose predicate is true (null -> dropped), input order ----------------
def select_mask(mask, mask_valid) -> np.ndarray:
    return np.asarray(mask, dtype=bool) & _valid(mask_valid, len(mask))


def filter_columns(mask, mask_valid, cols: Sequence[np.ndarray]) -> List[np.ndarray]:
    sel = select_mask(mask, mask_valid)
    return [np.asarray(c)[sel] for c in cols]


# ---- MaxAccumulator (K:538-561), literal ---------------------------------------------------------
class MaxAccumulator:
    """K:538-561: null skipped; first non-null seeds; replaced only on strictly greater."""

    def __init__(self):
        self.value = None

    def accumulate(self, value: Any) -> None:
        if value is not None:
            if self.value is None:
                self.value = value
            else:
                if isinstance(value, float):
                    is_max = value > self.value
                elif isinstance(value, int):  # build-added Long branch
                    is_max = value > self.value
                else:
                    raise TypeError(f"MAX is not implemented for data type {type(value).__name__}")
                if is_max:
                    self.value = value

    def finalValue(self) -> Any:  # noqa: N802
        return self.value


class MinAccumulator(MaxAccumulator):
    """Build-defined mirror of K:538-561 with `<`."""

    def accumulate(self, value: Any) -> None:
        if value is not None:
            if self.value is None:
                self.value = value
            elif value < self.value:
                self.value = value


class SumAccumulator:
    """Build-defined: nulls skipped; all-null -> null; int64 wraps; fp64 exact (fsum)."""

    def __init__(self, is_f64: bool):
        self.is_f64 = is_f64
        self.values: list = []

    def accumulate(self, value: Any) -> None:
        if value is not None:
            self.values.append(value)

    def finalValue(self) -> Any:  # noqa: N802
        if not self.values:
            return None
        if self.is_f64:
            return _fsum(self.values)
        s = sum(int(v) for v in self.values) & ((1 << 64) - 1)
        return s - (1 << 64) if s >= (1 << 63) else s


class CountAccumulator:
    def __init__(self, star: bool):
        self.star = star
        self.n = 0

    def accumulate(self, value: Any) -> None:
        if self.star or value is not None:
            self.n += 1

    def finalValue(self) -> Any:  # noqa: N802
        return self.n


class AvgAccumulator(SumAccumulator):
    def __init__(self):
        super().__init__(True)

    def finalValue(self) -> Any:  # noqa: N802
        if not self.values:
            return None
        return _fsum([float(v) for v in self.values]) / len(self.values)


def _fsum(values) -> float:
    vals = [float(v) for v in values]
    if any(math.isnan(v) for v in vals):
        return math.nan
    pos = any(v == math.inf for v in vals)
    neg = any(v == -math.inf for v in vals)
    if pos and neg:
        return math.nan
    if pos:
        return math.inf
    if neg:
        return -math.inf
    try:
        return math.fsum(vals)
    except OverflowError:
        return math.inf if sum(np.sign(vals)) > 0 else -math.inf


def make_accumulator(fn: int, is_f64: bool):
    if fn == AGG_MAX:
        return MaxAccumulator()
    if fn == AGG_MIN:
        return MinAccumulator()
    if fn == AGG_SUM:
        return SumAccumulator(is_f64)
    if fn == AGG_COUNT:
        return CountAccumulator(False)
    if fn == AGG_COUNT_STAR:
        return CountAccumulator(True)
    if fn == AGG_AVG:
        return AvgAccumulator()
    raise ValueError(fn)


# ---- HashAggregateExec.execute (K:615-651), literal ------------------------------------------------
def _key_of(v: Any) -> Any:
    """List.equals semantics of a key element: Double.equals (NaN == NaN, +0.0 != -0.0)."""
    if isinstance(v, float):
        if math.isnan(v):
            return ("f", "nan")
        return ("f", math.copysign(1.0, v), abs(v))
    return v


def hash_aggregate_rows(keys: Sequence[Sequence[Any]], inputs: Sequence[Sequence[Any]], fns: Sequence[int],
                        input_is_f64: Sequence[bool]) -> Dict[tuple, list]:
    """keys/inputs: per column, per row python values (None = null). Returns
    {key tuple (as python values) -> [final values]} — group order is unspecified (K:639)."""
    nrows = len(keys[0]) if keys else (len(inputs[0]) if inputs else 0)
    groups: Dict[tuple, Tuple[tuple, list]] = {}
    for row in range(nrows):  # K:620
        raw = tuple(k[row] for k in keys)  # K:621-626
        hk = tuple(_key_of(v) for v in raw)
        if hk not in groups:  # K:627 getOrPut
            groups[hk] = (raw, [make_accumulator(f, isf) for f, isf in zip(fns, input_is_f64)])
        for j, acc in enumerate(groups[hk][1]):  # K:628-631
            acc.accumulate(inputs[j][row] if fns[j] != AGG_COUNT_STAR else 1)
    return {tuple(canon(v) for v in raw): [a.finalValue() for a in accs] for raw, accs in groups.values()}


# ---- vectorised aggregates ---------------------------------------------------------------------------
def _minmax_f64(x: np.ndarray, is_max: bool) -> float:
    """MaxAccumulator semantics over the non-null values x (in row order)."""
    if math.isnan(x[0]):
        return math.nan  # a NaN seed is sticky
    y = x[~np.isnan(x)]
    m = y.max() if is_max else y.min()
    if m == 0.0:
        z = y[y == 0.0]
        return float(z[0])  # earliest of the +0.0 / -0.0 ties
    return float(m)


def global_aggregate(values: np.ndarray, valid=None, mask=None, mask_valid=None) -> dict:
    """All of COUNT(*), COUNT, SUM, MIN, MAX, AVG for one column (qe_agg_global)."""
    n = len(values)
    sel = np.ones(n, dtype=bool) if mask is None else select_mask(mask, mask_valid)
    nn = sel & _valid(valid, n)
    x = values[nn]
    out = {"rows": int(sel.sum()), "count": int(nn.sum())}
    if len(x) == 0:
        out.update(sum=None, min=None, max=None, avg=None)
        return out
    if values.dtype == np.float64:
        s = _fsum(x.tolist()) if len(x) < 2_000_000 else float(np.sum(x.astype(np.longdouble)))
        out.update(sum=s, min=_minmax_f64(x, False), max=_minmax_f64(x, True), avg=s / len(x))
    else:
        s = int(np.sum(x.astype(np.uint64), dtype=np.uint64).view(np.int64)) if len(x) else 0
        out.update(sum=s, min=int(x.min()), max=int(x.max()),
                   avg=float(np.sum(x.astype(np.longdouble)) / len(x)))
    return out


def group_aggregate(keys: Sequence[np.ndarray], key_valid: Sequence[Optional[np.ndarray]],
                    inputs: Sequence[Optional[np.ndarray]], input_valid: Sequence[Optional[np.ndarray]],
                    fns: Sequence[int], sel: Optional[np.ndarray] = None) -> Dict[tuple, list]:
    """Vectorised HashAggregateExec: {key tuple -> [final values]}; null key -> None in the tuple.
    fp64 keys follow Double.equals (one NaN group; +0.0 and -0.0 distinct). Key tuples hold
    canon() forms, because Python dicts would merge 0.0 and -0.0."""
    n = len(keys[0]) if keys else len(next(i for i in inputs if i is not None))
    if sel is None:
        sel = np.ones(n, dtype=bool)
    idx = np.nonzero(sel)[0]
    # encode each key column into a sortable int64 code per row (null -> its own code)
    codes = []
    decoders = []
    for k, kv in zip(keys, key_valid):
        kk = k[idx]
        kvv = _valid(kv, n)[idx]
        if kk.dtype == np.float64:
            bits = kk.view(np.int64).copy()
            bits[np.isnan(kk)] = 0x7FF8000000000000
        else:
            bits = kk.astype(np.int64)
        uniq, inv = np.unique(bits[kvv], return_inverse=True)
        code = np.full(len(kk), len(uniq), dtype=np.int64)  # null code = len(uniq)
        code[kvv] = inv
        codes.append(code)
        decoders.append((uniq, kk.dtype))
    if codes:
        combo = np.stack(codes, axis=1)
        ukeys, ginv = np.unique(combo, axis=0, return_inverse=True)
        ginv = ginv.reshape(-1)
    else:
        ukeys = np.zeros((1 if len(idx) else 0, 0), dtype=np.int64)
        ginv = np.zeros(len(idx), dtype=np.int64)
    ng = len(ukeys)
    order = np.argsort(ginv, kind="stable")
    bounds = np.searchsorted(ginv[order], np.arange(ng + 1))
    result: Dict[tuple, list] = {}
    cols = []
    for j, fn in enumerate(fns):
        if fn == AGG_COUNT_STAR:
            cols.append(np.diff(bounds).tolist())
            continue
        x = inputs[j][idx][order]
        xv = _valid(input_valid[j], n)[idx][order]
        vals = []
        for g in range(ng):
            seg = x[bounds[g]:bounds[g + 1]]
            segv = xv[bounds[g]:bounds[g + 1]]
            y = seg[segv]
            if fn == AGG_COUNT:
                vals.append(int(len(y)))
            elif len(y) == 0:
                vals.append(None)
            elif fn == AGG_SUM:
                if y.dtype == np.float64:
                    vals.append(float(np.sum(y.astype(np.longdouble))) if len(y) > 4096 else _fsum(y.tolist()))
                else:
                    vals.append(int(np.sum(y.astype(np.uint64), dtype=np.uint64).view(np.int64)))
            elif fn == AGG_AVG:
                vals.append(float(np.sum(y.astype(np.longdouble)) / len(y)))
            elif y.dtype == np.float64:
                vals.append(_minmax_f64(y, fn == AGG_MAX))
            else:
                vals.append(int(y.max() if fn == AGG_MAX else y.min()))
        cols.append(vals)
    for g in range(ng):
        kt = []
        for c, (uniq, dt) in enumerate(decoders):
            code = int(ukeys[g][c])
            if code == len(uniq):
                kt.append(None)
            elif dt == np.float64:
                kt.append(float(np.int64(uniq[code]).view(np.float64)))
            else:
                kt.append(int(uniq[code]))
        result[tuple(canon(x) for x in kt)] = [col[g] for col in cols]
    return result


def canon(v: Any) -> Any:
    """Comparable form of a result value (NaN equal to NaN, -0.0 distinct from +0.0)."""
    if isinstance(v, float):
        if math.isnan(v):
            return ("nan",)
        return (v, math.copysign(1.0, v))
    return v


def rows_equal(a: Any, b: Any, rel: float = 0.0) -> bool:
    if a is None or b is None:
        return a is None and b is None
    if isinstance(a, float) or isinstance(b, float):
        a, b = float(a), float(b)
        if math.isnan(a) or math.isnan(b):
            return math.isnan(a) and math.isnan(b)
        if rel == 0.0 or math.isinf(a) or math.isinf(b):
            return a == b and math.copysign(1, a) == math.copysign(1, b)
        return abs(a - b) <= rel * max(abs(a), abs(b), 1e-300)
    return a == b
