"""CPU tests: the oracle against the reference's fixture (employee.csv known answers), the
hand-derived golden vectors, and its own literal (row-at-a-time) forms. No GPU."""
import ctypes as C
import json
import math
import pathlib

import numpy as np
import pytest

from oracle import csv_ref, gen
from oracle import semantics as S

GOLD = pathlib.Path(__file__).parent / "golden"


def _f(x):
    if x is None:
        return None
    if isinstance(x, str):
        return float(x)
    return x


# ---- reference fixture: employee.csv (SURVEY §8c known answers) ----------------------------------
def test_employee_csv_schema_and_rows():
    kat = json.loads((GOLD / "employee_kat.json").read_text())
    batches = csv_ref.read_csv(str(GOLD / "employee.csv"))
    assert len(batches) == 1
    assert list(batches[0].keys()) == kat["columns"]
    assert len(batches[0]["id"]) == kat["rows"]
    assert batches[0]["last_name"][2] == "Pärsson"  # UTF-8 0xC3 0xA4 kept


def test_employee_filter_ca_is_empty():
    kat = json.loads((GOLD / "employee_kat.json").read_text())
    assert csv_ref.employee_filter_project(str(GOLD / "employee.csv"), "CA") == kat[
        "filter_state_CA_project_id_first_name"]


def test_employee_filter_uppsala():
    kat = json.loads((GOLD / "employee_kat.json").read_text())
    got = csv_ref.employee_filter_project(str(GOLD / "employee.csv"), "Uppsala", ("id",))
    assert [r[0] for r in got] == kat["filter_state_Uppsala_ids"]


def test_employee_group_max():
    kat = json.loads((GOLD / "employee_kat.json").read_text())
    assert csv_ref.employee_group_max(str(GOLD / "employee.csv")) == kat["group_state_max_salary"]


def test_csv_batching_1000_rows(tmp_path):
    p = tmp_path / "t.csv"
    p.write_text("x,y\n" + "".join(f" {i} ,{i % 7}\n" for i in range(2500)) + "\n\n")
    b = csv_ref.read_csv(str(p))
    assert [len(x["x"]) for x in b] == [1000, 1000, 500]
    assert b[0]["x"][0] == "0"  # trimmed


# ---- generator pinned by the golden vectors ---------------------------------------------------------
def test_generator_golden():
    g = json.loads((GOLD / "generator.json").read_text())
    for name, v in g.items():
        if "dist" not in v:
            continue
        vals, _ = gen.generate(v["dist"], v["param"], v["seed"], v["col"], v["row0"], len(v["values"]))
        if isinstance(v["values"][0], str):
            assert [float.fromhex(x) for x in v["values"]] == vals.tolist(), name
        else:
            assert v["values"] == vals.tolist(), name
    _, valid = gen.generate(gen.GEN_MOD, 1024, 42, 0, 0, 64, null_permille=100)
    assert valid.tolist() == g["nulls_permille100_c0"]["valid"]
    for x, y in g["splitmix64"].items():
        assert int(gen.splitmix64([int(x)])[0]) == y


def test_unit53_is_exact():
    v, _ = gen.generate(gen.GEN_UNIT53, 0, 42, 3, 0, 10000)
    assert v.min() >= -1024 and v.max() < 1024
    # every value is a multiple of 2^-42: exactly representable, fsum is the true sum
    assert np.all(np.ldexp(v + 1024.0, 42) == np.floor(np.ldexp(v + 1024.0, 42)))


# ---- build-defined semantics pinned by hand-derived vectors -----------------------------------------
def test_int64_arith_golden():
    g = json.loads((GOLD / "semantics.json").read_text())
    for name, op in (("int64_add_wrap", S.OP_ADD), ("int64_mul_wrap", S.OP_MUL), ("int64_div", S.OP_DIV)):
        a = np.array(g[name]["a"], dtype=np.int64)
        b = np.array(g[name]["b"], dtype=np.int64)
        r, v = S.arith(op, a, None, b, None)
        got = [int(x) if ok else None for x, ok in zip(r, v)]
        assert got == g[name]["out"], name


def _acc_run(acc, xs):
    for x in xs:
        acc.accumulate(_f(x))
    return acc.finalValue()


@pytest.mark.parametrize("case", ["max_order", "max_nan_later", "max_zero_tie_neg_first",
                                  "max_zero_tie_pos_first", "min_zero_tie", "max_all_null"])
def test_max_accumulator_golden(case):
    g = json.loads((GOLD / "semantics.json").read_text())[case]
    for fn, acc in (("max", S.MaxAccumulator()), ("min", S.MinAccumulator())):
        got = _acc_run(acc, g["in"])
        want = _f(g[fn])
        assert S.rows_equal(got, want), (case, fn, got, want)
        # the vectorised form agrees with the literal accumulator
        xs = [_f(x) for x in g["in"]]
        arr = np.array([x if x is not None else 0.0 for x in xs], dtype=np.float64)
        valid = np.array([x is not None for x in xs])
        res = S.global_aggregate(arr, valid)
        assert S.rows_equal(res[fn], want), (case, fn, res[fn], want)


def test_three_valued_logic_golden():
    g = json.loads((GOLD / "semantics.json").read_text())
    for name, op in (("and3", S.OP_AND), ("or3", S.OP_OR)):
        a, b = g[name]["a"], g[name]["b"]
        av = np.array([x is not None for x in a])
        bv = np.array([x is not None for x in b])
        r, v = S.bool3(op, np.array([bool(x) for x in a]), av, np.array([bool(x) for x in b]), bv)
        assert [bool(x) if ok else None for x, ok in zip(r, v)] == g[name]["out"], name


# ---- vectorised group-by == literal HashAggregateExec loop (K:615-651) -------------------------------
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_group_aggregate_matches_literal_loop(seed):
    rng = np.random.default_rng(seed)
    n = 3000
    k = rng.integers(-3, 4, n).astype(np.int64)
    kv = rng.random(n) > 0.1
    x = rng.normal(size=n)
    x[rng.random(n) < 0.05] = np.nan
    x[rng.random(n) < 0.05] = 0.0
    x[rng.random(n) < 0.05] = -0.0
    xv = rng.random(n) > 0.2
    y = rng.integers(-2**62, 2**62, n).astype(np.int64)
    fns = [S.AGG_MAX, S.AGG_MIN, S.AGG_SUM, S.AGG_COUNT, S.AGG_COUNT_STAR, S.AGG_MAX, S.AGG_SUM, S.AGG_AVG]
    ins = [x, x, x, x, None, y, y, y]
    insv = [xv, xv, xv, xv, None, None, None, None]
    vec = S.group_aggregate([k], [kv], ins, insv, fns)
    keys = [[int(a) if ok else None for a, ok in zip(k, kv)]]
    rows_in = []
    for arr, v in zip(ins, insv):
        if arr is None:
            rows_in.append([1] * n)
        elif arr.dtype == np.float64:
            rows_in.append([float(a) if (v is None or ok) else None for a, ok in zip(arr, v if v is not None else [True] * n)])
        else:
            rows_in.append([int(a) for a in arr])
    lit = S.hash_aggregate_rows(keys, rows_in, fns, [True, True, True, True, False, False, False, False])
    assert set(vec) == set(lit)
    for key in lit:
        for j, (a, b) in enumerate(zip(vec[key], lit[key])):
            rel = 1e-12 if fns[j] in (S.AGG_SUM, S.AGG_AVG) and isinstance(b, float) else 0.0
            assert S.rows_equal(a, b, rel), (key, j, a, b)


def test_global_aggregate_int_wrap_and_empty():
    x = np.array([2**63 - 1, 1, 5], dtype=np.int64)
    r = S.global_aggregate(x)
    assert r["sum"] == -2**63 + 5 and r["min"] == 1 and r["max"] == 2**63 - 1 and r["count"] == 3
    e = S.global_aggregate(np.zeros(0, dtype=np.float64))
    assert e["rows"] == 0 and e["sum"] is None and e["max"] is None


def test_fsum_special_values():
    assert math.isnan(S._fsum([1.0, math.nan]))
    assert S._fsum([math.inf, 1.0]) == math.inf
    assert math.isnan(S._fsum([math.inf, -math.inf]))


# ---- C restatement (CPU baseline) == numpy oracle -------------------------------------------------------
class _G(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("key", "sum", "count", "min", "max")]


def _oracle_lib():
    p = pathlib.Path(__file__).resolve().parents[1] / "oracle" / "build" / "libqe_oracle.so"
    if not p.exists():
        import subprocess

        subprocess.run(["make", "-C", str(p.parents[1])], check=True, capture_output=True)
    lib = C.CDLL(str(p))
    lib.qe_cpu_c4.restype = C.c_double
    lib.qe_cpu_c4.argtypes = [C.c_int64, C.c_int64, C.c_uint64, C.c_int, C.c_int64, C.c_int64,
                              C.POINTER(_G), C.c_int64, C.POINTER(C.c_int64)]
    lib.qe_cpu_c4_fast.restype = C.c_double
    lib.qe_cpu_c4_fast.argtypes = lib.qe_cpu_c4.argtypes
    return lib


@pytest.mark.parametrize("fast", [False, True])
@pytest.mark.parametrize("threads,row0", [(1, 0), (3, 12345)])
def test_cpu_baseline_matches_oracle(threads, row0, fast):
    """Both CPU legs of bench.py: the reference-faithful port and the tuned implementation."""
    lib = _oracle_lib()
    n = 100_000
    out = (_G * 2048)()
    ng = C.c_int64()
    secs = (lib.qe_cpu_c4_fast if fast else lib.qe_cpu_c4)(row0, n, 42, threads, 1 << 19, 1024, out, 2048,
                                                           C.byref(ng))
    assert secs >= 0
    k, _ = gen.generate(gen.GEN_MOD, 1024, 42, 0, row0, n)
    a, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 1, row0, n)
    b, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 2, row0, n)
    ref = S.group_aggregate([k], [None], [S.arith(S.OP_ADD, a, None, b, None)[0], None, a, b], [None] * 4,
                            [S.AGG_SUM, S.AGG_COUNT_STAR, S.AGG_MIN, S.AGG_MAX], a > (1 << 19))
    got = {(o.key,): [o.sum, o.count, o.min, o.max] for o in out[: ng.value]}
    assert got == ref


def test_double_key_equality_semantics():
    """Double.equals (K:621-627 keys are boxed Doubles): +0.0 and -0.0 are different groups,
    every NaN is one group — hand-derived expectation."""
    k = np.array([0.0, -0.0, 0.0, np.nan, float("nan"), -0.0, 1.0])
    x = np.arange(7, dtype=np.int64)
    got = S.group_aggregate([k], [None], [x], [None], [S.AGG_COUNT_STAR])
    want = {(S.canon(0.0),): [2], (S.canon(-0.0),): [2], (S.canon(math.nan),): [2], (S.canon(1.0),): [1]}
    assert got == want
    lit = S.hash_aggregate_rows([[float(v) for v in k]], [[1] * 7], [S.AGG_COUNT_STAR], [False])
    assert lit == want
