"""Regenerates the committed golden fixtures in tests/golden/ (run from the repo root).

* employee_kat.json — known answers on the reference's only fixture, kquerydiy/employee.csv
  (copied here as data: tests/golden/employee.csv), derived by hand from the file and the
  reference semantics: filter(state='CA') -> 0 rows; state='Uppsala' -> ids 1, 2;
  GROUP BY state MAX(CAST(salary AS double)) -> {Uppsala: 1337.0, Sthlm: 0.0}.
* generator.json — splitmix64 generator vectors (first rows of every distribution) that pin
  oracle/gen.py, the C baseline and the HIP generator to the same bits.
* semantics.json — small hand-checkable vectors for the build-defined semantics (int64 wrap,
  truncating division, x/0 -> null, NaN/+-0.0 MAX order rules, three-valued logic).
"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle import gen  # noqa: E402

OUT = ROOT / "tests" / "golden"


def main():
    kat = {
        "source": "folkol/query-engines kquerydiy/employee.csv (4 lines incl. header)",
        "filter_state_CA_project_id_first_name": [],
        "filter_state_Uppsala_ids": ["1", "2"],
        "group_state_max_salary": {"Uppsala": 1337.0, "Sthlm": 0.0},
        "columns": ["id", "first_name", "last_name", "state", "job_title", "salary"],
        "rows": 3,
    }
    (OUT / "employee_kat.json").write_text(json.dumps(kat, indent=1) + "\n")

    vec = {}
    for name, dist, param, col, dt in [
        ("mod1024_c0", gen.GEN_MOD, 1024, 0, "i"),
        ("mod2p20_c1", gen.GEN_MOD, 1 << 20, 1, "i"),
        ("raw_c2", gen.GEN_RAW, 0, 2, "i"),
        ("unit53_c3", gen.GEN_UNIT53, 0, 3, "f"),
        ("modf64_c5", gen.GEN_MOD_F64, 10000, 5, "f"),
    ]:
        v, _ = gen.generate(dist, param, 42, col, 1000, 16)
        vec[name] = {"dist": dist, "param": param, "col": col, "seed": 42, "row0": 1000,
                     "values": [float(x).hex() if dt == "f" else int(x) for x in v]}
    _, valid = gen.generate(gen.GEN_MOD, 1024, 42, 0, 0, 64, null_permille=100)
    vec["nulls_permille100_c0"] = {"valid": [bool(x) for x in valid]}
    vec["splitmix64"] = {str(x): int(gen.splitmix64([x])[0]) for x in (0, 1, 42, 2**63)}
    (OUT / "generator.json").write_text(json.dumps(vec, indent=1) + "\n")

    sem = {
        "int64_add_wrap": {"a": [2**63 - 1, -2**63], "b": [1, -1], "out": [-2**63, 2**63 - 1]},
        "int64_mul_wrap": {"a": [2**62, 3037000500], "b": [4, 3037000500], "out": [0, -9223372036709301616]},
        "int64_div": {"a": [7, -7, 7, -2**63, 5], "b": [2, 2, 0, -1, -3],
                      "out": [3, -3, None, -2**63, -1]},
        "max_order": {"in": ["nan", 1.0, 2.0], "max": "nan", "min": "nan"},
        "max_nan_later": {"in": [1.0, "nan", 2.0], "max": 2.0, "min": 1.0},
        "max_zero_tie_neg_first": {"in": [-1.0, -0.0, 0.0], "max": "-0.0", "min": -1.0},
        "max_zero_tie_pos_first": {"in": [0.0, -0.0], "max": "0.0", "min": "0.0"},
        "min_zero_tie": {"in": [-0.0, 0.0, 1.0], "max": 1.0, "min": "-0.0"},
        "max_all_null": {"in": [None, None], "max": None, "min": None},
        "and3": {"a": [True, True, True, False, False, False, None, None, None],
                 "b": [True, False, None, True, False, None, True, False, None],
                 "out": [True, False, None, False, False, False, None, False, None]},
        "or3": {"a": [True, True, True, False, False, False, None, None, None],
                "b": [True, False, None, True, False, None, True, False, None],
                "out": [True, True, True, True, False, None, True, None, None]},
    }
    (OUT / "semantics.json").write_text(json.dumps(sem, indent=1) + "\n")


if __name__ == "__main__":
    main()
