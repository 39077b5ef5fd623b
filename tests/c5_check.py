"""Shared by the C5 multi-rank tests: the exact C5 oracle over a row range (oracle/cpu_baseline.c
qe_cpu_c5_exact — test infrastructure) and the per-group comparison of an owner's finalized groups
with it. Exact mode: COUNT(*) / SUM(quantity) exact, fp64 SUMs and AVG bit for bit; fast mode
(QE_HASHAGG_FAST_FP64): fp64 within 1e-9 relative."""
import ctypes as C
import os
import pathlib
from fractions import Fraction

ROOT = pathlib.Path(__file__).resolve().parents[1]
REL = 1e-9


def c5_oracle(row0, n):
    """{(returnflag, linestatus): (count, sum_qty, [sum_price, sum_dp, sum_dpt] as floats)}."""
    lib = C.CDLL(str(ROOT / "oracle" / "build" / "libqe_oracle.so"))
    lib.qe_cpu_c5_exact.restype = C.c_double
    lib.qe_cpu_c5_exact.argtypes = [C.c_int64, C.c_int64, C.c_uint64, C.c_int, C.POINTER(C.c_int64)]
    out = (C.c_int64 * 48)()
    assert lib.qe_cpu_c5_exact(row0, n, 42, min(32, len(os.sched_getaffinity(0))), out) >= 0
    res = {}
    for g in range(6):
        o = list(out[g * 8:(g + 1) * 8])
        if o[0] == 0:
            continue
        sums = [float(Fraction((o[2 + 2 * k] << 64) + (o[3 + 2 * k] & ((1 << 64) - 1)), 1 << 80)) for k in range(3)]
        res[(g // 2, g % 2)] = (o[0], o[1], sums)
    return res


def check_groups(rows, want, exact):
    """rows: [(flag, status, sum_qty, sum_price, sum_dp, sum_dpt, avg_price, count)] -> (ok, why)."""
    got = {}
    for r in rows:
        key = (int(r[0]), int(r[1]))
        if key in got:
            return False, f"group {key} owned twice"
        got[key] = r[2:]
    if set(got) != set(want):
        return False, f"groups {sorted(got)} vs {sorted(want)}"
    for key, (cnt, sq, sums) in want.items():
        g = got[key]
        if int(g[5]) != cnt or int(g[0]) != sq:
            return False, f"{key}: count/sum_qty {int(g[5])}/{int(g[0])} vs {cnt}/{sq}"
        vals = [float(g[1]), float(g[2]), float(g[3]), float(g[4])]
        refs = sums + [sums[0] / cnt]
        for v, w in zip(vals, refs):
            if exact and v != w:
                return False, f"{key}: {vals} vs {refs} (exact)"
            if not exact and abs(v - w) > REL * abs(w):
                return False, f"{key}: {vals} vs {refs} (1e-9)"
    return True, ""
