#!/usr/bin/env python3
"""Per-mode mean counters and kernel durations of a kernel from tools/prof_fp64_sum.sh output.

  python tools/pmc_modes.py gpurun_out/fp64_pmc [kernel-prefix]
"""
import collections
import csv
import pathlib
import sys


def main():
    root = pathlib.Path(sys.argv[1])
    pre = sys.argv[2] if len(sys.argv) > 2 else "qe_fused"
    modes = sorted({p.name.rsplit("_", 1)[0] for p in root.iterdir() if p.is_dir()})
    table = collections.defaultdict(dict)
    for m in modes:
        tr = root / f"{m}_trace" / "run_kernel_trace.csv"
        if tr.exists():
            d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in csv.DictReader(open(tr))
                 if r["Kernel_Name"].startswith(pre)]
            if d:
                table["duration_ms"][m] = sorted(d)[len(d) // 2]
        for sub in ("sq", "lds"):
            f = root / f"{m}_{sub}" / "run_counter_collection.csv"
            if not f.exists():
                continue
            acc = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                if r["Kernel_Name"].startswith(pre):
                    acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            for c, v in acc.items():
                table[c][m] = sum(v.values()) / len(v)
    print(f"{'counter':24s}" + "".join(f"{m:>16s}" for m in modes))
    for c in sorted(table):
        print(f"{c:24s}" + "".join(f"{table[c].get(m, float('nan')):16.4g}" for m in modes))


if __name__ == "__main__":
    main()
