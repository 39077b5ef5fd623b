#!/usr/bin/env python3
"""Mean per-dispatch PMC counter values per kernel from rocprofv3 --pmc CSV output directories.

  python tools/pmc_table.py gpurun_out/pgrp_pmc [name-prefix ...]
"""
import csv
import pathlib
import sys
from collections import defaultdict


def main():
    root = pathlib.Path(sys.argv[1])
    prefixes = sys.argv[2:] or ["qe"]
    acc = defaultdict(lambda: defaultdict(dict))
    for f in sorted(root.glob("*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if not any(n.startswith(p) for p in prefixes):
                continue
            d = acc[n[:40]][r["Counter_Name"]]
            d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            vals = list(v.values())
            print(f"   {c:24s} {sum(vals) / len(vals):14.4g}  (n={len(vals)})")


if __name__ == "__main__":
    main()
