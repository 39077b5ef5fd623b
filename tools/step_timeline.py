#!/usr/bin/env python3
"""Kernel timeline between the last two fused-kernel launches of a rocprofv3 --kernel-trace run
(µs after the earlier one ends): where a bench step's time goes outside the fused kernel.

    python tools/step_timeline.py gpurun_out/<dir>
"""
import csv
import pathlib
import sys

f = next(pathlib.Path(sys.argv[1]).rglob("run_kernel_trace.csv"))
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "qe_fused"]
t0 = int(rows[idx[-2]]["End_Timestamp"])
for r in rows[idx[-2]:idx[-1] + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:9.2f}  {r['Kernel_Name'][:90]}")
