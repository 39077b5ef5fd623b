#!/usr/bin/env python3
"""Per-launch kernel durations from a rocprofv3 kernel trace CSV, grouped in launch order.

  python tools/kernel_table.py gpurun_out/pgrp/trace/run_kernel_trace.csv [name-prefix ...]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    prefixes = sys.argv[2:] or ["qe"]
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if any(n.startswith(p) for p in prefixes):
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            print(f"{n[:40]:40s} {ms:8.3f} ms  grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):7d} x "
                  f"{r['Workgroup_Size_X']:>4s}  lds {r['LDS_Block_Size']:>6s}  vgpr {r['VGPR_Count']}")


if __name__ == "__main__":
    main()
