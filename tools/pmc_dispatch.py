#!/usr/bin/env python3
"""Per-dispatch counter sums of the named kernels from rocprofv3 --pmc CSV directories.
  python tools/pmc_dispatch.py KERNEL[,KERNEL] DIR [DIR ...]"""
import collections
import csv
import glob
import sys

names = set(sys.argv[1].split(","))
for d in sys.argv[2:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg, order = collections.defaultdict(lambda: collections.defaultdict(float)), []
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] not in names:
                continue
            k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            if k not in agg:
                order.append(k)
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        print("==", f)
        for k in order:
            print(k, {c: "%.3g" % v for c, v in sorted(agg[k].items())})
