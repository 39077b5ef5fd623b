#!/usr/bin/env python3
"""Per-kernel table of the tripdata query (K:1336): average duration (kernel trace), HBM bytes per
launch from FETCH_SIZE (x2: the gfx950 correction for wide streaming reads, MI355X_MICROARCH.md)
and WRITE_SIZE, the rate those bytes move at, and the kernel's algorithmic bytes where stated.

  python tools/trip_traffic.py <trace_dir> <traffic_dir> [rows]  > profiles/r05_tripdata_kernels.md
"""
import collections
import csv
import pathlib
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def short(name):
    n = name.replace("qe::(anonymous namespace)::", "").replace("qe::", "")
    n = n[5:] if n.startswith("void ") else n
    return n.split("(")[0]


def main():
    trace, traffic = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2])
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 4_000_000
    stats = {r["Name"]: r for r in csv.DictReader(open(next(trace.glob("**/*kernel_stats.csv"))))}
    fetch = per_kernel(next((traffic / "fetch").glob("**/*counter_collection.csv")), "FETCH_SIZE")
    write = per_kernel(next((traffic / "write").glob("**/*counter_collection.csv")), "WRITE_SIZE")
    csv_bytes = 385_896_536 if rows == 4_000_000 else None
    # algorithmic bytes per launch (reads + writes) for the kernels whose traffic is fixed by the data
    alg = {
        "k_csv_count2": csv_bytes,
        "k_csv_terms<true>": csv_bytes and csv_bytes + 8 * rows,
        "k_dict_encode<true>": 4 * rows + 1 * rows + 8 * rows,  # offsets, 1-byte keys, int64 codes
        "qe_fused": 16 * rows,  # int64 code + fp64 fare
    }
    print("| kernel | calls | avg us | FETCH x2 (MB) | WRITE (MB) | moved (GB/s) | algorithmic (MB) |")
    print("|---|---|---|---|---|---|---|")
    for name, r in sorted(stats.items(), key=lambda kv: -float(kv[1]["TotalDurationNs"])):
        us = float(r["AverageNs"]) / 1e3
        f = fetch.get(name)
        w = write.get(name)
        if f is None and w is None:
            continue
        fb = 2 * 1024 * f if f is not None else 0.0  # FETCH_SIZE / WRITE_SIZE are in KB
        wb = 1024 * w if w is not None else 0.0
        rate = (fb + wb) / (us * 1e3) if us else 0.0
        sn = short(name)
        a = alg.get(sn)
        at = f"{a / 1e6:.1f}" if a else ""
        print(f"| {sn} | {r['Calls']} | {us:.1f} | {fb / 1e6:.1f} | {wb / 1e6:.1f} | {rate:.0f} | {at} |")


if __name__ == "__main__":
    main()
