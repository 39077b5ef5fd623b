#!/usr/bin/env python3
"""Summarise tools/prof_c2.sh output (gpurun_out/profc2/): qe_selproj dispatches grouped by launch
shape (grid size, VGPRs, LDS) -> calls, average duration (kernel trace), FETCH_SIZE x2 (gfx950
half-count correction, MI355X_MICROARCH.md) and WRITE_SIZE per dispatch, and the SQ counters as
ratios (waves waiting, VALU / VMEM issue). Writes a markdown table to stdout.

    python3 tools/selproj_pmc.py [gpurun_out/profc2] > profiles/r03_selproj_pmc.md
"""
import collections
import csv
import pathlib
import sys

D = pathlib.Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/profc2")
K = "qe_selproj"


def shape(r, grid_key="Grid_Size", wg_key="Workgroup_Size"):
    return (int(r[grid_key]), int(r[wg_key]), int(r["VGPR_Count"]), int(r["LDS_Block_Size"]))


def counters(sub):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    p = D / sub / "run_counter_collection.csv"
    if not p.exists():
        return out
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    shp = {}
    for r in csv.DictReader(open(p)):
        if K not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        shp[r["Dispatch_Id"]] = shape(r)
    for d, cs in per.items():
        for c, v in cs.items():
            out[shp[d]][c].append(v)
    return out


def main():
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(D / "trace" / "run_kernel_trace.csv")):
        if K in r["Kernel_Name"]:
            s = (int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]), int(r["VGPR_Count"]), int(r["LDS_Block_Size"]))
            dur[s].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    f, w, sq = counters("fetch"), counters("write"), counters("sq")
    print("| grid (threads) | block | VGPR | LDS B | calls | avg ms | read GB (FETCH x2) | write GB | read+write TB/s |"
          " SQ_WAIT_ANY/WAVE_CYCLES | SQ_WAIT_INST_ANY/WAVE_CYCLES | VMEM insts/wave-kcycle |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for s in sorted(dur, key=lambda s: -sum(dur[s]) / len(dur[s])):
        ms = sum(dur[s]) / len(dur[s])
        rd = (sum(f[s]["FETCH_SIZE"]) / len(f[s]["FETCH_SIZE"]) * 1024 * 2) if f[s]["FETCH_SIZE"] else float("nan")
        wr = (sum(w[s]["WRITE_SIZE"]) / len(w[s]["WRITE_SIZE"]) * 1024) if w[s]["WRITE_SIZE"] else float("nan")
        q = sq[s]
        avg = {c: sum(v) / len(v) for c, v in q.items()}
        cyc = avg.get("SQ_WAVE_CYCLES", float("nan"))
        print(f"| {s[0]} | {s[1]} | {s[2]} | {s[3]} | {len(dur[s])} | {ms:.4f} | {rd / 1e9:.3f} | {wr / 1e9:.3f} | "
              f"{(rd + wr) / (ms * 1e-3) / 1e12:.2f} | {avg.get('SQ_WAIT_ANY', float('nan')) / cyc:.3f} | "
              f"{avg.get('SQ_WAIT_INST_ANY', float('nan')) / cyc:.3f} | "
              f"{avg.get('SQ_INSTS_VMEM', float('nan')) / cyc * 1000:.2f} |")


if __name__ == "__main__":
    main()
