#!/usr/bin/env python3
"""Summarise tools/exp_variants.sh output: per variant label, kernel ms and step ms of each run."""
import json
import pathlib
import statistics
import sys

d = pathlib.Path(sys.argv[1])
labels = [l.split(":", 1)[1].strip() or "(defaults)" for l in (d / "variants.txt").read_text().splitlines()]
rows = {}
for i, lab in enumerate(labels, 1):
    try:
        j = json.loads((d / f"v{i}.json").read_text().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f"v{i} {lab}: {e}")
        continue
    rows.setdefault(lab, []).append((j["roofline"]["avg_kernel_ms"], j["ms_per_step"]))
for lab, v in rows.items():
    ks = [round(a, 4) for a, _ in v]
    ss = [round(b, 4) for _, b in v]
    print(f"{lab:40s} kernel med {statistics.median(ks):.4f} {ks}  step med {statistics.median(ss):.4f} {ss}")
