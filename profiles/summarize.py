"""Summarise a rocprofv3 run of bench.py (profiles/run_profile.sh output) into profiles/.

Writes profiles/<round>_kernel_stats.csv (copy of the kernel-trace --stats summary),
profiles/<round>_summary.md and profiles/traffic.json (tagged with the kernel signature the profiled
bench run printed — qe_hashagg_last_kernel_signature: the specialised kernel's compile key and launch
shape — and the git head; bench.py ignores traffic.json for any other kernel; HBM bytes per
fused-kernel launch from the
FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM: on gfx950 it counts
half the bytes of wide coalesced streaming reads; both counters are in KiB)."""
import csv
import json
import pathlib
import shutil
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
SRC = ROOT / "gpurun_out" / "prof"
OUT = ROOT / "profiles"
RND = sys.argv[1] if len(sys.argv) > 1 else "r01"
FUSED = ("qe_fused", "k_hashagg")


def per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or not any(f in r["Kernel_Name"] for f in FUSED):
            continue
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    stats = list(csv.DictReader(open(SRC / "trace" / "run_kernel_stats.csv")))
    shutil.copy(SRC / "trace" / "run_kernel_stats.csv", OUT / f"{RND}_kernel_stats.csv")
    fused = [r for r in stats if any(f in r["Name"] for f in FUSED)]
    lines = [f"# rocprofv3 summary ({RND})", "", "Command: `bash profiles/run_profile.sh` (bench.py, 1B rows, C4)", "",
             "| kernel | calls | avg ms | % |", "|---|---|---|---|"]
    for r in stats[:12]:
        lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} | {float(r['Percentage']):.1f} |")
    out = {}
    fetch = per_dispatch(SRC / "fetch" / "run_counter_collection.csv", "FETCH_SIZE")
    write = per_dispatch(SRC / "write" / "run_counter_collection.csv", "WRITE_SIZE")
    if fetch:
        f = sum(fetch) / len(fetch) * 1024 * 2  # KiB -> B, x2 gfx950 correction
        w = (sum(write) / len(write) * 1024) if write else 0.0
        import subprocess

        sig = None  # the profiled bench run's line (trace pass) names the kernel it launched
        for ln in open(SRC / "trace.log", errors="replace"):
            if ln.startswith("{") and '"kernel_signature"' in ln:
                sig = json.loads(ln)["roofline"]["kernel_signature"]
        try:
            head = subprocess.run(["git", "-C", str(ROOT), "rev-parse", "--short", "HEAD"], capture_output=True,
                                  text=True).stdout.strip()
        except OSError:
            head = ""
        out = {"rows": 1_000_000_000, "kernel_signature": sig, "git_head": head,
               "hbm_bytes_per_launch": f + w, "fetch_bytes_corrected": f, "write_bytes": w,
               "algorithmic_bytes": 24_000_000_000, "kernel": fused[0]["Name"] if fused else "",
               "avg_kernel_ms": float(fused[0]["AverageNs"]) / 1e6 if fused else None,
               "note": "FETCH_SIZE x1024 x2 (gfx950 half-count correction) + WRITE_SIZE x1024, per launch"}
        (OUT / "traffic.json").write_text(json.dumps(out, indent=1) + "\n")
        lines += ["", f"Fused kernel HBM traffic per launch: read {f / 1e9:.2f} GB (FETCH_SIZE x2), "
                      f"write {w / 1e6:.2f} MB; algorithmic 24.00 GB."]
    for name in ("sq", "lds"):
        p = SRC / name / "run_counter_collection.csv"
        if p.exists():
            cs = {}
            for r in csv.DictReader(open(p)):
                if any(f in r["Kernel_Name"] for f in FUSED):
                    cs.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                    cs[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            lines.append("")
            lines.append(f"{name} counters (fused kernel, mean per dispatch): " + ", ".join(
                f"{c}={sum(v.values()) / len(v):.4g}" for c, v in sorted(cs.items())))
    (OUT / f"{RND}_summary.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
