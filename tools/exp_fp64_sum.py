#!/usr/bin/env python3
"""C5 (and C4) fused GROUP BY kernel time with fp64 SUM / AVG in each accumulation mode, interleaved
on one box: the default (exact) state vs QE_HASHAGG_FAST_FP64 (fp64 atomics). One JSON line per (config, mode, round)
plus a summary line per (config, mode) with the median kernel time.

  python tools/exp_fp64_sum.py [C5] [C4] [--rounds R] [--mode exact|fast]
"""
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import torch  # noqa: E402

from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.columnar import Context  # noqa: E402
from kquery.datasource import C4_COLUMNS, C5_COLUMNS, generate_column  # noqa: E402
from kquery.workloads import C4_AGGS, C5_AGGS, C5_KEY_TYPES, c4_spec, c5_spec  # noqa: E402
from kquery import native as N  # noqa: E402


def main():
    argv = sys.argv[1:]
    rounds, modes = 3, ("exact", "fast")
    if "--rounds" in argv:
        i = argv.index("--rounds")
        rounds = int(argv[i + 1])
        del argv[i:i + 2]
    if "--mode" in argv:
        i = argv.index("--mode")
        modes = (argv[i + 1],)
        del argv[i:i + 2]
    args = argv
    which = args or ["C5"]
    ctx = Context.get(0)
    for cfg in which:
        specs, rows, aggs, keys, spec, bpr, ng = (
            (C5_COLUMNS, 1_250_000_000, C5_AGGS, C5_KEY_TYPES, c5_spec(), 38, 16) if cfg == "C5" else
            (C4_COLUMNS, 1_000_000_000, C4_AGGS, [N.TYPE_INT64], c4_spec(), 24, 1024))
        cols = [generate_column(s, rows, 0, 42, ctx) for s in specs]
        states = {m: HashAggregateState(ctx, keys, aggs, ng, fast_fp64=(m == "fast")) for m in modes}
        times = {m: [] for m in states}
        results = {}
        for r in range(rounds):
            for m, st in states.items():
                ks = []
                for it in range(13):
                    st.reset()
                    st.update_fused(cols, spec)
                    ks.append(st.last_kernel_time()[0])
                    if it == 12:
                        k, v = st.finalize()
                        results[m] = (k, v)
                med = statistics.median(ks[3:])
                times[m].append(med)
                print(json.dumps({"config": cfg, "mode": m, "round": r, "kernel_ms": med,
                                  "kind": st.last_kernel_kind()[0], "sig": st.last_kernel_signature()}), flush=True)
        for m in states:
            med = statistics.median(times[m])
            print(json.dumps({"config": cfg, "mode": m, "summary": True, "kernel_ms": med,
                              "gbs": rows * bpr / (med * 1e-3) / 1e9}), flush=True)
        torch.cuda.synchronize()
        del cols, states


if __name__ == "__main__":
    main()
