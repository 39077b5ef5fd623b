#!/usr/bin/env python3
"""Experiment: string-dictionary encode time by key cardinality (hot-key contention)."""
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from kquery import native as N  # noqa: E402
from kquery.columnar import Context, DeviceColumn  # noqa: E402
from kquery.strdict import StringDictionary  # noqa: E402


def main():
    ctx = Context.get(0)
    n = 4_000_000
    rng = np.random.default_rng(1)
    out = {}
    for card in (3, 100, 10_000, 1_000_000):
        words = [f"k{i}".encode() for i in range(card)]
        pick = rng.integers(0, card, n)
        lens = np.array([len(w) for w in words], dtype=np.int64)[pick]
        offs = np.zeros(n + 1, dtype=np.int32)
        offs[1:] = np.cumsum(lens)
        data = b"".join(words[i] for i in pick.tolist())
        col = DeviceColumn(N.TYPE_UTF8, n, torch.frombuffer(bytearray(data), dtype=torch.uint8).to(ctx.torch_device),
                           None, torch.from_numpy(offs).to(ctx.torch_device), ctx)
        ts = []
        for it in range(6):
            d = StringDictionary(ctx, 64)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            d.encode(col)
            e.record()
            e.synchronize()
            if it:
                ts.append(s.elapsed_time(e))
            d.close()
        out[card] = round(statistics.median(ts), 4)
        print(card, out[card], file=sys.stderr, flush=True)
    print(json.dumps({"rows": n, "ms_by_cardinality": out}))


if __name__ == "__main__":
    main()
