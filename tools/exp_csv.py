#!/usr/bin/env python3
"""Experiment: GPU CSV scan wall time vs kernel time on a tripdata-shaped file (run under
rocprofv3 --kernel-trace --stats to split the two)."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd"), str(ROOT / "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench_tripdata import make_csv  # noqa: E402
from kquery.columnar import Context  # noqa: E402
from kquery.csv_source import CsvDataSource  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
path = pathlib.Path("/tmp") / f"yc-synthetic-{rows}.csv"
if not path.exists():
    make_csv(path, rows)
ctx = Context.get(0)
ds = CsvDataSource(str(path), True, 0, ctx=ctx)
names = [f.name for f in ds.schema().fields]
idx = [names.index("VendorID"), names.index("fare_amount")]
raw = np.fromfile(path, dtype=np.uint8)
dev = torch.from_numpy(raw).to(ctx.torch_device)
for _ in range(3):
    ds._parse(ctx, dev, raw.size, idx)
torch.cuda.synchronize()
ts = []
for _ in range(10):
    t0 = time.perf_counter()
    ds._parse(ctx, dev, raw.size, idx)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print("parse wall ms (min/median):", min(ts) * 1e3, sorted(ts)[5] * 1e3, "bytes", raw.size)
