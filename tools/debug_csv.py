#!/usr/bin/env python3
"""Debug helper: first row where the GPU CSV scan differs from the oracle (seeded random file)."""
import pathlib
import random
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd"), str(ROOT / "tests")]

from oracle import csv_ref as R  # noqa: E402
from test_csv import random_csv  # noqa: E402

from kquery.columnar import Context  # noqa: E402
from kquery.csv_source import CsvDataSource  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
rng = random.Random(seed)
delim = rng.choice([",", ";", "\t", "|"])
data = random_csv(rng, rng.choice([0, 1, 5, 300, 5000]), rng.randint(1, 7), delim, rng.choice(["\n", "\r\n", "\r", "mixed"]))
with tempfile.TemporaryDirectory() as d:
    p = pathlib.Path(d) / "t.csv"
    p.write_bytes(data)
    ds = CsvDataSource(str(p), True, 0, ctx=Context.get(0))
    names = [f.name for f in ds.schema().fields]
    b = next(ds.scan(names))
    gpu = [b.field(i).to_pylist() for i in range(len(names))]
onames, od, rows = R.parse(data)
want = R.project(rows, range(len(onames)))
print("delim", repr(delim), "rows", len(rows), "gpu rows", len(gpu[0]))
recs = [r for r in R.split_records(data) if R.kept(r)][1:]
for i in range(min(len(rows), len(gpu[0]))):
    g = [c[i] for c in gpu]
    w = [c[i] for c in want]
    if g != w:
        print("row", i, "record", repr(recs[i]))
        print(" gpu ", g)
        print(" want", w)
        break
