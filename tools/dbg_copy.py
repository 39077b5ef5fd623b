import pathlib, random, sys, os
root = pathlib.Path("/root/repo")
sys.path[:0] = [str(root), str(root / "query-engines_amd"), str(root / "oracle"), str(root/"tests")]
import csv_ref as R
from kquery.columnar import Context
from kquery.csv_source import CsvDataSource
rng = random.Random(3)
body = []
for i in range(150_000):
    q = '"%s"' % ("x," * rng.randint(0, 30) + "\r\n" * rng.randint(0, 2)) if i % 7 == 0 else str(i)
    body.append(f"{i % 97},{q},{rng.random():.6f}")
data = ("k,v,f\r\n" + "\r\n".join(body) + "\r\n").encode()
p = pathlib.Path("/tmp/dbg.csv"); p.write_bytes(data)
ctx = Context.get(0)
ds = CsvDataSource(str(p), True, 0, ctx=ctx)
b = list(ds.scan(["k", "v", "f"]))[0]
_, _, rows = R.parse(data)
want = R.project(rows, range(3))
for c in range(3):
    got = b.field(c).to_pylist()
    bad = [i for i in range(len(want[c])) if got[i] != want[c][i]]
    print("col", c, "rows", len(got), len(want[c]), "bad", len(bad), "maxlen", b.field(c).max_len)
    for i in bad[:6]:
        print("  row", i, i % 64, repr(got[i]), repr(want[c][i]), repr(got[i-1]), repr(want[c][i-1]))
