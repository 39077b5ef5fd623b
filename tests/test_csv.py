"""GPU CSV scan (qe_csv_parse / CsvDataSource) against the oracle's byte-level restatement
(oracle/csv_ref.py), which is itself pinned by employee.csv and cross-checked with Python's csv
module where the two define the same result."""
import csv
import io
import random

import pytest

from oracle import csv_ref as R

WORDS = ["a", "b c", "Uppsala", "Sthlm", "Pärsson", "x,y", 'he said ""hi""', "line\nbreak", "crlf\r\nin", "1337",
         "", "  padded  ", "€uro", "#notcomment", "tab\there"]


def _field(rng, delim):
    w = rng.choice(WORDS)
    needs = any(ch in w for ch in (delim, "\n", "\r", '"')) or rng.random() < 0.2
    if needs:
        return '"' + w.replace('"', '""').replace('""""', '""') + '"'
    return w


def random_csv(rng, rows, ncols, delim=",", newline="\n"):
    lines = [delim.join(f"col{i}" for i in range(ncols))]
    for _ in range(rows):
        r = rng.random()
        if r < 0.03:
            lines.append("")  # blank line
        elif r < 0.05:
            lines.append("   \t ")
        elif r < 0.07:
            lines.append("#comment, with, delims")
        else:
            k = ncols if rng.random() < 0.9 else rng.randint(1, ncols + 2)  # ragged rows
            lines.append(delim.join(_field(rng, delim) for _ in range(k)))
    nl = newline if newline != "mixed" else None
    out = []
    for ln in lines:
        out.append(ln)
        out.append(nl or rng.choice(["\n", "\r\n", "\r"]))
    if rng.random() < 0.5:
        out.pop()  # no trailing terminator
    return "".join(out).encode()


# ---- CPU: oracle ------------------------------------------------------------------------------
def test_oracle_matches_python_csv_where_defined():
    rng = random.Random(1)
    for trial in range(40):
        ncols = rng.randint(1, 6)
        rows = []
        for _ in range(rng.randint(1, 30)):
            rows.append([rng.choice(["abc", "x y", 'q"uote', "a,b", "multi\nline", "", "ünï"]) for _ in range(ncols)])
        buf = io.StringIO()
        w = csv.writer(buf, lineterminator="\n", quoting=csv.QUOTE_MINIMAL)
        w.writerow([f"h{i}" for i in range(ncols)])
        for r in rows:
            if all(v == "" for v in r):
                r[0] = "z"  # the oracle skips blank records, csv does not
            w.writerow(r)
        data = buf.getvalue().encode()
        names, delim, got = R.parse(data)
        assert names == [f"h{i}" for i in range(ncols)]
        want = [[v.strip("".join(chr(c) for c in range(33))) for v in r] for r in rows]
        assert [[v.decode() for v in r] for r in got] == want


def test_oracle_rules():
    data = b'h1,h2\r\n\r\n  \n#c,d\n" a "" b ",  x  \r"q\nq",\n1,2,3\n4'
    names, delim, rows = R.parse(data)
    assert names == ["h1", "h2"] and delim == ord(",")
    assert rows == [[b'a " b', b"x"], [b"q\nq", b""], [b"1", b"2", b"3"], [b"4"]]
    assert R.project(rows, [1]) == [["x", "", "2", ""]]
    assert R.detect_delimiter(b"a;b") == ord(";") and R.detect_delimiter(b"a\tb") == 9


def test_host_header_helpers_match_oracle():
    from kquery.csv_source import _fields, _first_record

    rng = random.Random(5)
    for trial in range(30):
        data = random_csv(rng, rng.randint(0, 5), rng.randint(1, 5), rng.choice([",", ";", "\t", "|"]), "mixed")
        data = rng.choice([b"", b"\n\n", b"#x\n", b"  \r\n"]) + data
        rec = _first_record(data)
        recs = [r for r in R.split_records(data) if R.kept(r)]
        assert rec == (recs[0] if recs else None)
        if rec:
            d = R.detect_delimiter(rec)
            assert _fields(rec, d) == [R.value(f).decode("utf-8", "replace") for f in R.split_fields(rec, d)]


# ---- GPU -----------------------------------------------------------------------------------------
def _gpu_scan(ctx, tmp_path, data, projection=None, has_header=True, batch=0):
    from kquery.csv_source import CsvDataSource

    p = tmp_path / "t.csv"
    p.write_bytes(data)
    ds = CsvDataSource(str(p), has_header, batch, ctx=ctx)
    names = [f.name for f in ds.schema().fields]
    proj = projection if projection is not None else names
    batches = list(ds.scan(proj))
    cols = [[] for _ in proj]
    for b in batches:
        for i in range(len(proj)):
            vals = b.field(i).to_pylist()
            cols[i] += vals
            # the scan's longest-value bound (qe_csv_column_max_len): exact for a whole parse, an
            # upper bound for a batch cut from one
            longest = max((len(v.encode()) for v in vals), default=0)
            ml = b.field(i).max_len
            assert ml is not None and ml >= longest
            if len(batches) == 1 and not batch:
                assert ml == longest
    return names, proj, cols, batches


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_csv_random(gpu_ctx, tmp_path, seed):
    rng = random.Random(seed)
    delim = rng.choice([",", ";", "\t", "|"])
    data = random_csv(rng, rng.choice([0, 1, 5, 300, 5000]), rng.randint(1, 7), delim,
                      rng.choice(["\n", "\r\n", "\r", "mixed"]))
    names, proj, cols, _ = _gpu_scan(gpu_ctx, tmp_path, data)
    onames, _, rows = R.parse(data)
    assert names == onames
    assert cols == R.project(rows, range(len(onames)))


@pytest.mark.gpu
def test_gpu_csv_projection_and_batches(gpu_ctx, tmp_path):
    rng = random.Random(77)
    data = random_csv(rng, 20000, 6, ",", "\n")
    names, proj, cols, batches = _gpu_scan(gpu_ctx, tmp_path, data, ["col4", "col1"], batch=1000)
    onames, _, rows = R.parse(data)
    assert cols == R.project(rows, [4, 1])
    assert all(b.rowCount() == 1000 for b in batches[:-1]) and sum(b.rowCount() for b in batches) == len(rows)


@pytest.mark.gpu
def test_gpu_csv_large_segments(gpu_ctx, tmp_path):
    """~12 MB: many 64 KiB segments, quoted fields with newlines and delimiters crossing segment
    and lane boundaries, CRLF endings."""
    rng = random.Random(3)
    body = []
    for i in range(150_000):
        q = '"%s"' % ("x," * rng.randint(0, 30) + "\r\n" * rng.randint(0, 2)) if i % 7 == 0 else str(i)
        body.append(f"{i % 97},{q},{rng.random():.6f}")
    data = ("k,v,f\r\n" + "\r\n".join(body) + "\r\n").encode()
    names, proj, cols, _ = _gpu_scan(gpu_ctx, tmp_path, data)
    onames, _, rows = R.parse(data)
    assert cols == R.project(rows, range(3))


@pytest.mark.gpu
def test_gpu_csv_edge_files(gpu_ctx, tmp_path):
    cases = [b"a,b\n", b"a,b", b"a,b\r", b"a,b\n\n\n", b"\n\n#x\na,b\n1,2", b'a,b\n"open quote,1\n2,3',
             b"a\n \n\t\n", b"a,b\n1\n,\n", b'a\n"""\n']
    for data in cases:
        names, proj, cols, _ = _gpu_scan(gpu_ctx, tmp_path, data)
        onames, _, rows = R.parse(data)
        assert names == onames, data
        assert cols == R.project(rows, range(len(onames))), data


@pytest.mark.gpu
def test_gpu_csv_employee_fixture(gpu_ctx):
    import json
    import pathlib

    gold = pathlib.Path(__file__).parent / "golden"
    from kquery.csv_source import CsvDataSource

    ds = CsvDataSource(str(gold / "employee.csv"), True, 1000, ctx=gpu_ctx)
    assert [f.name for f in ds.schema().fields] == json.loads((gold / "employee_kat.json").read_text())["columns"]
    b = list(ds.scan(["state", "last_name"]))
    assert len(b) == 1 and b[0].field(0).to_pylist() == ["Uppsala", "Uppsala", "Sthlm"]
    assert b[0].field(1).to_pylist() == ["Johansson", "Person", "Pärsson"]


def test_missing_file_raises(tmp_path):
    from kquery.csv_source import CsvDataSource

    with pytest.raises(FileNotFoundError):
        CsvDataSource(str(tmp_path / "nope.csv")).schema()


@pytest.mark.gpu
def test_gpu_csv_long_lines_and_blank_lines(gpu_ctx, tmp_path):
    """Line blocks too long for a wave's LDS copy (k_csv_lines walks HBM for those), and large
    files with blank / comment lines in the middle (the kept-line path)."""
    rng = random.Random(9)
    body = []
    for i in range(40_000):
        w = rng.choice([1, 5, 300, 2000]) if (i // 500) % 3 == 1 else rng.choice([1, 3, 8])
        body.append(f"{i},{'y' * w},\"q\"\"{i % 13}\"")
    long_data = ("a,b,c\n" + "\n".join(body) + "\n").encode()
    mixed = body[:]
    for at in (5, 20_000, 39_990):
        mixed.insert(at, rng.choice(["", "   ", "#comment,x", "\t"]))
    for data in (long_data, ("a,b,c\n" + "\n".join(mixed) + "\n").encode()):
        names, proj, cols, _ = _gpu_scan(gpu_ctx, tmp_path, data)
        onames, _, rows = R.parse(data)
        assert names == onames
        assert cols == R.project(rows, range(len(onames)))


_SEG_CHILD = r'''
import pathlib, random, sys, tempfile
root = pathlib.Path(sys.argv[1])
sys.path[:0] = [str(root), str(root / "query-engines_amd"), str(root / "tests")]
from kquery.columnar import Context
from oracle import csv_ref as R
import test_csv as T
ctx = Context.get(0)
tmp = pathlib.Path(tempfile.mkdtemp())
for seed in range(8):
    rng = random.Random(100 + seed)
    delim = rng.choice([",", ";", "|"])
    data = T.random_csv(rng, rng.choice([1, 300, 5000]), rng.randint(1, 7), delim, rng.choice(["\n", "\r\n", "mixed"]))
    names, proj, cols, _ = T._gpu_scan(ctx, tmp, data)
    onames, _, rows = R.parse(data)
    assert names == onames and cols == R.project(rows, range(len(onames))), seed
body = [f"{i % 97},{i},\"q,{i}\",{i * 0.5}" for i in range(200_000)]
data = ("k,v,q,f\n" + "\n".join(body) + "\n").encode()
names, proj, cols, _ = T._gpu_scan(ctx, tmp, data)
onames, _, rows = R.parse(data)
assert cols == R.project(rows, range(4))
print("ok")
'''


@pytest.mark.gpu
def test_gpu_csv_segment_field_pass(tmp_path):
    """The opt-in segment field pass (QE_CSV_SEGFIELDS=1, read once per process: a child process)
    against the oracle: random files (blank / comment lines take the kept-line path), and a large
    all-records file with quoted fields, which it handles itself."""
    import os
    import pathlib
    import subprocess
    import sys

    root = pathlib.Path(__file__).resolve().parents[1]
    env = dict(os.environ, QE_CSV_SEGFIELDS="1")
    r = subprocess.run([sys.executable, "-c", _SEG_CHILD, str(root)], cwd=str(root), env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("newline", ["\n", "\r\n"])
def test_gpu_csv_chunked_overlapped_scan(gpu_ctx, tmp_path, monkeypatch, newline):
    """A large file scans in chunks (QE_CSV_CHUNK_MB; 1 MiB here), the next chunk uploading while
    this one parses: chunk boundaries land inside quoted fields with embedded newlines and
    delimiters, between '\\r' and '\\n', and in blank / comment lines; the concatenated batches equal
    one parse of the file (oracle), and there is more than one batch."""
    monkeypatch.setenv("QE_CSV_CHUNK_MB", "1")
    rng = random.Random(11 + len(newline))
    body = []
    for i in range(200_000):
        r = rng.random()
        if r < 0.01:
            body.append("")
        elif r < 0.02:
            body.append("#c,o,m")
        else:
            q = '"%s"' % ("a,b" + newline * rng.randint(0, 2) + 'x""y') if i % 5 == 0 else str(i)
            body.append(f"{i % 13},{q},{rng.random():.5f}")
    data = ("k,v,f" + newline + newline.join(body) + newline).encode()
    assert len(data) > 3 << 20  # three 1 MiB chunks at least
    names, proj, cols, batches = _gpu_scan(gpu_ctx, tmp_path, data)
    onames, _, rows = R.parse(data)
    assert names == onames
    assert len(batches) > 1
    assert cols == R.project(rows, range(3))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["plain", "short_lines", "no_trailing_newline", "one_quote_at_end", "cr_at_end"])
def test_gpu_csv_onepass_vs_general(gpu_ctx, tmp_path, monkeypatch, shape):
    """With QE_CSV_ONEPASS=1, files without '"' or '\\r' take the one-pass line-end list
    (k_csv_ends1, segments chained by look-back); a '"' or '\\r' anywhere (here only in the last
    line), or more line ends than its list holds (lines shorter than 16 bytes), sends the parse back
    to the general passes. The default (general) passes equal the oracle on every shape, and the
    one-pass scan (a fresh process: the switch is read once) gives the same columns."""
    import subprocess
    import sys

    rng = random.Random(len(shape))
    if shape == "short_lines":
        body = [f"{i % 7},{i % 3}" for i in range(300_000)]  # 4-byte lines: over the list's capacity
    else:
        body = [f"{i % 13},{rng.random():.6f},{'x' * (i % 40)},{i}" for i in range(120_000)]
    text = "k,v,s,i\n" + "\n".join(body)
    if shape == "one_quote_at_end":
        text += '\n1,"2",3,4'
    elif shape == "cr_at_end":
        text += "\r\n1,2,3,4"
    if shape != "no_trailing_newline":
        text += "\n"
    data = text.encode()
    assert len(data) > 1 << 20  # many 16 KiB segments
    names, proj, cols, _ = _gpu_scan(gpu_ctx, tmp_path, data)
    onames, _, rows = R.parse(data)
    assert names == onames
    assert cols == R.project(rows, range(len(names)))
    # the one-pass scan in a process of their own (the switch is read once per process)
    code = ("import sys, json; sys.path[:0] = [{root!r}, {root!r} + '/query-engines_amd']\n"
            "from kquery.columnar import Context\nfrom kquery.csv_source import CsvDataSource\n"
            "ds = CsvDataSource({path!r}, True, 0, ctx=Context.get(0))\n"
            "cols = [[] for _ in range(4)]\n"
            "for b in ds.scan(['k', 'v', 's', 'i'][:{n}]):\n"
            "    for i in range({n}): cols[i] += b.field(i).to_pylist()\n"
            "print(json.dumps(cols))\n")
    import pathlib

    root = str(pathlib.Path(__file__).resolve().parents[1])
    p = tmp_path / "t.csv"
    env = dict(__import__("os").environ, QE_CSV_ONEPASS="1")
    out = subprocess.run([sys.executable, "-c", code.format(root=root, path=str(p), n=len(names))], env=env,
                         capture_output=True, text=True, timeout=240, check=True).stdout
    assert __import__("json").loads(out.strip().splitlines()[-1]) == cols
