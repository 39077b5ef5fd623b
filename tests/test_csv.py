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
def _gpu_scan(ctx, tmp_path, data, projection=None, has_header=True, batch=0, chunk_bytes=0):
    from kquery.csv_source import CsvDataSource

    p = tmp_path / "t.csv"
    p.write_bytes(data)
    ds = CsvDataSource(str(p), has_header, batch, ctx=ctx, chunk_bytes=chunk_bytes)
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


@pytest.mark.gpu
@pytest.mark.parametrize("newline", ["\n", "\r\n"])
def test_gpu_csv_chunked_overlapped_scan(gpu_ctx, tmp_path, newline):
    """A large file scans in chunks (chunk_bytes; 1 MiB here), the next chunk uploading while
    this one parses: chunk boundaries land inside quoted fields with embedded newlines and
    delimiters, between '\\r' and '\\n', and in blank / comment lines; the concatenated batches equal
    one parse of the file (oracle), and there is more than one batch."""
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
    names, proj, cols, batches = _gpu_scan(gpu_ctx, tmp_path, data, chunk_bytes=1 << 20)
    onames, _, rows = R.parse(data)
    assert names == onames
    assert len(batches) > 1
    assert cols == R.project(rows, range(3))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["plain", "short_lines", "no_trailing_newline", "one_quote_at_end", "cr_at_end",
                                   "utf8", "tabs", "blank_and_comment_lines", "long_lines"])
def test_gpu_csv_fast_path_vs_oracle(gpu_ctx, tmp_path, shape):
    """A file without '"' or '\r' takes the classification pass (k_csv_classify: '\n' and delimiter
    bitmaps) with the bitmap line-end list and line walk; a '"' or '\r' anywhere (here only in the
    last line) sends it back to the general passes. Every shape equals the oracle: UTF-8 bytes whose
    low seven bits alias '\n' / ',' / '"' / '\r' (0x8A, 0xAC, 0xA2, 0x8D), tab delimiters, blank and
    comment lines (the kept-line path), lines longer than a 64-byte bitmap word, many 16 KiB
    segments."""
    rng = random.Random(len(shape))
    d = "\t" if shape == "tabs" else ","
    if shape == "short_lines":
        body = [f"{i % 7}{d}{i % 3}" for i in range(300_000)]
    elif shape == "utf8":
        words = ["Ê", "¬", "¢", "ō", "Pärsson", "x"]
        body = [f"{i % 13}{d}{rng.choice(words)}{d}{''.join(rng.choice(words) for _ in range(i % 9))}{d}{i}"
                for i in range(120_000)]
    elif shape == "long_lines":
        body = [f"{i % 13}{d}{'y' * rng.choice([1, 60, 200, 3000])}{d}{'z' * (i % 70)}{d}{i}" for i in range(20_000)]
    else:
        body = [f"{i % 13}{d}{rng.random():.6f}{d}{'x' * (i % 40)}{d}{i}" for i in range(120_000)]
    if shape == "blank_and_comment_lines":
        for at in (7, 50_000, 119_990):
            body.insert(at, rng.choice(["", "   ", "#comment,x", "\t"]))
    text = f"k{d}v{d}s{d}i\n" + "\n".join(body)
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
    # projections of single fields (the line walk's bit selection skips the others)
    for f in (names[-1], names[1]):
        _, _, c1, _ = _gpu_scan(gpu_ctx, tmp_path, data, [f])
        assert c1[0] == R.project(rows, [names.index(f)])[0]
