"""ORACLE (test infrastructure only — never imported by the product path).

CSV scan (CsvDataSource / ReaderIterator, folkol/query-engines kquerydiy/src/Main.kt K:204-357)
restated at byte level — the checker for query-engines_amd/csrc/qe_csv.hip:
  * CsvDataSource.inferSchema (K:332-356): the first kept record names the fields, all Utf8;
  * ReaderIterator.nextBatch/createBatch (K:239-273): batches of `batch_size` rows (1000, K:396),
    each value trimmed (K:263), a missing value reads as "" (K:263);
  * univocity CsvParser settings (K:290-297; library version unpinned, not in /root/reference):
    delimiter / line-separator detection, skipEmptyLines, default quote '"' with "" escapes and
    default comment char '#'. Restated as: '"' toggles the quoted state anywhere; outside quotes
    '\\n', '\\r\\n' and lone '\\r' end a record and the delimiter ends a field; records that are
    blank (all bytes <= 0x20) or start with '#' are skipped; the delimiter is the first of
    , ; TAB | found in the first kept record; a value is its bytes trimmed of <= 0x20, and a value
    wrapped in quotes loses them, "" becomes ", and it is trimmed again.
Pinned by the reference fixture employee.csv (tests/golden/employee_kat.json); the quote /
line-ending / comment rules are unpinned (univocity absent) and cross-checked against Python's
csv module where both define the same result (tests/test_csv.py).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

DELIMS = (b",", b";", b"\t", b"|")


def split_records(data: bytes) -> List[bytes]:
    recs: List[bytes] = []
    start, inq, n = 0, False, len(data)
    for i in range(n):
        c = data[i]
        if c == 0x22:
            inq = not inq
        elif not inq and (c == 0x0A or (c == 0x0D and (i + 1 >= n or data[i + 1] != 0x0A))):
            recs.append(data[start:i])
            start = i + 1
    if start < n:
        recs.append(data[start:])
    return recs


def kept(rec: bytes) -> bool:
    return len(rec) > 0 and rec[0] != 0x23 and any(b > 0x20 for b in rec)


def split_fields(rec: bytes, delim: int) -> List[bytes]:
    out, start, inq = [], 0, False
    for i, c in enumerate(rec):
        if c == 0x22:
            inq = not inq
        elif not inq and c == delim:
            out.append(rec[start:i])
            start = i + 1
    out.append(rec[start:])
    return out


def _trim(b: bytes) -> bytes:
    s, e = 0, len(b)
    while s < e and b[s] <= 0x20:
        s += 1
    while e > s and b[e - 1] <= 0x20:
        e -= 1
    return b[s:e]


def value(raw: bytes) -> bytes:
    v = _trim(raw)
    if len(v) >= 2 and v[0] == 0x22 and v[-1] == 0x22:
        v = _trim(v[1:-1]).replace(b'""', b'"')
    return v


def detect_delimiter(header: bytes) -> int:
    for d in DELIMS:
        if d in header:
            return d[0]
    return 0x2C


def parse(data: bytes, has_header: bool = True):
    """-> (field names, delimiter, rows as lists of byte values (all fields))."""
    recs = [r for r in split_records(data) if kept(r)]
    if not recs:
        return [], 0x2C, []
    delim = detect_delimiter(recs[0])
    first = split_fields(recs[0], delim)
    if has_header:
        names = [value(f).decode("utf-8", "replace") for f in first]
        body = recs[1:]
    else:
        names = [f"field_{i + 1}" for i in range(len(first))]
        body = recs
    return names, delim, [[value(f) for f in split_fields(r, delim)] for r in body]


def project(rows: List[List[bytes]], idx: Sequence[int]) -> List[List[str]]:
    """Columns for field positions `idx` (missing trailing fields -> "")."""
    return [[(r[i] if i < len(r) else b"").decode("utf-8", "replace") for r in rows] for i in idx]


def read_csv(path: str, batch_size: int = 1000) -> List[Dict[str, List[str]]]:
    with open(path, "rb") as f:
        names, _, rows = parse(f.read())
    batches = []
    for s in range(0, len(rows), batch_size):
        chunk = rows[s:s + batch_size]
        cols = project(chunk, range(len(names)))
        batches.append({name: cols[i] for i, name in enumerate(names)})
    return batches


def employee_filter_project(path: str, state: str = "CA", columns=("id", "first_name")) -> List[List[str]]:
    out: List[List[str]] = []
    for b in read_csv(path):
        for i, st in enumerate(b["state"]):
            if st.encode() == state.encode():
                out.append([b[c][i] for c in columns])
    return out


def employee_group_max(path: str, key: str = "state", value_col: str = "salary") -> Dict[str, Optional[float]]:
    """SELECT state, MAX(CAST(salary AS double)) ... GROUP BY state (K:1336 shape)."""
    from .semantics import MaxAccumulator

    groups: Dict[str, MaxAccumulator] = {}
    for b in read_csv(path):
        for k, v in zip(b[key], b[value_col]):
            acc = groups.setdefault(k, MaxAccumulator())
            acc.accumulate(float(v))  # Kotlin String.toDouble on these plain decimals
    return {k: a.finalValue() for k, a in groups.items()}
