"""ORACLE (test infrastructure only — never imported by the product path).

Config 1 (BASELINE.json configs[0]) on the CPU reference path: employee.csv
scan -> filter(state = 'CA') -> project(id, first_name), restating:
  * CsvDataSource.inferSchema (K:332-356): header row gives the field names, every column Utf8;
  * ReaderIterator.nextBatch/createBatch (K:239-273): batches of `batch_size` rows (1000, K:396),
    each value trimmed (K:263), missing values read as "" (K:263);
  * univocity settings (K:290-297): delimiter / line-separator detection, empty lines skipped.
    Only ',' and '\n' / '\r\n' occur in the fixture; detection is restated as "first of , ; \t
    found in the header".
The filter/project steps use the build-defined SelectionExec semantics (oracle/semantics.py).
"""
from __future__ import annotations

from typing import Dict, List, Optional


def read_csv(path: str, batch_size: int = 1000) -> List[Dict[str, List[str]]]:
    with open(path, "rb") as f:
        text = f.read().decode("utf-8")
    lines = [ln for ln in text.replace("\r\n", "\n").split("\n") if ln.strip() != ""]  # skipEmptyLines
    if not lines:
        return []
    header = lines[0]
    delim = next((d for d in (",", ";", "\t") if d in header), ",")
    names = [h.strip() for h in header.split(delim)]
    rows = [ln.split(delim) for ln in lines[1:]]
    batches = []
    for s in range(0, len(rows), batch_size):
        chunk = rows[s:s + batch_size]
        batch = {}
        for i, name in enumerate(names):
            batch[name] = [(r[i] if i < len(r) else "").strip() for r in chunk]  # K:263
        batches.append(batch)
    return batches


def employee_filter_project(path: str, state: str = "CA", columns=("id", "first_name")) -> List[List[str]]:
    out: List[List[str]] = []
    for b in read_csv(path):
        for i, st in enumerate(b["state"]):
            if st.encode() == state.encode():
                out.append([b[c][i] for c in columns])
    return out


def employee_group_max(path: str, key: str = "state", value: str = "salary") -> Dict[str, Optional[float]]:
    """SELECT state, MAX(CAST(salary AS double)) ... GROUP BY state (K:1336 shape)."""
    from .semantics import MaxAccumulator

    groups: Dict[str, MaxAccumulator] = {}
    for b in read_csv(path):
        for k, v in zip(b[key], b[value]):
            acc = groups.setdefault(k, MaxAccumulator())
            acc.accumulate(float(v))  # Kotlin String.toDouble on these plain decimals
    return {k: a.finalValue() for k, a in groups.items()}
