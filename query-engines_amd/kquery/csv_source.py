"""CsvDataSource (Main.kt:276-357) for config 1: host-side text parsing (CPU plumbing, out of the
HBM-bound path per SURVEY §2), producing device-resident Utf8 RecordBatches.

Follows the reference: the header row names the fields (inferSchema, K:332-356), every column is
Utf8 (K:348), batches hold `batchSize` rows (ReaderIterator.nextBatch, K:239-252; 1000 in
ExecutionContext.csv, K:396), each value is trimmed and a missing value reads as "" (K:263), empty
lines are skipped (K:294), a missing file raises FileNotFoundError (K:306-308)."""
from __future__ import annotations

import csv
import io
import os
from typing import Iterator, List, Optional, Sequence

from . import native as N
from .columnar import Context, DeviceColumn, Field, RecordBatch, Schema
from .datasource import DataSource


class CsvDataSource(DataSource):
    def __init__(self, filename: str, hasHeaders: bool = True, batchSize: int = 1000,  # noqa: N803
                 schema: Optional[Schema] = None, ctx: Optional[Context] = None):
        self.filename = filename
        self.hasHeaders = hasHeaders
        self.batchSize = batchSize
        self._schema = schema
        self.ctx = ctx

    def _rows(self) -> List[List[str]]:
        if not os.path.exists(self.filename):
            raise FileNotFoundError(os.path.abspath(self.filename))
        with open(self.filename, "rb") as f:
            text = f.read().decode("utf-8")
        sample = text.split("\n", 1)[0]
        delim = next((d for d in (",", ";", "\t") if d in sample), ",")
        return [r for r in csv.reader(io.StringIO(text), delimiter=delim) if any(x.strip() for x in r)]

    def schema(self) -> Schema:
        if self._schema is None:
            rows = self._rows()
            header = rows[0] if rows else []
            if self.hasHeaders:
                self._schema = Schema([Field(h.strip(), N.TYPE_UTF8) for h in header])
            else:
                self._schema = Schema([Field(f"field_{i + 1}", N.TYPE_UTF8) for i in range(len(header))])
        return self._schema

    def scan(self, projection: Sequence[str]) -> Iterator[RecordBatch]:
        rows = self._rows()
        schema = self.schema()
        read_schema = schema.select(projection) if projection else schema
        names = [f.name for f in schema.fields]
        idx = [names.index(f.name) for f in read_schema.fields]
        body = rows[1:] if self.hasHeaders else rows
        ctx = self.ctx or Context.get(0)
        for s in range(0, len(body), self.batchSize):
            chunk = body[s:s + self.batchSize]
            cols = [DeviceColumn.from_strings([(r[i] if i < len(r) else "").strip() for r in chunk], ctx=ctx)
                    for i in idx]
            yield RecordBatch(read_schema, cols)
