"""CsvDataSource (Main.kt:276-357) on the GPU CSV scan (qe_csv_parse).

The file's bytes go to HBM once; tokenising, trimming, unquoting and column building run on the
device (grammar: query-engines_amd/csrc/qe_csv.hip). The host only reads the first kept record to
resolve the header names and the delimiter (the reference's inferSchema, K:332-356, and
univocity's detection, K:290-297) and maps the projection to field positions, as
`settings.selectFields` does (K:319-321).

Like the reference: the header names the fields (or field_1.. without one), every column is
Utf8 (K:348), values are trimmed and a missing value reads as "" (K:263), a missing file raises
FileNotFoundError (K:306-308), and batches hold `batchSize` rows (K:239-252). Device batches are
zero-copy slices of one parsed table, so a large batchSize (default: the whole file) costs nothing.
"""
from __future__ import annotations

import os
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import native as N
from .columnar import Context, DeviceColumn, Field, RecordBatch, Schema
from .datasource import DataSource

_DELIMS = (b",", b";", b"\t", b"|")


def _first_record(data: bytes) -> Optional[bytes]:
    """First kept record (same record / skip rules as the device scan)."""
    start, inq, n = 0, False, len(data)
    for i in range(n):
        c = data[i]
        if c == 0x22:
            inq = not inq
        elif not inq and (c == 0x0A or (c == 0x0D and (i + 1 >= n or data[i + 1] != 0x0A))):
            rec = data[start:i]
            if rec and rec[0] != 0x23 and any(b > 0x20 for b in rec):
                return rec
            start = i + 1
    rec = data[start:]
    return rec if rec and rec[0] != 0x23 and any(b > 0x20 for b in rec) else None


def _fields(rec: bytes, delim: int) -> List[str]:
    out, start, inq = [], 0, False
    for i, c in enumerate(rec):
        if c == 0x22:
            inq = not inq
        elif not inq and c == delim:
            out.append(rec[start:i])
            start = i + 1
    out.append(rec[start:])
    vals = []
    for f in out:
        v = f.strip(bytes(range(0x21)))
        if len(v) >= 2 and v[:1] == b'"' and v[-1:] == b'"':
            v = v[1:-1].strip(bytes(range(0x21))).replace(b'""', b'"')
        vals.append(v.decode("utf-8", "replace"))
    return vals


def _head(filename: str, limit: int = 1 << 20) -> Tuple[bytes, bool]:
    with open(filename, "rb") as f:
        data = f.read(limit)
        return data, len(data) < limit


_UPLOAD_CTX: dict = {}


def _upload_ctx(device: int) -> Context:
    """The overlapped scan's upload context: its own stream, and kept, so its pinned staging
    buffers are allocated once per process (one scan at a time uses it: the scan joins its thread)."""
    if device not in _UPLOAD_CTX:
        import torch

        s = torch.cuda.Stream(torch.device("cuda", device))
        _UPLOAD_CTX[device] = (s, Context(device, s.cuda_stream))
    return _UPLOAD_CTX[device][1]


def _view(c: DeviceColumn, s: int, m: int, ctx: Context) -> DeviceColumn:
    """Rows [s, s + m) of a UTF8 column (its offsets sliced, the values shared)."""
    v = DeviceColumn(N.TYPE_UTF8, m, c.values, None, c.offsets[s:s + m + 1], ctx)
    v.max_len = c.max_len  # a bound for every row is one for these rows
    return v


class CsvDataSource(DataSource):
    def __init__(self, filename: str, hasHeaders: bool = True, batchSize: int = 0,  # noqa: N803
                 schema: Optional[Schema] = None, ctx: Optional[Context] = None, chunk_bytes: int = 0):
        """``chunk_bytes`` > 0: scan a file of at least two such chunks chunk by chunk, uploading the
        next while this one parses (one batch per chunk, like the JNI scan). Off by default: tripdata
        (386 MB, one box) took 10.4 ms file -> columns in 128 MB chunks against 8.9 ms for one staged
        upload + one parse (docs/experiments.md)."""
        self.chunk_bytes = int(chunk_bytes)
        self.filename = filename
        self.hasHeaders = hasHeaders
        self.batchSize = batchSize
        self._schema = schema
        self.ctx = ctx
        self._delim: Optional[int] = None

    def _check(self) -> None:
        if not os.path.exists(self.filename):
            raise FileNotFoundError(os.path.abspath(self.filename))

    def _infer(self) -> None:
        self._check()
        data, whole = _head(self.filename)
        rec = _first_record(data)
        while rec is None and not whole:  # header beyond the first MiB (blank / comment lines)
            data, whole = _head(self.filename, 2 * len(data))
            rec = _first_record(data)
        rec = rec or b""
        self._delim = next((d[0] for d in _DELIMS if d in rec), 0x2C)
        names = _fields(rec, self._delim) if rec else []
        if self._schema is None:
            if self.hasHeaders:
                self._schema = Schema([Field(h, N.TYPE_UTF8) for h in names])
            else:
                self._schema = Schema([Field(f"field_{i + 1}", N.TYPE_UTF8) for i in range(len(names))])

    def schema(self) -> Schema:
        if self._schema is None or self._delim is None:
            self._infer()
        return self._schema

    def scan(self, projection: Sequence[str]) -> Iterator[RecordBatch]:
        import torch

        self._check()
        schema = self.schema()
        read_schema = schema.select(projection) if projection else schema
        names = [f.name for f in schema.fields]
        idx = [names.index(f.name) for f in read_schema.fields]
        ctx = self.ctx or Context.get(0)
        size = os.path.getsize(self.filename)
        chunk = self.chunk_bytes
        if (not self.batchSize or self.batchSize <= 0) and chunk > 0 and size >= 2 * chunk:
            yield from self._scan_chunked(ctx, read_schema, idx, size, chunk)
            return
        dev = torch.empty(max(1, size), dtype=torch.uint8, device=ctx.torch_device)
        if size:  # file -> HBM: the library's staging threads pread() into pinned buffers and DMA them
            N.check(N.lib().qe_file_to_device(ctx.handle, os.fsencode(self.filename), 0, size,
                                              N.C.c_void_p(dev.data_ptr())))
        cols = self._parse(ctx, dev, size, idx)
        n = cols[0].length if cols else 0
        step = self.batchSize if self.batchSize and self.batchSize > 0 else max(n, 1)
        for s in range(0, n, step):
            m = min(step, n - s)
            yield RecordBatch(read_schema, [_view(c, s, m, ctx) for c in cols])

    def _scan_chunked(self, ctx: Context, read_schema: Schema, idx: List[int], size: int,
                      chunk: int) -> Iterator[RecordBatch]:
        """A large file in chunks of about `chunk` bytes, one batch each (like the JNI scan,
        NativeOperators.kt): a host thread uploads chunk k + 1 (qe_file_to_device on its own
        stream) while chunk k is parsed and its batch consumed, so the PCIe copy — the bound of a
        cold file scan — hides the device work. Chunk k is parsed from where chunk k - 1's last
        record ended (QE_CSV_PARTIAL_TAIL), so the records are exactly those of one parse."""
        import threading

        import torch

        dev = torch.empty(size, dtype=torch.uint8, device=ctx.torch_device)
        bounds = list(range(0, size, chunk)) + [size]
        if bounds[-1] - bounds[-2] < chunk // 2 and len(bounds) > 2:
            del bounds[-2]  # no small last chunk
        nchunks = len(bounds) - 1
        ready = [threading.Event() for _ in range(nchunks)]
        err: list = []
        up = _upload_ctx(ctx.device)
        path = os.fsencode(self.filename)

        def upload():
            try:
                for k in range(nchunks):
                    a, b = bounds[k], bounds[k + 1]
                    N.check(N.lib().qe_file_to_device(up.handle, path, a, b - a, N.C.c_void_p(dev.data_ptr() + a)))
                    ready[k].set()
            except BaseException as e:  # noqa: BLE001 - re-raised by the consumer
                err.append(e)
                for r in ready:
                    r.set()

        th = threading.Thread(target=upload, daemon=True)
        th.start()
        try:
            start, header = 0, self.hasHeaders
            for k in range(nchunks):
                ready[k].wait()
                if err:
                    raise err[0]
                end, last = bounds[k + 1], k == nchunks - 1
                cols, consumed = self._parse_region(ctx, dev, end - start, idx, offset=start, header=header,
                                                    partial=not last)
                if consumed == 0:  # no complete record in [start, end): the next chunk extends it
                    continue
                header = False
                start += consumed
                n = cols[0].length if cols else 0
                if n:
                    yield RecordBatch(read_schema, cols)
        finally:
            th.join()

    def _parse(self, ctx: Context, dev, nbytes: int, idx: List[int]) -> List[DeviceColumn]:
        return self._parse_region(ctx, dev, nbytes, idx)[0]

    def _parse_region(self, ctx: Context, dev, nbytes: int, idx: List[int], offset: int = 0,
                      header: Optional[bool] = None, partial: bool = False):
        """(columns of the projected fields of dev[offset, offset + nbytes), bytes consumed): with
        `partial` the records end at the last terminator and the rest continues in the next chunk."""
        import torch

        out: List[DeviceColumn] = []
        consumed = nbytes
        hdr = self.hasHeaders if header is None else header
        for s in range(0, len(idx), 32):  # qe_csv_parse projects up to 32 fields per call
            part = idx[s:s + 32]
            fi = (N.C.c_int32 * len(part))(*part)
            opt = N.QeCsvOptions(self._delim, 1 if hdr else 0, len(part), N.CSV_PARTIAL_TAIL if partial else 0, fi)
            h = N.C.c_void_p()
            N.check(N.lib().qe_csv_parse(ctx.handle, N.C.c_void_p(dev.data_ptr() + offset), nbytes, N.C.byref(opt),
                                         N.C.byref(h)))
            try:
                rows = N.C.c_int64()
                N.check(N.lib().qe_csv_rows(h, N.C.byref(rows)))
                used = N.C.c_int64()
                N.check(N.lib().qe_csv_consumed(h, N.C.byref(used)))
                consumed = used.value
                for c in range(len(part)):
                    nb = N.C.c_int64()
                    N.check(N.lib().qe_csv_column_bytes(h, c, N.C.byref(nb)))
                    col = DeviceColumn(N.TYPE_UTF8, rows.value,
                                       torch.empty(max(1, nb.value), dtype=torch.uint8, device=ctx.torch_device), None,
                                       torch.empty(rows.value + 1, dtype=torch.int32, device=ctx.torch_device), ctx)
                    cc = col.as_c()
                    N.check(N.lib().qe_csv_column_copy(h, c, N.C.byref(cc)))
                    ml = N.C.c_int64()
                    N.check(N.lib().qe_csv_column_max_len(h, c, N.C.byref(ml)))
                    col.max_len = ml.value  # (short keys then take packed dictionary codes)
                    out.append(col)
                # no sync: the column builds and the table's release are ordered on the ctx stream,
                # which is torch's current stream (the tensors' allocator stream)
            finally:
                N.lib().qe_csv_destroy(h)
        return out, consumed
