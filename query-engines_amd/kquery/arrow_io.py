"""Arrow C Data Interface interop (qe_batch_import / qe_batch_import_device / qe_batch_export).

This is the batch-level drop-in boundary of SURVEY §8b: Arrow Java hands a VectorSchemaRoot to
native code as a struct ArrowArray + ArrowSchema (org.apache.arrow.c.Data); here pyarrow plays
that producer/consumer role through the same two structs.
"""
from __future__ import annotations

import ctypes as C
from concurrent.futures import ThreadPoolExecutor
from typing import Iterable, Iterator, List, Optional, Sequence

from . import native as N
from .columnar import Context, DeviceColumn


class ArrowSchemaC(C.Structure):
    pass


ArrowSchemaC._fields_ = [
    ("format", C.c_char_p), ("name", C.c_char_p), ("metadata", C.c_char_p), ("flags", C.c_int64),
    ("n_children", C.c_int64), ("children", C.POINTER(C.POINTER(ArrowSchemaC))),
    ("dictionary", C.POINTER(ArrowSchemaC)), ("release", C.CFUNCTYPE(None, C.POINTER(ArrowSchemaC))),
    ("private_data", C.c_void_p),
]


class ArrowArrayC(C.Structure):
    pass


ArrowArrayC._fields_ = [
    ("length", C.c_int64), ("null_count", C.c_int64), ("offset", C.c_int64), ("n_buffers", C.c_int64),
    ("n_children", C.c_int64), ("buffers", C.POINTER(C.c_void_p)), ("children", C.POINTER(C.POINTER(ArrowArrayC))),
    ("dictionary", C.POINTER(ArrowArrayC)), ("release", C.CFUNCTYPE(None, C.POINTER(ArrowArrayC))),
    ("private_data", C.c_void_p),
]


class ArrowDeviceArrayC(C.Structure):
    _fields_ = [("array", ArrowArrayC), ("device_id", C.c_int64), ("device_type", C.c_int32),
                ("sync_event", C.c_void_p), ("reserved", C.c_int64 * 3)]


def _release(struct) -> None:
    if struct.release:
        struct.release(C.byref(struct))


class DeviceBatch:
    """A record batch in HBM owned by the library (qe_batch)."""

    def __init__(self, ctx: Context, handle: C.c_void_p):
        self.ctx = ctx
        self.handle = handle

    @classmethod
    def from_pyarrow(cls, batch, ctx: Optional[Context] = None) -> "DeviceBatch":
        """pyarrow.RecordBatch -> device (through the C data interface; H2D via pinned staging)."""
        ctx = ctx or Context.get(0)
        arr, sch = ArrowArrayC(), ArrowSchemaC()
        batch._export_to_c(C.addressof(arr), C.addressof(sch))
        try:
            h = C.c_void_p()
            N.check(N.lib().qe_batch_import(ctx.handle, C.byref(sch), C.byref(arr), C.byref(h)))
        finally:
            _release(arr)
            _release(sch)
        return cls(ctx, h)

    def close(self) -> None:
        if getattr(self, "handle", None) is not None:
            N.lib().qe_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def shape(self):
        nc, ln = C.c_int32(), C.c_int64()
        N.check(N.lib().qe_batch_num_columns(self.handle, C.byref(nc), C.byref(ln)))
        return nc.value, ln.value

    def column(self, i: int):
        """(QeColumn view, field name)."""
        col = N.QeColumn()
        name = C.c_char_p()
        N.check(N.lib().qe_batch_column(self.handle, i, C.byref(col), C.byref(name)))
        return col, name.value.decode()

    def columns(self):
        return [self.column(i) for i in range(self.shape()[0])]


def export_to_pyarrow(ctx: Context, cols: Sequence, names: Sequence[str]):
    """Device columns (QeColumn or DeviceColumn) -> pyarrow.RecordBatch (D2H, host copy owned by
    the returned batch through the Arrow release callback)."""
    import pyarrow as pa

    cc = [c.as_c() if isinstance(c, DeviceColumn) else c for c in cols]
    arr_cols = (N.QeColumn * max(1, len(cc)))(*cc)
    cnames = (C.c_char_p * max(1, len(names)))(*[n.encode() for n in names])
    arr, sch = ArrowArrayC(), ArrowSchemaC()
    N.check(N.lib().qe_batch_export(ctx.handle, arr_cols, len(cc), cnames, C.byref(sch), C.byref(arr)))
    return pa.RecordBatch._import_from_c(C.addressof(arr), C.addressof(sch))


def columns_from_batch(db: DeviceBatch) -> List[N.QeColumn]:
    return [c for c, _ in db.columns()]


_IMPORT_CTX: dict = {}


def prefetch_import(batches: Iterable, ctx: Context, import_ctx: Optional[Context] = None) -> Iterator[DeviceBatch]:
    """Host Arrow RecordBatches -> DeviceBatches, importing one batch ahead (H2D
    overlapped with compute). ScanExec.execute (K:569-571) hands batches to the operators one at a
    time. While the caller's kernels for batch i run on `ctx`'s stream, a worker thread imports
    batch i+1 through `import_ctx`. That ctx has its own HIP stream, so the import's pinned staging
    (8 host threads) and DMA run beside the compute. ctypes releases the GIL during
    qe_batch_import. The import has completed when a batch is yielded. A yielded batch stays
    valid until the caller asks for the next one. Then `ctx` is synchronised and the batch is
    closed, so its blocks are never reused while the caller's kernels still read them."""
    import torch

    if import_ctx is None:  # one import ctx (stream + pinned staging) per compute ctx, kept
        import_ctx = _IMPORT_CTX.get(id(ctx))
        if import_ctx is None:
            with torch.cuda.stream(torch.cuda.Stream(device=ctx.torch_device)):
                import_ctx = _IMPORT_CTX[id(ctx)] = Context.get(ctx.device)
    it = iter(batches)
    first = next(it, None)
    if first is None:
        return
    with ThreadPoolExecutor(max_workers=1) as pool:
        fut = pool.submit(DeviceBatch.from_pyarrow, first, import_ctx)
        while fut is not None:
            db = fut.result()
            nxt = next(it, None)
            fut = pool.submit(DeviceBatch.from_pyarrow, nxt, import_ctx) if nxt is not None else None
            try:
                yield db
            finally:
                ctx.synchronize()
                db.close()
