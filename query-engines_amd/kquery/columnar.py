"""Columnar data model: the reference's L1 layer (kquerydiy/src/Main.kt:19-61, :176-202)
with device-resident Arrow buffers.

* ``ArrowTypes`` / ``Field`` / ``Schema`` / ``RecordBatch`` mirror Main.kt:19-61 (names, the
  ``select`` exactly-one-match rule and its IllegalArgumentException, ``rowCount`` = first
  column's size).
* ``ColumnVector`` is the row-wise interface (``getValue(i)``, ``size()``, Main.kt:24-27).
* ``DeviceColumn`` is the MI355X replacement of ``ArrowFieldVector`` (Main.kt:176-202): an
  Arrow array (values + LSB validity bitmap [+ UTF-8 offsets]) in HBM. ``getValue`` keeps the
  reference's row-wise contract for callers such as ``printQueryResult`` (Main.kt:1344-1353)
  but the operators never use it: they hand whole buffers to the HIP kernels.
* ``HostColumn`` is the reference's CPU ``ArrowFieldVector`` over a pyarrow array (used for
  the CSV plumbing case, config 1).
"""
from __future__ import annotations

import dataclasses
import struct
from typing import Any, List, Optional, Sequence

import numpy as np

from . import native as N


class ArrowTypes:
    """Main.kt:19-22 knows DoubleType and StringType; the rest are build-added."""

    DoubleType = N.TYPE_FLOAT64
    StringType = N.TYPE_UTF8
    Int64Type = N.TYPE_INT64
    Int32Type = N.TYPE_INT32
    UInt8Type = N.TYPE_UINT8
    Date32Type = N.TYPE_DATE32
    BooleanType = N.TYPE_BOOL

    NAMES = {
        N.TYPE_FLOAT64: "FloatingPoint(DOUBLE)",
        N.TYPE_UTF8: "Utf8",
        N.TYPE_INT64: "Int(64, true)",
        N.TYPE_INT32: "Int(32, true)",
        N.TYPE_UINT8: "Int(8, false)",
        N.TYPE_DATE32: "Date(DAY)",
        N.TYPE_BOOL: "Bool",
    }


@dataclasses.dataclass(frozen=True)
class Field:
    """Main.kt:29-34 (every field nullable)."""

    name: str
    dataType: int

    def __repr__(self) -> str:
        return f"Field(name={self.name}, dataType={ArrowTypes.NAMES.get(self.dataType, self.dataType)})"


@dataclasses.dataclass(frozen=True)
class Schema:
    """Main.kt:36-54."""

    fields: tuple

    def __init__(self, fields: Sequence[Field]):
        object.__setattr__(self, "fields", tuple(fields))

    def select(self, names: Sequence[str]) -> "Schema":
        out = []
        for name in names:
            m = [f for f in self.fields if f.name == name]
            if len(m) == 1:
                out.append(m[0])
            else:  # Main.kt:49
                raise N.IllegalArgumentException(N.QE_ERR_INVALID_ARG, f"select: '{name}' matches {len(m)} fields")
        return Schema(out)


class ColumnVector:
    """Main.kt:24-27."""

    def getValue(self, i: int) -> Any:  # noqa: N802 (reference name)
        raise NotImplementedError

    def size(self) -> int:
        raise NotImplementedError


class RecordBatch:
    """Main.kt:56-61."""

    def __init__(self, schema: Schema, fields: List[ColumnVector]):
        self.schema = schema
        self.fields = list(fields)

    def rowCount(self) -> int:  # noqa: N802
        return self.fields[0].size()  # Main.kt:57: first column (raises on zero columns)

    def field(self, i: int) -> ColumnVector:
        return self.fields[i]


# ---------------------------------------------------------------------------------------------
# Device side
# ---------------------------------------------------------------------------------------------
class Context:
    """One qe_ctx per (device, stream): launches go to torch's current stream on that device."""

    _cache: dict = {}

    def __init__(self, device: int = 0, stream: Optional[int] = None):
        import torch

        self.device = device
        self.torch_device = torch.device("cuda", device)
        if stream is None:
            stream = torch.cuda.current_stream(self.torch_device).cuda_stream
        self.stream = stream
        h = N.C.c_void_p()
        N.check(N.lib().qe_ctx_create(device, N.C.c_void_p(stream), N.C.byref(h)))
        self.handle = h

    @classmethod
    def get(cls, device: int = 0) -> "Context":
        import torch

        stream = torch.cuda.current_stream(torch.device("cuda", device)).cuda_stream
        key = (device, stream)
        if key not in cls._cache:
            cls._cache[key] = Context(device, stream)
        return cls._cache[key]

    def synchronize(self) -> None:
        N.check(N.lib().qe_ctx_synchronize(self.handle))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and N._lib is not None:
            try:
                N._lib.qe_ctx_destroy(h)
            except Exception:
                pass


_TORCH_DTYPE = None


def _torch_dtype(type_id: int):
    import torch

    return {
        N.TYPE_INT64: torch.int64,
        N.TYPE_FLOAT64: torch.float64,
        N.TYPE_INT32: torch.int32,
        N.TYPE_DATE32: torch.int32,
        N.TYPE_UINT8: torch.uint8,
        N.TYPE_BOOL: torch.uint8,
        N.TYPE_UTF8: torch.uint8,
    }[type_id]


def _np_dtype(type_id: int):
    return {
        N.TYPE_INT64: np.int64,
        N.TYPE_FLOAT64: np.float64,
        N.TYPE_INT32: np.int32,
        N.TYPE_DATE32: np.int32,
        N.TYPE_UINT8: np.uint8,
    }[type_id]


def bitmap_bytes(n: int) -> int:
    """Validity / boolean bitmap bytes, padded to whole 32-bit words (kernels OR whole words)."""
    return ((n + 31) // 32) * 4


class DeviceCount:
    """A row count that lives in HBM (the selected rows of a stream-ordered selection,
    qe_filter_apply_async): read back once, on first use, after the ctx stream's work."""

    def __init__(self, tensor, ctx: "Context"):
        self.tensor = tensor  # int64 [1] on the device
        self.ctx = ctx
        self._v: Optional[int] = None

    def ptr(self):
        return N.C.c_void_p(self.tensor.data_ptr())

    def get(self) -> int:
        if self._v is None:
            self.ctx.synchronize()
            self._v = int(self.tensor.cpu().item())
        return self._v


class DeviceColumn(ColumnVector):
    """An Arrow array in HBM (offset 0). Replaces ArrowFieldVector (Main.kt:176-202).
    `length` may be pending: a column produced by a stream-ordered selection holds `capacity`
    rows of which the first DeviceCount rows are real; reading `length` resolves it (one sync)."""

    def __init__(self, type_id: int, length: int, values, validity=None, offsets=None, ctx: Optional[Context] = None):
        self.type = type_id
        self._length = int(length)
        self.pending: Optional[DeviceCount] = None
        self.values = values
        self.validity = validity
        self.offsets = offsets
        self.ctx = ctx or Context.get(values.device.index if values is not None else 0)
        self._c = None
        self.max_len = None  # UTF8: a host-known bound on the values' byte lengths (None: unknown)

    @property
    def length(self) -> int:
        if self.pending is not None:
            self._length = self.pending.get()
            self.pending = None
        return self._length

    @length.setter
    def length(self, n: int) -> None:
        self._length = int(n)
        self.pending = None

    @property
    def capacity(self) -> int:
        """Rows held: the length, or the upper bound of a pending one (no sync)."""
        return self._length

    # ---- allocation ------------------------------------------------------------------------
    @classmethod
    def empty(cls, type_id: int, n: int, nullable: bool = False, ctx: Optional[Context] = None) -> "DeviceColumn":
        import torch

        ctx = ctx or Context.get(0)
        dev = ctx.torch_device
        if type_id == N.TYPE_BOOL:
            values = torch.zeros(max(bitmap_bytes(n), 4), dtype=torch.uint8, device=dev)
        elif type_id in N.FIXED_WIDTH:
            values = torch.empty(max(n, 1), dtype=_torch_dtype(type_id), device=dev)
        else:
            raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"cannot allocate type {type_id}")
        validity = torch.zeros(max(bitmap_bytes(n), 4), dtype=torch.uint8, device=dev) if nullable else None
        return cls(type_id, n, values, validity, None, ctx)

    @classmethod
    def from_numpy(cls, type_id: int, values: np.ndarray, valid: Optional[np.ndarray] = None,
                   ctx: Optional[Context] = None) -> "DeviceColumn":
        """Upload host values (+ optional bool validity mask) into HBM."""
        import torch

        ctx = ctx or Context.get(0)
        n = len(values)
        dev = ctx.torch_device
        if type_id == N.TYPE_BOOL:
            bits = np.packbits(np.asarray(values, dtype=bool), bitorder="little")
            buf = np.zeros(max(bitmap_bytes(n), 4), dtype=np.uint8)
            buf[: len(bits)] = bits
            v = torch.from_numpy(buf).to(dev)
        else:
            arr = np.ascontiguousarray(values, dtype=_np_dtype(type_id))
            if n == 0:
                arr = np.zeros(1, dtype=_np_dtype(type_id))
            v = torch.from_numpy(arr).to(dev)
        vb = None
        if valid is not None:
            bits = np.packbits(np.asarray(valid, dtype=bool), bitorder="little")
            buf = np.zeros(max(bitmap_bytes(n), 4), dtype=np.uint8)
            buf[: len(bits)] = bits
            vb = torch.from_numpy(buf).to(dev)
        return cls(type_id, n, v, vb, None, ctx)

    @classmethod
    def from_strings(cls, strings: Sequence[Optional[str]], ctx: Optional[Context] = None) -> "DeviceColumn":
        """UTF-8 column (null entries allowed)."""
        import torch

        ctx = ctx or Context.get(0)
        enc = [s.encode() if s is not None else b"" for s in strings]
        offs = np.zeros(len(enc) + 1, dtype=np.int32)
        offs[1:] = np.cumsum([len(e) for e in enc]) if enc else []
        data = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
        valid = None
        if any(s is None for s in strings):
            bits = np.packbits(np.array([s is not None for s in strings]), bitorder="little")
            buf = np.zeros(max(bitmap_bytes(len(enc)), 4), dtype=np.uint8)
            buf[: len(bits)] = bits
            valid = torch.from_numpy(buf).to(ctx.torch_device)
        return cls(N.TYPE_UTF8, len(enc), torch.from_numpy(data).to(ctx.torch_device), valid,
                   torch.from_numpy(offs).to(ctx.torch_device), ctx)

    # ---- C ABI view ------------------------------------------------------------------------
    def as_c(self, pending_ok: bool = False) -> N.QeColumn:
        """The C view. pending_ok: a pending length stays unresolved and the view holds `capacity`
        rows (for the device-count calls, qe_eval_arith_dlen)."""
        ml = self.max_len if self.type == N.TYPE_UTF8 and self.max_len is not None else 0
        return N.QeColumn(
            self.type,
            int(min(ml, (1 << 31) - 1)),
            self._length if pending_ok else self.length,
            self.validity.data_ptr() if self.validity is not None else None,
            self.values.data_ptr() if self.values is not None else None,
            self.offsets.data_ptr() if self.offsets is not None else None,
        )

    @property
    def nullable(self) -> bool:
        return self.validity is not None

    # ---- host views --------------------------------------------------------------------------
    def valid_mask(self) -> np.ndarray:
        if self.validity is None:
            return np.ones(self.length, dtype=bool)
        bits = self.validity.cpu().numpy()
        return np.unpackbits(bits, bitorder="little")[: self.length].astype(bool)

    def to_numpy(self) -> np.ndarray:
        """Values (nulls keep whatever bits the buffer holds)."""
        if self.type == N.TYPE_BOOL:
            b = self.values.cpu().numpy()
            return np.unpackbits(b, bitorder="little")[: self.length].astype(bool)
        if self.type == N.TYPE_UTF8:
            offs = self.offsets.cpu().numpy()
            data = self.values.cpu().numpy().tobytes()
            return np.array([data[offs[i]:offs[i + 1]].decode() for i in range(self.length)], dtype=object)
        return self.values[: self.length].cpu().numpy()

    def to_pylist(self) -> list:
        vals = self.to_numpy()
        valid = self.valid_mask()
        out = []
        for i in range(self.length):
            if not valid[i]:
                out.append(None)
            elif self.type == N.TYPE_FLOAT64:
                out.append(float(vals[i]))
            elif self.type == N.TYPE_BOOL:
                out.append(bool(vals[i]))
            elif self.type == N.TYPE_UTF8:
                out.append(str(vals[i]))
            else:
                out.append(int(vals[i]))
        return out

    # ---- ColumnVector -----------------------------------------------------------------------
    def getValue(self, i: int) -> Any:  # noqa: N802
        """Row-wise access (Main.kt:178-197): null -> None; one device read per call."""
        if not 0 <= i < self.length:
            raise IndexError(i)
        if self.validity is not None:
            byte = int(self.validity[i >> 3].item())
            if not (byte >> (i & 7)) & 1:
                return None
        if self.type == N.TYPE_FLOAT64:
            return float(self.values[i].item())
        if self.type == N.TYPE_UTF8:
            s, e = (int(x) for x in self.offsets[i:i + 2].cpu().tolist())
            return bytes(self.values[s:e].cpu().numpy()).decode()
        if self.type == N.TYPE_BOOL:
            return bool((int(self.values[i >> 3].item()) >> (i & 7)) & 1)
        return int(self.values[i].item())

    def size(self) -> int:
        return self.length


class HostColumn(ColumnVector):
    """Reference ArrowFieldVector over a pyarrow array (Main.kt:176-202), CPU only.

    Supports Float8 and Utf8 like the reference; any other type raises IllegalStateException
    (Main.kt:195)."""

    def __init__(self, array):
        import pyarrow as pa

        self.array = array
        self._is_f64 = pa.types.is_float64(array.type)
        self._is_utf8 = pa.types.is_string(array.type)

    def getValue(self, i: int) -> Any:  # noqa: N802
        if not self.array[i].is_valid:
            return None
        if self._is_f64:
            return self.array[i].as_py()
        if self._is_utf8:
            return self.array[i].as_py()
        raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"getValue on {self.array.type}")

    def size(self) -> int:
        return len(self.array)


def f64_from_bits(bits: int) -> float:
    return struct.unpack("<d", struct.pack("<q", bits))[0]
