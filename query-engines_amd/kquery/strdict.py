"""Device string dictionary (qe_strdict_*): UTF-8 group keys for HashAggregateExec.

The reference keys its HashMap by ``String(bytes)`` (Main.kt:620-627) and compares keys by
content. Here every distinct byte string gets a dense int32 code on the device; the hash
aggregate groups by codes and finalize decodes them back to strings. A ``wide`` dictionary gives
int64 codes instead: a key of at most 7 bytes is packed into its own code (no dictionary work —
the reference's VendorID keys), longer keys get 2^62 | their dictionary code.
"""
from __future__ import annotations

from . import native as N
from .columnar import Context, DeviceColumn


class StringDictionary:
    def __init__(self, ctx: Context, expected_distinct: int = 1024, wide: bool = False):
        self.ctx = ctx
        self.wide = bool(wide)
        self.code_type = N.TYPE_INT64 if self.wide else N.TYPE_INT32
        self.expected_distinct = int(expected_distinct)
        self._handle = None
        if not self.wide:
            self._create()

    def _create(self):
        h = N.C.c_void_p()
        N.check(N.lib().qe_strdict_create(self.ctx.handle, self.expected_distinct, N.C.byref(h)))
        self._handle = h
        return h

    @property
    def handle(self):
        """The device dictionary; a wide one is created on its first long key (short keys are their
        own codes and never need it)."""
        return self._handle if self._handle is not None else self._create()

    def close(self) -> None:
        if getattr(self, "_handle", None) is not None:
            N.lib().qe_strdict_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        if self._handle is None:
            return 0
        n = N.C.c_int64()
        N.check(N.lib().qe_strdict_size(self.handle, N.C.byref(n)))
        return n.value

    def encode(self, col: DeviceColumn) -> DeviceColumn:
        """UTF8 column -> INT32 codes, or wide INT64 codes (nulls stay null)."""
        if col.type != N.TYPE_UTF8:
            raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"string dictionary input type {col.type}")
        out = DeviceColumn.empty(self.code_type, col.length, col.nullable, ctx=self.ctx)
        ic, oc = col.as_c(), out.as_c()
        if self.wide and col.max_len is not None and col.max_len <= 7:
            # every value is its own code: one stream-ordered kernel, no dictionary, no host round trip
            N.check(N.lib().qe_strdict_encode_packed(self.ctx.handle, N.C.byref(ic), N.C.byref(oc)))
        else:
            N.check(N.lib().qe_strdict_encode(self.handle, N.C.byref(ic), N.C.byref(oc)))
        return out

    def decode(self, codes: DeviceColumn, trusted: bool = False) -> DeviceColumn:
        """INT32 / wide INT64 codes -> UTF8 column. ``trusted``: codes this dictionary produced; wide
        codes are then decoded without a host round trip while every key is packed."""
        import torch

        cc = codes.as_c()
        if trusted and self.wide and self.size() == 0 and codes.length < (1 << 28):
            dev = self.ctx.torch_device
            n = codes.length
            out = DeviceColumn(N.TYPE_UTF8, n, torch.empty(max(1, 7 * n), dtype=torch.uint8, device=dev),
                               codes.validity.clone() if codes.validity is not None else None,
                               torch.empty(n + 1, dtype=torch.int32, device=dev), self.ctx)
            oc = out.as_c()
            N.check(N.lib().qe_strdict_decode_packed(self.ctx.handle, N.C.byref(cc), N.C.byref(oc)))
            return out
        nbytes = N.C.c_int64()
        N.check(N.lib().qe_strdict_decode_bytes(self.handle, N.C.byref(cc), N.C.byref(nbytes)))
        dev = self.ctx.torch_device
        n = codes.length
        out = DeviceColumn(N.TYPE_UTF8, n, torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=dev),
                           codes.validity.clone() if codes.validity is not None else None,
                           torch.empty(n + 1, dtype=torch.int32, device=dev), self.ctx)
        oc = out.as_c()
        N.check(N.lib().qe_strdict_decode(self.handle, N.C.byref(cc), N.C.byref(oc)))
        return out

    def encode_tuple(self, cols) -> DeviceColumn:
        """Composite key columns (fixed-width / BOOL, nullable) -> INT32 tuple codes (non-null)."""
        n = cols[0].length
        out = DeviceColumn.empty(N.TYPE_INT32, n, False, ctx=self.ctx)
        kc = (N.QeColumn * len(cols))(*[c.as_c() for c in cols])
        oc = out.as_c()
        N.check(N.lib().qe_strdict_encode_tuple(self.handle, kc, len(cols), N.C.byref(oc)))
        return out

    def decode_tuple(self, codes: DeviceColumn, types) -> list:
        outs = [DeviceColumn.empty(t, codes.length, True, ctx=self.ctx) for t in types]
        cc = codes.as_c()
        oc = (N.QeColumn * len(outs))(*[o.as_c() for o in outs])
        N.check(N.lib().qe_strdict_decode_tuple(self.handle, N.C.byref(cc), len(outs), oc))
        return outs
