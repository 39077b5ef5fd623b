"""Device hash-aggregate state (qe_hashagg_*): the engine behind HashAggregateExec
(Main.kt:615-651) and the two-phase partial -> merge aggregate of main() (Main.kt:1309-1325).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from . import native as N
from .columnar import Context, DeviceColumn


def output_type(fn: int, input_type: int) -> int:
    if fn in (N.AGG_COUNT, N.AGG_COUNT_STAR):
        return N.TYPE_INT64
    if fn == N.AGG_AVG:
        return N.TYPE_FLOAT64
    return input_type


class HashAggregateState:
    """Owns one qe_hashagg. Keys: ``key_types``; aggregates: (fn, input_type) pairs."""

    def __init__(self, ctx: Context, key_types: Sequence[int], aggs: Sequence[Tuple[int, int]],
                 expected_groups: int = 1024):
        self.ctx = ctx
        self.key_types = list(key_types)
        self.aggs = [(int(f), int(t)) for f, t in aggs]
        kt = (N.C.c_int32 * max(1, len(self.key_types)))(*self.key_types)
        ad = (N.QeAggDesc * max(1, len(self.aggs)))(*[N.QeAggDesc(f, t) for f, t in self.aggs])
        h = N.C.c_void_p()
        N.check(N.lib().qe_hashagg_create(ctx.handle, len(self.key_types), kt, len(self.aggs), ad,
                                          int(expected_groups), N.C.byref(h)))
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None) is not None:
            N.lib().qe_hashagg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- updates --------------------------------------------------------------------------------
    def update(self, keys: Sequence[DeviceColumn], inputs: Sequence[Optional[DeviceColumn]],
               mask: Optional[DeviceColumn] = None) -> None:
        kc = (N.QeColumn * max(1, len(keys)))(*[k.as_c() for k in keys])
        ic = (N.QeColumn * max(1, len(self.aggs)))(
            *[(x.as_c() if x is not None else N.QeColumn()) for x in inputs])
        mc = mask.as_c() if mask is not None else None
        N.check(N.lib().qe_hashagg_update(self.handle, kc, ic, N.C.byref(mc) if mc is not None else None))

    def update_fused(self, cols: Sequence[DeviceColumn], spec: N.QeFusedSpec) -> None:
        cc = (N.QeColumn * len(cols))(*[c.as_c() for c in cols])
        N.check(N.lib().qe_hashagg_update_fused(self.handle, cc, len(cols), N.C.byref(spec)))

    def set_row_base(self, row_base: int) -> None:
        N.check(N.lib().qe_hashagg_set_row_base(self.handle, int(row_base)))

    def last_kernel_time(self):
        """(ms, launches) of the aggregation kernel(s) of the last update (HIP events)."""
        ms = N.C.c_double()
        k = N.C.c_int32()
        N.check(N.lib().qe_hashagg_last_kernel_time(self.handle, N.C.byref(ms), N.C.byref(k)))
        return ms.value, k.value

    def last_kernel_kind(self):
        """(specialized: bool, note) for the last update's aggregation kernel."""
        k = N.C.c_int32()
        buf = N.C.create_string_buffer(512)
        N.check(N.lib().qe_hashagg_last_kernel_kind(self.handle, N.C.byref(k), buf, 512))
        return bool(k.value), buf.value.decode(errors="replace")

    def reset(self) -> None:
        N.check(N.lib().qe_hashagg_reset(self.handle))

    # ---- results ----------------------------------------------------------------------------------
    def num_groups(self) -> int:
        n = N.C.c_int64()
        N.check(N.lib().qe_hashagg_num_groups(self.handle, N.C.byref(n)))
        return n.value

    def finalize(self) -> Tuple[List[DeviceColumn], List[DeviceColumn]]:
        """One output batch (Main.kt:635-650): key columns, aggregate columns."""
        g = self.num_groups()
        keys = [DeviceColumn.empty(t, g, True, ctx=self.ctx) for t in self.key_types]
        aggs = [DeviceColumn.empty(output_type(f, t), g, f not in (N.AGG_COUNT, N.AGG_COUNT_STAR), ctx=self.ctx)
                for f, t in self.aggs]
        kc = (N.QeColumn * max(1, len(keys)))(*[k.as_c() for k in keys])
        ac = (N.QeColumn * max(1, len(aggs)))(*[a.as_c() for a in aggs])
        out = N.C.c_int64()
        N.check(N.lib().qe_hashagg_finalize(self.handle, kc, ac, N.C.byref(out)))
        for c in keys + aggs:
            c.length = out.value
        return keys, aggs

    # ---- partial records (exchange) -----------------------------------------------------------------
    def record_bytes(self) -> int:
        n = N.C.c_int64()
        N.check(N.lib().qe_hashagg_record_bytes(self.handle, N.C.byref(n)))
        return n.value

    def export_counts(self, nparts: int) -> List[int]:
        arr = (N.C.c_int64 * nparts)()
        N.check(N.lib().qe_hashagg_export_counts(self.handle, nparts, arr))
        return list(arr)

    def export(self, nparts: int):
        """-> (uint8 device tensor of records, per-partition counts)."""
        import torch

        counts = self.export_counts(nparts)
        rb = self.record_bytes()
        buf = torch.empty(max(1, sum(counts) * rb), dtype=torch.uint8, device=self.ctx.torch_device)
        N.check(N.lib().qe_hashagg_export(self.handle, nparts, N.C.c_void_p(buf.data_ptr())))
        return buf[: sum(counts) * rb], counts

    def import_records(self, records, nrecords: int) -> None:
        if nrecords == 0:
            return
        N.check(N.lib().qe_hashagg_import(self.handle, N.C.c_void_p(records.data_ptr()), int(nrecords)))
