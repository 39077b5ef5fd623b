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
    if fn == N.AGG_AVG or input_type == N.TYPE_FLOAT64:
        return N.TYPE_FLOAT64
    return N.TYPE_INT64  # integer inputs of every width accumulate (and come out) as int64


_KEY_BITS = {N.TYPE_INT32: 32, N.TYPE_DATE32: 32, N.TYPE_UINT8: 8}


def packable(key_types) -> bool:
    """Whether qe_hashagg packs these keys itself (one int64/fp64 key, or narrow keys whose values
    plus null bits fit 63 bits — qe_hashagg_create's rule)."""
    if len(key_types) == 0:
        return True
    if len(key_types) == 1 and key_types[0] in (N.TYPE_INT64, N.TYPE_FLOAT64):
        return True
    if any(t not in _KEY_BITS for t in key_types) or len(key_types) > N.MAX_KEYS:
        return False
    return sum(_KEY_BITS[t] + 1 for t in key_types) <= 63


def _carve(ctx: Context, n: int, specs) -> List[DeviceColumn]:
    """Fixed-width output columns of `n` rows from two device allocations (values; validity
    bitmaps), split with one unbind each — per-column slicing costs more host time than the
    finalize kernel. Validity is left uninitialised: qe_hashagg_finalize writes whole bitmaps."""
    import torch

    from .columnar import _torch_dtype, bitmap_bytes

    dev = ctx.torch_device
    vals = torch.empty((len(specs), max(n, 1)), dtype=torch.int64, device=dev).unbind(0)
    nv = sum(1 for _, nullable in specs if nullable)
    bits = torch.empty((max(nv, 1), max(bitmap_bytes(n), 4)), dtype=torch.uint8, device=dev).unbind(0) if nv else []
    out, b = [], 0
    for (t, nullable), v in zip(specs, vals):
        if t not in (N.TYPE_INT64, N.TYPE_FLOAT64):
            v = v.view(_torch_dtype(t))  # narrow key types: a prefix of the int64 row
        elif t == N.TYPE_FLOAT64:
            v = v.view(torch.float64)
        out.append(DeviceColumn(t, n, v, bits[b] if nullable else None, None, ctx))
        b += 1 if nullable else 0
    return out


def _trim(c: DeviceColumn, n: int) -> DeviceColumn:
    """The first n rows of a carved output column (views of its buffers)."""
    from .columnar import bitmap_bytes

    vb = c.validity[: max(bitmap_bytes(n), 4)] if c.validity is not None else None
    if c.type == N.TYPE_UTF8:
        return DeviceColumn(c.type, n, c.values, vb, c.offsets[: n + 1], c.ctx)
    if c.type == N.TYPE_BOOL:
        return DeviceColumn(c.type, n, c.values[: max(bitmap_bytes(n), 4)], vb, None, c.ctx)
    return DeviceColumn(c.type, n, c.values[: max(n, 1)], vb, None, c.ctx)


def _order_for_reader(ctx: Context) -> None:
    """Stream-ordered results (qe_hashagg_finalize) are read through torch on its current stream:
    when that is not the ctx's stream, wait for the ctx's queued work first."""
    import torch

    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)  # the same handle, without a Stream object
    cur = raw(ctx.device) if raw is not None else torch.cuda.current_stream(ctx.torch_device).cuda_stream
    if cur != ctx.stream:
        ctx.synchronize()


def dictionary_keys(key_types) -> Optional[int]:
    """None when qe_hashagg groups by these keys directly; otherwise the column slots a fused update
    adds for them: the key columns themselves (their codes take the UTF-8 slots in place), plus one
    for key-tuple codes when the coded keys still do not pack into 63 bits."""
    member = [N.TYPE_INT32 if t == N.TYPE_UTF8 else t for t in key_types]
    if len(key_types) == 1 and key_types[0] == N.TYPE_UTF8:
        member = [N.TYPE_INT64]  # a lone UTF-8 key: wide codes
    if not packable(member):
        return len(key_types) + 1
    return len(key_types) if N.TYPE_UTF8 in key_types else None


class HashAggregateState:
    """Owns one qe_hashagg. Keys: ``key_types`` (UTF-8 and key lists that do not pack included: the
    C state keeps their dictionaries); aggregates: (fn, input_type) pairs."""

    def __init__(self, ctx: Context, key_types: Sequence[int], aggs: Sequence[Tuple[int, int]],
                 expected_groups: int = 1024, async_update: bool = False, deterministic: bool = False,
                 fast_fp64: bool = False):
        """``async_update``: stream-ordered updates (qe_hashagg_set_async) — an update returns once
        its kernel is queued and is checked by the next call on the state (finalize, num_groups,
        the next update), which may re-read the update's columns; the state holds a reference to
        them until the next update or reset.
        fp64 SUM / AVG are exact by default (the correctly rounded exact sum, bit-identical run to
        run, like the reference's ordered row loop with exact arithmetic); ``deterministic`` names
        that default (QE_HASHAGG_DETERMINISTIC). ``fast_fp64``: plain fp64 atomics instead
        (QE_HASHAGG_FAST_FP64), without the 1e-9 guarantee for cancelling groups."""
        self.ctx = ctx
        self.expected_groups = int(expected_groups)
        self.key_types = list(key_types)
        self.aggs = [(int(f), int(t)) for f, t in aggs]
        kt = (N.C.c_int32 * max(1, len(self.key_types)))(*self.key_types)
        ad = (N.QeAggDesc * max(1, len(self.aggs)))(*[N.QeAggDesc(f, t) for f, t in self.aggs])
        h = N.C.c_void_p()
        N.check(N.lib().qe_hashagg_create_ex(ctx.handle, len(self.key_types), kt, len(self.aggs), ad,
                                             int(expected_groups),
                                             (N.HASHAGG_DETERMINISTIC if deterministic else 0) |
                                             (N.HASHAGG_FAST_FP64 if fast_fp64 else 0),
                                             N.C.byref(h)))
        self.deterministic = not fast_fp64
        self.handle = h
        kind, nd = N.C.c_int32(), N.C.c_int32()
        dt = (N.C.c_int32 * N.MAX_KEYS)()
        N.check(N.lib().qe_hashagg_key_layout(h, N.C.byref(kind), N.C.byref(nd), dt))
        self.key_layout = kind.value  # 0: raw key words, 1: string codes, 2: key-tuple codes
        self.device_key_types = list(dt)[: nd.value]
        self._out_rows = max(1, 2 * self.expected_groups)  # finalize's first output sizing guess
        self.async_update = bool(async_update)
        self._held = None  # async: the last update's columns, alive until the state settles it
        if async_update:
            N.check(N.lib().qe_hashagg_set_async(h, 1))

    def close(self) -> None:
        if getattr(self, "handle", None) is not None:
            N.lib().qe_hashagg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bind_key_dict(self, key: int, dictionary) -> None:
        """Key `key` (INT32, or a lone INT64 key of wide codes) takes codes the caller encodes with
        `dictionary` (kquery.strdict.StringDictionary): the state decodes through it at finalize
        (the key comes out as UTF-8) and merges / exchanges by content (qe_hashagg_bind_key_dict)."""
        N.check(N.lib().qe_hashagg_bind_key_dict(self.handle, int(key), dictionary.handle))
        self.key_types[key] = N.TYPE_UTF8
        self._bound = getattr(self, "_bound", []) + [dictionary]  # it must outlive the state
        self.key_layout = 1

    @property
    def keyed_by_dictionary(self) -> bool:
        """The table groups by dictionary codes local to this state: partials move by key content."""
        return self.key_layout != 0

    # ---- updates --------------------------------------------------------------------------------
    def update(self, keys: Sequence[DeviceColumn], inputs: Sequence[Optional[DeviceColumn]],
               mask: Optional[DeviceColumn] = None) -> None:
        """Keys as declared (UTF-8 columns included). A COUNT(*) input may be any column of the batch:
        with no keys and no other inputs its length is the row count (qe_hashagg_update)."""
        kc = (N.QeColumn * max(1, len(keys)))(*[k.as_c() for k in keys])
        ic = (N.QeColumn * max(1, len(self.aggs)))(
            *[(x.as_c() if x is not None else N.QeColumn()) for x in inputs])
        mc = mask.as_c() if mask is not None else None
        N.check(N.lib().qe_hashagg_update(self.handle, kc, ic, N.C.byref(mc) if mc is not None else None))
        if self.async_update:  # a pending update may re-read its columns when it is settled
            self._held = (keys, inputs, mask)

    def update_fused(self, cols: Sequence[DeviceColumn], spec: N.QeFusedSpec,
                     key_cols: Optional[Sequence[DeviceColumn]] = None) -> None:
        """Dictionary-keyed states take the declared key columns in `key_cols`: they join the launch
        as extra column slots after `cols` (the C state encodes them; codes of rows the predicate
        drops never form a group)."""
        cols = list(cols)
        if self.keyed_by_dictionary:
            if key_cols is None:
                raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED,
                                              "fused update with dictionary-encoded keys needs the key columns")
            if len(cols) + dictionary_keys(self.key_types) > N.MAX_COLS:
                raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"fused plan takes at most {N.MAX_COLS} columns")
            spec = N.QeFusedSpec.from_buffer_copy(spec)
            for k in range(len(key_cols)):
                spec.key_cols[k] = len(cols) + k
            cols += list(key_cols)
        cc = (N.QeColumn * len(cols))(*[c.as_c() for c in cols])
        N.check(N.lib().qe_hashagg_update_fused(self.handle, cc, len(cols), N.C.byref(spec)))
        if self.async_update:  # a pending update may re-read its columns when it is settled
            self._held = cols

    def slot_capacity(self, world: int) -> int:
        """Default records per slot of a `world`-rank exchange (qe_hashagg_slot_capacity)."""
        cap = N.C.c_int64()
        N.check(N.lib().qe_hashagg_slot_capacity(self.handle, int(world), N.C.byref(cap)))
        return cap.value

    def set_row_base(self, row_base: int) -> None:
        N.check(N.lib().qe_hashagg_set_row_base(self.handle, int(row_base)))

    def last_kernel_time(self):
        """(ms, launches) of the aggregation kernel(s) of the last update (HIP events)."""
        ms = N.C.c_double()
        k = N.C.c_int32()
        N.check(N.lib().qe_hashagg_last_kernel_time(self.handle, N.C.byref(ms), N.C.byref(k)))
        return ms.value, k.value

    def last_kernel_signature(self) -> str:
        """Hex signature of the last update's aggregation launch (kernel compile key + shape)."""
        sig = N.C.c_uint64()
        N.check(N.lib().qe_hashagg_last_kernel_signature(self.handle, N.C.byref(sig)))
        return f"{sig.value:016x}"

    def last_kernel_kind(self):
        """(specialized: bool, note) for the last update's aggregation kernel."""
        k = N.C.c_int32()
        buf = N.C.create_string_buffer(512)
        N.check(N.lib().qe_hashagg_last_kernel_kind(self.handle, N.C.byref(k), buf, 512))
        return bool(k.value), buf.value.decode(errors="replace")

    def reset(self) -> None:
        N.check(N.lib().qe_hashagg_reset(self.handle))
        # _held stays: the discarded update's kernel may still be reading those columns on the
        # ctx stream. The next update replaces it after queueing behind that kernel.

    # ---- results ----------------------------------------------------------------------------------
    def num_groups(self) -> int:
        n = N.C.c_int64()
        N.check(N.lib().qe_hashagg_num_groups(self.handle, N.C.byref(n)))
        return n.value

    def prepare_output(self) -> None:
        """Carve the next finalize's output columns now (at the last result's size), so that the
        host work is done before a call that waits for the device (kquery.exchange calls it
        before the import's read-back)."""
        if getattr(self, "_stash", None) is None and N.TYPE_UTF8 not in self.key_types:
            self._stash = self._carve_c(self._out_rows)

    def _carve_c(self, rows: int, key_bytes=None):
        import torch

        from .columnar import bitmap_bytes

        specs = ([(t, True) for t in self.key_types if t not in (N.TYPE_UTF8, N.TYPE_BOOL)] +
                 [(output_type(f, t), f not in (N.AGG_COUNT, N.AGG_COUNT_STAR)) for f, t in self.aggs])
        fixed = _carve(self.ctx, rows, specs) if specs else []
        dev = self.ctx.torch_device
        keys, it = [], iter(fixed)
        for k, t in enumerate(self.key_types):
            if t == N.TYPE_UTF8:  # offsets, values of the size finalize_sizes reported, validity
                nb = int(key_bytes[k]) if key_bytes is not None else 7 * rows
                keys.append(DeviceColumn(N.TYPE_UTF8, rows, torch.empty(max(1, nb), dtype=torch.uint8, device=dev),
                                         torch.empty(max(bitmap_bytes(rows), 4), dtype=torch.uint8, device=dev),
                                         torch.empty(rows + 1, dtype=torch.int32, device=dev), self.ctx))
            elif t == N.TYPE_BOOL:
                keys.append(DeviceColumn.empty(N.TYPE_BOOL, rows, True, ctx=self.ctx))
            else:
                keys.append(next(it))
        cols = keys + list(it)
        nk = len(self.key_types)
        kc = (N.QeColumn * max(1, nk))(*[k.as_c() for k in cols[:nk]])
        ac = (N.QeColumn * max(1, len(cols) - nk))(*[a.as_c() for a in cols[nk:]])
        return rows, cols, kc, ac

    def finalize(self) -> Tuple[List[DeviceColumn], List[DeviceColumn]]:
        """One output batch (Main.kt:635-650): key columns (as declared, UTF-8 included), aggregate
        columns.

        The outputs are carved before the call (or earlier, prepare_output), at the size of the
        last result (or 2x the expected groups), so that the host work is done before
        qe_hashagg_finalize waits for the aggregation; a larger result (QE_ERR_CAPACITY, with the
        exact count) carves again. UTF-8 keys are sized first (qe_hashagg_finalize_sizes)."""
        nk = len(self.key_types)
        out = N.C.c_int64(-1)
        stash, self._stash = getattr(self, "_stash", None), None
        if N.TYPE_UTF8 in self.key_types:
            # keys that are their own codes have a per-group byte bound: carve at the last result's
            # size while the update still runs, and let finalize report a larger count; otherwise
            # size them first (qe_hashagg_finalize_sizes, which waits for the update)
            bound = N.C.c_int64()
            packed = True
            for k, t in enumerate(self.key_types):
                if t == N.TYPE_UTF8:
                    N.check(N.lib().qe_hashagg_key_bytes_bound(self.handle, k, N.C.byref(bound)))
                    packed = packed and bound.value == 7
            if packed:
                stash = self._carve_c(self._out_rows)
            else:
                g = N.C.c_int64()
                kb = (N.C.c_int64 * max(1, nk))()
                N.check(N.lib().qe_hashagg_finalize_sizes(self.handle, N.C.byref(g), kb))
                stash = self._carve_c(max(1, g.value), list(kb))
        while True:
            rows, cols, kc, ac = stash if stash is not None else self._carve_c(self._out_rows)
            stash = None
            st = N.lib().qe_hashagg_finalize(self.handle, kc, ac, N.C.byref(out))
            if st == N.QE_ERR_CAPACITY and out.value > rows:
                self._out_rows = out.value
                continue
            N.check(st)
            break
        g = out.value
        self._out_rows = max(1, g)
        _order_for_reader(self.ctx)
        if g != rows:
            cols = [_trim(c, g) for c in cols]
        return cols[:nk], cols[nk:]

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
        """-> (uint8 device tensor of records, per-partition counts). Raw key words: refused for a
        dictionary-keyed state (export_keyed)."""
        import torch

        counts = self.export_counts(nparts)
        rb = self.record_bytes()
        buf = torch.empty(max(1, sum(counts) * rb), dtype=torch.uint8, device=self.ctx.torch_device)
        N.check(N.lib().qe_hashagg_export(self.handle, nparts, N.C.c_void_p(buf.data_ptr())))
        return buf[: sum(counts) * rb], counts

    def slot_bytes(self, slot_records: int) -> int:
        return N.SLOT_HEADER + int(slot_records) * self.record_bytes()

    def export_slots(self, nparts: int, slot_records: int):
        """-> uint8 device tensor of `nparts` fixed-capacity slots (qe_hashagg_export_slots):
        no host synchronisation, so the all-to-all can follow the aggregation kernel directly."""
        import torch

        buf = torch.empty(nparts * self.slot_bytes(slot_records), dtype=torch.uint8, device=self.ctx.torch_device)
        N.check(N.lib().qe_hashagg_export_slots(self.handle, int(nparts), int(slot_records),
                                                N.C.c_void_p(buf.data_ptr())))
        return buf

    def import_slots(self, slots, nslots: int, slot_records: int) -> Optional[int]:
        """Merges received slots; returns the records merged, or None when some sender's
        partition exceeded the slot capacity (nothing merged; the same on every rank)."""
        mx, n = N.C.c_int64(), N.C.c_int64()
        N.check(N.lib().qe_hashagg_import_slots(self.handle, N.C.c_void_p(slots.data_ptr()), int(nslots),
                                                int(slot_records), N.C.byref(mx), N.C.byref(n)))
        return None if mx.value > slot_records else n.value

    def import_records(self, records, nrecords: int) -> None:
        if nrecords == 0:
            return
        N.check(N.lib().qe_hashagg_import(self.handle, N.C.c_void_p(records.data_ptr()), int(nrecords)))

    # ---- partials by key content (every state; the only form for dictionary-keyed ones) -------------
    def export_keyed(self, nparts: int):
        """-> (uint8 device tensor of `nparts` keyed blocks back to back, their sizes)
        (qe_hashagg_export_keyed_sizes + qe_hashagg_export_keyed)."""
        import torch

        sizes = (N.C.c_int64 * nparts)()
        N.check(N.lib().qe_hashagg_export_keyed_sizes(self.handle, int(nparts), sizes))
        sizes = list(sizes)
        buf = torch.empty(max(1, sum(sizes)), dtype=torch.uint8, device=self.ctx.torch_device)
        N.check(N.lib().qe_hashagg_export_keyed(self.handle, int(nparts), N.C.c_void_p(buf.data_ptr())))
        return buf, sizes

    def import_keyed(self, blocks, sizes: Sequence[int]) -> int:
        """Merges keyed blocks (packed back to back, `sizes` bytes each) re-encoding their keys into
        this state's dictionaries; returns the records merged."""
        import numpy as np

        n = len(sizes)
        arr = (N.C.c_int64 * max(1, n))(*[int(x) for x in sizes])
        N.check(N.lib().qe_hashagg_import_keyed(self.handle, N.C.c_void_p(blocks.data_ptr()), n, arr))
        recs, off = 0, 0
        for sz in sizes:  # each block's header word 1 is its record count
            if sz:
                recs += int(np.frombuffer(blocks[off + 8: off + 16].cpu().numpy().tobytes(), dtype=np.int64)[0])
            off += int(sz)
        return recs

    def merge(self, other: "HashAggregateState") -> None:
        """Every group of `other` merged into this state (qe_hashagg_merge: by key content when
        either is dictionary-keyed) — main()'s partial -> final merge (Main.kt:1314-1325)."""
        N.check(N.lib().qe_hashagg_merge(self.handle, other.handle))
