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


def _device_column(ctx, type_id: int, vals, valid) -> DeviceColumn:
    """DeviceColumn from int64 device values (narrowed to `type_id`) and a bool validity tensor."""
    import torch

    from .columnar import bitmap_bytes

    n = vals.numel()
    dt = {N.TYPE_INT32: torch.int32, N.TYPE_DATE32: torch.int32, N.TYPE_UINT8: torch.uint8,
          N.TYPE_INT64: torch.int64}[type_id]
    v = vals.to(dt).contiguous() if n else torch.zeros(1, dtype=dt, device=vals.device)
    bits = torch.zeros(max(bitmap_bytes(n), 4) * 8, dtype=torch.uint8, device=vals.device)
    bits[:n] = valid.to(torch.uint8)
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=vals.device)
    vb = (bits.view(-1, 8) * w).sum(dim=1).to(torch.uint8)
    return DeviceColumn(type_id, n, v, vb, None, ctx)


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

    v = c.values[: max(n, 1)]
    vb = c.validity[: max(bitmap_bytes(n), 4)] if c.validity is not None else None
    return DeviceColumn(c.type, n, v, vb, None, c.ctx)


def _order_for_reader(ctx: Context) -> None:
    """Stream-ordered results (qe_hashagg_finalize) are read through torch on its current stream:
    when that is not the ctx's stream, wait for the ctx's queued work first."""
    import torch

    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)  # the same handle, without a Stream object
    cur = raw(ctx.device) if raw is not None else torch.cuda.current_stream(ctx.torch_device).cuda_stream
    if cur != ctx.stream:
        ctx.synchronize()


def dictionary_keys(key_types) -> Optional[int]:
    """None when qe_hashagg groups by these keys directly; otherwise the number of device key
    columns the dictionaries turn them into (UTF-8 keys -> one int32 code each; a key set that
    does not pack -> one tuple code)."""
    member = [N.TYPE_INT32 if t == N.TYPE_UTF8 else t for t in key_types]
    if not packable(member):
        return 1
    return len(member) if N.TYPE_UTF8 in key_types else None


class HashAggregateState:
    """Owns one qe_hashagg. Keys: ``key_types``; aggregates: (fn, input_type) pairs."""

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
        from .strdict import StringDictionary

        self.ctx = ctx
        self.expected_groups = int(expected_groups)
        self.key_types = list(key_types)
        self.aggs = [(int(f), int(t)) for f, t in aggs]
        # UTF-8 keys: grouped by their dictionary code, decoded in finalize. A lone UTF-8 key takes
        # wide INT64 codes (keys of up to 7 bytes packed in place, no dictionary traffic); in a
        # key set, INT32 codes keep the set packable into 63 bits
        wide = len(self.key_types) == 1
        self.dicts = {i: StringDictionary(ctx, expected_groups, wide=wide) for i, t in enumerate(self.key_types)
                      if t == N.TYPE_UTF8}
        self.member_types = [self.dicts[i].code_type if t == N.TYPE_UTF8 else t for i, t in enumerate(self.key_types)]
        # key sets that do not pack into 63 bits group by one code per distinct key tuple
        self.tuple_dict = None
        if not packable(self.member_types):
            if len(self.member_types) > N.MAX_KEYS:
                raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"at most {N.MAX_KEYS} group keys")
            self.tuple_dict = StringDictionary(ctx, expected_groups)
        self.device_key_types = [N.TYPE_INT32] if self.tuple_dict is not None else list(self.member_types)
        kt = (N.C.c_int32 * max(1, len(self.device_key_types)))(*self.device_key_types)
        ad = (N.QeAggDesc * max(1, len(self.aggs)))(*[N.QeAggDesc(f, t) for f, t in self.aggs])
        h = N.C.c_void_p()
        N.check(N.lib().qe_hashagg_create_ex(ctx.handle, len(self.device_key_types), kt, len(self.aggs), ad,
                                             int(expected_groups),
                                             (N.HASHAGG_DETERMINISTIC if deterministic else 0) |
                                             (N.HASHAGG_FAST_FP64 if fast_fp64 else 0),
                                             N.C.byref(h)))
        self.deterministic = not fast_fp64
        self.handle = h
        self._out_rows = max(1, 2 * self.expected_groups)  # finalize's first output sizing guess
        self.async_update = bool(async_update)
        self._held = None  # async: the last update's columns, alive until the state settles it
        if async_update:
            N.check(N.lib().qe_hashagg_set_async(h, 1))

    def close(self) -> None:
        for d in getattr(self, "dicts", {}).values():
            d.close()
        if getattr(self, "tuple_dict", None) is not None:
            self.tuple_dict.close()
        if getattr(self, "handle", None) is not None:
            N.lib().qe_hashagg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- updates --------------------------------------------------------------------------------
    def device_keys(self, keys: Sequence[DeviceColumn]) -> List[DeviceColumn]:
        """The key columns qe_hashagg groups by: dictionary codes for UTF-8 keys / key tuples."""
        keys = [self.dicts[i].encode(k) if i in self.dicts else k for i, k in enumerate(keys)]
        if self.tuple_dict is not None:
            keys = [self.tuple_dict.encode_tuple(keys)]
        return keys

    def update(self, keys: Sequence[DeviceColumn], inputs: Sequence[Optional[DeviceColumn]],
               mask: Optional[DeviceColumn] = None) -> None:
        """A COUNT(*) input may be any column of the batch: with no keys and no other inputs its
        length is the row count (qe_hashagg_update)."""
        keys = self.device_keys(keys)
        kc = (N.QeColumn * max(1, len(keys)))(*[k.as_c() for k in keys])
        ic = (N.QeColumn * max(1, len(self.aggs)))(
            *[(x.as_c() if x is not None else N.QeColumn()) for x in inputs])
        mc = mask.as_c() if mask is not None else None
        N.check(N.lib().qe_hashagg_update(self.handle, kc, ic, N.C.byref(mc) if mc is not None else None))
        if self.async_update:  # a pending update may re-read its columns when it is settled
            self._held = (keys, inputs, mask)

    def update_fused(self, cols: Sequence[DeviceColumn], spec: N.QeFusedSpec,
                     key_cols: Optional[Sequence[DeviceColumn]] = None) -> None:
        """Dictionary-keyed states take the original key columns in `key_cols`: they are encoded
        (over every row; codes of rows the predicate drops never form a group) and their codes
        join the fused launch as extra column slots after `cols`."""
        cols = list(cols)
        if self.keyed_by_dictionary:
            if key_cols is None:
                raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED,
                                              "fused update with dictionary-encoded keys needs the key columns")
            codes = self.device_keys(key_cols)
            if len(cols) + len(codes) > N.MAX_COLS:
                raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"fused plan takes at most {N.MAX_COLS} columns")
            spec = N.QeFusedSpec.from_buffer_copy(spec)
            for k in range(len(codes)):
                spec.key_cols[k] = len(cols) + k
            cols += codes
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
        if getattr(self, "_stash", None) is None:
            self._stash = self._carve_c(self._out_rows)

    def _carve_c(self, rows: int):
        specs = ([(t, True) for t in self.device_key_types] +
                 [(output_type(f, t), f not in (N.AGG_COUNT, N.AGG_COUNT_STAR)) for f, t in self.aggs])
        nk = len(self.device_key_types)
        cols = _carve(self.ctx, rows, specs)
        kc = (N.QeColumn * max(1, nk))(*[k.as_c() for k in cols[:nk]])
        ac = (N.QeColumn * max(1, len(cols) - nk))(*[a.as_c() for a in cols[nk:]])
        return rows, cols, kc, ac

    def finalize(self) -> Tuple[List[DeviceColumn], List[DeviceColumn]]:
        """One output batch (Main.kt:635-650): key columns, aggregate columns.

        The outputs are carved before the call (or earlier, prepare_output), at the size of the
        last result (or 2x the expected groups), so that the host work is done before
        qe_hashagg_finalize waits for the aggregation; a larger result (QE_ERR_CAPACITY, with the
        exact count) carves again."""
        nk = len(self.device_key_types)
        out = N.C.c_int64(-1)
        stash, self._stash = getattr(self, "_stash", None), None
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
        keys, aggs = cols[:nk], cols[nk:]
        if self.tuple_dict is not None:
            keys = self.tuple_dict.decode_tuple(keys[0], self.member_types)
        keys = [self.dicts[i].decode(k, trusted=True) if i in self.dicts else k for i, k in enumerate(keys)]
        return keys, aggs

    # ---- partial records (exchange) -----------------------------------------------------------------
    def record_bytes(self) -> int:
        n = N.C.c_int64()
        N.check(N.lib().qe_hashagg_record_bytes(self.handle, N.C.byref(n)))
        return n.value

    def _check_exportable(self) -> None:
        if self.dicts or self.tuple_dict is not None:  # codes are local to this state's dictionary
            raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED,
                                          "dictionary-keyed partials move by key content: use "
                                          "kquery.exchange.exchange_partials (export_all / import_keyed)")

    # ---- dictionary-keyed states: keys travel as their content (kquery/exchange.py) -----------------
    @property
    def keyed_by_dictionary(self) -> bool:
        return bool(self.dicts) or self.tuple_dict is not None

    def _wide_key(self) -> bool:
        """One INT64 device key (a lone UTF-8 key's wide codes): records carry it whole, with the
        null group flagged in the record's second word, instead of packed narrow keys."""
        return self.device_key_types == [N.TYPE_INT64]

    def _packing(self):
        """(shift, nullbit, width) per device key, as qe_hashagg_create packs narrow keys."""
        if self._wide_key():
            return []
        out, bit = [], 0
        for t in self.device_key_types:
            w = _KEY_BITS[t]
            out.append((bit, bit + w, w))
            bit += w + 1
        return out

    def record_key_columns(self, records, n: int) -> List[DeviceColumn]:
        """The original key columns (UTF8 included) of `n` exported records of this state."""
        import torch

        if n == 0:
            return self._empty_keys()
        rec = records[: n * self.record_bytes()].view(torch.int64).view(n, -1)
        packed = rec[:, 0]
        members = []
        if self._wide_key():  # one INT64 key (wide string codes): the key word and the null flag
            members.append(_device_column(self.ctx, N.TYPE_INT64, packed, rec[:, 1] == 0))
        for (shift, nullbit, w), t in zip(self._packing(), self.device_key_types):
            vals = (packed >> shift) & ((1 << w) - 1)
            valid = ((packed >> nullbit) & 1) == 0
            members.append(_device_column(self.ctx, t, vals, valid))
        if self.tuple_dict is not None:
            members = self.tuple_dict.decode_tuple(members[0], self.member_types)
        return [self.dicts[i].decode(k) if i in self.dicts else k for i, k in enumerate(members)]

    def _empty_keys(self) -> List[DeviceColumn]:
        import torch

        out = []
        for t in self.key_types:
            if t == N.TYPE_UTF8:
                out.append(DeviceColumn(N.TYPE_UTF8, 0, torch.zeros(1, dtype=torch.uint8, device=self.ctx.torch_device),
                                        None, torch.zeros(1, dtype=torch.int32, device=self.ctx.torch_device), self.ctx))
            else:
                out.append(DeviceColumn.empty(t, 0, True, ctx=self.ctx))
        return out

    def packed_keys(self, key_cols: Sequence[DeviceColumn]):
        """(int64 device key words, null-group flags) of rows given as original key columns
        (encodes new strings / tuples into this state's dictionaries)."""
        import torch

        members = [self.dicts[i].encode(k) if i in self.dicts else k for i, k in enumerate(key_cols)]
        if self.tuple_dict is not None:
            members = [self.tuple_dict.encode_tuple(members)]
        n = members[0].length
        packed = torch.zeros(n, dtype=torch.int64, device=self.ctx.torch_device)
        knull = torch.zeros(n, dtype=torch.int64, device=self.ctx.torch_device)
        if self._wide_key():
            m = members[0]
            valid = torch.from_numpy(m.valid_mask()).to(self.ctx.torch_device)
            packed = torch.where(valid, m.values[:n].to(torch.int64), packed)
            knull = (~valid).to(torch.int64)
        for (shift, nullbit, w), m in zip(self._packing(), members):
            vals = m.values[:n].to(torch.int64) & ((1 << w) - 1)
            valid = torch.from_numpy(m.valid_mask()).to(self.ctx.torch_device)
            packed |= torch.where(valid, vals << shift, torch.zeros_like(vals)) | ((~valid).to(torch.int64) << nullbit)
        return packed, knull

    def import_keyed(self, records, n: int, key_cols: Sequence[DeviceColumn]) -> None:
        """Import records whose keys come from another state: rewrite their key field from the
        key columns' content, then merge (qe_hashagg_import)."""
        import torch

        if n == 0:
            return
        rec = records[: n * self.record_bytes()].view(torch.int64).view(n, -1)
        rec[:, 0], rec[:, 1] = self.packed_keys(key_cols)  # (narrow packed keys: null flag 0)
        N.check(N.lib().qe_hashagg_import(self.handle, N.C.c_void_p(records.data_ptr()), int(n)))

    def export_all(self):
        """All partial records, unbucketed: (uint8 device tensor, count)."""
        import torch

        counts = self._export_counts_raw(1)
        rb = self.record_bytes()
        buf = torch.empty(max(1, counts[0] * rb), dtype=torch.uint8, device=self.ctx.torch_device)
        N.check(N.lib().qe_hashagg_export(self.handle, 1, N.C.c_void_p(buf.data_ptr())))
        return buf, counts[0]

    def _export_counts_raw(self, nparts: int) -> List[int]:
        arr = (N.C.c_int64 * nparts)()
        N.check(N.lib().qe_hashagg_export_counts(self.handle, nparts, arr))
        return list(arr)

    def export_counts(self, nparts: int) -> List[int]:
        self._check_exportable()
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

    def slot_bytes(self, slot_records: int) -> int:
        return N.SLOT_HEADER + int(slot_records) * self.record_bytes()

    def export_slots(self, nparts: int, slot_records: int):
        """-> uint8 device tensor of `nparts` fixed-capacity slots (qe_hashagg_export_slots):
        no host synchronisation, so the all-to-all can follow the aggregation kernel directly."""
        import torch

        self._check_exportable()
        buf = torch.empty(nparts * self.slot_bytes(slot_records), dtype=torch.uint8, device=self.ctx.torch_device)
        N.check(N.lib().qe_hashagg_export_slots(self.handle, int(nparts), int(slot_records),
                                                N.C.c_void_p(buf.data_ptr())))
        return buf

    def import_slots(self, slots, nslots: int, slot_records: int) -> Optional[int]:
        """Merges received slots; returns the records merged, or None when some sender's
        partition exceeded the slot capacity (nothing merged; the same on every rank)."""
        self._check_exportable()
        mx, n = N.C.c_int64(), N.C.c_int64()
        N.check(N.lib().qe_hashagg_import_slots(self.handle, N.C.c_void_p(slots.data_ptr()), int(nslots),
                                                int(slot_records), N.C.byref(mx), N.C.byref(n)))
        return None if mx.value > slot_records else n.value

    def import_records(self, records, nrecords: int) -> None:
        self._check_exportable()
        if nrecords == 0:
            return
        N.check(N.lib().qe_hashagg_import(self.handle, N.C.c_void_p(records.data_ptr()), int(nrecords)))
