"""ORACLE (test infrastructure only).

CPU restatement of the partial-aggregate record format and the exchange partition function of
qe_hashagg_export / qe_hashagg_import (query-engines_amd/csrc/qe_dev.hpp: agg_rec_bytes,
write_record_head; qe_hashagg.hip: partition_of), so the multi-process exchange can be tested with
gloo on CPU (tests/test_distributed.py) exactly as RCCL runs it on GPUs.

Record: [0] key i64, [8] flags u64 (bit0 null key), [16] COUNT(*) u64, then per aggregate
acc (8 B) + non-null count (8 B) (+ 4 x 8 B first-row indices for fp64 MIN/MAX; not used here).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Sequence, Tuple

import numpy as np

from .gen import MASK64

NULL_SALT = 0x6A09E667F3BCC909
AGG_SUM, AGG_MIN, AGG_MAX, AGG_COUNT, AGG_COUNT_STAR = 1, 2, 3, 4, 5


def fmix64(k: int) -> int:
    k &= MASK64
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & MASK64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & MASK64
    k ^= k >> 33
    return k


def partition_of(key: int, knull: bool, nparts: int) -> int:
    h = fmix64((key & MASK64) ^ (NULL_SALT if knull else 0))
    return ((h >> 32) * nparts) >> 32


def record_bytes(naggs: int) -> int:
    return 24 + 16 * naggs


def encode(groups: Dict[int, Tuple[int, List[Tuple[int, int]]]], fns: Sequence[int], nparts: int):
    """groups: key -> (count_star, [(acc, nn) per aggregate]) for int64 SUM/MIN/MAX/COUNT.
    Returns (payload bytes partition-major, counts per partition)."""
    buckets: List[List[bytes]] = [[] for _ in range(nparts)]
    for key, (cstar, aggs) in groups.items():
        rec = struct.pack("<qQQ", key, 0, cstar)
        for (acc, nn) in aggs:
            rec += struct.pack("<qQ", acc, nn)
        buckets[partition_of(key, False, nparts)].append(rec)
    return b"".join(b"".join(b) for b in buckets), [len(b) for b in buckets]


SLOT_HEADER = 64


def encode_slots(groups: Dict[int, Tuple[int, List[Tuple[int, int]]]], fns: Sequence[int], nparts: int,
                 slot_records: int) -> bytes:
    """qe_hashagg_export_slots' layout: per partition a 64-byte header (word 0 = the partition's
    full count, word 1 = the largest count over all partitions) then `slot_records` record
    places, the first min(count, slot_records) filled."""
    payload, counts = encode(groups, fns, nparts)
    rb = record_bytes(len(fns))
    out, off = b"", 0
    for c in counts:
        recs = payload[off: off + min(c, slot_records) * rb]
        off += c * rb
        hdr = struct.pack("<QQ", c, max(counts)) + bytes(SLOT_HEADER - 16)
        out += hdr + recs + bytes(slot_records * rb - len(recs))
    return out


def decode_slots(buf: bytes, nslots: int, slot_records: int, naggs: int):
    """Received slots -> (records, largest count any sender reported) — qe_hashagg_import_slots'
    reading; when the largest count exceeds slot_records the records are incomplete."""
    rb = record_bytes(naggs)
    sb = SLOT_HEADER + slot_records * rb
    recs, mx = [], 0
    for i in range(nslots):
        c, m = struct.unpack_from("<QQ", buf, i * sb)
        mx = max(mx, m)
        recs += decode(buf[i * sb + SLOT_HEADER: i * sb + SLOT_HEADER + min(c, slot_records) * rb], naggs)
    return recs, mx


def decode(payload: bytes, naggs: int) -> List[Tuple[int, int, List[Tuple[int, int]]]]:
    rb = record_bytes(naggs)
    out = []
    for off in range(0, len(payload), rb):
        key, _flags, cstar = struct.unpack_from("<qQQ", payload, off)
        aggs = [struct.unpack_from("<qQ", payload, off + 24 + 16 * j) for j in range(naggs)]
        out.append((key, cstar, aggs))
    return out


def combine(fns: Sequence[int], into: Dict[int, Tuple[int, List[Tuple[int, int]]]], key: int, cstar: int,
            aggs: Sequence[Tuple[int, int]]) -> None:
    """Merge semantics of qe_dev.hpp gcombine for int64 aggregates."""
    if key not in into:
        into[key] = (cstar, [tuple(a) for a in aggs])
        return
    c0, a0 = into[key]
    merged = []
    for f, (x, xn), (y, yn) in zip(fns, a0, aggs):
        if f == AGG_SUM:
            v = (x + y) & MASK64
            merged.append((v - (1 << 64) if v >= 1 << 63 else v, xn + yn))
        elif f == AGG_MIN:
            merged.append((min(x, y), xn + yn))
        elif f == AGG_MAX:
            merged.append((max(x, y), xn + yn))
        else:
            merged.append((0, xn + yn))
    into[key] = (c0 + cstar, merged)


def partials_c4(k: np.ndarray, a: np.ndarray, b: np.ndarray, threshold: int):
    """Partial state of SUM(a+b), COUNT(*), MIN(a), MAX(b) WHERE a > threshold GROUP BY k."""
    sel = a > threshold
    out: Dict[int, Tuple[int, List[Tuple[int, int]]]] = {}
    ks, as_, bs = k[sel], a[sel], b[sel]
    for key in np.unique(ks):
        m = ks == key
        s = int(np.sum((as_[m] + bs[m]).astype(np.uint64), dtype=np.uint64).view(np.int64))
        n = int(m.sum())
        out[int(key)] = (n, [(s, n), (0, 0), (int(as_[m].min()), n), (int(bs[m].max()), n)])
    return out
