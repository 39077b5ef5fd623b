"""Multi-GPU hash-sharded aggregate exchange (north star: "HashAggregateExec shards
by key-hash across the 8 GPUs of one node with an RCCL all-to-all of partial aggregates").

Each rank partial-aggregates its own row range (one process per GPU), exports its groups as
fixed-size records bucketed by destination = hash(key) mod world_size (qe_hashagg_export), and
ONE all-to-all moves every bucket to its owner, which merges them (qe_hashagg_import). This is
the reference's partial -> final merge of main() (Main.kt:1309-1325) with the 12 coroutine
partitions replaced by ranks. With backend "nccl" (= RCCL on ROCm) the payload moves over xGMI
point-to-point links, all peers at once; with "gloo" the same code runs on CPU tensors (tests).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def all_to_all_records(payload: torch.Tensor, counts: List[int], record_bytes: int,
                       group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, int]:
    """payload: uint8 records, partition-major (counts[p] records for rank p).
    Returns (received uint8 records, number of records)."""
    world = dist.get_world_size(group)
    assert len(counts) == world
    dev = payload.device
    send_counts = torch.tensor(counts, dtype=torch.int64, device=dev)
    recv_counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    rc = [int(x) for x in recv_counts.cpu().tolist()]
    out = torch.empty(max(1, sum(rc) * record_bytes), dtype=torch.uint8, device=dev)
    in_split = [c * record_bytes for c in counts]
    out_split = [c * record_bytes for c in rc]
    if payload.numel() == 0:
        payload = torch.empty(0, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out[: sum(out_split)], payload[: sum(in_split)], out_split, in_split, group=group)
    return out[: sum(out_split)], sum(rc)


def _a2a_bytes(chunks: List[torch.Tensor], group=None) -> Tuple[torch.Tensor, List[int]]:
    """Variable-size all-to-all of uint8 tensors (chunks[p] goes to rank p). Returns the received
    bytes concatenated in source-rank order and the size from each source. gloo runs on CPU
    tensors: device tensors are staged through host memory for it."""
    world = dist.get_world_size(group)
    dev = chunks[0].device
    stage = dist.get_backend(group) == "gloo" and dev.type != "cpu"
    send = torch.cat([c.reshape(-1) for c in chunks]) if any(c.numel() for c in chunks) else \
        torch.empty(0, dtype=torch.uint8, device=dev)
    sizes = torch.tensor([c.numel() for c in chunks], dtype=torch.int64)
    rsizes = torch.empty(world, dtype=torch.int64)
    if not stage and dev.type != "cpu":
        sizes, rsizes = sizes.to(dev), rsizes.to(dev)
    dist.all_to_all_single(rsizes, sizes, group=group)
    rs = [int(x) for x in rsizes.cpu().tolist()]
    out = torch.empty(sum(rs), dtype=torch.uint8, device="cpu" if stage else dev)
    dist.all_to_all_single(out, send.cpu() if stage else send, rs, [c.numel() for c in chunks], group=group)
    return (out.to(dev) if stage else out), rs


def exchange_keyed_partials(partial, owner, group: Optional[dist.ProcessGroup] = None) -> int:
    """Dictionary-keyed partials (UTF-8 or composite keys): codes are local to a state, so groups
    travel with their key CONTENT, through the same C entry points a JNI host uses:
    qe_hashagg_export_keyed (records + key values, routed by a content hash of the keys), one
    all-to-all of the blocks, qe_hashagg_import_keyed (the owner re-encodes the keys into its own
    dictionaries). Returns the records this rank merged."""
    world = dist.get_world_size(group)
    blocks, sizes = partial.export_keyed(world)
    chunks, off = [], 0
    for sz in sizes:
        chunks.append(blocks[off: off + sz])
        off += sz
    rblocks, rsz = _a2a_bytes(chunks, group)
    return owner.import_keyed(rblocks, rsz)


def all_to_all_slots(send: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Equal-split all-to-all of `world` fixed-size slots (slot p goes to rank p). No sizes are
    exchanged first and nothing waits on the host: with RCCL it queues behind the export kernel
    on the device. gloo (CPU tests) stages device tensors through host memory."""
    stage = dist.get_backend(group) == "gloo" and send.device.type != "cpu"
    src = send.cpu() if stage else send
    out = torch.empty_like(src)
    dist.all_to_all_single(out, src, group=group)
    return out.to(send.device) if stage else out


def exchange_partials(partial, owner, group: Optional[dist.ProcessGroup] = None,
                      slot_records: Optional[int] = None) -> int:
    """Moves every group of `partial` (this rank's HashAggregateState) to the rank that owns its
    key and merges what this rank receives into `owner`. Returns the records received.

    Fast path: fixed-capacity slots of `slot_records` groups per destination (default:
    qe_hashagg_slot_capacity — the create-time expected groups spread over the ranks with
    headroom, 1.5x an even share plus 32, at most the expected groups — the same on every rank
    whatever groups each rank's data produced), ONE all-to-all, no host round trip
    before it. If any rank had more groups for one owner than a slot holds, every rank sees it in
    the slot headers and all of them fall back to the variable-size exchange (counts all-to-all,
    then records)."""
    if getattr(partial, "keyed_by_dictionary", False) or getattr(owner, "keyed_by_dictionary", False):
        return exchange_keyed_partials(partial, owner, group)
    world = dist.get_world_size(group)
    cap = int(slot_records or partial.slot_capacity(world))
    recv = all_to_all_slots(partial.export_slots(world, cap), group)
    owner.prepare_output()  # host work of the owner's finalize, before the import's read-back
    n = owner.import_slots(recv, world, cap)
    if n is not None:
        return n
    recs, counts = partial.export(world)
    recv, n = all_to_all_records(recs, counts, partial.record_bytes(), group)
    owner.import_records(recv, n)
    return n


class NativeComm:
    """An RCCL communicator owned by the C library (qe_comm_*): the exchange a JNI host would use,
    with no torch.distributed collective on the data path. Rank 0's unique id reaches the other
    ranks through the process group's object broadcast (a JNI host would use its own transport)."""

    def __init__(self, ctx, group: Optional[dist.ProcessGroup] = None):
        from . import native as N

        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        uid = (N.C.c_char * N.COMM_ID_BYTES)()
        if rank == 0:
            N.check(N.lib().qe_comm_unique_id(uid))
        if world > 1:
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=0, group=group)
            uid = (N.C.c_char * N.COMM_ID_BYTES).from_buffer_copy(box[0])
        h = N.C.c_void_p()
        N.check(N.lib().qe_comm_create(ctx.handle, world, rank, uid, N.C.byref(h)))
        self.handle, self.ctx, self.world, self.rank = h, ctx, world, rank

    def close(self) -> None:
        from . import native as N

        if getattr(self, "handle", None) is not None:
            N.lib().qe_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def exchange_partials_native(partial, owner, comm: NativeComm, slot_records: int = 0) -> int:
    """exchange_partials through the C ABI (qe_hashagg_exchange): export slots, one grouped RCCL
    send/recv on the ctx stream, import with one read-back; same fallback rule. Returns the records
    this rank merged."""
    from . import native as N

    owner.prepare_output()  # host work of the owner's finalize, before the import's read-back
    n = N.C.c_int64()
    N.check(N.lib().qe_hashagg_exchange(comm.handle, partial.handle, owner.handle, int(slot_records), N.C.byref(n)))
    return n.value


def _all_gather_bytes(part, world: int, group):
    if world == 1:
        return part
    if dist.get_backend(group) == "gloo":  # CPU collectives: stage through host memory
        got = [torch.empty_like(part, device="cpu") for _ in range(world)]
        dist.all_gather(got, part.cpu(), group=group)
        return torch.cat(got).to(part.device)
    parts = torch.empty(world * part.numel(), dtype=torch.uint8, device=part.device)
    dist.all_gather_into_tensor(parts, part, group=group)
    return parts


def global_aggregate(col, mask=None, row_base: int = 0, group: Optional[dist.ProcessGroup] = None):
    """SUM/MIN/MAX/COUNT/AVG without GROUP BY over a column whose rows are split across ranks
    (SURVEY §8e "global aggregate: one exchange"): this rank's 128-byte partial
    (qe_agg_global_partial, row indices offset by `row_base` — this rank's first global row),
    ONE all-gather, and the same fixed-order merge on every rank (qe_agg_global_merge), so every
    rank returns identical bits. When the merged fp64 sum cannot be proven correctly rounded (the
    ranks' sums cancel) the merge says so on every rank alike (QE_NEED_EXACT) and a second round
    gathers each rank's exact sum words (qe_agg_global_exact_partial, 320 bytes) for
    qe_agg_global_merge_exact: the sum is then math.fsum's over all ranks' rows.
    Without an initialised process group: this column alone."""
    from . import native as N

    ctx = col.ctx
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    part = torch.empty(N.GLOBAL_PARTIAL_BYTES, dtype=torch.uint8, device=ctx.torch_device)
    cc = col.as_c()
    mc = mask.as_c() if mask is not None else None
    mp = N.C.byref(mc) if mc is not None else None
    N.check(N.lib().qe_agg_global_partial(ctx.handle, N.C.byref(cc), mp, int(row_base), N.C.c_void_p(part.data_ptr())))
    parts = _all_gather_bytes(part, world, group)
    out = N.QeGlobalAgg()
    st = N.lib().qe_agg_global_merge(ctx.handle, col.type, N.C.c_void_p(parts.data_ptr()), world, N.C.byref(out))
    if st == N.QE_NEED_EXACT:
        words = torch.empty(N.GLOBAL_EXACT_BYTES, dtype=torch.uint8, device=ctx.torch_device)
        N.check(N.lib().qe_agg_global_exact_partial(ctx.handle, N.C.byref(cc), mp, N.C.c_void_p(words.data_ptr())))
        allw = _all_gather_bytes(words, world, group)
        st = N.lib().qe_agg_global_merge_exact(ctx.handle, N.C.c_void_p(allw.data_ptr()), world, N.C.byref(out))
    N.check(st)
    return out
