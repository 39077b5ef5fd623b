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


def exchange_partials(partial, owner, group: Optional[dist.ProcessGroup] = None) -> int:
    """Moves every group of `partial` (this rank's HashAggregateState) to the rank that owns its
    key and merges what this rank receives into `owner`. Returns the records received."""
    world = dist.get_world_size(group)
    recs, counts = partial.export(world)
    recv, n = all_to_all_records(recs, counts, partial.record_bytes(), group)
    owner.import_records(recv, n)
    return n
