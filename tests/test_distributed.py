"""N > 1 path on CPU: two processes over gloo run the hash-sharded partial-aggregate exchange
(kquery/exchange.py all_to_all_records — the same code RCCL runs on GPUs) on records in the
C ABI's format (oracle/records.py), and the owners' merged groups equal the single-process
aggregate. World size 2, 127.0.0.1 rendezvous."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gen, records as R

FNS = [R.AGG_SUM, R.AGG_COUNT_STAR, R.AGG_MIN, R.AGG_MAX]
ROWS = 40_000
THR = 1 << 19


def _data(row0, n):
    k, _ = gen.generate(gen.GEN_MOD, 1024, 42, 0, row0, n)
    a, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 1, row0, n)
    b, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 2, row0, n)
    return k, a, b


def _worker(rank, world, port, q, slot_records=None):
    import sys
    import pathlib

    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "query-engines_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kquery.exchange import all_to_all_records, all_to_all_slots

    k, a, b = _data(rank * ROWS, ROWS)
    parts = R.partials_c4(k, a, b, THR)
    recs = None
    if slot_records is not None:  # the fast path: fixed slots, one all-to-all (exchange_partials)
        send = torch.frombuffer(bytearray(R.encode_slots(parts, FNS, world, slot_records)), dtype=torch.uint8)
        got, mx = R.decode_slots(bytes(all_to_all_slots(send).numpy().tobytes()), world, slot_records, len(FNS))
        seen = [None] * world
        dist.all_gather_object(seen, mx > slot_records)
        assert len(set(seen)) == 1  # every rank takes the same path
        recs = None if mx > slot_records else got
    if recs is None:
        payload, counts = R.encode(parts, FNS, world)
        t = torch.frombuffer(bytearray(payload), dtype=torch.uint8) if payload else torch.empty(0, dtype=torch.uint8)
        recv, n = all_to_all_records(t, counts, R.record_bytes(len(FNS)))
        recs = R.decode(bytes(recv.numpy().tobytes()), len(FNS))
    owned = {}
    for key, cstar, aggs in recs:
        assert R.partition_of(key, False, world) == rank
        R.combine(FNS, owned, key, cstar, aggs)
    gathered = [None] * world
    dist.all_gather_object(gathered, owned)
    if rank == 0:
        q.put(gathered)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,slot_records", [(2, None), (2, 1024), (2, 100), (3, 400)])
def test_exchange_gloo_matches_single_process(world, slot_records):
    """slot_records None: variable-size exchange; 1024 / 400: fixed slots hold every partition;
    100: slots overflow (≈512 groups per owner), every rank falls back together."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, slot_records)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = {}
    for owned in gathered:
        assert not (set(merged) & set(owned))  # every group has exactly one owner
        merged.update(owned)
    k, a, b = _data(0, world * ROWS)
    ref = R.partials_c4(k, a, b, THR)
    assert merged == ref


def test_partition_function_balanced():
    keys = np.arange(1024)
    for p in (2, 4, 8):
        counts = np.bincount([R.partition_of(int(x), False, p) for x in keys], minlength=p)
        assert counts.min() > 1024 / p * 0.7
