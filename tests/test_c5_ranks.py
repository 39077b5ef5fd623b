"""C5 (BASELINE configs[4]: 10B lineitem rows, multi-key GROUP BY "across 8 MI355X") rehearsed across
two ranks on one GPU (VERDICT r04 "rehearse C5 across ranks"; Main.kt:1314-1325 partial -> merge):

* test_c5_two_ranks_gloo — two processes (torch.distributed.run, gloo), the torch exchange
  (kquery.exchange.exchange_partials): fixed slots and the overflow fallback, exact and fast fp64;
* test_c5_two_ranks_native_loopback — two threads of one process, each with its own qe_ctx, through
  the C ABI's own exchange (qe_hashagg_exchange: export slots -> grouped send/recv -> import, and
  its counts + records fallback) with the in-process transport in place of RCCL
  (qe_comm_create_loopback).

Every owner's groups, unioned, are compared per group with the exact C oracle over both ranks'
rows (tests/c5_check.py)."""
import json
import os
import pathlib
import socket
import subprocess
import sys
import threading

import pytest

from c5_check import c5_oracle, check_groups

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_c5_two_ranks_gloo():
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "tests" / "dist_c5_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(line[0][len("RESULT "):])
    assert set(res) == {"exact-slots", "exact-overflow", "fast-slots", "fast-overflow"}, res
    assert all(v["ok"] for v in res.values()), res


@pytest.mark.parametrize("fast", [False, True], ids=["exact", "fast"])
@pytest.mark.parametrize("slot_records", [0, 1], ids=["slots", "overflow"])
def test_c5_two_ranks_native_loopback(gpu_ctx, fast, slot_records):
    import torch

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import Context
    from kquery.datasource import C5_COLUMNS, generate_column
    from kquery.exchange import exchange_partials_native
    from kquery.workloads import C5_AGGS, C5_KEY_TYPES, c5_spec

    world, row0, sizes = 2, 7_000_000_000, (2_000_003, 1_500_000)
    hub = N.C.c_void_p()
    N.check(N.lib().qe_comm_loopback_hub_create(world, N.C.byref(hub)))
    out, errors = [None] * world, []

    class Comm:  # what exchange_partials_native reads of a NativeComm
        pass

    def rank_main(r):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                ctx = Context.get(0)
                base = row0 + sum(sizes[:r])
                cols = [generate_column(sp, sizes[r], base, 42, ctx) for sp in C5_COLUMNS]
                partial = HashAggregateState(ctx, C5_KEY_TYPES, C5_AGGS, 16, fast_fp64=fast)
                owner = HashAggregateState(ctx, C5_KEY_TYPES, C5_AGGS, 16, fast_fp64=fast)
                partial.set_row_base(base)
                partial.update_fused(cols, c5_spec())
                h = N.C.c_void_p()
                N.check(N.lib().qe_comm_create_loopback(ctx.handle, world, r, hub, N.C.byref(h)))
                comm = Comm()
                comm.handle = h
                try:
                    exchange_partials_native(partial, owner, comm, slot_records)
                finally:
                    N.lib().qe_comm_destroy(h)
                kk, aa = owner.finalize()
                ctx.synchronize()
                out[r] = [list(x) for x in zip(*([c.to_pylist() for c in kk] + [c.to_pylist() for c in aa]))]
        except Exception as e:  # reported by the main thread
            errors.append(repr(e))

    threads = [threading.Thread(target=rank_main, args=(r,), daemon=True) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(100)
    N.lib().qe_comm_loopback_hub_destroy(hub)
    assert not errors, errors
    assert all(o is not None for o in out)
    ok, why = check_groups([row for rows in out for row in rows], c5_oracle(row0, sum(sizes)), exact=not fast)
    assert ok, why
