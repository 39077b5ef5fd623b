#!/usr/bin/env python3
"""Ingest path: an Arrow host RecordBatch (what Arrow Java exports for the
reference's VectorSchemaRoot) -> qe_batch_import (pinned double-buffered H2D) -> device columns,
then the C4 query on them. Reports the PCIe-inclusive rate next to the device-only rate, and a
plain pinned torch copy of the same bytes as the link ceiling."""
import ctypes as C
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

import pyarrow as pa  # noqa: E402
import torch  # noqa: E402

from kquery import native as N  # noqa: E402
from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.arrow_io import DeviceBatch, prefetch_import  # noqa: E402
from kquery.columnar import Context, DeviceColumn  # noqa: E402
from kquery.workloads import C4_AGGS, c4_spec  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    ctx = Context.get(0)
    rng = np.random.default_rng(1)
    k = rng.integers(0, 1024, rows)
    a = rng.integers(0, 1 << 20, rows)
    b = rng.integers(0, 1 << 20, rows)
    rb = pa.RecordBatch.from_arrays([pa.array(k), pa.array(a), pa.array(b)], names=["k", "a", "b"])
    nbytes = 24 * rows
    # link ceiling: pinned host tensor -> device
    host = torch.from_numpy(np.concatenate([k, a, b]).view(np.uint8)).pin_memory()
    dev = torch.empty_like(host, device=ctx.torch_device)
    for _ in range(2):
        dev.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    pinned_gbs = nbytes / (time.perf_counter() - t0) / 1e9
    del dev, host
    # qe_batch_import (pageable Arrow buffers -> pinned staging -> HBM)
    DeviceBatch.from_pyarrow(rb.slice(0, 1000), ctx).close()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        db = DeviceBatch.from_pyarrow(rb, ctx)
        ctx.synchronize()
        ts.append(time.perf_counter() - t0)
        if _ < 2:
            db.close()
    imp = min(ts)
    cols = [db.column(i)[0] for i in range(3)]
    st = HashAggregateState(ctx, [N.TYPE_INT64], C4_AGGS, 1024)
    cc = (N.QeColumn * 3)(*cols)
    spec = c4_spec()

    def run():
        st.reset()
        N.check(N.lib().qe_hashagg_update_fused(st.handle, cc, 3, C.byref(spec)))
        return st.finalize()

    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    keys, _ = run()
    torch.cuda.synchronize()
    q = time.perf_counter() - t0
    db.close()
    # the same rows as 8 batches through the operator loop: import then query per batch, against
    # prefetch_import (batch i+1's import beside batch i's kernels)
    nb = 8
    parts = [rb.slice(i * rows // nb, rows // nb) for i in range(nb)]

    def batch_query(d, st):
        cc = (N.QeColumn * 3)(*[d.column(i)[0] for i in range(3)])
        N.check(N.lib().qe_hashagg_update_fused(st.handle, cc, 3, C.byref(spec)))

    def sequential():
        st.reset()
        for p in parts:
            d = DeviceBatch.from_pyarrow(p, ctx)
            batch_query(d, st)
            ctx.synchronize()
            d.close()
        return st.finalize()

    def pipelined():
        st.reset()
        for d in prefetch_import(parts, ctx):
            batch_query(d, st)
        return st.finalize()

    res = {}
    for name, fn in (("sequential", sequential), ("pipelined", pipelined)):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            k2, v2 = fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        res[name] = {"s": best, "rows_per_s": rows / best, "groups": k2[0].length,
                     "count_star_total": int(v2[1].to_numpy().sum())}
    print(json.dumps({
        "rows": rows, "bytes": nbytes, "import_s": imp, "import_GBps": nbytes / imp / 1e9,
        "pinned_copy_GBps": pinned_gbs, "query_s": q, "groups": keys[0].length,
        "rows_per_s_pcie_inclusive": rows / (imp + q), "rows_per_s_device_only": rows / q,
        "batches": nb, "batched": res,
    }))


if __name__ == "__main__":
    main()
