#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json metric): rows/s of filter + project + GROUP BY over
device-resident synthetic RecordBatches, config 4:

    SELECT k, SUM(a + b), COUNT(*), MIN(a), MAX(b) FROM t WHERE a > 2^19 GROUP BY k
    k = u0 mod 1024, a = u1 mod 2^20, b = u2 mod 2^20 (int64; splitmix64 counter generator)

One step = one full query over this rank's 1B-row batch (inputs resident in HBM before the
timed region): fused filter -> project -> partial hash-aggregate kernel, then (N > 1) the
hash-sharded all-to-all of partial aggregates over RCCL and the owner-side merge, then the
final one-batch materialisation. Weak scaling: every rank owns 1B rows.

    python bench.py [--gpus N --steps K --warmup W]      (N > 1: launched by torch.distributed.run)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "query-engines_amd"))

METRIC = "rows/sec filter+project+group-by over 1B-row Arrow batch; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
BYTES_PER_ROW = 24     # k, a, b int64: algorithmic bytes read per row


def c4_spec(N, threshold=1 << 19):
    from kquery.workloads import c4_spec as spec

    return spec(threshold)


def _cpu_lib():
    lib_path = ROOT / "oracle" / "build" / "libqe_oracle.so"
    if not lib_path.exists():
        import subprocess

        subprocess.run(["make", "-C", str(ROOT / "oracle")], check=True, capture_output=True)

    class G(C.Structure):
        _fields_ = [(n, C.c_int64) for n in ("key", "sum", "count", "min", "max")]

    lib = C.CDLL(str(lib_path))
    for fn in (lib.qe_cpu_c4, lib.qe_cpu_c4_fast):
        fn.restype = C.c_double
        fn.argtypes = [C.c_int64, C.c_int64, C.c_uint64, C.c_int, C.c_int64, C.c_int64,
                       C.POINTER(G), C.c_int64, C.POINTER(C.c_int64)]
    return lib, G


def cpu_baseline(sample_rows: int, threads: int):
    """Timed CPU legs (rank 0, N = 1) on bounded samples of the same rows:
    * `value`: the oracle's reference-faithful C restatement of the query (oracle/cpu_baseline.c:
      row-at-a-time Selection -> Projection -> HashMap aggregate with boxed keys and virtual
      accumulators, partition-parallel like Main.kt:1309-1325) on `threads` threads;
    * `single_thread`: the same port on one thread (1 thread and all threads);
    * `tuned`: a tuned C implementation (no boxing or materialisation, per-thread open-addressing
      tables), so the GPU is also compared with a fast CPU engine.
    Returns (the port's groups over the sample, key -> (SUM, COUNT, MIN, MAX); the JSON object)."""
    lib, G = _cpu_lib()
    out = (G * 2048)()
    ng = C.c_int64()
    secs = lib.qe_cpu_c4(0, sample_rows, 42, threads, 1 << 19, 1024, out, 2048, C.byref(ng))
    groups = {int(g.key): (int(g.sum), int(g.count), int(g.min), int(g.max)) for g in out[:ng.value]}
    one_rows = min(sample_rows, 100_000_000)
    secs1 = lib.qe_cpu_c4(0, one_rows, 42, 1, 1 << 19, 1024, out, 2048, C.byref(ng))
    secs_t = lib.qe_cpu_c4_fast(0, sample_rows, 42, threads, 1 << 19, 1024, out, 2048, C.byref(ng))
    return groups, {"value": sample_rows / secs, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"rows 0..{sample_rows - 1} of the same C4 table (seed 42), {threads} threads, "
                      f"{secs:.3f} s; C restatement of the reference operator chain (oracle/cpu_baseline.c)",
            "single_thread": {"value": one_rows / secs1, "cores": 1,
                              "sample": f"rows 0..{one_rows - 1}, 1 thread, {secs1:.3f} s"},
            "tuned": ({"value": sample_rows / secs_t, "cores": threads,
                       "sample": f"rows 0..{sample_rows - 1}, {threads} threads, {secs_t:.3f} s; "
                                 "per-thread open-addressing tables (qe_cpu_c4_fast)"} if secs_t > 0 else None)}


def load_traffic(rows: int):
    """HBM bytes per fused-kernel launch from the committed rocprofv3 PMC summary (profiles/),
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 counts half of wide streaming reads)."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        t = json.loads(p.read_text())
        if int(t.get("rows", -1)) == rows:
            return float(t["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=1_000_000_000, help="rows per GPU")
    ap.add_argument("--cpu-sample-rows", type=int, default=0, help="default: the same rows as one GPU")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--exchange", action="store_true",
                    help="run the multi-GPU exchange leg even with one rank (tests the N > 1 step on one GPU)")
    ap.add_argument("--exchange-impl", default="torch", choices=["torch", "native"],
                    help="torch: all-to-all through torch.distributed (default); native: the C ABI's own "
                         "RCCL communicator (qe_hashagg_exchange)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend (nccl = RCCL over xGMI; gloo only to rehearse N > 1 "
                         "ranks sharing one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import Context
    from kquery.datasource import C4_COLUMNS, generate_column

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    # one rank per GPU; more ranks than GPUs only in a gloo rehearsal (ranks then share devices)
    device = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1 or args.exchange:
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29511"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.dist_backend)
    from kquery.exchange import NativeComm, exchange_partials, exchange_partials_native

    ctx = Context.get(device)
    rows = args.rows
    row0 = rank * rows
    cols = [generate_column(s, rows, row0, 42, ctx) for s in C4_COLUMNS]
    ctx.synchronize()
    aggs = [(N.AGG_SUM, N.TYPE_INT64), (N.AGG_COUNT_STAR, N.TYPE_INT64), (N.AGG_MIN, N.TYPE_INT64),
            (N.AGG_MAX, N.TYPE_INT64)]
    # stream-ordered updates: the columns stay resident, so the update's counters are read back
    # by finalize (one host wait per step) instead of by the update itself
    partial = HashAggregateState(ctx, [N.TYPE_INT64], aggs, 1024, async_update=True)
    exchange = world > 1 or args.exchange
    owner = HashAggregateState(ctx, [N.TYPE_INT64], aggs, 1024) if exchange else None
    comm = NativeComm(ctx) if exchange and args.exchange_impl == "native" else None
    spec = c4_spec(N)
    kernel_ms = []
    kinds = []

    def step():
        partial.reset()
        partial.set_row_base(row0)
        partial.update_fused(cols, spec)
        final = partial
        if exchange:
            owner.reset()
            if comm is not None:
                exchange_partials_native(partial, owner, comm)
            else:
                exchange_partials(partial, owner)
            final = owner
        out = final.finalize()
        kernel_ms.append(partial.last_kernel_time())
        return out

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    kinds.append(partial.last_kernel_kind())
    kernel_ms.clear()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        keys, res = step()
    torch.cuda.synchronize()
    kinds.append(partial.last_kernel_kind())
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # stream-read ceiling over the same 24 B/row (k, a, b), median of 5
    cc = (N.QeColumn * 3)(*[c.as_c() for c in cols])
    sr = []
    for _ in range(5):
        ms = C.c_double()
        N.check(N.lib().qe_stream_read(ctx.handle, cc, 3, C.byref(ms)))
        sr.append(ms.value)
    stream_gbs = rows * BYTES_PER_ROW / (sorted(sr)[2] * 1e-3) / 1e9

    # Result checks before any number is printed: every group present once across owners, and
    # COUNT(*) adds up to the rows an independent torch kernel counts as passing the predicate.
    a_col = cols[1].values[:rows]
    selected = int((a_col > (1 << 19)).sum().item())
    groups = torch.tensor([keys[0].length, int(res[1].to_numpy().sum()), selected], dtype=torch.int64, device="cuda")
    if world > 1:
        dist.all_reduce(groups)
    n_groups, count_total, selected_total = (int(x) for x in groups.tolist())
    if n_groups != 1024 or count_total != selected_total:
        sys.exit(f"bench: wrong result: {n_groups} groups (want 1024), COUNT(*) total {count_total} "
                 f"(want {selected_total})")
    ms_step = elapsed / args.steps * 1e3
    launches = sum(k for _, k in kernel_ms)
    avg_kernel_ms = sum(m for m, _ in kernel_ms) / max(1, launches)
    achieved = rows * BYTES_PER_ROW / (avg_kernel_ms * 1e-3) / 1e9
    traffic = load_traffic(rows)
    line = {
        "metric": METRIC,
        "value": world * rows / (ms_step * 1e-3),
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (counter-based splitmix64 generator, seed 42), device-resident before timing",
        "config": {
            "workload": "C4: SELECT k, SUM(a+b), COUNT(*), MIN(a), MAX(b) WHERE a > 2^19 GROUP BY k",
            "rows_per_gpu": rows,
            "groups": 1024,
            "columns": "k, a, b int64 (Arrow, no nulls)",
            "parallelism": f"hash-sharded partial aggregate x{world}" + (
                (" + RCCL send/recv (qe_hashagg_exchange)" if comm is not None else
                 " + RCCL all-to-all" if args.dist_backend == "nccl" else f" + {args.dist_backend} all-to-all (rehearsal)")
                if exchange else ""),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": ("qe_fused (hipRTC plan-specialised filter+project+LDS hash aggregate)" if kinds[-1][0]
                       else f"k_hashagg generic interpreter ({kinds[-1][1]})"),
            "avg_kernel_ms": avg_kernel_ms,
            "bytes_per_launch": rows * BYTES_PER_ROW,
            "stream_read_ceiling_gbs": stream_gbs,
        },
        "check": {"groups": n_groups, "count_star_total": count_total, "count_star_torch": selected_total},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        sample = args.cpu_sample_rows or rows
        cpu_groups, line["cpu_baseline"] = cpu_baseline(sample, threads)
        if sample == rows:
            # the CPU port ran over exactly these rows: every group's SUM/COUNT/MIN/MAX must agree
            kv = keys[0].to_numpy()
            rv = [r.to_numpy() for r in res]
            gpu_groups = {int(kv[i]): tuple(int(r[i]) for r in rv) for i in range(keys[0].length)}
            if gpu_groups != cpu_groups:
                bad = sorted(k for k in set(gpu_groups) | set(cpu_groups) if gpu_groups.get(k) != cpu_groups.get(k))
                sys.exit(f"bench: {len(bad)} groups differ from the CPU port, e.g. key {bad[0]}: "
                         f"gpu {gpu_groups.get(bad[0])} cpu {cpu_groups.get(bad[0])}")
            line["check"]["cpu_port_groups_equal"] = True
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
