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


def cpu_model() -> str:
    """The host CPU's model name (what `lscpu` prints as "Model name"), from /proc/cpuinfo."""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.lower().startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpus():
    """CPUs the cgroup quota allows (cpu.max), or None when unlimited / unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def usable_cpus() -> int:
    """CPUs this process can actually run on: its affinity set, capped by the cgroup CPU quota
    (on the GPU box the affinity lists the whole machine while the quota grants a share of it;
    threads beyond the quota only time-slice)."""
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpus()
    return max(1, min(n, int(-(-q // 1)))) if q else n


def cpu_baseline(sample_rows: int, threads: int):
    """Timed CPU legs (rank 0, N = 1) on bounded samples of the same rows:
    * `value`: the oracle's C restatement of the reference operator chain (oracle/cpu_baseline.c:
      row-at-a-time Selection -> Projection -> HashMap aggregate whose keys are per-row List +
      boxed Long objects from a per-thread bump allocator, boxed accumulator inputs through virtual
      accumulators, partition-parallel like Main.kt:1309-1325) on `threads` threads — every CPU
      this process may use (usable_cpus: the affinity set capped by the cgroup quota);
    * `threads_affinity`: the same with one thread per CPU of the affinity set;
    * `threads_16`: the same at 16 threads (the GPU box's CPU share per GPU);
    * `single_thread`: the same on one thread (1 thread and all threads);
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
    secs16 = lib.qe_cpu_c4(0, sample_rows, 42, 16, 1 << 19, 1024, out, 2048, C.byref(ng)) if threads != 16 else secs
    naff = len(os.sched_getaffinity(0))
    secs_aff = (lib.qe_cpu_c4(0, sample_rows, 42, naff, 1 << 19, 1024, out, 2048, C.byref(ng))
                if naff != threads else secs)
    secs_t = lib.qe_cpu_c4_fast(0, sample_rows, 42, threads, 1 << 19, 1024, out, 2048, C.byref(ng))
    return groups, {"value": sample_rows / secs, "unit": "rows/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "cgroup_cpus": cgroup_cpus(), "affinity_cpus": naff,
            "sample": f"rows 0..{sample_rows - 1} of the same C4 table (seed 42), {threads} threads "
                      f"(every usable CPU: sched_getaffinity {naff}, cgroup quota {cgroup_cpus()}), {secs:.3f} s; "
                      "C restatement of the reference operator chain with per-row boxed key List / Long objects "
                      "(oracle/cpu_baseline.c)",
            "threads_16": {"value": sample_rows / secs16, "cores": 16, "sample": f"same rows, 16 threads, {secs16:.3f} s"},
            "threads_affinity": {"value": sample_rows / secs_aff, "cores": naff,
                                 "sample": f"same rows, one thread per CPU of sched_getaffinity, {secs_aff:.3f} s"},
            "single_thread": {"value": one_rows / secs1, "cores": 1,
                              "sample": f"rows 0..{one_rows - 1}, 1 thread, {secs1:.3f} s"},
            "tuned": ({"value": sample_rows / secs_t, "cores": threads,
                       "sample": f"rows 0..{sample_rows - 1}, {threads} threads, {secs_t:.3f} s; "
                                 "per-thread open-addressing tables (qe_cpu_c4_fast)"} if secs_t > 0 else None)}


def load_traffic(rows: int, signature: str):
    """HBM bytes per fused-kernel launch from the committed rocprofv3 PMC summary
    (profiles/traffic.json, written by profiles/summarize.py; FETCH_SIZE doubled per
    MI355X_MICROARCH.md §HBM: gfx950 counts half of wide streaming reads). Used only when it was
    measured at these rows on the identical kernel and launch: `signature` is this run's
    qe_hashagg_last_kernel_signature (hash of the specialised kernel's compile key — toolchain,
    options, generated source — and its launch shape). Any kernel change leaves `traffic` null
    until the PMC passes are re-run. Returns (bytes, note)."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None, "no profiles/traffic.json"
    try:
        t = json.loads(p.read_text())
    except ValueError:
        return None, "unreadable profiles/traffic.json"
    if int(t.get("rows", -1)) != rows:
        return None, f"profiles/traffic.json is for {t.get('rows')} rows"
    have = t.get("kernel_signature")
    if have != signature:
        return None, f"stale: profiles/traffic.json measured kernel {have}, this run launched {signature}"
    return float(t["hbm_bytes_per_launch"]), (f"profiles/traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of this "
                                              f"kernel {have}, git {t.get('git_head', '?')})")


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N ranks with torch.distributed.run as a child
    process (this process never touches the GPU, so no exec after GPU init), pass rank 0's JSON
    line through, and return the child's exit code. With nccl (RCCL) each rank needs its own GPU:
    fewer visible GPUs than N is an error, never a silent 1-rank run. gloo may rehearse N ranks on
    fewer GPUs (ranks then share devices)."""
    import socket
    import subprocess

    if args.dist_backend == "nccl":
        import torch  # device_count() does not initialise HIP on this image

        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench: --gpus {args.gpus} needs {args.gpus} visible GPUs for one RCCL rank each, found {have} "
                  "(--dist-backend gloo rehearses more ranks than GPUs)", file=sys.stderr)
            return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(pathlib.Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    # stdout carries rank 0's JSON line only: anything else the ranks print there (gloo's
    # connection lines, library notices) goes to stderr
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in proc.stdout:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
    sys.stdout.flush()
    return proc.wait()


def rank_plan(world: int, rank: int, local: int, backend: str, ndev: int, exchange: bool) -> dict:
    """This rank's device and process-group plan from the launcher environment. One RCCL rank per
    GPU: rank `local` drives cuda:`local` and binds its communicator to it (device_id); more ranks
    than GPUs only in a gloo rehearsal (ranks then share devices, no device_id)."""
    plan = {"world_size": world, "rank": rank, "local_rank": local, "backend": backend, "visible_gpus": ndev,
            "device": local % max(1, ndev), "device_id": None, "process_group": world > 1 or exchange}
    if world > 1 and backend == "nccl" and ndev < world:
        plan["error"] = f"bench: {world} RCCL ranks need {world} visible GPUs, found {ndev}"
    if plan["process_group"] and backend == "nccl":
        plan["device_id"] = f"cuda:{plan['device']}"
    return plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--rows", type=lambda v: int(float(v)), default=1_000_000_000, help="rows per GPU (1e9 ok)")
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
    ap.add_argument("--slot-records", type=int, default=0,
                    help="N > 1: records per exchange slot (0: qe_hashagg_slot_capacity); a small value forces "
                         "the variable-size fallback")
    ap.add_argument("--verify-cpu", action="store_true",
                    help="check every owner's groups against the CPU port over all ranks' rows (default for N > 1)")
    ap.add_argument("--no-verify-cpu", action="store_true", help="N > 1: skip that check")
    ap.add_argument("--dry-run", action="store_true",
                    help="print this rank's device plan (backend, device, device_id) as JSON and exit before any "
                         "GPU or process-group call (launcher-environment check)")
    ap.add_argument("--assume-gpus", type=int, default=-1, help="--dry-run only: visible GPU count to plan for")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: this process only launches them (no torch, no GPU call here)
        return launch_ranks(args)

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
    ndev = args.assume_gpus if args.dry_run and args.assume_gpus >= 0 else torch.cuda.device_count()
    plan = rank_plan(world, rank, local, args.dist_backend, ndev, args.exchange)
    if args.dry_run:
        print(json.dumps(plan), flush=True)
        return 0 if "error" not in plan else 2
    if "error" in plan:
        sys.exit(plan["error"])
    device = plan["device"]
    torch.cuda.set_device(device)
    if plan["process_group"]:
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29511"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        if plan["device_id"] is not None:
            dist.init_process_group(plan["backend"], device_id=torch.device(plan["device_id"]))
        else:
            dist.init_process_group(plan["backend"])
        world = dist.get_world_size()
        rank = dist.get_rank()
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
    exch_ev = []  # (after the update is queued, after the owner's import) per timed step
    kinds = []
    timing = [False]

    def step():
        partial.reset()
        partial.set_row_base(row0)
        partial.update_fused(cols, spec)
        final = partial
        if exchange:
            if timing[0]:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            owner.reset()
            if comm is not None:
                exchange_partials_native(partial, owner, comm, args.slot_records)
            else:
                exchange_partials(partial, owner, slot_records=args.slot_records or None)
            if timing[0]:
                e1.record()
                exch_ev.append((e0, e1))
            final = owner
        out = final.finalize()
        kernel_ms.append(partial.last_kernel_time())
        return out

    def barrier():
        if world > 1:
            dist.barrier()

    # the same read ceiling before any warm-up (the device straight from idle), for the record
    cc0 = (N.QeColumn * 3)(*[c.as_c() for c in cols])
    ms0 = C.c_double()
    shape0 = C.create_string_buffer(128)
    N.check(N.lib().qe_stream_read_best(ctx.handle, cc0, 3, 1, C.byref(ms0), shape0, 128))
    cold_gbs = rows * BYTES_PER_ROW / (ms0.value * 1e-3) / 1e9
    t_w = time.perf_counter()
    for _ in range(args.warmup):
        step()
    # Clock warm-up (untimed, like the W warm-up steps): on a box fresh from idle the first
    # process's kernels and stream reads ran ~7 % slower (2.65e11 vs 2.85e11 rows/s, ceiling 6.70 vs
    # 7.02 TB/s, same box, back-to-back processes); keep stepping until the device has been busy
    # for QE_BENCH_PREWARM_S seconds (default 2) before the timed region. One rank only: ranks
    # must run the same number of steps (each holds collectives), so N > 1 runs none.
    prewarm_s = float(os.environ.get("QE_BENCH_PREWARM_S", "2")) if world == 1 else 0.0
    prewarm_steps = 0
    while time.perf_counter() - t_w < prewarm_s:
        step()
        torch.cuda.synchronize()
        prewarm_steps += 1
    kinds.append(partial.last_kernel_kind())
    kernel_ms.clear()
    barrier()
    torch.cuda.synchronize()
    timing[0] = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        keys, res = step()
    torch.cuda.synchronize()
    kinds.append(partial.last_kernel_kind())
    barrier()
    elapsed = time.perf_counter() - t0
    timing[0] = False
    launches = sum(k for _, k in kernel_ms)
    avg_kernel_ms = sum(m for m, _ in kernel_ms) / max(1, launches)
    # exchange leg on the device timeline: from the aggregation kernel's queue position to the end
    # of the owner's import (waits for the slowest peer's kernel inside the all-to-all)
    avg_exch_ms = (sum(a.elapsed_time(b) for a, b in exch_ev) / len(exch_ev)) if exch_ev else None
    if world > 1:
        t = torch.tensor([elapsed, avg_kernel_ms, avg_exch_ms or 0.0], dtype=torch.float64, device="cuda")
        if args.dist_backend == "gloo":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, max_kernel_ms, avg_exch_ms = (float(x) for x in t.tolist())
    else:
        max_kernel_ms = avg_kernel_ms

    # stream-read ceiling over the same 24 B/row (k, a, b): best launch shape, median of 5 each
    cc = (N.QeColumn * 3)(*[c.as_c() for c in cols])
    ms = C.c_double()
    shape = C.create_string_buffer(128)
    N.check(N.lib().qe_stream_read_best(ctx.handle, cc, 3, 5, C.byref(ms), shape, 128))
    stream_gbs = rows * BYTES_PER_ROW / (ms.value * 1e-3) / 1e9

    # Result checks before any number is printed: every group present once across owners, and
    # COUNT(*) adds up to the rows an independent torch kernel counts as passing the predicate.
    a_col = cols[1].values[:rows]
    selected = int((a_col > (1 << 19)).sum().item())
    groups = torch.tensor([keys[0].length, int(res[1].to_numpy().sum()), selected], dtype=torch.int64, device="cuda")
    if world > 1:
        if args.dist_backend == "gloo":
            groups = groups.cpu()
        dist.all_reduce(groups)
    n_groups, count_total, selected_total = (int(x) for x in groups.tolist())
    if n_groups != 1024 or count_total != selected_total:
        sys.exit(f"bench: wrong result: {n_groups} groups (want 1024), COUNT(*) total {count_total} "
                 f"(want {selected_total})")
    kv = keys[0].to_numpy()
    rv = [r.to_numpy() for r in res]
    my_groups = {int(kv[i]): tuple(int(r[i]) for r in rv) for i in range(keys[0].length)}
    check = {"groups": n_groups, "count_star_total": count_total, "count_star_torch": selected_total}
    if world > 1 and (args.verify_cpu or not args.no_verify_cpu):
        # union of the owners' groups == the CPU port over every rank's rows (rows 0 .. world*rows)
        everyone = [None] * world
        dist.all_gather_object(everyone, my_groups)
        if rank == 0:
            union = {}
            for g in everyone:
                for k, v in g.items():
                    if k in union:
                        sys.exit(f"bench: group {k} owned by two ranks")
                    union[k] = v
            lib, G = _cpu_lib()
            out = (G * 2048)()
            ng = C.c_int64()
            # the tuned CPU leg (per-thread open-addressing tables, oracle/cpu_baseline.c), after the
            # timed region: 8 ranks x 1B rows take seconds, not minutes
            lib.qe_cpu_c4_fast(0, world * rows, 42, usable_cpus(), 1 << 19, 1024, out, 2048, C.byref(ng))
            want = {int(g.key): (int(g.sum), int(g.count), int(g.min), int(g.max)) for g in out[:ng.value]}
            if union != want:
                bad = sorted(k for k in set(union) | set(want) if union.get(k) != want.get(k))
                sys.exit(f"bench: {len(bad)} groups differ from the CPU port over all ranks' rows, e.g. key {bad[0]}: "
                         f"gpu {union.get(bad[0])} cpu {want.get(bad[0])}")
            check["cpu_port_groups_equal_all_ranks"] = True
    ms_step = elapsed / args.steps * 1e3
    achieved = rows * BYTES_PER_ROW / (avg_kernel_ms * 1e-3) / 1e9
    signature = partial.last_kernel_signature()
    traffic, traffic_note = load_traffic(rows, signature)
    line = {
        "metric": METRIC,
        "value": world * rows / (ms_step * 1e-3),
        "unit": "rows/s",
        "n_gpus": world,
        "world_size": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "kernel_ms": max_kernel_ms,
        "exchange_ms": avg_exch_ms,
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
            "traffic_source": traffic_note,
            "kernel_signature": signature,
            "kernel": ("qe_fused (hipRTC plan-specialised filter+project+LDS hash aggregate)" if kinds[-1][0]
                       else f"k_hashagg generic interpreter ({kinds[-1][1]})"),
            "avg_kernel_ms": avg_kernel_ms,
            "bytes_per_launch": rows * BYTES_PER_ROW,
            "stream_read_ceiling_gbs": stream_gbs,
            "stream_read_cold_gbs": cold_gbs,
            "prewarm_steps": prewarm_steps,
            "stream_read_ceiling_shape": shape.value.decode(),
        },
        "check": check,
    }
    if world > 1 or exchange:
        line["comm"] = {"backend": args.dist_backend, "impl": args.exchange_impl,
                        "rccl_version": (".".join(str(x) for x in torch.cuda.nccl.version())
                                         if args.dist_backend == "nccl" else None)}
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = args.cpu_threads or usable_cpus()
        sample = args.cpu_sample_rows or rows
        cpu_groups, line["cpu_baseline"] = cpu_baseline(sample, threads)
        if sample == rows:
            # the CPU port ran over exactly these rows: every group's SUM/COUNT/MIN/MAX must agree
            if my_groups != cpu_groups:
                bad = sorted(k for k in set(my_groups) | set(cpu_groups) if my_groups.get(k) != cpu_groups.get(k))
                sys.exit(f"bench: {len(bad)} groups differ from the CPU port, e.g. key {bad[0]}: "
                         f"gpu {my_groups.get(bad[0])} cpu {cpu_groups.get(bad[0])}")
            line["check"]["cpu_port_groups_equal"] = True
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
