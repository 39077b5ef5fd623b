"""Worker for tests/test_c5_ranks.py::test_c5_two_ranks_gloo (torch.distributed.run, 2 ranks sharing
cuda:0, gloo): each rank runs the C5 fused plan (BASELINE configs[4], Q1-like) over its own row
range of the generator with its row base, exchange_partials moves each (returnflag, linestatus)
group to its owner (hash(key) mod world) — through the fixed slots and, with one-record slots,
through the overflow fallback — and rank 0 compares the union of the owners' groups with the exact
C oracle over both ranks' rows (tests/c5_check.py), in the default exact mode and the opt-in
fp64-atomics mode. Main.kt:1309-1325 (partials per partition, merged)."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd"), str(ROOT / "tests")]

import torch.distributed as dist  # noqa: E402

from c5_check import c5_oracle, check_groups  # noqa: E402

ROW0, N0, N1 = 5_000_000_000, 3_000_001, 2_500_000


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import Context
    from kquery.datasource import C5_COLUMNS, generate_column
    from kquery.exchange import exchange_partials
    from kquery.workloads import C5_AGGS, C5_KEY_TYPES, c5_spec

    ctx = Context.get(0)
    row0 = ROW0 if rank == 0 else ROW0 + N0
    n = N0 if rank == 0 else N1
    cols = [generate_column(s, n, row0, 42, ctx) for s in C5_COLUMNS]
    want = c5_oracle(ROW0, N0 + N1) if rank == 0 else None
    results = {}
    for fast in (False, True):
        for cap in (None, 1):
            partial = HashAggregateState(ctx, C5_KEY_TYPES, C5_AGGS, 16, fast_fp64=fast)
            owner = HashAggregateState(ctx, C5_KEY_TYPES, C5_AGGS, 16, fast_fp64=fast)
            partial.set_row_base(row0)
            partial.update_fused(cols, c5_spec())
            exchange_partials(partial, owner, slot_records=cap)
            kk, aa = owner.finalize()
            ctx.synchronize()
            mine = [list(r) for r in zip(*([c.to_pylist() for c in kk] + [c.to_pylist() for c in aa]))]
            every = [None] * world
            dist.all_gather_object(every, mine)
            if rank == 0:
                ok, why = check_groups([r for rows in every for r in rows], want, exact=not fast)
                results[f"{'fast' if fast else 'exact'}-{'overflow' if cap else 'slots'}"] = {"ok": ok, "why": why}
    if rank == 0:
        print("RESULT " + json.dumps(results), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
