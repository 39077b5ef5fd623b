"""bench.py's multi-rank step (VERDICT r02 "make the 8-GPU run real"): `bench.py --gpus N` with no
launcher environment starts N ranks itself (torch.distributed.run as a child process), and each
rank runs the exact timed step — stream-ordered fused C4 update with its global row base, the slot
exchange of partial aggregates (or its variable-size fallback), the owner's merge, finalize. Rank 0
then checks the union of every owner's groups against the CPU port over all ranks' rows (the
default for N > 1; oracle/cpu_baseline.c restating Main.kt:615-651 and the K:1309-1325 merge).

On the one-GPU box the ranks share cuda:0 over gloo (RCCL cannot put two ranks on one device); the
RCCL leg itself is covered by tests/test_native_comm.py and the driver's multi-GPU runs."""
import json
import os
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _run(args, timeout=600):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def _line(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    return json.loads(lines[0])


def test_bench_refuses_more_ranks_than_gpus():
    """Plain `--gpus N` (RCCL) on a machine with fewer than N GPUs fails loudly: no 1-rank line."""
    import torch

    n = max(2, torch.cuda.device_count() + 1)
    r = _run(["--gpus", str(n), "--rows", "1e6", "--steps", "1", "--warmup", "0", "--no-cpu"], timeout=120)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "visible GPUs" in r.stderr


@pytest.mark.parametrize("local", range(8))
def test_bench_rank_plan_eight_gpus(local):
    """The driver's 8-GPU run (`torch.distributed.run --nproc-per-node 8 bench.py --gpus 8`): in that
    launcher environment every rank drives the GPU of its LOCAL_RANK and binds its RCCL
    communicator to it (init_process_group device_id). A dry run prints the plan without touching
    a GPU or the process group."""
    env = dict(os.environ, WORLD_SIZE="8", RANK=str(local), LOCAL_RANK=str(local), MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29599")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--dry-run", "--assume-gpus", "8"],
                       capture_output=True, text=True, timeout=300, env=env)
    plan = _line(r)
    assert plan["backend"] == "nccl" and plan["world_size"] == 8 and plan["rank"] == local
    assert plan["device"] == local and plan["device_id"] == f"cuda:{local}" and plan["process_group"]


def test_bench_rank_plan_refuses_shared_rccl_gpus():
    """Eight RCCL ranks with fewer visible GPUs: the plan is an error, never ranks sharing a device."""
    env = dict(os.environ, WORLD_SIZE="8", RANK="5", LOCAL_RANK="5")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--dry-run", "--assume-gpus", "4"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2 and "need 8 visible GPUs" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("slot_records", [0, 40])
def test_bench_two_ranks_self_launch(slot_records):
    """slot_records 0: the fixed-slot fast path; 40: every slot overflows (1024 groups / 2 owners),
    so all ranks take the counts + records fallback."""
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--rows", "1e7", "--steps", "2", "--warmup", "1",
              "--slot-records", str(slot_records)])  # (the CPU check is the N > 1 default)
    line = _line(r)
    assert line["n_gpus"] == 2 and line["world_size"] == 2
    assert line["value"] > 0 and line["exchange_ms"] is not None and line["exchange_ms"] > 0
    assert line["check"]["groups"] == 1024
    assert line["check"]["count_star_total"] == line["check"]["count_star_torch"]
    assert line["check"]["cpu_port_groups_equal_all_ranks"] is True
    assert "gloo all-to-all" in line["config"]["parallelism"]
