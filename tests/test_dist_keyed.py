"""Partials across ranks: dictionary-keyed (exchange_keyed_partials) and numeric keys through the
fixed-capacity slot exchange and its overflow fallback, and deterministic (fixed-point) fp64 sums
that must equal math.fsum over both ranks' rows after the exchange. Two processes on the one GPU, gloo
backend (RCCL cannot put two ranks on one device); see tests/dist_keyed_worker.py."""
import json
import os
import pathlib
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_keyed_exchange_two_ranks():
    root = pathlib.Path(__file__).resolve().parents[1]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(root / "tests" / "dist_keyed_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(line[0][len("RESULT "):])
    assert all(res[m]["ok"] for m in ("utf8", "tuple", "slots", "slots_overflow", "deterministic", "global")), res
