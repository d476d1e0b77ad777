"""GPU: bench.py's N>1 path end to end on a 1-GPU box (`--share-gpu`): two ranks under
torch.distributed.run prepare DIFFERENT global report ranges on cuda:0, exchange their shard records
over gloo and merge them on the device; each rank checks its own aggregate against its range and the
merged record against the union (CyclicPool). The driver's 8-GPU scaling run takes the same code path
with RCCL instead of gloo; the CPU tests (test_distributed.py) cover the range arithmetic at worlds 2
and 3 without the engine.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.timeout(300)
def test_two_ranks_on_one_gpu_verify():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--share-gpu", "--reports-per-gpu", "20000", "--pool", "4096", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--no-secondary"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_reports_per_step"] == 40000
    assert out["verified"] is True and out["verification"]["all_ranks"] is True, out.get("verification")
    # the self-checking fields the 8-GPU run carries: the collective's world, ranks verified, timing spread
    assert out["rccl_world"] == 2 and out["ranks_verified"] == 2
    assert out["elapsed_spread"] >= 1.0
