"""GPU: the N > 1 path executed — two ranks, each with the real engine on its report shard, shard
records all-gathered over torch.distributed (gloo, host-staged: a 1-GPU box has no RCCL peer) and
merged on the device. Result == the golden fixture's whole-batch aggregate share, count, checksum
(compute_aggregate_share, aggregator/src/aggregator/aggregate_share.rs:55-96).
"""
from __future__ import annotations

import hashlib
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("name", ["sumvec_8x1000_88.json", "fixedpoint16_37.json", "count.json"])
def test_two_ranks_engine_shards_and_device_merge(name):
    world, port = 2, _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), name],
                              env=dict(env, RANK=str(r), LOCAL_RANK="0"), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    for p in procs:
        so, se = p.communicate(timeout=240)
        assert p.returncode == 0, se[-2000:]
        outs.append(json.loads(so.strip().splitlines()[-1]))
    doc = json.load(open(os.path.join(HERE, "golden", name)))
    want_sha = hashlib.sha256(bytes.fromhex(doc["aggregate_share"])).hexdigest() if "aggregate_share" in doc \
        else doc["aggregate_share_sha256"]
    for o in outs:
        assert o["agg_sha"] == want_sha
        assert o["count"] == doc["report_count"] and o["checksum"] == doc["checksum"]
    assert sum(o["own_count"] for o in outs) == doc["report_count"]
    assert outs[0]["shard"][1] == outs[1]["shard"][0]  # contiguous shards


@pytest.mark.parametrize("name", ["sumvec_8x1000_88.json", "fixedpoint16_37.json", "count.json"])
def test_rccl_world1_shard_combine(name):
    """the RCCL branch of ShardCombiner executed -- an nccl (RCCL) process group of world
    size 1 on the box's GPU, device-tensor all-gather ordered against the engine's own stream by stream
    waits (no host sync between export, gather and merge; two combines queued back to back), merged
    record == the golden fixture."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(HERE, "dist_worker.py"), name, "nccl"], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    o = json.loads(p.stdout.strip().splitlines()[-1])
    doc = json.load(open(os.path.join(HERE, "golden", name)))
    want_sha = hashlib.sha256(bytes.fromhex(doc["aggregate_share"])).hexdigest() if "aggregate_share" in doc \
        else doc["aggregate_share_sha256"]
    assert o["backend"] == "nccl"
    assert o["agg_sha"] == want_sha and o["count"] == doc["report_count"] and o["checksum"] == doc["checksum"]


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N never silently measures fewer GPUs (here: N beyond the visible ones)."""
    import torch

    n = torch.cuda.device_count() + 1
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", str(n)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "GPU(s) visible" in (r.stderr + r.stdout)
