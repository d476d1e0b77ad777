"""Multi-rank report sharding + shard-record combine over torch.distributed (gloo, CPU).

Mirrors Janus's sharded batch aggregations: every writer adds into one shard row
(aggregation_job_writer.rs:527) and compute_aggregate_share merges all of them
(aggregate_share.rs:55-96). Each rank prepares its contiguous report range (here with the
C oracle, the checker — the GPU ranks use the engine, tests/test_gpu_parity.py), packs its
shard record, all-gathers the records and merges them; the result must equal the golden
fixture's whole-batch aggregate share, count and checksum.
"""
from __future__ import annotations

import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from janus_amd import distributed as D

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _load(name):
    doc = json.load(open(os.path.join(GOLDEN, name)))
    reps = doc["reports"]
    n = len(reps)

    def cat(k):
        return np.frombuffer(b"".join(bytes.fromhex(r[k]) for r in reps), np.uint8).reshape(n, -1)

    return doc, n, cat("nonce"), cat("public_share") if reps[0]["public_share"] else np.zeros((n, 0), np.uint8), \
        cat("helper_input_share"), cat("leader_prep_share")


def _rank_main(rank, world, port, name, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import oracle as O

        doc, n, nonces, ps, his, lps = _load(name)
        v = doc["vdaf"]
        orc = O.Prio3Oracle(v["algo_id"], v["bits"], v["length"], v["chunk_length"])
        a, b = D.shard_range(n, rank, world)
        res = orc.helper_prep_batch(bytes.fromhex(doc["verify_key"]), nonces[a:b], ps[a:b], his[a:b], lps[a:b])
        rec = torch.from_numpy(D.pack_record(res["agg"], res["count"], res["checksum"]))
        gathered = D.all_gather_records(rec)
        agg, count, checksum = D.merge_records(gathered.numpy(), orc.sizes.field_bytes)
        q.put((rank, agg.hex(), count, checksum.hex(), gathered.shape[0]))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure in the parent
        q.put((rank, "error", repr(e), "", 0))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["sumvec_small.json", "count.json", "histogram_16_4.json"])
def test_sharded_combine_gloo(world, name):
    doc = json.load(open(os.path.join(GOLDEN, name)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, agg, count, checksum, nrec in out:
        assert agg != "error", count
        assert nrec == world
        assert agg == doc["aggregate_share"]
        assert count == doc["report_count"]
        assert checksum == doc["checksum"]


def test_shard_range_partition():
    for n in (0, 1, 7, 64, 1000, 1_250_000):
        for world in (1, 2, 3, 8):
            spans = [D.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        D.shard_range(10, 2, 2)


def test_merge_rejects_noncanonical():
    p = D.P128
    good = (5).to_bytes(16, "little")
    bad = p.to_bytes(16, "little")
    assert D.merge_aggregate_shares([good, good], 16) == (10).to_bytes(16, "little")
    assert D.merge_aggregate_shares([(p - 1).to_bytes(16, "little"), (2).to_bytes(16, "little")], 16) == \
        (1).to_bytes(16, "little")
    with pytest.raises(ValueError):
        D.merge_aggregate_shares([good, bad], 16)
    with pytest.raises(ValueError):
        D.merge_aggregate_shares([good, good[:8]], 16)


def test_record_roundtrip():
    agg = bytes(range(32))
    rec = D.pack_record(agg, 123456789, bytes(range(100, 132)))
    assert rec.size == D.record_bytes(2, 16)
    assert D.unpack_record(rec, 16) == (agg, 123456789, bytes(range(100, 132)))


def test_bench_refuses_world_mismatch():
    """bench.py --gpus 2 under a launcher world of another size exits non-zero (no silent 1-GPU run)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                       env=dict(os.environ, WORLD_SIZE="3"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr
