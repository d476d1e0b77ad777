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


_NO_GPU_RUNTIME = """
import sys, types
class _Untouchable(types.ModuleType):
    def __getattr__(self, k):
        raise SystemExit("torch touched before the launcher: torch." + k)
sys.modules["torch"] = _Untouchable("torch")
am = types.ModuleType("amdsmi")
def _fail(*a):
    raise RuntimeError("amdsmi unavailable")
am.amdsmi_init = _fail
sys.modules["amdsmi"] = am
sys.path.insert(0, ROOT)
import bench
"""


def test_bench_refuses_when_gpus_cannot_be_counted():
    """With amdsmi failing and no KFD topology, bench.py --gpus 2 refuses (exit != 0) before any launcher,
    and never reaches torch (whose device count could initialise HIP in this process)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _NO_GPU_RUNTIME.replace("ROOT", repr(root)) + "bench.ensure_world(2, sysfs_root='/nonexistent/kfd')\n"
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "cannot count the node's GPUs" in r.stderr and "torch touched" not in r.stderr


def test_count_gpus_from_kfd_topology(tmp_path):
    """Without amdsmi, the GPU count comes from the KFD topology (nodes with SIMDs), limited by the
    visibility variables; torch is never imported for it."""
    import subprocess
    import sys

    for i, simds in enumerate((0, 1024, 1024, 0, 1024)):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 16\nsimd_count {simds}\nmax_waves_per_simd 8\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _NO_GPU_RUNTIME.replace("ROOT", repr(root)) + f"print(bench.count_gpus({str(tmp_path)!r}))\n"
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES",
                                                             "CUDA_VISIBLE_DEVICES")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "3", r.stderr
    r = subprocess.run([sys.executable, "-c", code], env=dict(env, HIP_VISIBLE_DEVICES="0,1"), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "2", r.stderr


def _bench_shard_rank(rank, world, port, name, R, q):
    """One rank of bench.py's N > 1 verification on CPU: the rank's global reports [r R, (r+1) R) of the
    cyclic pool tiling (here prepared by the oracle instead of the engine), its shard record checked
    against bench.CyclicPool's expectation, the records all-gathered (gloo) and merged, the merge
    checked against the expectation over every rank's range."""
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bench
        from oracle import oracle as O

        doc, K, nonces, ps, his, lps = _load(name)
        v = doc["vdaf"]
        vk = bytes.fromhex(doc["verify_key"])
        orc = O.Prio3Oracle(v["algo_id"], v["bits"], v["length"], v["chunk_length"])
        fb = orc.sizes.field_bytes
        p = D.P64 if fb == 8 else D.P128
        prep = lambda a, b: orc.helper_prep_batch(vk, nonces[a:b], ps[a:b], his[a:b], lps[a:b])  # noqa: E731
        full = prep(0, K)
        block = 3
        blocks = [bench.field_elems(prep(b, min(K, b + block))["agg"], fb) for b in range(0, K, block)]
        cyc = bench.CyclicPool(full["verdicts"] == 0, blocks, block, lambda a, r: bench.field_elems(prep(a, r)["agg"], fb), p)
        start, stop = D.shard_range(R * world, rank, world)
        idx = (start + np.arange(stop - start)) % K
        mine = orc.helper_prep_batch(vk, nonces[idx], ps[idx], his[idx], lps[idx])  # what the rank's engine computes
        exp, cnt = cyc.range(start, stop)
        enc = b"".join(x.to_bytes(fb, "little") for x in exp)
        own_ok = mine["agg"] == enc and mine["count"] == cnt
        rec = torch.from_numpy(D.pack_record(mine["agg"], mine["count"], mine["checksum"]))
        agg, count, _ = D.merge_records(D.all_gather_records(rec).numpy(), fb)
        all_exp, all_cnt = cyc.range(0, R * world)
        merged_ok = agg == b"".join(x.to_bytes(fb, "little") for x in all_exp) and count == all_cnt
        # a rank that merged its own record twice instead of its neighbour's would not match
        dup = D.merge_aggregate_shares([mine["agg"]] * world, fb)
        q.put((rank, own_ok, merged_ok, dup != agg or world == 1, ""))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure in the parent
        q.put((rank, False, False, False, repr(e)))


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("name,R", [("sumvec_small.json", 23), ("count.json", 17)])
def test_bench_distinct_shard_expectations(world, name, R):
    """bench.py's N > 1 verification: ranks hold distinct global report ranges, and the expected rank
    and merged aggregates follow from the range offsets (bench.CyclicPool), not from `x world`."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_shard_rank, args=(r, world, port, name, R, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, own_ok, merged_ok, distinct, err in out:
        assert not err, err
        assert own_ok and merged_ok and distinct, (rank, own_ok, merged_ok, distinct)


def test_cyclic_pool_ranges_match_direct_sums():
    """CyclicPool.range == the direct sum over the tiled range, for ranges crossing block and pool
    boundaries (small integers instead of field elements)."""
    import bench

    rng = np.random.default_rng(3)
    K, block, p = 11, 4, 2**61 - 1
    vals = rng.integers(0, 1000, size=(K, 3))
    fin = rng.random(K) < 0.8
    contrib = [[int(x) if fin[i] else 0 for x in vals[i]] for i in range(K)]
    blocks = [[sum(contrib[i][j] for i in range(b, min(K, b + block))) for j in range(3)] for b in range(0, K, block)]
    partial = lambda a, r: [sum(contrib[i][j] for i in range(a, r)) for j in range(3)]  # noqa: E731
    cyc = bench.CyclicPool(fin, blocks, block, partial, p)
    for lo, hi in [(0, 0), (0, 5), (3, 9), (7, 30), (12, 13), (0, 44), (5, 100), (40, 41)]:
        want = [sum(contrib[g % K][j] for g in range(lo, hi)) % p for j in range(3)]
        assert cyc.range(lo, hi) == (want, sum(int(fin[g % K]) for g in range(lo, hi))), (lo, hi)
        assert cyc.range(lo, hi, 3) == ([3 * w % p for w in want], 3 * sum(int(fin[g % K]) for g in range(lo, hi)))
