"""GPU parity: the HIP engine (through the C ABI) against the golden fixtures and the C oracle.

Bar: bit-exact verdicts, prepare messages, output shares, aggregate shares, report
counts and checksums (integer/byte work). The oracle is the checker only.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os

import numpy as np
import pytest

from janus_amd.engine import HelperEngine
from janus_amd.vdaf import Prio3
from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.json"))
                if not os.path.basename(p).startswith("hpke"))


def _vdaf(doc) -> Prio3:
    v = doc["vdaf"]
    return Prio3(v["algo_id"], v["bits"], v["length"], v["chunk_length"], v.get("num_proofs", 1))


def _arrays(doc):
    reps = doc["reports"]
    n = len(reps)

    def cat(key):
        return np.frombuffer(b"".join(bytes.fromhex(r[key]) for r in reps), np.uint8).reshape(n, -1)

    return n, cat("nonce"), cat("public_share") if reps[0]["public_share"] else None, \
        cat("helper_input_share"), cat("leader_prep_share")


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-5] for p in GOLDEN])
@pytest.mark.parametrize("slow", [False, True], ids=["fast", "slowpath"])
def test_golden(path, slow):
    doc = json.load(open(path))
    vdaf = _vdaf(doc)
    n, nonces, ps, his, lps = _arrays(doc)
    with HelperEngine(vdaf, bytes.fromhex(doc["verify_key"])) as eng:
        if slow:
            eng.debug(1, 1)
        res = eng.helper_initialized_batch(nonces, ps if ps is not None else b"", his, lps, want_out_shares=True)
        for i, rep in enumerate(doc["reports"]):
            assert int(res.verdicts[i]) == rep["verdict"], (i, rep["tamper"])
            if rep["verdict"] == 0:
                assert res.prep_msgs[i].tobytes().hex() == rep["prep_msg"]
                assert hashlib.sha256(res.out_shares[i].tobytes()).hexdigest() == rep["out_share_sha256"], i
        eng.accumulate(n)
        agg, count, checksum = eng.aggregate_share(0)
        if "aggregate_share" in doc:
            assert agg.hex() == doc["aggregate_share"]
        else:
            assert hashlib.sha256(agg).hexdigest() == doc["aggregate_share_sha256"]
        assert count == doc["report_count"]
        assert checksum.hex() == doc["checksum"]


def _random_batch(orc: O.Prio3Oracle, vk, n, seed, tamper_every=7):
    rng = np.random.default_rng(seed)
    a, (algo, bits, length, chunk, _) = orc.algo, orc.params
    if a in (O.SUMVEC, O.SUMVEC_F64_MULTIPROOF):
        meas = rng.integers(0, 1 << bits, size=(n, length), dtype=np.uint64)
    elif a == O.SUM:
        meas = rng.integers(0, 1 << bits, size=(n, 1), dtype=np.uint64)
    elif a == O.HISTOGRAM:
        meas = rng.integers(0, length, size=(n, 1), dtype=np.uint64)
    else:
        meas = rng.integers(0, 2, size=(n, 1), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
    for i in range(0, n, tamper_every):  # flip one random bit of the leader prep share
        j = int(rng.integers(0, lps.shape[1]))
        lps[i, j] ^= 1 << int(rng.integers(0, 8))
    return nonces, ps, his, lps


CASES = {
    "count": Prio3.count(),
    "sum32": Prio3.sum(32),
    # Sum's v uses geometric sums over the bits of C = bits: one call, odd and non-power-of-2 counts
    "sum1": Prio3.sum(1),
    "sum5": Prio3.sum(5),
    "sum17": Prio3.sum(17),
    "sum31": Prio3.sum(31),
    # bits > 32 (Janus's VdafInstance::Prio3Sum{bits} has no 32-bit cap, core/src/vdaf.rs:65-108)
    "sum33": Prio3.sum(33),
    "sum64": Prio3.sum(64),
    "sumvec_33x5_7": Prio3.sum_vec(33, 5, 7),
    "sumvec_64x20_9": Prio3.sum_vec(64, 20, 9),
    "sumvec_small": Prio3.sum_vec(3, 37, 5),
    "sumvec_8x1000_88": Prio3.sum_vec(8, 1000, 88),
    "histogram_256_16": Prio3.histogram(256, 16),
    "histogram_100_7": Prio3.histogram(100, 7),
}


@pytest.mark.parametrize("name", list(CASES))
def test_random_batches_vs_oracle(name):
    vdaf = CASES[name]
    vk = bytes(range(100, 116))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    n = 200 if name == "sumvec_8x1000_88" else 333
    nonces, ps, his, lps = _random_batch(orc, vk, n, seed=sum(map(ord, name)))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    with HelperEngine(vdaf, vk) as eng:
        res = eng.helper_initialized_batch(nonces, ps, his, lps, want_out_shares=True)
        np.testing.assert_array_equal(res.verdicts, want["verdicts"])
        fin = want["verdicts"] == 0
        assert fin.sum() > n // 2
        np.testing.assert_array_equal(res.prep_msgs[fin], want["prep_msgs"][fin])
        np.testing.assert_array_equal(res.out_shares[fin], want["out_shares"][fin])
        eng.accumulate(n)
        agg, count, cs = eng.aggregate_share(0)
        assert agg == want["agg"] and count == want["count"] and cs == want["checksum"]
        # fused path gives the same aggregation (into another segment)
        v2, m2 = eng.prep_and_aggregate(nonces, ps, his, lps, segment=7)
        np.testing.assert_array_equal(v2, want["verdicts"])
        agg7, count7, cs7 = eng.aggregate_share(7)
        assert agg7 == want["agg"] and count7 == want["count"] and cs7 == want["checksum"]


def test_count_grid_stride_select():
    """300k Count reports: more than the select kernel's 1024 x 256 threads, so every thread folds
    several reports' SHA-256 into the checksum; 4096 accumulate chunks of the single element."""
    vdaf = Prio3.count()
    vk = bytes(range(16))
    orc = O.Prio3Oracle(vdaf.algo_id)
    n = 300_000
    nonces, ps, his, lps = _random_batch(orc, vk, n, seed=0xC0)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    with HelperEngine(vdaf, vk) as eng:
        v, _ = eng.prep_and_aggregate(nonces, ps, his, lps, segment=0)
        np.testing.assert_array_equal(v, want["verdicts"])
        agg, count, cs = eng.aggregate_share(0)
    assert agg == want["agg"] and count == want["count"] and cs == want["checksum"]


def test_mask_and_segments():
    vdaf = Prio3.histogram(64, 8)
    vk = bytes(16)
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    n = 777
    nonces, ps, his, lps = _random_batch(orc, vk, n, seed=5)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    rng = np.random.default_rng(9)
    mask = rng.integers(0, 2, size=n).astype(np.uint8)
    seg = rng.integers(0, 3, size=n).astype(np.uint32)
    with HelperEngine(vdaf, vk) as eng:
        eng.helper_initialized_batch(nonces, ps, his, lps)
        eng.accumulate(n, mask, seg)
        for s in range(3):
            sel = (want["verdicts"] == 0) & (mask == 1) & (seg == s)
            exp = orc.aggregate([want["out_shares"][i].tobytes() for i in np.nonzero(sel)[0]])
            cs = bytes(32)
            for i in np.nonzero(sel)[0]:
                cs = bytes(a ^ b for a, b in zip(cs, O.sha256(nonces[i].tobytes())))
            agg, count, checksum = eng.aggregate_share(s)
            assert agg == exp and count == int(sel.sum()) and checksum == cs


def test_empty_and_tiny_batches():
    vdaf = Prio3.sum_vec(8, 1000, 88)
    vk = bytes(range(16))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    nonces, ps, his, lps = _random_batch(orc, vk, 3, seed=1, tamper_every=100)
    with HelperEngine(vdaf, vk) as eng:
        res = eng.helper_initialized_batch(nonces[:0], ps[:0], his[:0], lps[:0])
        assert res.verdicts.shape == (0,)
        eng.accumulate(0)
        for k in (1, 2, 3):
            res = eng.helper_initialized_batch(nonces[:k], ps[:k], his[:k], lps[:k])
            want = orc.helper_prep_batch(vk, nonces[:k], ps[:k], his[:k], lps[:k])
            np.testing.assert_array_equal(res.verdicts, want["verdicts"])


def test_full_size_cycled_pool_property():
    """2^15 SumVec(8x1000/88) reports = a pool of 64 distinct reports cycled 512 times:
    aggregate == 512 * pool aggregate (mod p), count == 512 * pool count."""
    vdaf = Prio3.sum_vec(8, 1000, 88)
    vk = bytes(range(16))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    K, reps = 64, 512
    nonces, ps, his, lps = _random_batch(orc, vk, K, seed=11, tamper_every=9)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    p = 2**128 - 28 * 2**64 + 1
    pool = [int.from_bytes(want["agg"][16 * i:16 * i + 16], "little") for i in range(1000)]
    exp = b"".join(((reps * x) % p).to_bytes(16, "little") for x in pool)
    tile = lambda a: np.ascontiguousarray(np.tile(a, (reps, 1)))  # noqa: E731
    with HelperEngine(vdaf, vk) as eng:
        v, _ = eng.prep_and_aggregate(tile(nonces), tile(ps), tile(his), tile(lps))
        np.testing.assert_array_equal(v, np.tile(want["verdicts"], reps))
        agg, count, cs = eng.aggregate_share(0)
        assert count == reps * want["count"]
        assert agg == exp
        assert cs == bytes(32)  # each report id appears an even number of times


def test_multi_part_combine():
    """Per-GPU partial aggregates combined on device (the RCCL all-gather + mod-p add step)."""
    import torch

    vdaf = Prio3.sum_vec(8, 1000, 88)
    vk = bytes(range(16))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    nonces, ps, his, lps = _random_batch(orc, vk, 96, seed=3)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    parts = torch.zeros((3, 16000), dtype=torch.uint8, device="cuda")
    engs = [HelperEngine(vdaf, vk) for _ in range(3)]
    for k, eng in enumerate(engs):
        sl = slice(32 * k, 32 * (k + 1))
        eng.prep_and_aggregate(nonces[sl], ps[sl], his[sl], lps[sl])
        eng.export_aggregate_device(0, parts[k].data_ptr())
        eng.sync()
    out = torch.zeros(16000, dtype=torch.uint8, device="cuda")
    engs[0].combine_device(parts.data_ptr(), 3, out.data_ptr())
    engs[0].sync()
    assert out.cpu().numpy().tobytes() == want["agg"]
    for e in engs:
        e.close()


@pytest.mark.parametrize("name", ["count", "sumvec_small", "histogram_256_16"])
def test_shard_records_device_merge(name):
    """Shard records exported per engine, merged on the device (the step after the RCCL
    all-gather, janus_amd/distributed.py) == host merge == oracle over the whole batch."""
    import torch

    from janus_amd import distributed as D

    vdaf = CASES[name]
    vk = bytes(range(16))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    n, world = 150, 3
    nonces, ps, his, lps = _random_batch(orc, vk, n, seed=21)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    engs = [HelperEngine(vdaf, vk) for _ in range(world)]
    nb = engs[0].record_bytes()
    assert nb == D.record_bytes(vdaf.output_len, vdaf.field_bytes)
    recs = torch.zeros((world, nb), dtype=torch.uint8, device="cuda")
    for r, eng in enumerate(engs):
        a, b = D.shard_range(n, r, world)
        eng.prep_and_aggregate(nonces[a:b], ps[a:b], his[a:b], lps[a:b])
        eng.export_record_device(0, recs[r].data_ptr())
        eng.sync()
    out = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    engs[0].combine_records_device(recs.data_ptr(), world, out.data_ptr())
    engs[0].sync()
    agg, count, cs = D.unpack_record(out.cpu().numpy(), vdaf.field_bytes)
    assert (agg, count, cs) == (want["agg"], want["count"], want["checksum"])
    assert D.merge_records(recs.cpu().numpy(), vdaf.field_bytes) == (agg, count, cs)
    for e in engs:
        e.close()


@pytest.mark.parametrize("split", [3, 5, 6, 7], ids=["lanes", "fused", "pairs", "words"])
@pytest.mark.parametrize("name", ["sumvec_8x1000_88", "histogram_256_16", "sum64", "sumvec_small", "sumvec_64x20_9",
                                  "sum5", "sum32"])
def test_k1_split_variants(name, split):
    """The four helper K1 kernels == the oracle, fast and slow path: the word-per-lane kernel (each sponge
    over 25 lanes, a report per wave, the truncation in its own kernel; the engine's choice up to one
    report-wave per SIMD, i.e. every small test batch), the lane-pair kernel (every sponge split over two
    lanes), the lane-split kernel (S and J sponges in the two halves of a wave) and the fused two-sponge
    kernel (the engine's choice for large launches). n = 150 spans three 64-report blocks and a partial
    workgroup. sum5 has its whole joint_rand_part message in one block; sum64 and sumvec_64x20_9
    (bits > 32) run the fused kernel when pairs or words are asked for."""
    vdaf = CASES[name]
    vk = bytes(range(60, 76))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    n = 150
    nonces, ps, his, lps = _random_batch(orc, vk, n, seed=split * 7 + sum(map(ord, name)))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    with HelperEngine(vdaf, vk) as eng:
        eng.debug(3, split)
        res = eng.helper_initialized_batch(nonces, ps, his, lps, want_out_shares=True)
        np.testing.assert_array_equal(res.verdicts, want["verdicts"])
        fin = want["verdicts"] == 0
        np.testing.assert_array_equal(res.prep_msgs[fin], want["prep_msgs"][fin])
        np.testing.assert_array_equal(res.out_shares[fin], want["out_shares"][fin])
        eng.accumulate(n)
        assert eng.aggregate_share(0) == (want["agg"], want["count"], want["checksum"])
        eng.debug(1, 1)  # slow path behind either K1 kernel
        res = eng.helper_initialized_batch(nonces, ps, his, lps)
        np.testing.assert_array_equal(res.verdicts, want["verdicts"])


@pytest.mark.parametrize("name", ["sumvec_8x1000_88", "histogram_256_16", "sumvec_64x20_9", "sumvec_small"])
def test_k3_ring_padded_groups(name):
    """The ParallelSum FLP part kernel (the depth-4 LDS-DMA ring, 4 slot groups per workgroup) == the
    oracle, helper (verdicts, messages, output shares, aggregate) and leader (prep shares).
    sumvec_64x20_9 and sumvec_small have a padded last group and workgroup."""
    vdaf = CASES[name]
    vk = bytes(range(90, 106))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    n = 150
    nonces, ps, his, lps = _random_batch(orc, vk, n, seed=231 + sum(map(ord, name)))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    with HelperEngine(vdaf, vk) as eng:
        res = eng.helper_initialized_batch(nonces, ps, his, lps, want_out_shares=True)
        np.testing.assert_array_equal(res.verdicts, want["verdicts"])
        fin = want["verdicts"] == 0
        np.testing.assert_array_equal(res.prep_msgs[fin], want["prep_msgs"][fin])
        np.testing.assert_array_equal(res.out_shares[fin], want["out_shares"][fin])
        eng.accumulate(n)
        assert eng.aggregate_share(0) == (want["agg"], want["count"], want["checksum"])
    rng = np.random.default_rng(21)
    meas = rng.integers(0, 1 << vdaf.bits, size=(24, vdaf.length), dtype=np.uint64) \
        if vdaf.algo_id == O.SUMVEC else rng.integers(0, vdaf.length, size=(24, 1), dtype=np.uint64)
    ln = rng.integers(0, 256, size=(24, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(24, orc.sizes.client_rand), dtype=np.uint8)
    shards = [orc.shard(meas[i], ln[i].tobytes(), rands[i].tobytes()) for i in range(24)]
    lps_, lis_ = (np.stack([np.frombuffer(s[k], np.uint8) for s in shards]) for k in (0, 1))
    with HelperEngine(vdaf, vk) as eng:
        init = eng.leader_initialized_batch(ln, lps_, lis_)
    for i in range(24):
        rc, share, _, _ = orc.prep_init(vk, 0, ln[i].tobytes(), lps_[i].tobytes(), lis_[i].tobytes())
        assert rc == 0 and init.prep_shares[i].tobytes() == share, i


@pytest.mark.parametrize("name", ["sumvec_small", "histogram_256_16"])
def test_mixed_k1_launch(name):
    """A helper launch past one lane-split wave per SIMD (40,960 reports on MI355X: round_reports / 4 = 32,768)
    runs its first 32,768 reports lane-split on the engine stream and the rest as lane pairs on the side stream
    (prep_core, bufs_tail). Every verdict, finished prep message and output share, and the aggregate, == the
    oracle's (a 512-report pool tiled)."""
    vdaf = CASES[name]
    vk = bytes(range(140, 156))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    K, n = 512, 40960
    nonces, ps, his, lps = _random_batch(orc, vk, K, seed=4096 + sum(map(ord, name)))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    idx = np.arange(n) % K
    with HelperEngine(vdaf, vk) as eng:
        res = eng.helper_initialized_batch(nonces[idx], ps[idx], his[idx], lps[idx], want_out_shares=True)
        np.testing.assert_array_equal(res.verdicts, want["verdicts"][idx])
        fin = want["verdicts"][idx] == 0
        np.testing.assert_array_equal(res.prep_msgs[fin], want["prep_msgs"][idx][fin])
        np.testing.assert_array_equal(res.out_shares[fin], want["out_shares"][idx][fin])
        eng.accumulate(n)
        agg, count, cs = eng.aggregate_share(0)
        assert count == int(fin.sum())
        assert agg == orc.aggregate([want["out_shares"][i].tobytes() for i in idx[fin]])
        exp_cs = bytes(32)
        for i, f in zip(idx, fin):  # XOR of SHA-256(id): tiled ids cancel in pairs
            if f:
                exp_cs = bytes(a ^ b for a, b in zip(exp_cs, O.sha256(nonces[i].tobytes())))
        assert cs == exp_cs
