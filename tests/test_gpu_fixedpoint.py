"""GPU parity of Prio3FixedPointBoundedL2VecSum (BASELINE configs[4]; Janus builds it at
aggregator/src/aggregator.rs:916-932 with FixedI16<U15> / FixedI32<U31>).

Helper prep (fast and slow XOF paths), leader prep_init, the leader <-> helper ping-pong and
accumulation are compared with the C oracle byte for byte (verdicts, prep shares, prepare
messages, output shares, aggregate shares, counts, checksums). Reports whose claimed squared norm
is wrong (a client with a vector of norm >= 1) must be rejected exactly like the oracle rejects
them. Parity with prio 0.16.1 itself is unpinned; the aggregate of the reference's
own end-to-end measurements decodes to the reference's expected result.
"""
from __future__ import annotations

import numpy as np
import pytest

from janus_amd.engine import HelperEngine
from janus_amd.vdaf import Prio3
from oracle import oracle as O
from tests.golden.make_golden import fixedpoint_measurements

pytestmark = pytest.mark.gpu

P128 = 2**128 - 28 * 2**64 + 1

CASES = {
    "fp16_len3": (16, 3),
    "fp32_len3": (32, 3),
    "fp16_len37": (16, 37),      # short last chunks in both gadgets
    "fp32_len100": (32, 100),
    "fp16_len1000": (16, 1000),
    "fp16_len10000": (16, 10000),  # configs[4]
}


def _batch(orc, vdaf, vk, n, seed, tamper_every=7):
    rng = np.random.default_rng(seed)
    meas = fixedpoint_measurements(vdaf.bits, vdaf.length, rng, n)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
    for i in range(0, n, tamper_every):  # one random bit of the leader prep share
        j = int(rng.integers(0, lps.shape[1]))
        lps[i, j] ^= 1 << int(rng.integers(0, 8))
    return meas, nonces, ps, his, lps


@pytest.mark.parametrize("slow", [False, True], ids=["fast", "slowpath"])
@pytest.mark.parametrize("name", list(CASES))
def test_helper_vs_oracle(name, slow):
    bits, length = CASES[name]
    vdaf = Prio3.fixedpoint_boundedl2_vec_sum(bits, length)
    vk = bytes(range(50, 66))
    orc = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, length, 0)
    n = 48 if length >= 10000 else (96 if length >= 1000 else 200)
    _, nonces, ps, his, lps = _batch(orc, vdaf, vk, n, seed=sum(map(ord, name)))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    with HelperEngine(vdaf, vk) as eng:
        assert (eng.prep_share_len, eng.output_len) == (orc.sizes.prep_share, length)
        if slow:
            eng.debug(1, 1)
        res = eng.helper_initialized_batch(nonces, ps, his, lps, want_out_shares=True)
        np.testing.assert_array_equal(res.verdicts, want["verdicts"])
        fin = want["verdicts"] == 0
        assert 0 < fin.sum() < n  # tampered and norm-violating reports are rejected
        assert (want["verdicts"] == 3).any()
        np.testing.assert_array_equal(res.prep_msgs[fin], want["prep_msgs"][fin])
        np.testing.assert_array_equal(res.out_shares[fin], want["out_shares"][fin])
        eng.accumulate(n)
        agg, count, cs = eng.aggregate_share(0)
        assert agg == want["agg"] and count == want["count"] and cs == want["checksum"]
        v2, _ = eng.prep_and_aggregate(nonces, ps, his, lps, segment=3)
        np.testing.assert_array_equal(v2, want["verdicts"])
        assert eng.aggregate_share(3) == (want["agg"], want["count"], want["checksum"])


@pytest.mark.parametrize("name", ["fp16_len3", "fp32_len100", "fp16_len10000"])
def test_leader_prep_init_vs_oracle(name):
    bits, length = CASES[name]
    vdaf = Prio3.fixedpoint_boundedl2_vec_sum(bits, length)
    vk = bytes(range(16))
    orc = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, length, 0)
    n = 12 if length >= 10000 else 40
    rng = np.random.default_rng(3 + length)
    meas = fixedpoint_measurements(bits, length, rng, n)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, lis = [], []
    for i in range(n):
        a, b, _ = orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes())
        ps.append(a)
        lis.append(b)
    ps = np.frombuffer(b"".join(ps), np.uint8).reshape(n, -1)
    lis = np.frombuffer(b"".join(lis), np.uint8).reshape(n, -1).copy()
    lis[2, 0:16] = 0xFF  # an explicit element >= p: prepare_init_failure
    with HelperEngine(vdaf, vk) as eng:
        init = eng.leader_initialized_batch(nonces, ps, lis)
    for i in range(n):
        rc, share, _, _ = orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())
        assert int(init.verdicts[i]) == (1 if rc else 0), i
        if rc == 0:
            assert init.prep_shares[i].tobytes() == share, i
    assert init.verdicts[2] == 1 and init.verdicts.sum() == 1


@pytest.mark.parametrize("name", ["fp16_len37", "fp16_len10000"])
def test_ping_pong_leader_helper(name):
    """configs[4]: leader+helper ping-pong prep with joint randomness, both roles on the device.
    Leader + helper aggregates = the sum of the offset-encoded entries of the accepted reports."""
    bits, length = CASES[name]
    vdaf = Prio3.fixedpoint_boundedl2_vec_sum(bits, length)
    vk = bytes(range(9, 25))
    orc = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, length, 0)
    n = 24
    rng = np.random.default_rng(17)
    meas = fixedpoint_measurements(bits, length, rng, n)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    shards = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(n)]
    ps, lis, his = (np.frombuffer(b"".join(s[k] for s in shards), np.uint8).reshape(n, -1) for k in range(3))
    with HelperEngine(vdaf, vk) as leader, HelperEngine(vdaf, vk) as helper:
        init = leader.leader_initialized_batch(nonces, ps, lis)
        assert not init.verdicts.any()
        lps = init.prep_shares.copy()
        lps[1, 40] ^= 4  # a tampered leader verifier share
        hres = helper.helper_initialized_batch(nonces, ps, his, lps)
        want = orc.helper_prep_batch(vk, nonces, ps, his, lps)
        np.testing.assert_array_equal(hres.verdicts, want["verdicts"])
        violators = [i for i in range(n) if i % 6 == 4]
        assert all(hres.verdicts[i] == 3 for i in violators) and hres.verdicts[1] != 0
        msgs = hres.prep_msgs.copy()
        msgs[7, 0] ^= 1  # corrupted Finish: leader prepare_next fails
        fin = leader.leader_continued_batch(msgs)
        assert fin.verdicts[7] == 4
        accept = ((hres.verdicts == 0) & (fin.verdicts == 0)).astype(np.uint8)
        leader.accumulate(n, accept_mask=accept)
        helper.accumulate(n, accept_mask=accept)
        agg_l, cnt_l, cs_l = leader.aggregate_share(0)
        agg_h, cnt_h, cs_h = helper.aggregate_share(0)
    ok = accept.astype(bool)
    assert cnt_l == cnt_h == int(ok.sum()) == n - len(violators) - 2
    assert cs_l == cs_h
    total = [(int.from_bytes(agg_l[16 * i:16 * i + 16], "little") + int.from_bytes(agg_h[16 * i:16 * i + 16], "little"))
             % P128 for i in range(length)]
    enc = (meas.astype(object) ^ (1 << (bits - 1)))  # to_field_integer of every entry
    assert total == [int(enc[ok, j].sum()) for j in range(length)]


@pytest.mark.parametrize("bits", [16, 32])
def test_reference_e2e_result(bits):
    """interop_binaries/tests/end_to_end.rs:689-765: four length-3 measurements aggregate (leader
    engine + helper engine) and decode to [0.5, 0.5, 0.6875]."""
    vdaf = Prio3.fixedpoint_boundedl2_vec_sum({16: "BitSize16", 32: "BitSize32"}[bits], 3)
    q, e, s = 0.25, 0.125, 0.0625
    meas = [[q, e, e], [s, e, s], [e, e, q], [s, e, q]]
    vk = bytes(range(16))
    orc = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, 3, 0)
    shards = [orc.shard(vdaf.encode_fixedpoint(m), bytes([i]) * 16, bytes([i + 7]) * 80) for i, m in enumerate(meas)]
    nonces = np.array([[i] * 16 for i in range(4)], np.uint8)
    ps, lis, his = (np.frombuffer(b"".join(x[k] for x in shards), np.uint8).reshape(4, -1) for k in range(3))
    with HelperEngine(vdaf, vk) as leader, HelperEngine(vdaf, vk) as helper:
        init = leader.leader_initialized_batch(nonces, ps, lis)
        hres = helper.helper_initialized_batch(nonces, ps, his, init.prep_shares)
        fin = leader.leader_continued_batch(hres.prep_msgs)
        assert not hres.verdicts.any() and not fin.verdicts.any()
        leader.accumulate(4)
        helper.accumulate(4)
        agg_l, _, _ = leader.aggregate_share(0)
        agg_h, _, _ = helper.aggregate_share(0)
    total = b"".join(((int.from_bytes(agg_l[i:i + 16], "little") + int.from_bytes(agg_h[i:i + 16], "little")) % P128)
                     .to_bytes(16, "little") for i in range(0, 48, 16))
    assert vdaf.decode_fixedpoint_result(total, 4) == [0.5, 0.5, 0.6875]


@pytest.mark.parametrize("split,padded", [(0, False), (3, False), (6, False), (7, False), (5, False), (0, True)],
                         ids=["auto", "lanes", "pairs", "words", "fused", "auto-padded-rows"])
def test_two_jobs_in_flight(split, padded):
    """configs[4]'s bench shape (tools/bench_fixedpoint.py, two jobs in flight): while the helper engine
    prepares job i-1 on its stream, the leader engine initializes job i on its own; then the leader
    finishes job i-1. Inputs live in HBM (a 24-report pool tiled to 4,096 reports per job), the helper's
    K1 is each of its kernels in turn, and after three jobs the verdicts of the last job and both
    aggregates must be exactly the oracle's (24-report pool x multiplicity x 3 jobs)."""
    import torch

    bits, length = CASES["fp16_len10000"]
    vdaf = Prio3.fixedpoint_boundedl2_vec_sum(bits, length)
    vk = bytes(range(30, 46))
    orc = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, length, 0)
    K, R, jobs = 24, 4096, 3
    rng = np.random.default_rng(91)
    meas = fixedpoint_measurements(bits, length, rng, K)
    nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
    shards = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(K)]
    ps, lis, his = (np.frombuffer(b"".join(s[k] for s in shards), np.uint8).reshape(K, -1) for k in range(3))
    lps = np.stack([np.frombuffer(orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())[1],
                                  np.uint8) for i in range(K)])
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    fin = want["verdicts"] == 0
    assert 0 < fin.sum() < K  # the pool holds norm violators
    dev = torch.device("cuda", 0)

    def tile(x):
        return torch.from_numpy(np.array(x).reshape(K, -1)).to(dev).repeat(-(-R // K), 1)[:R].contiguous()

    # padded: the leader's input-share rows at a 128-byte multiple stride (jx_leader_prep_init_device_ex),
    # with garbage in the padding (it must never be read)
    stride = -(-lis.shape[1] // 128) * 128 if padded else 0
    if padded:
        rows = np.full((K, stride), 0xA5, np.uint8)
        rows[:, :lis.shape[1]] = lis
        d_lis = tile(rows)
    else:
        d_lis = tile(lis)
    d_n, d_ps, d_his = tile(nonces), tile(ps), tile(his)
    d_lps = [torch.empty((R, vdaf.prep_share_len), dtype=torch.uint8, device=dev) for _ in range(2)]
    d_msgs = torch.empty((R, 16), dtype=torch.uint8, device=dev)
    d_hv = torch.empty(R, dtype=torch.uint8, device=dev)
    d_lv = torch.empty(R, dtype=torch.uint8, device=dev)
    with HelperEngine(vdaf, vk) as leader, HelperEngine(vdaf, vk) as helper:
        if split:
            helper.debug(3, split)
        prev = None
        for i in range(jobs + 1):
            bid = leader.leader_init_device(R, d_n.data_ptr(), d_ps.data_ptr(), d_lis.data_ptr(),
                                            d_lps[i % 2].data_ptr(), lis_stride=stride) if i < jobs else None
            if prev is not None:
                helper.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(),
                                                 d_lps[(i - 1) % 2].data_ptr(), R, 0, d_msgs.data_ptr(),
                                                 d_hv.data_ptr())
                helper.sync()
                leader.leader_finish_device(prev, R, d_msgs.data_ptr(), d_hv.data_ptr(), d_lv.data_ptr())
                leader.accumulate_device(prev, R)
            leader.sync()
            prev = bid
        agg_l, cnt_l, cs_l = leader.aggregate_share(0)
        agg_h, cnt_h, cs_h = helper.aggregate_share(0)
    tiled_v = np.tile(want["verdicts"], -(-R // K))[:R]
    np.testing.assert_array_equal(d_hv.cpu().numpy(), tiled_v)
    np.testing.assert_array_equal(d_lv.cpu().numpy() == 0, tiled_v == 0)
    mult = np.bincount(np.arange(R) % K, minlength=K) * jobs
    enc = meas.astype(object) ^ (1 << (bits - 1))
    total = [(int.from_bytes(agg_l[16 * j:16 * j + 16], "little") + int.from_bytes(agg_h[16 * j:16 * j + 16], "little"))
             % P128 for j in range(length)]
    assert total == [int((enc[fin, j] * mult[fin]).sum()) % P128 for j in range(length)]
    assert cnt_l == cnt_h == int(mult[fin].sum()) and cs_l == cs_h
