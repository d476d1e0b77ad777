"""GPU parity for Prio3SumVecField64MultiproofHmacSha256Aes128 (Janus
core/src/vdaf.rs:173-199): the HIP kernels of janus_amd/csrc/jx_mp64.hip, through the C ABI,
against the C oracle (pinned to the independent Python restatement, tests/test_oracle_crosscheck.py)
and the golden fixtures tests/golden/sumvec_f64mp_*.json (replayed by test_gpu_parity.test_golden).

Bar: bit-exact verdicts, prepare messages (32 bytes), output shares, aggregate shares, counts and
checksums. Parameter sets: Janus's own tests (janus.rs:369-374, taskprov_tests.rs:1266), a padded
chunk with three proofs, and the headline SumVec shape with two and three proofs.
"""
from __future__ import annotations

import numpy as np
import pytest

from janus_amd.engine import HelperEngine
from janus_amd.vdaf import Prio3
from oracle import oracle as O

pytestmark = pytest.mark.gpu

VK = bytes(range(200, 232))
CASES = {
    "p2_16x15_16": (2, 16, 15, 16),
    "p2_8x12_14": (2, 8, 12, 14),
    "p3_1x7_3": (3, 1, 7, 3),
    "p2_8x1000_88": (2, 8, 1000, 88),
    "p3_8x1000_88": (3, 8, 1000, 88),
    "p8_2x33_4": (8, 2, 33, 4),
}


def _setup(name, n, seed, tamper_every=7):
    proofs, bits, length, chunk = CASES[name]
    vdaf = Prio3.sum_vec_field64_multiproof_hmacsha256_aes128(proofs, bits, length, chunk)
    orc = O.Prio3Oracle(O.SUMVEC_F64_MULTIPROOF, bits, length, chunk, proofs)
    rng = np.random.default_rng(seed)
    meas = rng.integers(0, 1 << bits, size=(n, length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, lout = orc.client_leader_batch(VK, meas, nonces, rands, nthreads=16, want_leader_out=True)
    for i in range(0, n, tamper_every) if tamper_every else ():
        j = int(rng.integers(0, lps.shape[1]))
        lps[i, j] ^= 1 << int(rng.integers(0, 8))
    return vdaf, orc, meas, nonces, rands, ps, his, lps, lout


@pytest.mark.parametrize("slow", [False, True], ids=["fast", "slowpath"])
@pytest.mark.parametrize("name", list(CASES))
def test_random_batches_vs_oracle(name, slow):
    n = 130 if "1000" in name else 333
    vdaf, orc, _, nonces, ps, his, lps = (lambda t: (t[0], t[1], t[2], t[3], t[5], t[6], t[7]))(
        _setup(name, n, seed=sum(map(ord, name))))
    want = orc.helper_prep_batch(VK, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    with HelperEngine(vdaf, VK) as eng:
        assert eng.prep_msg_len == 32 and eng.field_bytes == 8
        if slow:
            eng.debug(1, 1)
        res = eng.helper_initialized_batch(nonces, ps, his, lps, want_out_shares=True)
        np.testing.assert_array_equal(res.verdicts, want["verdicts"])
        fin = want["verdicts"] == 0
        assert fin.sum() > n // 2
        assert set(np.unique(want["verdicts"])) <= {0, 2, 3, 4}
        np.testing.assert_array_equal(res.prep_msgs[fin], want["prep_msgs"][fin])
        np.testing.assert_array_equal(res.out_shares[fin], want["out_shares"][fin])
        eng.accumulate(n)
        agg, count, cs = eng.aggregate_share(0)
        assert agg == want["agg"] and count == want["count"] and cs == want["checksum"]
        v2, m2 = eng.prep_and_aggregate(nonces, ps, his, lps, segment=3)
        np.testing.assert_array_equal(v2, want["verdicts"])
        np.testing.assert_array_equal(m2[fin], want["prep_msgs"][fin])
        assert eng.aggregate_share(3) == (want["agg"], want["count"], want["checksum"])


@pytest.mark.parametrize("name", ["p2_16x15_16", "p3_8x1000_88"])
def test_leader_helper_ping_pong(name):
    """Leader prepare_init on the GPU -> helper prepare on the GPU -> leader prepare_next on the
    helper's prep message: both output shares sum to the measurement (aggregation_job_driver.rs
    :345,588 / aggregator.rs:1947)."""
    n = 96
    vdaf, orc, meas, nonces, rands, ps, his, lps_want, lout = _setup(name, n, seed=77, tamper_every=0)
    proofs, bits, length, chunk = CASES[name]
    # the leader's explicit input shares
    lis = np.zeros((n, orc.sizes.leader_input_share), np.uint8)
    for i in range(n):
        _, lin, _ = orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes())
        lis[i] = np.frombuffer(lin, np.uint8)
    with HelperEngine(vdaf, VK) as leader, HelperEngine(vdaf, VK) as helper:
        init = leader.leader_initialized_batch(nonces, ps, lis)
        assert (init.verdicts == 0).all()
        np.testing.assert_array_equal(init.prep_shares, lps_want)  # == the oracle's leader prep shares
        hres = helper.helper_initialized_batch(nonces, ps, his, init.prep_shares, want_out_shares=True)
        assert (hres.verdicts == 0).all()
        lres = leader.leader_continued_batch(hres.prep_msgs, want_out_shares=True)
        assert (lres.verdicts == 0).all()
        np.testing.assert_array_equal(lres.out_shares, lout)
        p = 2**64 - 2**32 + 1
        for i in range(n):
            a = np.frombuffer(lres.out_shares[i].tobytes(), "<u8").astype(object)
            b = np.frombuffer(hres.out_shares[i].tobytes(), "<u8").astype(object)
            assert [int(x) % p for x in (a + b)] == [int(x) for x in meas[i]]
        # a wrong prep message fails the leader's prepare_next
        bad = hres.prep_msgs.copy()
        bad[5, 0] ^= 1
        leader.leader_initialized_batch(nonces, ps, lis)
        assert leader.leader_continued_batch(bad).verdicts.tolist() == [4 if i == 5 else 0 for i in range(n)]


def test_shard_records_device_merge():
    import torch

    from janus_amd import distributed as D

    n, world = 120, 3
    vdaf, orc, _, nonces, _, ps, his, lps, _ = _setup("p2_16x15_16", n, seed=5)
    want = orc.helper_prep_batch(VK, nonces, ps, his, lps, nthreads=16)
    engs = [HelperEngine(vdaf, VK) for _ in range(world)]
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
    assert D.unpack_record(out.cpu().numpy(), vdaf.field_bytes) == (want["agg"], want["count"], want["checksum"])
    for e in engs:
        e.close()


def test_bad_parameters_rejected():
    from janus_amd._lib import EngineError
    with pytest.raises(ValueError):
        Prio3.sum_vec_field64_multiproof_hmacsha256_aes128(1, 8, 10, 4)
    vdaf = Prio3.sum_vec_field64_multiproof_hmacsha256_aes128(2, 8, 10, 4)
    with pytest.raises(ValueError):
        HelperEngine(vdaf, bytes(16))  # needs a 32-byte verify key
    with pytest.raises(EngineError):
        HelperEngine(Prio3(4, 8, 10, 4, 9), bytes(32))  # more proofs than the kernels support
