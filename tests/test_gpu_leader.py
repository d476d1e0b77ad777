"""GPU parity of the leader role and the full leader <-> helper ping-pong on the device.

Leader prepare_init (agg_id 0, leader_initialized, aggregation_job_driver.rs:344-362) is
compared byte for byte with the C oracle's prep_init; leader prepare_next (leader_continued,
:588-602) with the helper's outbound prep messages. The end-to-end property is the one
Janus's integration tests check (integration_tests/tests/integration/common.rs:298-510):
leader aggregate + helper aggregate = sum of the (truncated) measurements of the accepted
reports, mod p.
"""
from __future__ import annotations

import numpy as np
import pytest

from janus_amd.engine import HelperEngine
from janus_amd.vdaf import Prio3
from oracle import oracle as O

pytestmark = pytest.mark.gpu

P128 = 2**128 - 28 * 2**64 + 1
P64 = 2**64 - 2**32 + 1

CASES = {
    "count": Prio3.count(),
    "sum8": Prio3.sum(8),
    "sum32": Prio3.sum(32),
    "sum64": Prio3.sum(64),
    "sumvec_48x6_5": Prio3.sum_vec(48, 6, 5),
    "sumvec_small": Prio3.sum_vec(3, 37, 5),
    "sumvec_8x1000_88": Prio3.sum_vec(8, 1000, 88),
    "histogram_16_4": Prio3.histogram(16, 4),
    "histogram_256_16": Prio3.histogram(256, 16),
}


def _measurements(v: Prio3, rng, n):
    if v.algo_id == O.COUNT:
        return rng.integers(0, 2, size=(n, 1), dtype=np.uint64)
    if v.algo_id == O.SUM:
        return rng.integers(0, 1 << v.bits, size=(n, 1), dtype=np.uint64)
    if v.algo_id == O.HISTOGRAM:
        return rng.integers(0, v.length, size=(n, 1), dtype=np.uint64)
    return rng.integers(0, 1 << v.bits, size=(n, v.length), dtype=np.uint64)


def _shard(orc, v: Prio3, n, seed):
    rng = np.random.default_rng(seed)
    meas = _measurements(v, rng, n)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, lis, his = [], [], []
    for i in range(n):
        a, b, c = orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes())
        ps.append(a)
        lis.append(b)
        his.append(c)
    cat = lambda xs, w: np.frombuffer(b"".join(xs), np.uint8).reshape(n, w) if w else np.zeros((n, 0), np.uint8)  # noqa: E731
    return meas, nonces, cat(ps, orc.sizes.public_share), cat(lis, orc.sizes.leader_input_share), \
        cat(his, orc.sizes.helper_input_share)


def _expected_total(v: Prio3, meas, accepted):
    """Sum of the truncated measurements of accepted reports (the aggregate result)."""
    if v.algo_id in (O.COUNT, O.SUM):
        return [int(meas[accepted, 0].astype(object).sum())]
    if v.algo_id == O.HISTOGRAM:
        return [int(np.sum(meas[accepted, 0] == b)) for b in range(v.length)]
    return [int(meas[accepted, j].astype(object).sum()) for j in range(v.length)]


def _decode(agg: bytes, fb: int):
    return [int.from_bytes(agg[i:i + fb], "little") for i in range(0, len(agg), fb)]


@pytest.mark.parametrize("name", list(CASES))
def test_leader_prep_init_matches_oracle(name):
    v = CASES[name]
    vk = bytes(range(32, 48))
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    n = 24 if name == "sumvec_8x1000_88" else 70
    meas, nonces, ps, lis, his = _shard(orc, v, n, seed=sum(map(ord, name)) + 1)
    fb = v.field_bytes
    lis = lis.copy()
    lis[3, 0:fb] = 0xFF  # first measurement element >= p: decode failure -> prepare_init_failure
    lis[5, lis.shape[1] - (17 if v.joint_rand_len else 1)] ^= 0xFF  # last proof element altered: still valid
    with HelperEngine(v, vk) as eng:
        init = eng.leader_initialized_batch(nonces, ps, lis)
    for i in range(n):
        rc, share, out, corr = orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())
        assert int(init.verdicts[i]) == (1 if rc else 0), i
        if rc == 0:
            assert init.prep_shares[i].tobytes() == share, i
    assert init.verdicts[3] == 1 and init.verdicts.sum() == 1


@pytest.mark.parametrize("name", list(CASES))
def test_ping_pong_leader_helper_on_device(name):
    v = CASES[name]
    vk = bytes(range(100, 116))
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    n = 20 if name == "sumvec_8x1000_88" else 64
    meas, nonces, ps, lis, his = _shard(orc, v, n, seed=7 + sum(map(ord, name)))
    with HelperEngine(v, vk) as leader, HelperEngine(v, vk) as helper:
        init = leader.leader_initialized_batch(nonces, ps, lis)
        assert not init.verdicts.any()
        lps = init.prep_shares.copy()
        lps[2, 0] ^= 1  # one tampered leader prep share: helper rejects it
        hres = helper.helper_initialized_batch(nonces, ps, his, lps)
        want = orc.helper_prep_batch(vk, nonces, ps, his, lps)
        np.testing.assert_array_equal(hres.verdicts, want["verdicts"])
        assert hres.verdicts[2] != 0 and (hres.verdicts != 0).sum() == 1
        msgs = hres.prep_msgs.copy()
        if v.joint_rand_len:
            msgs[4, 7] ^= 0x10  # a corrupted Finish message: leader's prepare_next fails
        fin = leader.leader_continued_batch(msgs, want_out_shares=True)
        if v.joint_rand_len:
            assert fin.verdicts[4] == 4
        # the leader accumulates the reports the helper finished (the helper's PrepareResp)
        accept = ((hres.verdicts == 0) & (fin.verdicts == 0)).astype(np.uint8)
        leader.accumulate(n, accept_mask=accept)
        helper.accumulate(n, accept_mask=accept)
        agg_l, cnt_l, cs_l = leader.aggregate_share(0)
        agg_h, cnt_h, cs_h = helper.aggregate_share(0)
    ok = accept.astype(bool)
    assert cnt_l == cnt_h == int(ok.sum())
    assert cs_l == cs_h
    p = P64 if v.field_bytes == 8 else P128
    total = [(a + b) % p for a, b in zip(_decode(agg_l, v.field_bytes), _decode(agg_h, v.field_bytes))]
    assert total == [x % p for x in _expected_total(v, meas, ok)]
    # leader output shares of finished reports == the oracle's leader prep_init output shares
    for i in np.nonzero(fin.verdicts == 0)[0][:8]:
        _, _, out, _ = orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())
        assert fin.out_shares[i].tobytes() == out


def test_dap_handlers_end_to_end():
    """The DAP-level mirrors: leader_aggregate_init -> helper handle_aggregate_init (with one
    replayed report and one malformed leader message) -> leader_process_helper_response; the
    two batch aggregations add up to the measurements of the reports both sides finished."""
    from janus_amd.aggregator import (LeaderReport, handle_aggregate_init, leader_aggregate_init,
                                      leader_process_helper_response)
    from janus_amd.messages import HpkeCiphertext, PingPongMessage, PrepareError, PrepareInit, ReportMetadata

    v = Prio3.sum_vec(4, 50, 7)
    vk = bytes(range(7, 23))
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    n = 40
    meas, nonces, ps, lis, his = _shard(orc, v, n, seed=99)
    reports = [LeaderReport(ReportMetadata(nonces[i].tobytes(), 1_700_000_000 + i), ps[i].tobytes(),
                            lis[i].tobytes(), HpkeCiphertext(1, b"enc", b"ct")) for i in range(n)]
    reports[6] = LeaderReport(reports[6].metadata, reports[6].public_share, reports[6].leader_input_share[:-1],
                              reports[6].helper_encrypted_input_share)  # truncated leader share
    with HelperEngine(v, vk) as leader, HelperEngine(v, vk) as helper:
        step = leader_aggregate_init(leader, reports)
        assert step.failed == {6: PrepareError.InvalidMessage}
        inits = list(step.prepare_inits)
        k9 = step.stepped.index(9)
        bad = inits[k9]
        inits[k9] = PrepareInit(bad.report_share, PingPongMessage.initialize(bad.message.prep_share[:-1]))
        helper_shares = [his[i].tobytes() for i in step.stepped]
        replayed = {nonces[12].tobytes()}
        out = handle_aggregate_init(helper, inits, helper_shares, replayed=replayed)
        by_id = {r.report_id: r.result for r in out.responses}
        assert by_id[nonces[9].tobytes()].error == PrepareError.VdafPrepError
        assert by_id[nonces[12].tobytes()].error == PrepareError.ReportReplayed
        assert out.step_failures["leader_prep_share_decode_failure"] == 1
        lead = leader_process_helper_response(leader, step, out.responses)
        ok = np.zeros(n, bool)
        ok[[i for i in range(n) if lead.finished[i]]] = True
        assert not ok[[6, 9, 12]].any() and ok.sum() == n - 3
        agg_l, cnt_l, _ = leader.aggregate_share(0)
        agg_h, cnt_h, _ = helper.aggregate_share(0)
    assert cnt_l == cnt_h == n - 3
    total = [(a + b) % P128 for a, b in zip(_decode(agg_l, 16), _decode(agg_h, 16))]
    assert total == _expected_total(v, meas, ok)
