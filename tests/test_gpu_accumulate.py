"""GPU: batch accumulation into many batch aggregations, batch ids, device-pointer leader role.

Accumulation mirrors AggregationJobWriter::update_batch_aggregations_from_report_aggregations
(aggregator/src/aggregator/aggregation_job_writer.rs:608-708) -> BatchAggregation::merged_with
(aggregator_core/src/datastore/models.rs:1275-1330): per batch identifier, aggregate share +=
output share, count += 1, checksum ^= SHA-256(report id). Every expectation comes from the C oracle.
"""
from __future__ import annotations

import time

import numpy as np
import pytest

from janus_amd._lib import EngineError
from janus_amd.engine import HELPER_STEP_FAILURE, HelperEngine
from janus_amd.vdaf import Prio3
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _batch(vdaf, vk, n, seed, tamper_every=9):
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    rng = np.random.default_rng(seed)
    if vdaf.algo_id == O.HISTOGRAM:
        meas = rng.integers(0, vdaf.length, size=(n, 1), dtype=np.uint64)
    elif vdaf.algo_id == O.COUNT:
        meas = rng.integers(0, 2, size=(n, 1), dtype=np.uint64)
    else:
        meas = rng.integers(0, 1 << vdaf.bits, size=(n, vdaf.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
    for i in range(0, n, tamper_every):
        lps[i, int(rng.integers(0, lps.shape[1]))] ^= 1 << int(rng.integers(0, 8))
    return orc, nonces, ps, his, lps


def _expected(orc, want, nonces, sel):
    idx = np.nonzero(sel)[0]
    agg = orc.aggregate([want["out_shares"][i].tobytes() for i in idx]) if len(idx) else \
        bytes(orc.sizes.output_len * orc.sizes.field_bytes)
    cs = bytes(32)
    for i in idx:
        cs = bytes(a ^ b for a, b in zip(cs, O.sha256(nonces[i].tobytes())))
    return agg, int(len(idx)), cs


@pytest.mark.parametrize("nseg", [2, 64, 700])
def test_many_segments_one_pass(nseg):
    """Reports of one batch spread over nseg batch aggregations (arbitrary u32 ids, random order,
    accept mask), merged in one pass: every segment equals the oracle's merge of its reports."""
    vdaf = Prio3.histogram(32, 4)
    vk = bytes(range(16))
    n = 3000
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=nseg)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    rng = np.random.default_rng(99)
    ids = rng.choice(np.arange(1, 1 << 31, dtype=np.uint64), size=nseg, replace=False).astype(np.uint32)
    seg = ids[rng.integers(0, nseg, size=n)]
    mask = (rng.random(n) < 0.9).astype(np.uint8)
    with HelperEngine(vdaf, vk) as eng:
        res = eng.helper_initialized_batch(nonces, ps, his, lps)
        np.testing.assert_array_equal(res.verdicts, want["verdicts"])
        eng.accumulate(n, mask, seg, batch_id=res.batch_id)
        for s in ids[: min(nseg, 40)]:
            sel = (want["verdicts"] == 0) & (mask == 1) & (seg == s)
            assert eng.aggregate_share(int(s)) == _expected(orc, want, nonces, sel), int(s)
        # the sum over all segments is the batch total
        total = [0] * vdaf.length
        cnt = 0
        for s in ids:
            agg, c, _ = eng.aggregate_share(int(s))
            cnt += c
            for j in range(vdaf.length):
                total[j] += int.from_bytes(agg[16 * j:16 * j + 16], "little")
        sel = (want["verdicts"] == 0) & (mask == 1)
        agg_all, cnt_all, _ = _expected(orc, want, nonces, sel)
        assert cnt == cnt_all
        p = 2**128 - 28 * 2**64 + 1
        assert [x % p for x in total] == [int.from_bytes(agg_all[16 * j:16 * j + 16], "little") for j in range(vdaf.length)]


def test_segments_cost_is_not_linear():
    """One pass regardless of the number of segments: 1024 segments cost well under 1024x one."""
    import torch

    vdaf = Prio3.sum_vec(8, 1000, 88)
    vk = bytes(range(16))
    K, R = 64, 65536
    orc, nonces, ps, his, lps = _batch(vdaf, vk, K, seed=7)
    dev = torch.device("cuda", 0)
    tile = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev).repeat(R // K, 1).contiguous()  # noqa: E731
    d_n, d_ps, d_his, d_lps = tile(nonces), tile(ps), tile(his), tile(lps)
    times = {}
    with HelperEngine(vdaf, vk) as eng:
        for nseg in (1, 64, 1024):
            segs = torch.from_numpy(np.random.default_rng(nseg).integers(0, nseg, size=R).astype(np.int32)).to(dev)
            ids = list(range(10_000, 10_000 + nseg))
            for rep in range(2):
                eng.timing(True)
                eng.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), R,
                                              d_segments=segs.data_ptr(), segment_ids=ids)
                eng.sync()
                times[nseg] = eng.timing_read()["accumulate"]["ms"]
        eng.reset_aggregates()
    assert times[1024] < 8 * times[1] + 2.0, times  # ms; a pass per segment would be ~1000x
    print("accumulate ms by segments:", times)


def test_fused_device_segments_match_oracle():
    import torch

    vdaf = Prio3.sum_vec(2, 50, 9)
    vk = bytes(range(16))
    n = 2000
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=3)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    rng = np.random.default_rng(5)
    dense = rng.integers(0, 6, size=n).astype(np.uint32)  # 5 = out of range: skipped
    ids = [7, 70, 700, 7000, 70000]
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.array(a, copy=True)).to(dev)  # noqa: E731  (writable copy)
    d_seg = T(dense.astype(np.int32))
    import os
    eng = HelperEngine(vdaf, vk)
    eng.debug(5, 512)  # 512 reports per launch
    with eng:
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        keep = [T(nonces), T(ps), T(his), T(lps)]  # hold the tensors: a freed block is reused at once
        eng.prep_and_aggregate_device(*[t.data_ptr() for t in keep], n, d_out_verdicts=d_v.data_ptr(),
                                      d_segments=d_seg.data_ptr(), segment_ids=ids)
        eng.sync()
        np.testing.assert_array_equal(d_v.cpu().numpy(), want["verdicts"])
        for k, s in enumerate(ids):
            sel = (want["verdicts"] == 0) & (dense == k)
            assert eng.aggregate_share(s) == _expected(orc, want, nonces, sel)


@pytest.mark.parametrize("name,vdaf", [("sumvec", Prio3.sum_vec(2, 50, 9)), ("histogram", Prio3.histogram(40, 5)),
                                       ("sum", Prio3.sum(7))])
def test_fused_device_multi_launch(name, vdaf):
    """A fused device call over five launches into one aggregation gives the oracle's verdicts, prep
    messages and aggregate (the staging is reused launch after launch)."""
    import os

    import torch

    vk = bytes(range(16))
    n = 2300
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=11)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.array(a, copy=True)).to(dev)  # noqa: E731  (writable copy)
    eng = HelperEngine(vdaf, vk)
    eng.debug(5, 512)  # 512 reports per launch
    with eng:
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_m = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
        keep = [T(nonces), T(ps) if ps is not None else None, T(his), T(lps)]
        eng.prep_and_aggregate_device(keep[0].data_ptr(), keep[1].data_ptr() if keep[1] is not None else None,
                                      keep[2].data_ptr(), keep[3].data_ptr(), n, d_out_prep_msgs=d_m.data_ptr(),
                                      d_out_verdicts=d_v.data_ptr())
        eng.sync()
        np.testing.assert_array_equal(d_v.cpu().numpy(), want["verdicts"])
        fin = want["verdicts"] == 0
        if vdaf.algo_id != O.COUNT:
            np.testing.assert_array_equal(d_m.cpu().numpy()[fin], want["prep_msgs"][fin])
        assert eng.aggregate_share(0) == (want["agg"], want["count"], want["checksum"])


def _leader_job(orc, vdaf, n, seed):
    rng = np.random.default_rng(seed)
    meas = rng.integers(0, 1 << vdaf.bits, size=(n, vdaf.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    sh = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(n)]
    ps, lis, his = (np.frombuffer(b"".join(s[k] for s in sh), np.uint8).reshape(n, -1) for k in range(3))
    return nonces, ps, lis, his


def test_interleaved_jobs_on_one_engine():
    """three aggregation jobs in flight on ONE engine -- two leader jobs (init A, init B,
    helper job C prepared in between, finish B, finish A) and one helper job -- each keeps its own
    resident batch; every job's deltas equal the oracle's and are repeatable; a batch finishes and
    accumulates at most once and a released batch is refused."""
    vdaf = Prio3.sum_vec(4, 30, 7)
    vk = bytes(range(5, 21))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    sizes = {"A": 70, "B": 50, "C": 90}
    jobs = {k: _leader_job(orc, vdaf, sizes[k], seed) for k, seed in (("A", 1), ("B", 2), ("C", 3))}
    with HelperEngine(vdaf, vk) as eng, HelperEngine(vdaf, vk) as peer:
        nA, psA, lisA, hisA = jobs["A"]
        nB, psB, lisB, hisB = jobs["B"]
        nC, psC, lisC, hisC = jobs["C"]
        a = eng.leader_initialized_batch(nA, psA, lisA)
        b = eng.leader_initialized_batch(nB, psB, lisB)
        # job C: this engine is the helper; its leader runs on the peer engine
        c_lead = peer.leader_initialized_batch(nC, psC, lisC)
        c = eng.helper_initialized_batch(nC, psC, hisC, c_lead.prep_shares)
        assert len({a.batch_id, b.batch_id, c.batch_id}) == 3
        assert eng.resident_batches()[0] == 3
        # the helper answers A and B (on the peer engine); B finishes before A
        hb = peer.helper_initialized_batch(nB, psB, hisB, b.prep_shares)
        ha = peer.helper_initialized_batch(nA, psA, hisA, a.prep_shares)
        fb = eng.leader_continued_batch(hb.prep_msgs, init=b)
        fa = eng.leader_continued_batch(ha.prep_msgs, init=a)
        assert not fa.verdicts.any() and not fb.verdicts.any() and not c.verdicts.any()
        with pytest.raises(EngineError, match="call out of order"):
            eng.leader_continued_batch(ha.prep_msgs, init=a)  # finished once
        for name, res in (("A", a), ("B", b)):
            nonces, ps, lis, _ = jobs[name]
            n = sizes[name]
            outs = [orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())[2] for i in range(n)]
            seg = (np.arange(n) % 3).astype(np.uint32)
            mask = (np.arange(n) % 5 != 0).astype(np.uint8)
            recs = eng.aggregate_records(res.batch_id, n, mask, seg, 3)
            assert recs == eng.aggregate_records(res.batch_id, n, mask, seg, 3)  # repeatable: a retried transaction
            for k in range(3):
                sel = [i for i in range(n) if seg[i] == k and mask[i]]
                cs = bytes(32)
                for i in sel:
                    cs = bytes(x ^ y for x, y in zip(cs, O.sha256(nonces[i].tobytes())))
                assert recs[k] == (orc.aggregate([outs[i] for i in sel]), len(sel), cs), (name, k)
        # the helper job's records match the oracle's helper prep
        want = orc.helper_prep_batch(vk, nC, psC, hisC, c_lead.prep_shares, nthreads=16, want_out_shares=True)
        assert eng.aggregate_records(c.batch_id, sizes["C"]) == [(want["agg"], want["count"], want["checksum"])]
        assert eng.aggregate_share(0)[1] == 0  # records never touch the running aggregations
        eng.accumulate(sizes["A"], batch_id=a.batch_id)
        with pytest.raises(EngineError, match="call out of order"):
            eng.accumulate(sizes["A"], batch_id=a.batch_id)  # released by the accumulate: no double count
        eng.release(b.batch_id)
        with pytest.raises(EngineError, match="call out of order"):
            eng.aggregate_records(b.batch_id, sizes["B"])
        with pytest.raises(EngineError, match="invalid argument"):
            eng.aggregate_records(c.batch_id, sizes["C"] + 1)
        eng.release(c.batch_id)
        assert eng.resident_batches()[0] == 0
        assert eng.aggregate_share(0)[1] == sizes["A"]


def test_records_device_match_host_and_skip_out_of_range():
    import torch

    from janus_amd import distributed as D

    vdaf = Prio3.histogram(40, 5)
    vk = bytes(range(16))
    n = 1000
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=21)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    rng = np.random.default_rng(4)
    idx = rng.integers(0, 9, size=n).astype(np.uint32)  # 8 = out of range: skipped
    mask = (rng.random(n) < 0.8).astype(np.uint8)
    with HelperEngine(vdaf, vk) as eng:
        res = eng.helper_initialized_batch(nonces, ps, his, lps)
        host = eng.aggregate_records(res.batch_id, n, mask, idx, 8)
        dev = torch.device("cuda", 0)
        rb = eng.record_bytes()
        d_out = torch.zeros(8 * rb, dtype=torch.uint8, device=dev)
        d_m, d_i = torch.from_numpy(mask.copy()).to(dev), torch.from_numpy(idx.astype(np.int32)).to(dev)
        torch.cuda.synchronize()
        eng.aggregate_records_device(res.batch_id, n, d_m.data_ptr(), d_i.data_ptr(), 8, d_out.data_ptr())
        eng.sync()
        out = d_out.cpu().numpy()
        assert [D.unpack_record(out[k * rb:(k + 1) * rb], 16) for k in range(8)] == host
        for k in range(8):
            sel = (want["verdicts"] == 0) & (mask == 1) & (idx == k)
            assert host[k] == _expected(orc, want, nonces, sel), k


def test_repeated_segment_ids_refused():
    """a segment-id table repeating an id would race two reduce rows on one
    aggregation; the device entry points refuse it."""
    import torch

    vdaf = Prio3.sum_vec(2, 50, 9)
    vk = bytes(range(16))
    n = 200
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=5)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.array(a, copy=True)).to(dev)  # noqa: E731
    keep = [T(nonces), T(ps), T(his), T(lps)]
    d_seg = T((np.arange(n) % 2).astype(np.int32))
    with HelperEngine(vdaf, vk) as eng:
        with pytest.raises(EngineError, match="repeated"):
            eng.prep_and_aggregate_device(*[t.data_ptr() for t in keep], n, d_segments=d_seg.data_ptr(),
                                          segment_ids=[7, 7])
        res = eng.helper_initialized_batch(nonces, ps, his, lps)
        with pytest.raises(EngineError, match="repeated"):
            eng.accumulate_device(res.batch_id, n, None, d_seg.data_ptr(), (3, 3))
        eng.accumulate_device(res.batch_id, n, None, d_seg.data_ptr(), (3, 4))
        eng.sync()
        assert eng.aggregate_share(3)[1] + eng.aggregate_share(4)[1] == int((res.verdicts == 0).sum())


def test_interleaved_count_jobs_and_double_accumulate():
    """Two interleaved leader jobs of the same size (init A, init B, finish A) on one engine: A finishes
    against its own device state, not B's; a batch accumulates at most once."""
    vdaf = Prio3.count()
    vk = bytes(range(16))
    orc = O.Prio3Oracle(vdaf.algo_id)
    rng = np.random.default_rng(1)
    n = 40
    meas = rng.integers(0, 2, size=(2 * n, 1), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(2 * n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(2 * n, orc.sizes.client_rand), dtype=np.uint8)
    sh = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(2 * n)]
    lis = np.frombuffer(b"".join(s[1] for s in sh), np.uint8).reshape(2 * n, -1)
    his = np.frombuffer(b"".join(s[2] for s in sh), np.uint8).reshape(2 * n, -1)
    empty = np.zeros((n, 0), np.uint8)
    with HelperEngine(vdaf, vk) as leader, HelperEngine(vdaf, vk) as helper:
        a = leader.leader_initialized_batch(nonces[:n], empty, lis[:n])
        b = leader.leader_initialized_batch(nonces[n:], empty, lis[n:])
        assert a.batch_id != b.batch_id
        with pytest.raises(EngineError, match="call out of order"):
            leader.accumulate(n, batch_id=a.batch_id)  # a leader batch accumulates after its finish
        fa = leader.leader_continued_batch(None, init=a)
        assert not fa.verdicts.any()
        leader.release(a.batch_id)
        hres = helper.helper_initialized_batch(nonces[n:], empty, his[n:], b.prep_shares)
        fin = leader.leader_continued_batch(None, init=b)
        assert not fin.verdicts.any() and not hres.verdicts.any()
        leader.accumulate(n, batch_id=b.batch_id)
        with pytest.raises(EngineError, match="call out of order"):
            leader.accumulate(n, batch_id=b.batch_id)  # no double count
        helper.accumulate(n)
        (agg_l, c_l, _), (agg_h, c_h, _) = leader.aggregate_share(0), helper.aggregate_share(0)
    assert c_l == c_h == n
    p = 2**64 - 2**32 + 1
    assert (int.from_bytes(agg_l, "little") + int.from_bytes(agg_h, "little")) % p == int(meas[n:].sum())



def test_device_leader_ping_pong_with_peer_verdicts():
    """Both roles with inputs resident in HBM: leader init (device) -> helper prep (device, fused) ->
    leader finish with the helper's verdicts -> leader accumulate (device, two segments)."""
    import torch

    vdaf = Prio3.sum_vec(4, 30, 7)
    vk = bytes(range(3, 19))
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    n = 300
    rng = np.random.default_rng(8)
    meas = rng.integers(0, 16, size=(n, vdaf.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    sh = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(n)]
    ps, lis, his = (np.frombuffer(b"".join(s[k] for s in sh), np.uint8).reshape(n, -1) for k in range(3))
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.array(a, copy=True)).to(dev)  # noqa: E731  (writable copy)
    d_n, d_ps, d_lis, d_his = T(nonces), T(ps), T(lis), T(his)
    d_lps = torch.zeros((n, vdaf.prep_share_len), dtype=torch.uint8, device=dev)
    d_hv = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_msgs = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
    d_lv = torch.zeros(n, dtype=torch.uint8, device=dev)
    seg = (np.arange(n) % 2).astype(np.int32)
    with HelperEngine(vdaf, vk) as leader, HelperEngine(vdaf, vk) as helper:
        bid = leader.leader_init_device(n, d_n.data_ptr(), d_ps.data_ptr(), d_lis.data_ptr(), d_lps.data_ptr())
        leader.sync()
        d_lps[5, 3] ^= 1  # helper rejects report 5
        torch.cuda.synchronize()
        helper.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), n,
                                         0, d_msgs.data_ptr(), d_hv.data_ptr())
        helper.sync()
        d_msgs[9, 0] ^= 1  # leader prepare_next fails on report 9
        torch.cuda.synchronize()
        leader.leader_finish_device(bid, n, d_msgs.data_ptr(), d_hv.data_ptr(), d_lv.data_ptr())
        d_seg = T(seg)
        leader.accumulate_device(bid, n, None, d_seg.data_ptr(), (11, 12))
        leader.sync()
        lv = d_lv.cpu().numpy()
        assert lv[5] == HELPER_STEP_FAILURE and lv[9] == 4 and (lv != 0).sum() == 2
        assert d_hv.cpu().numpy()[5] != 0
        ok = lv == 0
        for k, s in enumerate((11, 12)):
            agg, cnt, _ = leader.aggregate_share(s)
            sel = ok & (seg == k)
            assert cnt == int(sel.sum())
            # leader output shares == the oracle's leader prep_init output shares
            outs = [orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())[2]
                    for i in np.nonzero(sel)[0]]
            assert agg == orc.aggregate(outs)


@pytest.mark.parametrize("name", ["count", "sumvec"])
def test_device_combine_rejects_non_canonical(name):
    """the device merge must refuse a non-canonical element (>= p) like the host merge."""
    import torch

    from janus_amd import distributed as D

    vdaf = Prio3.count() if name == "count" else Prio3.sum_vec(1, 4, 2)
    fb = vdaf.field_bytes
    with HelperEngine(vdaf, bytes(16)) as eng:
        nb = eng.record_bytes()
        recs = torch.zeros((2, nb), dtype=torch.uint8, device="cuda")
        recs[1, :fb] = 0xFF
        out = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        eng.combine_records_device(recs.data_ptr(), 2, out.data_ptr())
        with pytest.raises(EngineError, match="non-canonical"):
            eng.sync()
        eng.sync()  # the flag is cleared once reported
        with pytest.raises(ValueError, match="not canonical"):
            D.merge_records(recs.cpu().numpy(), fb)


def test_handler_batch_aggregations_with_writer():
    """handle_aggregate_init over several batch identifiers with a BatchAggregationWriter: per-job deltas
    from the resident batch merged in a transaction that is rolled back twice and retried (the rows
    equal one clean attempt's), plus the host half (client timestamp interval over every report
    aggregation, failed ones included; None share for a batch without finished reports)."""
    from janus_amd.aggregator import handle_aggregate_init
    from janus_amd.batch_aggregation import BatchAggregationWriter, Interval
    from janus_amd.messages import HpkeCiphertext, PingPongMessage, PrepareInit, ReportMetadata, ReportShare

    vdaf = Prio3.sum_vec(2, 10, 4)
    vk = bytes(range(16))
    n = 60
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=31, tamper_every=7)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    times = [1_700_000_000 + 17 * i for i in range(n)]
    segs = [100 + (i % 3) for i in range(n)]
    segs[0] = 999  # a batch identifier whose only report fails (tampered: index 0)
    inits = [PrepareInit(ReportShare(ReportMetadata(nonces[i].tobytes(), times[i]), ps[i].tobytes(),
                                     HpkeCiphertext(1, b"e", b"c")), PingPongMessage.initialize(lps[i].tobytes()))
             for i in range(n)]
    w = BatchAggregationWriter(field_bytes=16, shard_count=2)
    with HelperEngine(vdaf, vk) as eng:
        out = handle_aggregate_init(eng, inits, [his[i].tobytes() for i in range(n)], segs, writer=w,
                                    inject_tx_failures=2)
        assert want["verdicts"][0] != 0 and not out.finished[0]
        assert w.datastore.attempts == 3 and eng.resident_batches()[0] == 0  # the job's batch is released
        assert eng.aggregate_share(100)[1] == 0  # deltas only: the running aggregations are untouched
        rows = {s: w.batch_aggregation(s) for s in w.segments()}
    assert rows[999].aggregate_share is None and rows[999].report_count == 0
    assert rows[999].client_timestamp_interval == Interval.from_time(times[0])
    for s in (100, 101, 102):
        idx = [i for i in range(n) if segs[i] == s]
        sel = np.zeros(n, bool)
        sel[[i for i in idx if want["verdicts"][i] == 0]] = True
        agg, cnt, cs = _expected(orc, want, nonces, sel)
        r = rows[s]
        assert (r.aggregate_share, r.report_count, r.checksum) == (agg, cnt, cs)
        t = [times[i] for i in idx]
        assert r.client_timestamp_interval == Interval(min(t), max(t) + 1 - min(t))


def test_leader_collected_batch_fails_at_init_and_batches_are_released():
    """Leader with a BatchAggregationWriter: reports of an already collected batch fail with
    BatchCollected at the initial write and are not sent to the helper (aggregation_job_writer.rs:
    557-605); a mismatched helper response releases the job's engine batch; the finished job leaves no
    resident batch behind."""
    from janus_amd.aggregator import (LeaderReport, handle_aggregate_init, leader_aggregate_init,
                                      leader_process_helper_response)
    from janus_amd.batch_aggregation import AGGREGATING, BatchAggregation, BatchAggregationWriter
    from janus_amd.messages import HpkeCiphertext, PrepareError, ReportMetadata

    vdaf = Prio3.sum_vec(2, 10, 4)
    vk = bytes(range(16))
    n = 30
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    rng = np.random.default_rng(77)
    meas = rng.integers(0, 4, size=(n, vdaf.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    shards = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(n)]
    reports = [LeaderReport(ReportMetadata(nonces[i].tobytes(), 1_700_000_000 + i), shards[i][0], shards[i][1],
                            HpkeCiphertext(1, b"e", b"c")) for i in range(n)]
    segs = [7 if i % 3 == 0 else 8 for i in range(n)]
    w = BatchAggregationWriter(field_bytes=16)
    w.datastore.rows[(7, 0)] = BatchAggregation(7, 0, state=AGGREGATING).collected()  # batch 7 was collected
    with HelperEngine(vdaf, vk) as leader, HelperEngine(vdaf, vk) as helper:
        step = leader_aggregate_init(leader, reports, segs, writer=w)
        assert {i for i, e in step.failed.items() if e == PrepareError.BatchCollected} == {i for i in range(n)
                                                                                          if segs[i] == 7}
        assert all(segs[i] == 8 for i in step.stepped) and len(step.stepped) == sum(s == 8 for s in segs)
        # a helper response that does not match the request: the step fails and its engine batch is released
        with pytest.raises(ValueError):
            leader_process_helper_response(leader, step, [], segs, writer=w)
        assert leader.resident_batches()[0] == 0
        # a fresh step of the same job goes through
        w2 = BatchAggregationWriter(field_bytes=16)
        step = leader_aggregate_init(leader, reports, segs, writer=w2)
        hout = handle_aggregate_init(helper, step.prepare_inits, [shards[i][2] for i in step.stepped],
                                     [segs[i] for i in step.stepped])
        out = leader_process_helper_response(leader, step, hout.responses, segs, writer=w2)
        assert out.finished.sum() == n and leader.resident_batches()[0] == 0 and helper.resident_batches()[0] == 0
        assert w2.batch_aggregation(8).report_count == sum(s == 8 for s in segs)


def test_helper_batch_keep_false_and_resident_scope():
    """helper_initialized_batch(keep=False) leaves no resident batch; resident() releases on exit unless
    accumulate consumed the batch; releasing a consumed batch is an error unless missing_ok."""
    vdaf = Prio3.sum_vec(2, 10, 4)
    vk = bytes(range(16))
    orc, nonces, ps, his, lps = _batch(vdaf, vk, 40, seed=5)
    with HelperEngine(vdaf, vk) as eng:
        res = eng.helper_initialized_batch(nonces, ps, his, lps, keep=False)
        assert res.batch_id == 0 and eng.resident_batches()[0] == 0
        res = eng.helper_initialized_batch(nonces, ps, his, lps)
        with eng.resident(res.batch_id):
            assert eng.resident_batches()[0] == 1
        assert eng.resident_batches()[0] == 0
        res = eng.helper_initialized_batch(nonces, ps, his, lps)
        with eng.resident(res.batch_id):
            eng.accumulate(40, batch_id=res.batch_id)  # consumes it; the scope's release is a no-op
        assert eng.resident_batches()[0] == 0
        with pytest.raises(EngineError, match="no resident"):
            eng.release(res.batch_id)
        eng.release(res.batch_id, missing_ok=True)


@pytest.mark.parametrize("vdaf", [Prio3.count(), Prio3.sum_vec(4, 12, 4)], ids=["count-field64", "sumvec-field128"])
def test_small_accumulate_boundary(vdaf):
    """jx_accumulate of an unmasked batch of <= ACC_SMALL (1,024) reports runs the one-kernel accumulate
    (accumulate_small_kernel: no staging, no partials); 1,025 reports or an accept mask take select +
    accumulate + reduce_partials. Both sides of the boundary, added into one aggregation, == the oracle."""
    vk = bytes(range(120, 136))
    n = 2049
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=1024)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    parts = [(0, 1024), (1024, 2049)]  # the small path, then the large one
    rng = np.random.default_rng(5)
    mask = rng.integers(0, 2, size=n).astype(bool)
    with HelperEngine(vdaf, vk) as eng:
        for a, b in parts:
            res = eng.helper_initialized_batch(nonces[a:b], ps[a:b], his[a:b], lps[a:b])
            np.testing.assert_array_equal(res.verdicts, want["verdicts"][a:b])
            eng.accumulate(b - a, batch_id=res.batch_id)
        assert eng.aggregate_share(0) == (want["agg"], want["count"], want["checksum"])
        # a masked small batch (staged mask upload, the three-kernel path) into a second aggregation
        eng.reset_aggregates()
        res = eng.helper_initialized_batch(nonces[:512], ps[:512], his[:512], lps[:512])
        eng.accumulate(512, accept_mask=mask[:512].astype(np.uint8), batch_id=res.batch_id)
        sel = (want["verdicts"][:512] == 0) & mask[:512]
        exp = _expected(orc, want, nonces, np.concatenate([sel, np.zeros(n - 512, bool)]))
        assert eng.aggregate_share(0) == exp


@pytest.mark.parametrize("vdaf", [Prio3.count(), Prio3.sum_vec(4, 12, 4), Prio3.histogram(40, 5)],
                         ids=["count-field64", "sumvec-field128", "histogram"])
def test_deferred_accumulate_of_many_jobs(vdaf):
    """jx_accumulate of job-sized batches (<= 1,024 reports, no mask, one segment) is deferred and run as one
    accumulate_multi launch per aggregation (up to 64 batches, auto-flushed when 64 wait): 150 jobs of 1 to 1,024
    reports into three aggregations, with masked jobs (accumulated at once) interleaved, equal the oracle per
    aggregation; a reset flushes first (deferred jobs before it are zeroed), and the immediate path (debug
    option 8 = 0) gives the same aggregates."""
    vk = bytes(range(40, 56))
    rng = np.random.default_rng(77)
    sizes = [int(s) for s in rng.choice([1, 2, 7, 30, 63, 64, 65, 100, 129], size=146)] + [1024, 1024, 5, 1]
    n = sum(sizes)
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=4242)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    mask = rng.integers(0, 2, size=n).astype(np.uint8)
    jobs, off = [], 0
    for k, s in enumerate(sizes):
        jobs.append((off, off + s, k % 3 + 10, k % 17 == 5))  # (first, end, aggregation id, masked)
        off += s

    def run(eng):
        for a, b, seg, masked in jobs:
            res = eng.helper_initialized_batch(nonces[a:b], ps[a:b], his[a:b], lps[a:b])
            np.testing.assert_array_equal(res.verdicts, want["verdicts"][a:b])
            eng.accumulate(b - a, accept_mask=mask[a:b] if masked else None,
                           segments=np.full(b - a, seg, np.uint32), batch_id=res.batch_id)
        return {seg: eng.aggregate_share(seg) for seg in (10, 11, 12)}

    exp = {}
    for seg in (10, 11, 12):
        sel = np.zeros(n, bool)
        for a, b, sg, masked in jobs:
            if sg == seg:
                sel[a:b] = (want["verdicts"][a:b] == 0) & ((mask[a:b] != 0) if masked else True)
        exp[seg] = _expected(orc, want, nonces, sel)
    with HelperEngine(vdaf, vk) as eng:
        got = run(eng)
        assert got == exp
        m = eng.memory()
        assert m["resident_batches"] == 0
        # deferred jobs before a reset are applied, then zeroed
        a, b = jobs[0][0], jobs[0][1]
        res = eng.helper_initialized_batch(nonces[a:b], ps[a:b], his[a:b], lps[a:b])
        eng.accumulate(b - a, batch_id=res.batch_id)
        eng.reset_aggregates()
        assert eng.aggregate_share(0)[1] == 0
    with HelperEngine(vdaf, vk) as eng:
        eng.debug(8, 0)
        assert run(eng) == exp
