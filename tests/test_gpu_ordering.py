"""GPU: the producer / consumer ordering contract of the device-pointer ABI (include/jx_prio3.h,
"Conventions"; jx_engine_wait_stream / jx_engine_join_stream).

The engine runs on its own non-blocking HIP stream. Inputs that a caller writes on torch's stream
AFTER the engine exists, behind a long producer kernel, must be read only once written, and torch
must be able to read the outputs with no host synchronization. Janus calls prio synchronously on
owned values (aggregator/src/aggregator.rs:1945-1967), so a drop-in must not introduce this race.

Every value is checked against the C oracle: helper verdicts, prep messages and the aggregate; the
leader's prep shares; the leader's finish verdicts and its batch-aggregation records.
"""
from __future__ import annotations

import numpy as np
import pytest

from janus_amd.engine import HelperEngine
from janus_amd.vdaf import Prio3
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SLEEP_CYCLES = 400_000_000  # torch.cuda._sleep: a producer kernel of a few hundred ms


def _reports(v, vk, n, seed):
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    rng = np.random.default_rng(seed)
    meas = rng.integers(0, 1 << v.bits, size=(n, v.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, lis, his = [], [], []
    for i in range(n):
        a, b, c = orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes())
        ps.append(a)
        lis.append(b)
        his.append(c)
    cat = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(n, -1)  # noqa: E731
    return orc, nonces, cat(ps), cat(lis), cat(his)


def _produce(pairs, torch):
    """The producer: a long kernel on torch's current stream, then the copies that write the inputs."""
    torch.cuda._sleep(SLEEP_CYCLES)
    for dst, src in pairs:
        dst.copy_(src, non_blocking=True)


def test_inputs_produced_after_engine_creation_on_torch_stream():
    import torch

    v = Prio3.sum_vec(4, 60, 7)
    vk = bytes(range(40, 56))
    n = 1536
    orc, nonces, ps, lis, his = _reports(v, vk, n, seed=11)
    dev = torch.device("cuda", 0)
    # the engines exist (and hold their staging) before any input is produced
    leader, helper = HelperEngine(v, vk), HelperEngine(v, vk)
    leader.set_capacity(n)
    helper.set_capacity(n)
    pinned = lambda a: torch.from_numpy(np.array(a, copy=True)).pin_memory()  # noqa: E731
    h_n, h_ps, h_lis, h_his = pinned(nonces), pinned(ps), pinned(lis), pinned(his)
    mask = np.ones(n, np.uint8)
    mask[5::17] = 0  # reports the leader's writer leaves out
    seg = (np.arange(n) % 3).astype(np.uint32)
    h_mask, h_seg = pinned(mask), pinned(seg.view(np.int32))
    d_n, d_ps, d_lis, d_his = (torch.empty(t.shape, dtype=torch.uint8, device=dev) for t in (h_n, h_ps, h_lis, h_his))
    d_mask = torch.empty(n, dtype=torch.uint8, device=dev)
    d_seg = torch.empty(n, dtype=torch.int32, device=dev)
    d_lps = torch.empty((n, helper.prep_share_len), dtype=torch.uint8, device=dev)
    d_lver = torch.empty(n, dtype=torch.uint8, device=dev)
    d_hver = torch.empty(n, dtype=torch.uint8, device=dev)
    d_msgs = torch.empty((n, helper.prep_msg_len), dtype=torch.uint8, device=dev)
    d_fver = torch.empty(n, dtype=torch.uint8, device=dev)
    rb = leader.record_bytes()
    d_rec = torch.empty(3 * rb, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    try:
        # leader init -> helper prep + aggregate -> leader finish -> leader records, each call issued at
        # once behind its producers; the only ordering is through torch's current stream
        _produce([(d_n, h_n), (d_ps, h_ps), (d_lis, h_lis), (d_his, h_his)], torch)
        bid = leader.leader_init_device(n, d_n.data_ptr(), d_ps.data_ptr(), d_lis.data_ptr(), d_lps.data_ptr(),
                                        d_lver.data_ptr())
        d_lps[3::50, 0] ^= 1  # torch tampers with some leader prep shares between the two engines
        helper.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), n,
                                         d_out_prep_msgs=d_msgs.data_ptr(), d_out_verdicts=d_hver.data_ptr())
        leader.leader_finish_device(bid, n, d_msgs.data_ptr(), d_hver.data_ptr(), d_fver.data_ptr())
        _produce([(d_mask, h_mask), (d_seg, h_seg)], torch)
        leader.aggregate_records_device(bid, n, d_mask.data_ptr(), d_seg.data_ptr(), 3, d_rec.data_ptr())
        # torch reads every output on its own stream: no engine sync, no device-wide synchronize
        lps_got, lver, hver, msgs, fver, rec = (t.cpu().numpy() for t in (d_lps, d_lver, d_hver, d_msgs, d_fver, d_rec))
        h_agg, h_cnt, h_cs = helper.aggregate_share(0)
    finally:
        leader.close()
        helper.close()

    assert not lver.any()
    for i in list(range(0, n, 97)) + [3, 53]:
        rc, share, _, _ = orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())
        sent = bytearray(share)
        if i % 50 == 3:
            sent[0] ^= 1
        assert rc == 0 and lps_got[i].tobytes() == bytes(sent), i
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps_got, nthreads=16)
    np.testing.assert_array_equal(hver, want["verdicts"])
    assert (hver[3::50] != 0).all() and (hver != 0).sum() == len(range(3, n, 50))
    fin = hver == 0  # a rejected report's prep message is not sent (PrepareStepResult::Reject)
    np.testing.assert_array_equal(msgs[fin], want["prep_msgs"][fin])
    assert (h_agg, h_cnt, h_cs) == (want["agg"], want["count"], want["checksum"])
    np.testing.assert_array_equal(fver, np.where(want["verdicts"] != 0, 5, 0))
    louts = [orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())[2] for i in range(n)]
    from janus_amd.distributed import unpack_record

    for k in range(3):
        sel = [i for i in range(n) if fver[i] == 0 and mask[i] and seg[i] == k]
        cs = bytes(32)
        for i in sel:
            cs = bytes(a ^ b for a, b in zip(cs, O.sha256(nonces[i].tobytes())))
        got = unpack_record(rec[k * rb:(k + 1) * rb], 16)
        assert got == (orc.aggregate([louts[i] for i in sel]), len(sel), cs), k


def test_unordered_call_is_the_callers_responsibility():
    """stream=False leaves ordering to the caller: with an explicit wait_stream / join_stream pair
    around the call, the result is the oracle's; the wrappers' default does exactly that."""
    import torch

    v = Prio3.sum_vec(2, 40, 6)
    vk = bytes(range(16))
    n = 512
    orc, nonces, ps, lis, his = _reports(v, vk, n, seed=5)
    lps = np.zeros((n, 0), np.uint8)
    with HelperEngine(v, vk) as leader:
        init = leader.leader_initialized_batch(nonces, ps, lis)
        lps = init.prep_shares
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    dev = torch.device("cuda", 0)
    srcs = [torch.from_numpy(np.array(a, copy=True)).pin_memory() for a in (nonces, ps, his, lps)]
    dsts = [torch.empty(s.shape, dtype=torch.uint8, device=dev) for s in srcs]
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    with HelperEngine(v, vk) as eng:
        eng.set_capacity(n)
        with torch.cuda.stream(side):  # a producer on a non-default stream
            _produce(list(zip(dsts, srcs)), torch)
        eng.wait_stream(side)
        eng.prep_and_aggregate_device(*[d.data_ptr() for d in dsts], n, d_out_verdicts=d_v.data_ptr(), stream=False)
        eng.join_stream(side)
        with torch.cuda.stream(side):
            got = d_v.cpu().numpy()
        agg, cnt, _ = eng.aggregate_share(0)
    np.testing.assert_array_equal(got, want["verdicts"])
    assert (agg, cnt) == (want["agg"], want["count"])


def test_event_ordering():
    """jx_engine_wait_event / jx_engine_record_event with caller-owned torch events."""
    import torch

    v = Prio3.sum(8)
    vk = bytes(range(16))
    n = 2048
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    rng = np.random.default_rng(4)
    meas = rng.integers(0, 256, size=(n, 1), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    dev = torch.device("cuda", 0)
    srcs = [torch.from_numpy(np.array(a, copy=True)).pin_memory() for a in (nonces, ps, his, lps)]
    dsts = [torch.empty(s.shape, dtype=torch.uint8, device=dev) for s in srcs]
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    produced, done = torch.cuda.Event(), torch.cuda.Event()
    with HelperEngine(v, vk) as eng:
        eng.set_capacity(n)
        _produce(list(zip(dsts, srcs)), torch)
        produced.record()
        eng.wait_event(produced)
        eng.prep_and_aggregate_device(*[d.data_ptr() for d in dsts], n, d_out_verdicts=d_v.data_ptr(), stream=False)
        eng.record_event(done)
        torch.cuda.current_stream(dev).wait_event(done)
        got = d_v.cpu().numpy()
        agg, cnt, _ = eng.aggregate_share(0)
    np.testing.assert_array_equal(got, want["verdicts"])
    assert (agg, cnt) == (want["agg"], want["count"])
