"""GPU: coalesced prepares at Janus's job granularity, and the device arena shared by engines.

Janus prepares one aggregation job of 10-100 reports per request (aggregator/src/aggregator.rs:
1712-2013; docs/samples/basic_config/aggregation_job_creator.yaml:23-26) with many requests in flight
(binary_utils/job_driver.rs:116). With coalescing on (jx_engine_coalesce), concurrent jobs of every
engine (task) of one Prio3 instance share launches; each job must still get exactly its own verdicts,
prep messages, batch and records, with its own task's verify key. Every expectation comes from the C
oracle.
"""
from __future__ import annotations

import threading

import numpy as np
import pytest

from janus_amd.engine import HelperEngine
from janus_amd.vdaf import Prio3
from oracle import oracle as O

pytestmark = pytest.mark.gpu

P128 = 2**128 - 28 * 2**64 + 1
P64 = 2**64 - 2**32 + 1


def _oracle(v: Prio3):
    return O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length, v.num_proofs)


def _meas(v: Prio3, rng, n):
    if v.algo_id == O.COUNT:
        return rng.integers(0, 2, size=(n, 1), dtype=np.uint64)
    if v.algo_id == O.SUM:
        return rng.integers(0, 1 << v.bits, size=(n, 1), dtype=np.uint64)
    if v.algo_id == O.HISTOGRAM:
        return rng.integers(0, v.length, size=(n, 1), dtype=np.uint64)
    return rng.integers(0, 1 << v.bits, size=(n, v.length), dtype=np.uint64)


def _pool(v: Prio3, vk: bytes, n: int, seed: int, tamper_every=9):
    """n client reports (C-oracle client + leader), every tamper_every-th with a flipped bit in its leader
    prep share, and the oracle's helper results."""
    orc = _oracle(v)
    rng = np.random.default_rng(seed)
    meas = _meas(v, rng, n)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
    for i in range(0, n, tamper_every):
        lps[i, int(rng.integers(0, lps.shape[1]))] ^= 1 << int(rng.integers(0, 8))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    return orc, nonces, ps, his, lps, want


def _record(orc, want, nonces, idx):
    """(aggregate share, count, checksum) the oracle gives for the finished reports among idx."""
    fin = [i for i in idx if want["verdicts"][i] == 0]
    agg = orc.aggregate([want["out_shares"][i].tobytes() for i in fin]) if fin else \
        bytes(orc.sizes.output_len * orc.sizes.field_bytes)
    cs = bytes(32)
    for i in fin:
        cs = bytes(a ^ b for a, b in zip(cs, O.sha256(nonces[i].tobytes())))
    return agg, len(fin), cs


def _run_threads(fn, nthreads):
    errs = []

    def wrap(t):
        try:
            fn(t)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    th = [threading.Thread(target=wrap, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    if errs:
        raise errs[0]


def test_64_threads_of_100_report_jobs_two_tasks():
    """64 host threads, 100-report SumVec 8x1000/88 jobs (valid and tampered), split over two engines
    (tasks) with different verify keys: every job's verdicts, Finish{prep_msg}s and batch-aggregation
    record equal the oracle's, and the jobs really shared launches."""
    v = Prio3.sum_vec(8, 1000, 88)
    vks = [bytes(range(16)), bytes(range(100, 116))]
    K = 1024
    pools = [_pool(v, vk, K, seed=71 + k) for k, vk in enumerate(vks)]
    engs = [HelperEngine(v, vk) for vk in vks]
    try:
        for e in engs:
            e.coalesce(True)
        n, jobs_per_thread = 100, 2
        results = {}

        def worker(t):
            k = t % 2
            eng = engs[k]
            orc, nonces, ps, his, lps, want = pools[k]
            for j in range(jobs_per_thread):
                off = ((t // 2) * jobs_per_thread + j) * 37 % K
                idx = (off + np.arange(n)) % K
                res = eng.helper_initialized_batch(nonces[idx], ps[idx], his[idx], lps[idx])
                rec = eng.aggregate_records(res.batch_id, n)[0]
                eng.release(res.batch_id)
                results[(t, j)] = (k, idx, res.verdicts.copy(), res.prep_msgs.copy(), rec)

        _run_threads(worker, 64)
        assert len(results) == 64 * jobs_per_thread
        tampered = 0
        for (t, j), (k, idx, verdicts, msgs, rec) in results.items():
            orc, nonces, ps, his, lps, want = pools[k]
            np.testing.assert_array_equal(verdicts, want["verdicts"][idx], err_msg=f"job {t}/{j}")
            fin = want["verdicts"][idx] == 0
            tampered += int((~fin).sum())
            np.testing.assert_array_equal(msgs[fin], want["prep_msgs"][idx][fin], err_msg=f"job {t}/{j}")
            assert rec == _record(orc, want, nonces, idx), f"job {t}/{j}"
        assert tampered > 0
        m = engs[0].memory()
        assert m["coalesced_jobs"] == 64 * jobs_per_thread
        # the jobs shared launches at scale: closed-loop callers gather into few launches per round trip
        assert m["coalesced_jobs"] >= 8 * m["coalesced_launches"], m
        assert m["resident_batches"] == 0 and engs[1].memory()["resident_batches"] == 0
    finally:
        for e in engs:
            e.close()


CASES = {
    "count": Prio3.count(),
    "sum32": Prio3.sum(32),
    "sumvec_4x50_7": Prio3.sum_vec(4, 50, 7),
    "histogram_40_5": Prio3.histogram(40, 5),
    "multiproof_p2_8x12_14": Prio3.sum_vec_field64_multiproof_hmacsha256_aes128(2, 8, 12, 14),
}


def _shard(orc, v: Prio3, n, seed):
    rng = np.random.default_rng(seed)
    meas = _meas(v, rng, n)
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


@pytest.mark.parametrize("name", list(CASES))
def test_coalesced_ping_pong_both_roles(name):
    """Leader prepare_init and helper prepare of ragged jobs (1..150 reports) from 16 threads, both
    coalesced, three tasks (verify keys) per role: leader prep shares and verdicts equal the oracle's
    prep_init, the helper's verdicts and prep messages equal the oracle's, and per task leader +
    helper aggregates add up to the accepted measurements."""
    v = CASES[name]
    orc = _oracle(v)
    vklen = v.verify_key_len
    vks = [bytes((7 * k + i) % 256 for i in range(vklen)) for k in range(3)]
    sizes = [1, 7, 64, 65, 100, 150, 13, 128]
    n = sum(sizes)
    meas, nonces, ps, lis, his = _shard(orc, v, n, seed=sum(map(ord, name)))
    starts = np.concatenate([[0], np.cumsum(sizes)])
    leaders = [HelperEngine(v, vk) for vk in vks]
    helpers = [HelperEngine(v, vk) for vk in vks]
    try:
        for e in leaders + helpers:
            e.coalesce(True)
        out = {}

        def job(t):
            j, k = t // 3, t % 3  # job j of task k (every task prepares every slice)
            a, b = int(starts[j]), int(starts[j + 1])
            init = leaders[k].leader_initialized_batch(nonces[a:b], ps[a:b], lis[a:b])
            lps = init.prep_shares.copy()
            if b - a > 3:
                lps[2, 0] ^= 1  # the helper rejects this one
            hres = helpers[k].helper_initialized_batch(nonces[a:b], ps[a:b], his[a:b], lps)
            fin = leaders[k].leader_continued_batch(hres.prep_msgs, init=init)
            accept = ((hres.verdicts == 0) & (fin.verdicts == 0)).astype(np.uint8)
            leaders[k].accumulate(b - a, accept_mask=accept, batch_id=fin.batch_id)
            helpers[k].accumulate(b - a, accept_mask=accept, batch_id=hres.batch_id)
            out[(j, k)] = (init, lps, hres, accept)

        _run_threads(job, 3 * len(sizes))
        p = P64 if v.field_bytes == 8 else P128
        for k, vk in enumerate(vks):
            ok = np.zeros(n, bool)
            for j in range(len(sizes)):
                a, b = int(starts[j]), int(starts[j + 1])
                init, lps, hres, accept = out[(j, k)]
                for i in range(a, b):
                    rc, share, _, _ = orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())
                    assert int(init.verdicts[i - a]) == (1 if rc else 0), (name, k, i)
                    if rc == 0:
                        assert init.prep_shares[i - a].tobytes() == share, (name, k, i)
                want = orc.helper_prep_batch(vk, nonces[a:b], ps[a:b], his[a:b], lps)
                np.testing.assert_array_equal(hres.verdicts, want["verdicts"])
                f = want["verdicts"] == 0
                if v.joint_rand_len:
                    np.testing.assert_array_equal(hres.prep_msgs[f], want["prep_msgs"][f])
                ok[a:b] = accept.astype(bool)
            agg_l, cnt_l, cs_l = leaders[k].aggregate_share(0)
            agg_h, cnt_h, cs_h = helpers[k].aggregate_share(0)
            assert cnt_l == cnt_h == int(ok.sum()) and cs_l == cs_h
            fb = v.field_bytes
            dec = lambda g: [int.from_bytes(g[i:i + fb], "little") for i in range(0, len(g), fb)]  # noqa: E731
            total = [(x + y) % p for x, y in zip(dec(agg_l), dec(agg_h))]
            if v.algo_id in (O.COUNT, O.SUM):
                exp = [int(meas[ok, 0].astype(object).sum()) % p]
            elif v.algo_id == O.HISTOGRAM:
                exp = [int(np.sum(meas[ok, 0] == c)) for c in range(v.length)]
            else:
                exp = [int(meas[ok, c].astype(object).sum()) % p for c in range(v.length)]
            assert total == exp, (name, k)
        assert leaders[0].memory()["coalesced_jobs"] >= 2 * 3 * len(sizes)
    finally:
        for e in leaders + helpers:
            e.close()


def test_large_jobs_bypass_and_mix():
    """Jobs over a quarter of a launch take the direct path, small ones coalesce; both give the oracle's
    results on one engine, interleaved from several threads."""
    v = Prio3.histogram(256, 16)
    vk = bytes(range(50, 66))
    K = 3000
    orc, nonces, ps, his, lps, want = _pool(v, vk, K, seed=5)
    with HelperEngine(v, vk) as eng:
        eng.debug(5, 1024)  # launches of 1,024: jobs over 256 reports go direct
        eng.coalesce(True, window_us=300)
        sizes = [10, 300, 40, 1000, 256, 257, 3]
        res = {}

        def worker(t):
            a = (t * 400) % (K - 1000)
            m = sizes[t % len(sizes)]
            r = eng.helper_initialized_batch(nonces[a:a + m], ps[a:a + m], his[a:a + m], lps[a:a + m],
                                             want_out_shares=(t == 3))
            res[t] = (a, m, r)
            eng.accumulate(m, batch_id=r.batch_id, segments=np.full(m, t, np.uint32))

        _run_threads(worker, 14)
        for t, (a, m, r) in res.items():
            np.testing.assert_array_equal(r.verdicts, want["verdicts"][a:a + m])
            f = want["verdicts"][a:a + m] == 0
            np.testing.assert_array_equal(r.prep_msgs[f], want["prep_msgs"][a:a + m][f])
            if r.out_shares is not None:
                np.testing.assert_array_equal(r.out_shares[f], want["out_shares"][a:a + m][f])
            agg, cnt, cs = eng.aggregate_share(t)
            assert (agg, cnt, cs) == _record(orc, want, nonces, range(a, a + m)), t


def test_two_engines_share_the_arena_pipelined_calls():
    """Two SumVec 8x1000/88 engines (tasks) with different verify keys on one GPU, each running
    1.25M-report pipelined fused calls from its own thread, interleaved: both aggregates and every
    verdict equal the oracle's; the staging both use comes out of one device arena (jx_engine_memory)."""
    import torch

    v = Prio3.sum_vec(8, 1000, 88)
    vks = [bytes(range(16)), bytes(range(16, 32))]
    K, R = 2048, 1_250_000
    pools = [_pool(v, vk, K, seed=300 + k, tamper_every=50) for k, vk in enumerate(vks)]
    dev = torch.device("cuda", 0)
    idx = np.arange(R) % K
    d_idx = torch.from_numpy(idx).to(dev)
    tiles = []
    for orc, nonces, ps, his, lps, want in pools:
        tiles.append([torch.from_numpy(np.ascontiguousarray(a)).to(dev).index_select(0, d_idx).contiguous()
                      for a in (nonces, ps, his, lps)])
    del d_idx
    engs = [HelperEngine(v, vk) for vk in vks]
    outs = [(torch.empty(R, dtype=torch.uint8, device=dev), torch.empty((R, 16), dtype=torch.uint8, device=dev))
            for _ in engs]
    torch.cuda.synchronize()
    try:
        calls = 2

        def worker(k):
            d_n, d_ps, d_his, d_lps = tiles[k]
            d_v, d_m = outs[k]
            for _ in range(calls):
                engs[k].prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(),
                                                  R, 0, d_m.data_ptr(), d_v.data_ptr(), stream=False)
            engs[k].sync()

        _run_threads(worker, 2)
        mult = np.bincount(idx, minlength=K) * calls
        for k, (orc, nonces, ps, his, lps, want) in enumerate(pools):
            d_v, d_m = outs[k]
            got_v = d_v.cpu().numpy()
            np.testing.assert_array_equal(got_v, want["verdicts"][idx])
            f = got_v == 0
            np.testing.assert_array_equal(d_m.cpu().numpy()[f], want["prep_msgs"][idx][f])
            fin = want["verdicts"] == 0
            # sum_i mult_i * out_i by 32-bit limbs (exact in uint64: mult < 2^12, K < 2^11)
            words = want["out_shares"].reshape(K, v.length, 4, 4).astype(np.uint64)
            words = words[..., 0] | (words[..., 1] << 8) | (words[..., 2] << 16) | (words[..., 3] << 24)
            sums = np.einsum("k,kew->ew", np.where(fin, mult, 0).astype(np.uint64), words)
            exp = b"".join((sum(int(sums[e, w]) << (32 * w) for w in range(4)) % P128).to_bytes(16, "little")
                           for e in range(v.length))
            agg, cnt, _ = engs[k].aggregate_share(0)
            assert cnt == int(np.where(fin, mult, 0).sum())
            assert agg == exp
        m = engs[0].memory()
        assert m["arena_engines"] >= 2
        assert m["arena_allocated"] <= m["arena_budget"]
        assert m["last_pipelines"] >= 1
        assert m["arena_reuses"] > 0  # later launches reuse the first ones' staging
    finally:
        for e in engs:
            e.close()


def test_mixed_k1_launch_two_verify_keys():
    """A coalesced helper launch past one lane-split K1 wave per SIMD takes the mixed K1 (the first
    round_reports / 4 reports lane-split on the lane's stream, the rest as lane pairs on a side stream,
    prep_core / bufs_tail). With jobs of two tasks in that launch, every report of the tail must still use its
    own task's verify key: two 24,000-report jobs of engines with different keys (48,000 reports, past the
    32,768-report split on MI355X and under a K1 round's half), gathered into ONE launch (debug option 7), each
    equal to the oracle."""
    v = Prio3.sum_vec(4, 50, 7)
    vks = [bytes(range(16)), bytes(range(40, 56))]
    K, n = 1024, 24000
    pools = [_pool(v, vk, K, seed=900 + k, tamper_every=37) for k, vk in enumerate(vks)]
    engs = [HelperEngine(v, vk) for vk in vks]
    try:
        for e in engs:
            e.coalesce(True, window_us=1_000_000)
        engs[0].debug(7, 2)  # the gather waits for both jobs (one launch of 48,000 reports)
        m0 = engs[0].memory()
        out = {}

        def worker(k):
            orc, nonces, ps, his, lps, want = pools[k]
            idx = (311 * k + np.arange(n)) % K
            r = engs[k].helper_initialized_batch(nonces[idx], ps[idx], his[idx], lps[idx])
            out[k] = (idx, r.verdicts.copy(), r.prep_msgs.copy(), engs[k].aggregate_records(r.batch_id, n)[0])
            engs[k].release(r.batch_id)

        _run_threads(worker, 2)
        m1 = engs[0].memory()
        assert m1["coalesced_launches"] - m0["coalesced_launches"] == 1
        assert m1["coalesced_reports"] - m0["coalesced_reports"] == 2 * n
        for k in range(2):
            orc, nonces, ps, his, lps, want = pools[k]
            idx, verdicts, msgs, rec = out[k]
            np.testing.assert_array_equal(verdicts, want["verdicts"][idx], err_msg=f"task {k}")
            fin = want["verdicts"][idx] == 0
            assert (~fin).sum() > 0 and fin.sum() > 0
            np.testing.assert_array_equal(msgs[fin], want["prep_msgs"][idx][fin], err_msg=f"task {k}")
            agg, cnt, cs = rec
            exp_agg, exp_cnt, exp_cs = _record(orc, want, nonces, list(idx))
            assert (cnt, cs, agg) == (exp_cnt, exp_cs, exp_agg), f"task {k}"
    finally:
        engs[0].debug(7, 0)
        for e in engs:
            e.close()


def test_mixed_roles_32_leader_32_helper_threads():
    """An aggregator that is leader for one task and helper for another on one Prio3 instance
    (aggregator_core/src/task.rs:598): 32 threads of 100-report leader prepare_init jobs interleaved with 32
    threads of helper jobs, all coalesced. Each role gathers in its own lane, so a leader job never closes a
    helper gather (and back): every job equals the oracle, and both roles share launches as they would alone."""
    v = Prio3.sum_vec(8, 1000, 88)
    vk_l, vk_h = bytes(range(16)), bytes(range(50, 66))
    K, n, per_thread = 512, 100, 3
    orc = _oracle(v)
    meas, nonces, ps, lis, his = _shard(orc, v, K, seed=123)
    lead = [orc.prep_init(vk_l, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes()) for i in range(K)]
    horc, hn, hps, hhis, hlps, hwant = _pool(v, vk_h, K, seed=124)
    leader, helper = HelperEngine(v, vk_l), HelperEngine(v, vk_h)
    try:
        leader.coalesce(True)
        helper.coalesce(True)
        m0 = leader.memory()
        out = {}

        def worker(t):
            for j in range(per_thread):
                idx = ((t // 2) * 37 + j * 11 + np.arange(n)) % K
                if t % 2 == 0:
                    r = leader.leader_initialized_batch(nonces[idx], ps[idx], lis[idx])
                    leader.release(r.batch_id)
                    out[(t, j)] = ("leader", idx, r.verdicts.copy(), r.prep_shares.copy())
                else:
                    r = helper.helper_initialized_batch(hn[idx], hps[idx], hhis[idx], hlps[idx])
                    helper.release(r.batch_id)
                    out[(t, j)] = ("helper", idx, r.verdicts.copy(), r.prep_msgs.copy())

        _run_threads(worker, 64)
        m1 = leader.memory()
        for (t, j), (role, idx, verdicts, x) in out.items():
            if role == "leader":
                for k, i in enumerate(idx):
                    rc, share, _, _ = lead[i]
                    assert int(verdicts[k]) == (1 if rc else 0), (t, j, i)
                    if rc == 0:
                        assert x[k].tobytes() == share, (t, j, i)
            else:
                np.testing.assert_array_equal(verdicts, hwant["verdicts"][idx], err_msg=f"job {t}/{j}")
                f = hwant["verdicts"][idx] == 0
                np.testing.assert_array_equal(x[f], hwant["prep_msgs"][idx][f], err_msg=f"job {t}/{j}")
        d = {k: m1[k] - m0[k] for k in ("coalesced_helper_launches", "coalesced_helper_jobs",
                                        "coalesced_leader_launches", "coalesced_leader_jobs")}
        assert d["coalesced_helper_jobs"] == d["coalesced_leader_jobs"] == 32 * per_thread, d
        # closed-loop callers of each role share launches (>= 4 jobs per launch; alone: ~16-32)
        assert d["coalesced_helper_jobs"] >= 4 * d["coalesced_helper_launches"], d
        assert d["coalesced_leader_jobs"] >= 4 * d["coalesced_leader_launches"], d
        assert m1["coalesce_pinned_bytes"] > 0
    finally:
        leader.close()
        helper.close()


def test_two_engines_under_a_small_arena_budget():
    """Two SumVec engines of different tasks run fused device calls from their own threads under a 6 GB arena
    budget (JX_ARENA_GB, read once per process: run in a child process), with launch sizes that change every
    call, so the arena keeps trimming idle slabs of one engine for the other's check-outs (outside its lock).
    Both aggregates and every verdict equal the oracle's, and the arena did free slabs."""
    import json
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, JX_ARENA_GB="6")
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "arena_trim_worker.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["verified"], res
    assert res["arena_frees"] > 0 and res["arena_allocated_max"] <= res["arena_budget"], res
