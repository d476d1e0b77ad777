"""GPU: the helper's loop from the ENCRYPTED report share, with the HPKE open inside the prepare launch
(jx_helper_prep_encrypted_batch, alone and coalesced; janus_amd.aggregator.handle_aggregate_init_encrypted).

The reference does, per report (aggregator/src/aggregator.rs:1763-1967): the task's and then the global keypair
for the report's config id (:1781-1832), PlaintextInputShare decode and extension checks (:1834-1893), the
helper input share and public share decodes (:1895-1925), the report-too-early check (:1929-1940), then
helper_initialized + evaluate. Every expectation here comes from a restatement of that loop on the test side:
oracle/hpke_oracle.py opens (pinned by the RFC 9180 vector the reference ships), a small PlaintextInputShare
decoder below, and the C oracle's helper prepare. Each PrepareResp list must equal it exactly.
"""
from __future__ import annotations

import random
import threading

import numpy as np
import pytest

from janus_amd import hpke
from janus_amd.aggregator import handle_aggregate_init_encrypted
from janus_amd.engine import OPEN_STATUS, HelperEngine
from janus_amd.messages import (EXTENSION_TASKPROV, EXTENSION_TBD, Extension, HpkeCiphertext, PingPongMessage,
                                PlaintextInputShare, PrepareError, PrepareInit, PrepareResp, PrepareStepResult,
                                ReportMetadata, ReportShare)
from janus_amd.vdaf import Prio3
from oracle import hpke_oracle as H
from oracle import oracle as O

pytestmark = pytest.mark.gpu

P128 = 2**128 - 28 * 2**64 + 1
INFO = H.dap_info()


def _aad(task_id: bytes, rid: bytes, time: int, ps: bytes) -> bytes:
    """InputShareAad (messages/src/lib.rs:1854-1858), restated."""
    return task_id + rid + time.to_bytes(8, "big") + len(ps).to_bytes(4, "big") + ps


def _decode_plaintext(pt: bytes):
    """PlaintextInputShare (messages/src/lib.rs:1323-1326), restated: ([(type, data)], payload) or None."""
    if len(pt) < 2:
        return None
    end = 2 + int.from_bytes(pt[:2], "big")
    if end > len(pt):
        return None
    exts, i = [], 2
    while i < end:
        if i + 4 > end:
            return None
        t, dl = int.from_bytes(pt[i:i + 2], "big"), int.from_bytes(pt[i + 2:i + 4], "big")
        if t not in (0x0000, 0xFF00) or i + 4 + dl > end:
            return None
        exts.append((t, pt[i + 4:i + 4 + dl]))
        i += 4 + dl
    if end + 4 > len(pt):
        return None
    plen = int.from_bytes(pt[end:end + 4], "big")
    if end + 4 + plen != len(pt):
        return None
    return exts, pt[end + 4:]


def reference_responses(orc, vk, v: Prio3, task_id, keys, inits, require_taskprov=False, deadline=None):
    """The reference's per-report loop on the test side. keys: {config_id: [(sk, pk) of the task keypair or
    None, (sk, pk) of the global keypair or None]}. Returns (PrepareResps, finished mask, the oracle's output
    shares of the finished reports)."""
    n = len(inits)
    res: list = [None] * n
    survivors = []
    for i, pi in enumerate(inits):
        rs = pi.report_share
        ct = rs.encrypted_input_share
        ks = [k for k in keys.get(ct.config_id, []) if k]
        if not ks:
            res[i] = PrepareStepResult(2, error=PrepareError.HpkeUnknownConfigId)
            continue
        aad = _aad(task_id, rs.metadata.report_id, rs.metadata.time, rs.public_share)
        pt = None
        for sk, pk in ks:
            if len(ct.encapsulated_key) == 32 and len(ct.payload) >= 16:
                pt = H.open_base(sk, pk, INFO, ct.encapsulated_key, aad, ct.payload)
            if pt is not None:
                break
        if pt is None:
            res[i] = PrepareStepResult(2, error=PrepareError.HpkeDecryptError)
            continue
        dec = _decode_plaintext(pt)
        bad = dec is None
        if not bad:
            exts, payload = dec
            types = [t for t, _ in exts]
            tp = [d for t, d in exts if t == 0xFF00]
            bad = (len(set(types)) != len(types) or (require_taskprov and not (len(tp) == 1 and tp[0] == b""))
                   or (not require_taskprov and tp) or len(payload) != v.helper_input_share_len
                   or len(rs.public_share) != v.public_share_len)
        if bad:
            res[i] = PrepareStepResult(2, error=PrepareError.InvalidMessage)
            continue
        if deadline is not None and rs.metadata.time > deadline:
            res[i] = PrepareStepResult(2, error=PrepareError.ReportTooEarly)
            continue
        if pi.message.kind != PingPongMessage.INITIALIZE or len(pi.message.prep_share) != v.prep_share_len:
            res[i] = PrepareStepResult(2, error=PrepareError.VdafPrepError)
            continue
        survivors.append((i, payload))
    finished = np.zeros(n, bool)
    outs = {}
    if survivors:
        idx = [i for i, _ in survivors]
        m = len(idx)
        cat = lambda xs, w: np.frombuffer(b"".join(xs), np.uint8).reshape(m, w)  # noqa: E731
        want = orc.helper_prep_batch(
            vk, cat([inits[i].report_share.metadata.report_id for i in idx], 16),
            cat([inits[i].report_share.public_share for i in idx], v.public_share_len),
            cat([p for _, p in survivors], v.helper_input_share_len),
            cat([inits[i].message.prep_share for i in idx], v.prep_share_len), nthreads=16, want_out_shares=True)
        for j, i in enumerate(idx):
            if want["verdicts"][j]:
                res[i] = PrepareStepResult(2, error=PrepareError.VdafPrepError)
            else:
                msg = want["prep_msgs"][j].tobytes()[: v.prep_msg_len]
                res[i] = PrepareStepResult(0, message=PingPongMessage.finish(msg))
                finished[i] = True
                outs[i] = want["out_shares"][j].tobytes()
    return [PrepareResp(inits[i].report_share.metadata.report_id, res[i]) for i in range(n)], finished, outs


def _keypair(rnd):
    sk = rnd.randbytes(32)
    return sk, H.x25519_base(sk)


def _make_inits(rnd, orc, v: Prio3, vk, task_id, n, kind_of, seal_key, cfg_of, seed, time0=1_700_000_000):
    """n PrepareInits of client reports sealed with seal_key(i) under config id cfg_of(i); kind_of(i) picks a
    mutation (see _mutate)."""
    rng = np.random.default_rng(seed)
    if v.algo_id == O.COUNT:
        meas = rng.integers(0, 2, size=(n, 1), dtype=np.uint64)
    elif v.algo_id == O.HISTOGRAM:
        meas = rng.integers(0, v.length, size=(n, 1), dtype=np.uint64)
    elif v.algo_id == O.SUM:
        meas = rng.integers(0, 1 << v.bits, size=(n, 1), dtype=np.uint64)
    else:
        meas = rng.integers(0, 1 << v.bits, size=(n, v.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
    inits = []
    for i in range(n):
        kind = kind_of(i)
        md = ReportMetadata(nonces[i].tobytes(), time0 + i)
        exts, payload, pub, lp = (), his[i].tobytes(), ps[i].tobytes(), lps[i].tobytes()
        if kind == "dup_ext":
            exts = (Extension(EXTENSION_TBD, b"x"), Extension(EXTENSION_TBD, b"y"))
        elif kind == "taskprov":
            exts = (Extension(EXTENSION_TASKPROV),)
        elif kind == "taskprov_data":
            exts = (Extension(EXTENSION_TASKPROV, b"cfg"),)
        elif kind == "dup_taskprov":
            exts = (Extension(EXTENSION_TASKPROV), Extension(EXTENSION_TASKPROV))
        elif kind == "tbd_ext":
            exts = (Extension(EXTENSION_TBD, b"ext-data"),)
        elif kind == "long_payload":
            payload += b"\x00"
        elif kind == "tamper_lps":
            lp = bytearray(lp)
            lp[rnd.randrange(len(lp))] ^= 1 << rnd.randrange(8)
            lp = bytes(lp)
        elif kind == "odd_ps":
            pub = pub + b"\x00"
        pt = PlaintextInputShare(exts, payload).encode()
        if kind == "bad_ext_type":
            pt = (6).to_bytes(2, "big") + (0x1234).to_bytes(2, "big") + (2).to_bytes(2, "big") + b"zz" + pt[2:]
        elif kind == "truncated_exts":
            pt = (10).to_bytes(2, "big") + pt[2:6]
        aad = _aad(task_id, md.report_id, md.time, pub)
        enc, ct = H.seal_base(seal_key(i)[1], INFO, aad, pt, rnd.randbytes(32))
        if kind == "corrupt_ct":
            ct = bytearray(ct)
            ct[rnd.randrange(len(ct))] ^= 1 << rnd.randrange(8)
            ct = bytes(ct)
        elif kind == "short_enc":
            enc = enc[:31]
        elif kind == "short_ct":
            ct = ct[:12]
        msg = PingPongMessage.initialize(lp)
        if kind == "finish_msg":
            msg = PingPongMessage.finish(bytes(v.prep_msg_len))
        inits.append(PrepareInit(ReportShare(md, pub, HpkeCiphertext(cfg_of(i), enc, ct)), msg))
    return inits


def _aggregate(orc, v, outs: list[bytes]) -> bytes:
    if not outs:
        return bytes(orc.sizes.output_len * orc.sizes.field_bytes)
    return orc.aggregate(outs)


KINDS = ["valid", "valid", "valid", "tamper_lps", "corrupt_ct", "unknown_cfg", "dup_ext", "taskprov", "bad_ext_type",
         "long_payload", "global_fallback", "global_only", "short_enc", "truncated_exts", "tbd_ext", "short_ct",
         "odd_ps", "finish_msg", "too_early"]


@pytest.mark.parametrize("coalesce", [False, True])
def test_every_open_failure_and_fallback_key(coalesce):
    """One job holding every failure the loop maps before helper_initialized (and the trial of the global
    keypair after the task's): handle_aggregate_init_encrypted's PrepareResps, the engine's aggregate and the
    per-label counters equal the reference's; the raw open status codes are checked too."""
    rnd = random.Random(31 + coalesce)
    v = Prio3.sum_vec(4, 50, 7)
    vk = bytes(range(16))
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    task_id = rnd.randbytes(32)
    kt, g7, g11 = _keypair(rnd), _keypair(rnd), _keypair(rnd)
    n = 4 * len(KINDS)
    kind_of = lambda i: KINDS[i % len(KINDS)]  # noqa: E731
    seal = lambda i: {"global_fallback": g7, "global_only": g11}.get(kind_of(i), kt)  # noqa: E731
    cfg = lambda i: {"unknown_cfg": 9, "global_only": 11}.get(kind_of(i), 7)  # noqa: E731
    inits = _make_inits(rnd, orc, v, vk, task_id, n, kind_of, seal, cfg, seed=5)
    deadline = 1_700_000_000 + n - 3  # the last reports come from "too far in the future"
    inits = [p if kind_of(i) != "too_early" else
             PrepareInit(ReportShare(ReportMetadata(p.report_share.metadata.report_id, deadline + 100),
                                     p.report_share.public_share, p.report_share.encrypted_input_share), p.message)
             for i, p in enumerate(inits)]
    # the too-early reports were sealed for their original time: re-seal them for the new one
    for i, p in enumerate(inits):
        if kind_of(i) == "too_early":
            rs = p.report_share
            aad = _aad(task_id, rs.metadata.report_id, rs.metadata.time, rs.public_share)
            pt = H.open_base(kt[0], kt[1], INFO, rs.encrypted_input_share.encapsulated_key,
                             _aad(task_id, rs.metadata.report_id, 1_700_000_000 + i, rs.public_share),
                             rs.encrypted_input_share.payload)
            enc, ct = H.seal_base(kt[1], INFO, aad, pt, rnd.randbytes(32))
            inits[i] = PrepareInit(ReportShare(rs.metadata, rs.public_share, HpkeCiphertext(7, enc, ct)), p.message)
    want, fin, outs = reference_responses(orc, vk, v, task_id, {7: [kt, g7], 11: [None, g11]}, inits, deadline=deadline)
    with hpke.HpkeOpener(*kt, INFO) as ot, hpke.HpkeOpener(*g7, INFO) as o7, hpke.HpkeOpener(*g11, INFO) as o11, \
            HelperEngine(v, vk) as eng:
        if coalesce:
            eng.coalesce(True)
        got = handle_aggregate_init_encrypted(eng, ot, 7, task_id, inits, global_keypairs={7: o7, 11: o11},
                                              report_deadline=deadline)
        agg, count, _ = eng.aggregate_share(0)
        # the raw statuses of the device call
        rows = [i for i in range(n) if kind_of(i) in ("corrupt_ct", "unknown_cfg", "dup_ext", "taskprov",
                                                        "bad_ext_type", "long_payload", "short_enc", "truncated_exts",
                                                        "short_ct", "valid", "global_fallback")]
        sel = [inits[i] for i in rows]
        key_index = np.array([(0xFF, 0xFF) if p.report_share.encrypted_input_share.config_id == 9 else
                              (0xFE, 0xFF) if len(p.report_share.encrypted_input_share.encapsulated_key) != 32 else
                              (0, 1) for p in sel], np.uint8)
        r = eng.helper_initialized_encrypted_batch(
            np.frombuffer(b"".join(p.report_share.metadata.report_id for p in sel), np.uint8).reshape(-1, 16),
            [p.report_share.metadata.time for p in sel],
            np.frombuffer(b"".join(p.report_share.public_share for p in sel), np.uint8), task_id, [ot, o7], key_index,
            np.frombuffer(b"".join(p.report_share.encrypted_input_share.encapsulated_key.ljust(32, b"\0")[:32]
                                   for p in sel), np.uint8).reshape(-1, 32),
            [p.report_share.encrypted_input_share.payload for p in sel],
            np.frombuffer(b"".join(p.message.prep_share for p in sel), np.uint8), keep=False)
        if coalesce:
            assert eng.memory()["coalesced_encrypted_jobs"] >= 2
    assert got.responses == want
    assert (got.finished == fin).all() and fin.sum() > 0
    assert count == int(fin.sum()) and agg == _aggregate(orc, v, [outs[i] for i in sorted(outs)])
    expect_status = {"corrupt_ct": 1, "short_enc": 1, "short_ct": 1, "bad_ext_type": 2, "truncated_exts": 2,
                     "dup_ext": 3, "taskprov": 4, "long_payload": 6, "unknown_cfg": 7, "valid": 0, "global_fallback": 0}
    assert list(r.open_status) == [expect_status[kind_of(i)] for i in rows]
    assert all((r.verdicts[j] == 6) == (r.open_status[j] != 0) for j in range(len(rows)))
    labels = {OPEN_STATUS[expect_status[k]][0] for k in expect_status if expect_status[k]}
    assert labels <= set(got.step_failures)


def test_require_taskprov():
    """A taskprov task (require_taskprov): only reports with exactly one, empty taskprov extension open
    (aggregator.rs:1869-1879); a duplicate is a duplicate_extension first."""
    rnd = random.Random(77)
    v = Prio3.sum(8)
    vk = bytes(range(16, 32))
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    task_id = rnd.randbytes(32)
    kt = _keypair(rnd)
    kinds = ["taskprov", "valid", "taskprov_data", "dup_taskprov", "taskprov", "tbd_ext"]
    n = 24
    inits = _make_inits(rnd, orc, v, vk, task_id, n, lambda i: kinds[i % len(kinds)], lambda i: kt, lambda i: 3, seed=9)
    want, fin, _ = reference_responses(orc, vk, v, task_id, {3: [kt, None]}, inits, require_taskprov=True)
    with hpke.HpkeOpener(*kt, INFO) as ot, HelperEngine(v, vk) as eng:
        got = handle_aggregate_init_encrypted(eng, ot, 3, task_id, inits, require_taskprov=True)
    assert got.responses == want and fin.sum() == 2 * n // len(kinds)
    assert got.step_failures["missing_or_malformed_taskprov_extension"] == 3 * n // len(kinds)
    assert got.step_failures["duplicate_extension"] == n // len(kinds)


def _pool(rnd, v, vk, task_id, K, kt, seed):
    """K sealed PrepareInits: valid, tampered leader prep share (every 9th), corrupted ciphertext (every 13th),
    unknown config id (every 17th)."""
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)

    def kind(i):
        return ("unknown_cfg" if i % 17 == 5 else "corrupt_ct" if i % 13 == 4 else "tamper_lps" if i % 9 == 2
                else "valid")

    inits = _make_inits(rnd, orc, v, vk, task_id, K, kind, lambda i: kt, lambda i: 9 if kind(i) == "unknown_cfg" else 1,
                        seed=seed)
    want, fin, outs = reference_responses(orc, vk, v, task_id, {1: [kt, None]}, inits)
    return orc, inits, want, fin, outs


def test_64_threads_of_100_report_encrypted_jobs_two_tasks():
    """64 host threads, 100-report encrypted SumVec 8x1000/88 jobs of two tasks (verify keys, task ids, HPKE
    keys), coalesced: every job's PrepareResp list equals the reference's, including HpkeDecryptError and
    HpkeUnknownConfigId, the jobs' opens ran inside shared launches, and each task's aggregate equals the
    oracle's over the jobs' accepted reports."""
    rnd = random.Random(4242)
    v = Prio3.sum_vec(8, 1000, 88)
    K = 256
    tasks = []
    for k in range(2):
        vk, task_id, kt = bytes((37 * k + i) % 256 for i in range(16)), rnd.randbytes(32), _keypair(rnd)
        tasks.append((vk, task_id, kt) + _pool(rnd, v, vk, task_id, K, kt, seed=600 + k))
    openers = [hpke.HpkeOpener(*t[2], INFO) for t in tasks]
    engs = [HelperEngine(v, t[0]) for t in tasks]
    try:
        for e in engs:
            e.coalesce(True)
        m0 = engs[0].memory()
        n, per_thread = 100, 2
        results = {}

        errs = []

        def worker(t):
            try:
                k = t % 2
                vk, task_id, kt, orc, inits, want, fin, outs = tasks[k]
                for j in range(per_thread):
                    off = ((t // 2) * per_thread + j) * 41 % K
                    idx = [(off + i) % K for i in range(n)]
                    out = handle_aggregate_init_encrypted(engs[k], openers[k], 1, task_id, [inits[i] for i in idx])
                    results[(t, j)] = (k, idx, out)
            except BaseException as e:  # noqa: BLE001 - re-raised below
                errs.append(e)

        th = [threading.Thread(target=lambda t=t: worker(t)) for t in range(64)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            raise errs[0]
        assert len(results) == 64 * per_thread
        mult = [np.zeros(K, np.int64) for _ in tasks]
        kinds = set()
        for (t, j), (k, idx, out) in results.items():
            vk, task_id, kt, orc, inits, want, fin, outs = tasks[k]
            assert out.responses == [want[i] for i in idx], f"job {t}/{j}"
            for i in idx:
                mult[k][i] += int(fin[i])
                r = want[i].result
                kinds.add(r.error if r.kind == 2 else "ok")
        assert {"ok", PrepareError.VdafPrepError, PrepareError.HpkeDecryptError, PrepareError.HpkeUnknownConfigId} <= kinds
        m1 = engs[0].memory()
        jobs = m1["coalesced_encrypted_jobs"] - m0["coalesced_encrypted_jobs"]
        launches = m1["coalesced_helper_launches"] - m0["coalesced_helper_launches"]
        # shared launches (Python threads parse each job's messages under the GIL, so their jobs arrive spread
        # out; the native driver measures coalescing at scale: bench.py secondary.jobs, tools/jobs_driver.cpp)
        assert jobs == 64 * per_thread and jobs >= 2 * launches, (jobs, launches)
        for k, (vk, task_id, kt, orc, inits, want, fin, outs) in enumerate(tasks):
            agg, cnt, _ = engs[k].aggregate_share(0)
            assert cnt == int(mult[k].sum())
            dec = lambda b: [int.from_bytes(b[i:i + 16], "little") for i in range(0, len(b), 16)]  # noqa: E731
            exp = [0] * v.length
            for i in range(K):
                if mult[k][i]:
                    exp = [(x + int(mult[k][i]) * y) % P128 for x, y in zip(exp, dec(outs[i]))]
            assert dec(agg) == exp
    finally:
        for e in engs:
            e.close()
        for o in openers:
            o.close()


def test_plain_and_encrypted_jobs_share_a_launch():
    """A plain job (helper_initialized_batch) and an encrypted job of another task in ONE coalesced launch
    (debug option 7): the open kernel leaves the plain job's rows alone, and both equal the oracle."""
    rnd = random.Random(8)
    v = Prio3.histogram(40, 5)
    vks = [bytes(range(16)), bytes(range(3, 19))]
    task_id = rnd.randbytes(32)
    kt = _keypair(rnd)
    orc, inits, want, fin, outs = _pool(rnd, v, vks[1], task_id, 120, kt, seed=77)
    # the plain job: C-oracle reports of task 0
    orc0 = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    rng = np.random.default_rng(3)
    n0 = 90
    meas = rng.integers(0, v.length, size=(n0, 1), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n0, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n0, orc0.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc0.client_leader_batch(vks[0], meas, nonces, rands, nthreads=16)
    lps[5, 0] ^= 1
    want0 = orc0.helper_prep_batch(vks[0], nonces, ps, his, lps, nthreads=16)
    engs = [HelperEngine(v, vk) for vk in vks]
    with hpke.HpkeOpener(*kt, INFO) as ot:
        try:
            for e in engs:
                e.coalesce(True, window_us=1_000_000)
            # a first encrypted job: from then on the coalescer's helper lanes carry the encrypted-input regions
            first = handle_aggregate_init_encrypted(engs[1], ot, 1, task_id, inits[:10])
            assert first.responses == want[:10]
            engs[0].debug(7, 2)
            m0 = engs[0].memory()
            out = {}

            def plain():
                out["plain"] = engs[0].helper_initialized_batch(nonces, ps, his, lps, keep=False)

            def enc():
                out["enc"] = handle_aggregate_init_encrypted(engs[1], ot, 1, task_id, inits)

            th = [threading.Thread(target=plain), threading.Thread(target=enc)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            m1 = engs[0].memory()
            assert m1["coalesced_launches"] - m0["coalesced_launches"] == 1
            np.testing.assert_array_equal(out["plain"].verdicts, want0["verdicts"])
            assert out["enc"].responses == want
        finally:
            engs[0].debug(7, 0)
            for e in engs:
                e.close()
