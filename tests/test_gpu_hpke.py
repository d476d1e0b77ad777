"""GPU parity of batched HPKE open (janus_amd/csrc/jx_hpke.hip) against the RFC 9180 vector the
reference ships (tests/golden/hpke_rfc9180.json, from core/src/test-vectors.json) and against
oracle/hpke_oracle.py on DAP-shaped report shares (InputShareAad, input-share application
info), including every failure the helper maps to PrepareError::HpkeDecryptError."""
from __future__ import annotations

import json
import os
import random

import pytest

from janus_amd import hpke
from oracle import hpke_oracle as H

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "hpke_rfc9180.json")


def test_rfc9180_vector_on_gpu():
    for v in json.load(open(GOLDEN))["vectors"]:
        sk, pk = bytes.fromhex(v["skRm"]), bytes.fromhex(v["pkRm"])
        e = v["encryptions"][0]
        with hpke.HpkeOpener(sk, pk, bytes.fromhex(v["info"])) as op:
            out = op.open_batch([bytes.fromhex(v["enc"])], [bytes.fromhex(e["ct"])], [bytes.fromhex(e["aad"])])
        assert out[0] is not None and out[0].hex() == e["pt"]


def test_dap_batch_vs_oracle():
    rnd = random.Random(2024)
    sk = rnd.randbytes(32)
    pk = H.x25519_base(sk)
    info = hpke.application_info()
    assert info == H.dap_info()
    task = rnd.randbytes(32)
    encs, cts, aads, want = [], [], [], []
    n = 150
    for i in range(n):
        rid = rnd.randbytes(16)
        ps = rnd.randbytes(32)
        aad = hpke.input_share_aad(task, rid, 1_700_000_000 + i, ps)
        # PlaintextInputShare: u16 extensions length (0) || u32 payload length || payload (helper share)
        pt = (0).to_bytes(2, "big") + (48).to_bytes(4, "big") + rnd.randbytes(48 + (i % 5) * 7)
        enc, ct = H.seal_base(pk, info, aad, pt, rnd.randbytes(32))
        kind = i % 10
        if kind == 3:  # tampered ciphertext byte
            ct = bytearray(ct)
            ct[rnd.randrange(len(ct))] ^= 1 << rnd.randrange(8)
            ct = bytes(ct)
        elif kind == 5:  # wrong associated data (e.g. another task)
            aad = aad[:-1] + bytes([aad[-1] ^ 0x80])
        elif kind == 7:  # encapsulated key of a low-order point: all-zero DH -> error
            enc = bytes(32)
        elif kind == 9:  # truncated below the tag size
            ct = ct[:15]
        elif kind == 1:  # malformed encapsulated key length: fails alone, not the whole batch
            enc = enc[:31] if i % 20 == 1 else enc + b"\0"
        encs.append(enc)
        cts.append(ct)
        aads.append(aad)
        want.append(H.open_base(sk, pk, info, enc, aad, ct) if len(ct) >= 16 and len(enc) == 32 else None)
    with hpke.HpkeOpener(sk, pk, info) as op:
        got = op.open_batch(encs, cts, aads)
    assert got == want
    assert sum(x is None for x in got) == 5 * n // 10
    # a different application info (aggregate-share label) cannot open input shares
    with hpke.HpkeOpener(sk, pk, hpke.application_info(hpke.LABEL_AGGREGATE_SHARE, hpke.ROLE_HELPER,
                                                       hpke.ROLE_COLLECTOR)) as op:
        assert all(x is None for x in op.open_batch(encs[:10], cts[:10], aads[:10]))


def test_helper_aggregate_init_with_hpke_on_gpu():
    """handle_aggregate_init_encrypted: batched HPKE open + plaintext checks + batched prepare +
    accumulate, against the C oracle's verdicts and aggregate (aggregator.rs:1763-2013)."""
    import numpy as np

    from janus_amd.aggregator import handle_aggregate_init_encrypted
    from janus_amd.engine import HelperEngine
    from janus_amd.messages import (EXTENSION_TASKPROV, EXTENSION_TBD, Extension, HpkeCiphertext, PingPongMessage,
                                    PlaintextInputShare, PrepareError, PrepareInit, ReportMetadata, ReportShare)
    from janus_amd.vdaf import Prio3
    from oracle import oracle as O

    rnd = random.Random(77)
    v = Prio3.sum_vec(8, 1000, 88)
    vk = bytes(range(16))
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    n = 48
    rng = np.random.default_rng(5)
    meas = rng.integers(0, 256, size=(n, v.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
    sk = rnd.randbytes(32)
    pk = H.x25519_base(sk)
    info = hpke.application_info()
    task = rnd.randbytes(32)
    inits = []
    for i in range(n):
        md = ReportMetadata(nonces[i].tobytes(), 1_700_000_000 + i)
        exts = ()
        if i % 12 == 4:
            exts = (Extension(EXTENSION_TBD, b"x"), Extension(EXTENSION_TBD, b"y"))  # duplicate -> InvalidMessage
        if i % 12 == 6:
            exts = (Extension(EXTENSION_TASKPROV),)  # unexpected taskprov -> InvalidMessage
        pt = PlaintextInputShare(exts, his[i].tobytes()).encode()
        aad = hpke.input_share_aad(task, md.report_id, md.time, ps[i].tobytes())
        enc, ct = H.seal_base(pk, info, aad, pt, rnd.randbytes(32))
        cfg = 7
        if i % 12 == 8:
            ct = ct[:-1] + bytes([ct[-1] ^ 1])  # tag mismatch -> HpkeDecryptError
        if i % 12 == 10:
            cfg = 9  # unknown HPKE config -> HpkeUnknownConfigId
        inits.append(PrepareInit(ReportShare(md, ps[i].tobytes(), HpkeCiphertext(cfg, enc, ct)),
                                 PingPongMessage.initialize(lps[i].tobytes())))
    with hpke.HpkeOpener(sk, pk, info) as op, HelperEngine(v, vk) as eng:
        out = handle_aggregate_init_encrypted(eng, op, 7, task, inits)
        agg, count, checksum = eng.aggregate_share(0)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
    expected_err = {4: PrepareError.InvalidMessage, 6: PrepareError.InvalidMessage,
                    8: PrepareError.HpkeDecryptError, 10: PrepareError.HpkeUnknownConfigId}
    ok = np.zeros(n, bool)
    for i, resp in enumerate(out.responses):
        assert resp.report_id == nonces[i].tobytes()
        if i % 12 in expected_err:
            assert resp.result.kind == 2 and resp.result.error == expected_err[i % 12], i
        elif want["verdicts"][i] != 0:
            assert resp.result.kind == 2 and resp.result.error == PrepareError.VdafPrepError
        else:
            assert resp.result.kind == 0 and resp.result.message.prep_msg == want["prep_msgs"][i].tobytes()
            ok[i] = True
    assert (out.finished == ok).all() and count == ok.sum()
    assert agg == orc.aggregate([want["out_shares"][i].tobytes() for i in np.nonzero(ok)[0]])
