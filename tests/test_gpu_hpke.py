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
        encs.append(enc)
        cts.append(ct)
        aads.append(aad)
        want.append(H.open_base(sk, pk, info, enc, aad, ct) if len(ct) >= 16 else None)
    with hpke.HpkeOpener(sk, pk, info) as op:
        got = op.open_batch(encs, cts, aads)
    assert got == want
    assert sum(x is None for x in got) == 4 * n // 10
    # a different application info (aggregate-share label) cannot open input shares
    with hpke.HpkeOpener(sk, pk, hpke.application_info(hpke.LABEL_AGGREGATE_SHARE, hpke.ROLE_HELPER,
                                                       hpke.ROLE_COLLECTOR)) as op:
        assert all(x is None for x in op.open_batch(encs[:10], cts[:10], aads[:10]))
