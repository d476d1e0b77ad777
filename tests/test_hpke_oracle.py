"""The HPKE oracle (oracle/hpke_oracle.py) pinned by the RFC 9180 vector the reference ships
(core/src/test-vectors.json -> tests/golden/hpke_rfc9180.json) and by the component KATs of
FIPS 197 (AES-128), the GCM specification (test case 2) and RFC 7748 (X25519)."""
import json
import os

from oracle import hpke_oracle as H

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "hpke_rfc9180.json")


def test_aes128_fips197():
    rk = H.aes128_expand(bytes(range(16)))
    assert H.aes128_encrypt_block(rk, bytes.fromhex("00112233445566778899aabbccddeeff")).hex() == \
        "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_gcm_test_case_2():
    ct = H.aes128gcm_seal(bytes(16), bytes(12), b"", bytes(16))
    assert ct.hex() == "0388dace60b6a392f328c2b971b2fe78" + "ab6e47d42cec13bdf53a67b21257bddf"
    assert H.aes128gcm_open(bytes(16), bytes(12), b"", ct) == bytes(16)
    assert H.aes128gcm_open(bytes(16), bytes(12), b"x", ct) is None


def test_x25519_rfc7748():
    k = bytes.fromhex("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4")
    u = bytes.fromhex("e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c")
    assert H.x25519(k, u).hex() == "c3da55379de9c6908e94ea4df28d084f32eccf03491c71f754b4075577a28552"


def test_rfc9180_vector_from_reference():
    for v in json.load(open(GOLDEN))["vectors"]:
        sk, pk, enc = bytes.fromhex(v["skRm"]), bytes.fromhex(v["pkRm"]), bytes.fromhex(v["enc"])
        info = bytes.fromhex(v["info"])
        assert H.x25519_base(sk) == pk
        ss = H.decap(enc, sk, pk)
        key, nonce = H.key_schedule(ss, info)
        assert nonce.hex() == v["base_nonce"]
        e0 = v["encryptions"][0]  # sequence number 0: nonce == base_nonce
        assert e0["nonce"] == v["base_nonce"]
        pt = H.open_base(sk, pk, info, enc, bytes.fromhex(e0["aad"]), bytes.fromhex(e0["ct"]))
        assert pt.hex() == e0["pt"]


def test_seal_open_roundtrip_and_tamper():
    sk = bytes(range(1, 33))
    pk = H.x25519_base(sk)
    info = H.dap_info()
    enc, ct = H.seal_base(pk, info, b"aad", b"input share payload", bytes(range(40, 72)))
    assert H.open_base(sk, pk, info, enc, b"aad", ct) == b"input share payload"
    assert H.open_base(sk, pk, info, enc, b"aad!", ct) is None
    bad = bytearray(ct)
    bad[3] ^= 1
    assert H.open_base(sk, pk, info, enc, b"aad", bytes(bad)) is None
    assert H.open_base(sk, pk, H.dap_info(sender=2), enc, b"aad", ct) is None
