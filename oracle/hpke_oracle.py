"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the HPKE suite Janus uses to protect
report shares: RFC 9180 base mode, DHKEM(X25519, HKDF-SHA256) / HKDF-SHA256 / AES-128-GCM
(KEM 0x0020, KDF 0x0001, AEAD 0x0001; Janus core/src/hpke.rs:167-230 via hpke-dispatch,
suite of docs/samples/tasks.yaml:54-58).

Only tests/ may import this module, as the checker of the batched HPKE-open kernels
(janus_amd/csrc/jx_hpke.hip). It is pinned by the RFC 9180 test vector for this suite that
the reference itself ships (core/src/test-vectors.json, used by core/src/hpke.rs:508-513),
copied as data into tests/golden/hpke_rfc9180.json.

Components: X25519 (RFC 7748 §5), HMAC/HKDF-SHA256 (RFC 2104 / RFC 5869, via hashlib),
AES-128 (FIPS 197), GCM (NIST SP 800-38D).
"""
from __future__ import annotations

import hashlib
import hmac

# ----------------------------------------------------------------------------- X25519

P25519 = 2**255 - 19
A24 = 121665


def _clamp(k: bytes) -> int:
    b = bytearray(k)
    b[0] &= 248
    b[31] &= 127
    b[31] |= 64
    return int.from_bytes(b, "little")


def x25519(k: bytes, u: bytes) -> bytes:
    """RFC 7748 §5: scalar multiplication on Curve25519 (Montgomery ladder)."""
    p = P25519
    kk = _clamp(k)
    x1 = int.from_bytes(u, "little") & ((1 << 255) - 1)
    x2, z2, x3, z3, swap = 1, 0, x1, 1, 0
    for t in reversed(range(255)):
        kt = (kk >> t) & 1
        swap ^= kt
        if swap:
            x2, x3, z2, z3 = x3, x2, z3, z2
        swap = kt
        a = (x2 + z2) % p
        aa = a * a % p
        b = (x2 - z2) % p
        bb = b * b % p
        e = (aa - bb) % p
        c = (x3 + z3) % p
        d = (x3 - z3) % p
        da = d * a % p
        cb = c * b % p
        x3 = (da + cb) ** 2 % p
        z3 = x1 * (da - cb) ** 2 % p
        x2 = aa * bb % p
        z2 = e * (aa + A24 * e) % p
    if swap:
        x2, x3, z2, z3 = x3, x2, z3, z2
    return (x2 * pow(z2, p - 2, p) % p).to_bytes(32, "little")


def x25519_base(k: bytes) -> bytes:
    return x25519(k, (9).to_bytes(32, "little"))


# ----------------------------------------------------------------------------- AES-128


def _gmul(a: int, b: int) -> int:
    r = 0
    for _ in range(8):
        if b & 1:
            r ^= a
        hi = a & 0x80
        a = (a << 1) & 0xFF
        if hi:
            a ^= 0x1B
        b >>= 1
    return r


def _make_sbox():
    inv = [0] * 256
    for x in range(1, 256):
        for y in range(1, 256):
            if _gmul(x, y) == 1:
                inv[x] = y
                break
    sbox = []
    for x in range(256):
        b = inv[x]
        s = b
        for i in range(1, 5):
            s ^= ((b << i) | (b >> (8 - i))) & 0xFF
        sbox.append(s ^ 0x63)
    return sbox


SBOX = _make_sbox()


def aes128_expand(key: bytes) -> list[bytes]:
    w = [list(key[4 * i:4 * i + 4]) for i in range(4)]
    rcon = 1
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = [SBOX[t[1]] ^ rcon, SBOX[t[2]], SBOX[t[3]], SBOX[t[0]]]
            rcon = _gmul(rcon, 2)
        w.append([w[i - 4][j] ^ t[j] for j in range(4)])
    return [bytes(sum(w[4 * r:4 * r + 4], [])) for r in range(11)]


def aes128_encrypt_block(rk: list[bytes], block: bytes) -> bytes:
    s = [block[i] ^ rk[0][i] for i in range(16)]  # column-major state: s[4c + r]
    for rnd in range(1, 11):
        s = [SBOX[x] for x in s]
        s = [s[(i + 4 * (i % 4)) % 16] for i in range(16)]  # ShiftRows
        if rnd != 10:
            t = []
            for c in range(4):
                a = s[4 * c:4 * c + 4]
                t += [_gmul(a[0], 2) ^ _gmul(a[1], 3) ^ a[2] ^ a[3],
                      a[0] ^ _gmul(a[1], 2) ^ _gmul(a[2], 3) ^ a[3],
                      a[0] ^ a[1] ^ _gmul(a[2], 2) ^ _gmul(a[3], 3),
                      _gmul(a[0], 3) ^ a[1] ^ a[2] ^ _gmul(a[3], 2)]
            s = t
        s = [s[i] ^ rk[rnd][i] for i in range(16)]
    return bytes(s)


# ----------------------------------------------------------------------------- GCM

_R = 0xE1 << 120


def _ghash_mul(x: int, y: int) -> int:
    z, v = 0, y
    for i in range(128):
        if (x >> (127 - i)) & 1:
            z ^= v
        v = (v >> 1) ^ _R if v & 1 else v >> 1
    return z


def _ghash(h: int, aad: bytes, ct: bytes) -> int:
    def blocks(b):
        b = b + bytes(-len(b) % 16)
        return [int.from_bytes(b[i:i + 16], "big") for i in range(0, len(b), 16)]

    y = 0
    for x in blocks(aad) + blocks(ct) + [((8 * len(aad)) << 64) | (8 * len(ct))]:
        y = _ghash_mul(y ^ x, h)
    return y


def _inc32(block: bytes) -> bytes:
    c = (int.from_bytes(block[12:], "big") + 1) & 0xFFFFFFFF
    return block[:12] + c.to_bytes(4, "big")


def _gctr(rk, icb: bytes, data: bytes) -> bytes:
    out, cb = bytearray(), icb
    for i in range(0, len(data), 16):
        ks = aes128_encrypt_block(rk, cb)
        out += bytes(a ^ b for a, b in zip(data[i:i + 16], ks))
        cb = _inc32(cb)
    return bytes(out)


def aes128gcm_seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> bytes:
    rk = aes128_expand(key)
    h = int.from_bytes(aes128_encrypt_block(rk, bytes(16)), "big")
    j0 = nonce + b"\x00\x00\x00\x01"
    ct = _gctr(rk, _inc32(j0), pt)
    s = _ghash(h, aad, ct).to_bytes(16, "big")
    return ct + _gctr(rk, j0, s)


def aes128gcm_open(key: bytes, nonce: bytes, aad: bytes, ct_tag: bytes) -> bytes | None:
    if len(ct_tag) < 16:
        return None
    ct, tag = ct_tag[:-16], ct_tag[-16:]
    rk = aes128_expand(key)
    h = int.from_bytes(aes128_encrypt_block(rk, bytes(16)), "big")
    j0 = nonce + b"\x00\x00\x00\x01"
    s = _ghash(h, aad, ct).to_bytes(16, "big")
    if not hmac.compare_digest(_gctr(rk, j0, s), tag):
        return None
    return _gctr(rk, _inc32(j0), ct)


# ----------------------------------------------------------------------------- HPKE (RFC 9180)

KEM_ID, KDF_ID, AEAD_ID = 0x0020, 0x0001, 0x0001
SUITE_KEM = b"KEM" + KEM_ID.to_bytes(2, "big")
SUITE = b"HPKE" + KEM_ID.to_bytes(2, "big") + KDF_ID.to_bytes(2, "big") + AEAD_ID.to_bytes(2, "big")


def hkdf_extract(salt: bytes, ikm: bytes) -> bytes:
    return hmac.new(salt, ikm, hashlib.sha256).digest()


def hkdf_expand(prk: bytes, info: bytes, n: int) -> bytes:
    out, t, i = b"", b"", 1
    while len(out) < n:
        t = hmac.new(prk, t + info + bytes([i]), hashlib.sha256).digest()
        out += t
        i += 1
    return out[:n]


def labeled_extract(suite: bytes, salt: bytes, label: bytes, ikm: bytes) -> bytes:
    return hkdf_extract(salt, b"HPKE-v1" + suite + label + ikm)


def labeled_expand(suite: bytes, prk: bytes, label: bytes, info: bytes, n: int) -> bytes:
    return hkdf_expand(prk, n.to_bytes(2, "big") + b"HPKE-v1" + suite + label + info, n)


def key_schedule(shared_secret: bytes, info: bytes) -> tuple[bytes, bytes]:
    """mode_base: (key, base_nonce)."""
    psk_id_hash = labeled_extract(SUITE, b"", b"psk_id_hash", b"")
    info_hash = labeled_extract(SUITE, b"", b"info_hash", info)
    ksc = b"\x00" + psk_id_hash + info_hash
    secret = labeled_extract(SUITE, shared_secret, b"secret", b"")
    return labeled_expand(SUITE, secret, b"key", ksc, 16), labeled_expand(SUITE, secret, b"base_nonce", ksc, 12)


def decap(enc: bytes, sk: bytes, pk: bytes) -> bytes | None:
    dh = x25519(sk, enc)
    if dh == bytes(32):
        return None
    eae_prk = labeled_extract(SUITE_KEM, b"", b"eae_prk", dh)
    return labeled_expand(SUITE_KEM, eae_prk, b"shared_secret", enc + pk, 32)


def encap(ske: bytes, pk: bytes) -> tuple[bytes, bytes]:
    enc = x25519_base(ske)
    dh = x25519(ske, pk)
    eae_prk = labeled_extract(SUITE_KEM, b"", b"eae_prk", dh)
    return labeled_expand(SUITE_KEM, eae_prk, b"shared_secret", enc + pk, 32), enc


def open_base(sk: bytes, pk: bytes, info: bytes, enc: bytes, aad: bytes, ct: bytes) -> bytes | None:
    ss = decap(enc, sk, pk)
    if ss is None:
        return None
    key, nonce = key_schedule(ss, info)
    return aes128gcm_open(key, nonce, aad, ct)


def seal_base(pk: bytes, info: bytes, aad: bytes, pt: bytes, ske: bytes) -> tuple[bytes, bytes]:
    """Deterministic seal with the given ephemeral secret key (tests only). Returns (enc, ct)."""
    ss, enc = encap(ske, pk)
    key, nonce = key_schedule(ss, info)
    return enc, aes128gcm_seal(key, nonce, aad, pt)


def dap_info(label: bytes = b"dap-09 input share", sender: int = 1, recipient: int = 3) -> bytes:
    """HpkeApplicationInfo (core/src/hpke.rs:69-84): label || sender role || recipient role
    (Role: Collector 0, Client 1, Leader 2, Helper 3; messages/src/lib.rs:512-517)."""
    return label + bytes([sender, recipient])
