"""Pin the oracle's XOF: TurboSHAKE128 KATs (RFC 9861) and SHAKE128 (hashlib) at 24 rounds."""
import hashlib
import os

import pytest

from oracle import oracle as O
from oracle import pyref

# RFC 9861 TurboSHAKE128 test vectors (message, D, output length, expected tail)
KATS = [
    (b"", 0x1F, 32, "1e415f1c5983aff2169217277d17bb538cd945a397ddec541f1ce41af2c1b74c"),
    (b"", 0x1F, 64, "1e415f1c5983aff2169217277d17bb538cd945a397ddec541f1ce41af2c1b74c"
                    "3e8ccae2a4dae56c84a04c2385c03c15e8193bdf58737363321691c05462c8df"),
    (b"\xff\xff\xff", 0x01, 32, "bf323f940494e88ee1c540fe660be8a0c93f43d15ec006998462fa994eed5dab"),
    (b"\xff", 0x06, 32, "8ec9c66465ed0d4a6c35d13506718d687a25cb05c74cca1e42501abd83874a67"),
]


@pytest.mark.parametrize("msg,D,n,want", KATS)
def test_turboshake_kat_c(msg, D, n, want):
    assert O.turboshake128(msg, D, n).hex() == want


@pytest.mark.parametrize("msg,D,n,want", KATS)
def test_turboshake_kat_pyref(msg, D, n, want):
    assert pyref.turboshake128(msg, D, n).hex() == want


def test_turboshake_long_output_tail():
    # last 32 bytes of TurboSHAKE128(M = empty, D = 0x1F, 10032)
    assert O.turboshake128(b"", 0x1F, 10032)[-32:].hex() == \
        "a3b9b0385900ce761f22aed548e754da10a5242d62e8c658e3f3a923a7555607"


@pytest.mark.parametrize("n", [0, 1, 135, 136, 167, 168, 169, 335, 336, 1000])
def test_keccak_24_rounds_is_shake128(n):
    m = os.urandom(n)
    assert pyref.shake128_24(m, 400) == hashlib.shake_128(m).digest(400)


@pytest.mark.parametrize("n", [0, 1, 41, 42, 167, 168, 169, 1000, 5000])
def test_c_and_pyref_turboshake_agree(n):
    m = os.urandom(n)
    assert O.turboshake128(m, 1, 500) == pyref.turboshake128(m, 1, 500)


def test_c_keccak_matches_pyref_permutation():
    import random
    rnd = random.Random(3)
    st = [rnd.getrandbits(64) for _ in range(25)]
    lanes = [[st[x + 5 * y] for y in range(5)] for x in range(5)]
    for rounds in (12, 24):
        out = O.keccak_p1600(st, rounds)
        ref = pyref.keccak_p(lanes, rounds)
        assert out == [ref[i % 5][i // 5] for i in range(25)]


def test_sha256():
    for n in (0, 3, 16, 55, 56, 64, 100):
        m = os.urandom(n)
        assert O.sha256(m) == hashlib.sha256(m).digest()


def test_field_constants():
    p128 = 2**128 - 28 * 2**64 + 1
    p64 = 2**64 - 2**32 + 1
    g64 = O.field_op(True, 5, None)
    g128 = O.field_op(False, 5, None)
    assert g64 == pow(7, (p64 - 1) >> 32, p64) == 1753635133440165772
    assert g128 == pow(7, (p128 - 1) >> 66, p128) == 145091266659756586618791329697897684742
    assert pow(g64, 2**31, p64) != 1 and pow(g64, 2**32, p64) == 1
    assert pow(g128, 2**65, p128) != 1 and pow(g128, 2**66, p128) == 1


def test_field_ops_vs_bigint():
    import random
    rnd = random.Random(7)
    for f64, p in ((True, 2**64 - 2**32 + 1), (False, 2**128 - 28 * 2**64 + 1)):
        for _ in range(300):
            a, b = rnd.randrange(p), rnd.randrange(p)
            assert O.field_op(f64, 0, a, b) == (a + b) % p
            assert O.field_op(f64, 1, a, b) == (a - b) % p
            assert O.field_op(f64, 2, a, b) == a * b % p
        for a in (1, 2, p - 1, rnd.randrange(1, p)):
            assert O.field_op(f64, 3, a) * a % p == 1
