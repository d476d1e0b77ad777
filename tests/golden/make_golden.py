"""Generate the golden fixtures in tests/golden/*.json from the C oracle (oracle/prio3_oracle.c).

The reference tree holds no Prio3 vectors, so these fixtures pin
GPU <-> C oracle <-> pure-Python restatement agreement; parity with prio 0.16.1 itself is
unpinned. Inputs are seeded; re-running this script reproduces the files byte for byte.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

VK = bytes(range(16))
VK32 = bytes(range(32))  # VERIFY_KEY_LENGTH_HMACSHA256_AES128, core/src/vdaf.rs:24

CONFIGS = {
    "count": dict(algo=O.COUNT, bits=0, length=0, chunk=0, n=12),
    "sum8": dict(algo=O.SUM, bits=8, length=0, chunk=0, n=12),
    "sum32": dict(algo=O.SUM, bits=32, length=0, chunk=0, n=10),
    "sumvec_small": dict(algo=O.SUMVEC, bits=2, length=10, chunk=4, n=12),
    "sumvec_8x1000_88": dict(algo=O.SUMVEC, bits=8, length=1000, chunk=88, n=6),
    "histogram_16_4": dict(algo=O.HISTOGRAM, bits=0, length=16, chunk=4, n=12),
    "histogram_256_16": dict(algo=O.HISTOGRAM, bits=0, length=256, chunk=16, n=8),
    # Prio3SumVecField64MultiproofHmacSha256Aes128: the parameter sets of Janus's own tests
    # (integration_tests/tests/integration/janus.rs:369-374, taskprov_tests.rs:1266) and the
    # headline SumVec shape with two and three proofs
    "sumvec_f64mp_2_16x15_16": dict(algo=O.SUMVEC_F64_MULTIPROOF, bits=16, length=15, chunk=16, proofs=2, n=12),
    "sumvec_f64mp_2_8x12_14": dict(algo=O.SUMVEC_F64_MULTIPROOF, bits=8, length=12, chunk=14, proofs=2, n=12),
    "sumvec_f64mp_3_1x7_3": dict(algo=O.SUMVEC_F64_MULTIPROOF, bits=1, length=7, chunk=3, proofs=3, n=12),
    "sumvec_f64mp_2_8x1000_88": dict(algo=O.SUMVEC_F64_MULTIPROOF, bits=8, length=1000, chunk=88, proofs=2, n=6),
    "sumvec_f64mp_3_8x1000_88": dict(algo=O.SUMVEC_F64_MULTIPROOF, bits=8, length=1000, chunk=88, proofs=3, n=6),
    # Prio3FixedPointBoundedL2VecSum: the reference's e2e shape (length 3, both bitsizes), a length
    # with short last chunks in both gadgets, and the BASELINE configs[4] shape (16-bit, 10000)
    "fixedpoint16_3": dict(algo=O.FIXEDPOINT_L2, bits=16, length=3, chunk=0, n=12),
    "fixedpoint32_3": dict(algo=O.FIXEDPOINT_L2, bits=32, length=3, chunk=0, n=12),
    "fixedpoint16_37": dict(algo=O.FIXEDPOINT_L2, bits=16, length=37, chunk=0, n=12),
    "fixedpoint32_100": dict(algo=O.FIXEDPOINT_L2, bits=32, length=100, chunk=0, n=12),
    "fixedpoint16_10000": dict(algo=O.FIXEDPOINT_L2, bits=16, length=10000, chunk=0, n=6),
}


def measurements(cfg, rng, n):
    a = cfg["algo"]
    if a == O.COUNT:
        return rng.integers(0, 2, size=(n, 1), dtype=np.uint64)
    if a == O.SUM:
        return rng.integers(0, 1 << cfg["bits"], size=(n, 1), dtype=np.uint64)
    if a == O.HISTOGRAM:
        return rng.integers(0, cfg["length"], size=(n, 1), dtype=np.uint64)
    if a == O.FIXEDPOINT_L2:
        return fixedpoint_measurements(cfg["bits"], cfg["length"], rng, n)
    return rng.integers(0, 1 << cfg["bits"], size=(n, cfg["length"]), dtype=np.uint64)


def fixedpoint_measurements(bits, length, rng, n, violate_every=6):
    """FixedI{bits}<U{bits-1}> bit patterns with squared L2 norm < 1/4, except every
    `violate_every`-th report (index 4 mod 6): entries of 1/2 and -1/2 whose squared norm >= 1
    (a client lying about its norm; the FLP must reject it)."""
    half = 1 << (bits - 1)
    lim = max(1, int(half / (2 * np.sqrt(length))))
    vals = rng.integers(-lim, lim, size=(n, length), dtype=np.int64)
    for i in range(n):
        if violate_every and i % violate_every == 4 and length >= 4:
            vals[i] = np.where(np.arange(length) % 2 == 0, half // 2, -(half // 2))
    return (vals & ((1 << bits) - 1)).astype(np.uint64)


def tamper(lps: np.ndarray, sizes: O.Sizes, rng) -> list[str]:
    """Per report: '' (honest) or a description of the tampering applied to the leader prep share."""
    kinds = []
    n = lps.shape[0]
    for i in range(n):
        k = i % 6
        if k == 1:  # flip a bit in a verifier element (decide fails, or decode if it crosses p)
            lps[i, 1 + sizes.field_bytes] ^= 0x01
            kinds.append("verifier_bitflip")
        elif k == 3:  # verifier element >= p: decode failure
            lps[i, 0:sizes.field_bytes] = 0xFF
            kinds.append("verifier_ge_p")
        elif k == 5 and sizes.joint_rand_len:  # leader joint-rand part altered: prepare_next failure
            lps[i, -1] ^= 0x80
            kinds.append("joint_rand_part")
        else:
            kinds.append("")
    return kinds


def make(name, cfg):
    rng = np.random.default_rng(sum(map(ord, name)) * 7919)
    proofs = cfg.get("proofs", 1)
    orc = O.Prio3Oracle(cfg["algo"], cfg["bits"], cfg["length"], cfg["chunk"], proofs)
    s = orc.sizes
    VK = VK32 if s.verify_key == 32 else bytes(range(16))
    n = cfg["n"]
    meas = measurements(cfg, rng, n)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, s.client_rand), dtype=np.uint8)
    ps, his, lps, lout = orc.client_leader_batch(VK, meas, nonces, rands, nthreads=8, want_leader_out=True)
    kinds = tamper(lps, s, rng)
    res = orc.helper_prep_batch(VK, nonces, ps, his, lps, nthreads=8, want_out_shares=True)
    reports = []
    for i in range(n):
        v = int(res["verdicts"][i])
        out = res["out_shares"][i].tobytes() if v == 0 else b""
        m = [int(x) for x in meas[i]]
        rep = {
            "measurement": m if len(m) <= 1000 else
            {"sha256_u64le": hashlib.sha256(meas[i].astype("<u8").tobytes()).hexdigest()},
            "nonce": nonces[i].tobytes().hex(),
            "public_share": ps[i].tobytes().hex(),
            "helper_input_share": his[i].tobytes().hex(),
            "leader_prep_share": lps[i].tobytes().hex(),
            "tamper": kinds[i],
            "verdict": v,
            "prep_msg": res["prep_msgs"][i].tobytes().hex() if v == 0 else "",
            "out_share_sha256": hashlib.sha256(out).hexdigest() if v == 0 else "",
        }
        if v == 0 and len(out) <= 4096:
            rep["out_share"] = out.hex()
        if v == 0:
            rep["leader_out_share_sha256"] = hashlib.sha256(lout[i].tobytes()).hexdigest()
        reports.append(rep)
    doc = {
        "generator": "tests/golden/make_golden.py (C oracle oracle/prio3_oracle.c)",
        "parity": "pins GPU == C oracle == pyref; parity with prio 0.16.1 unpinned (SURVEY.md 8c)",
        "vdaf": {"algo_id": cfg["algo"], "bits": cfg["bits"], "length": cfg["length"],
                 "chunk_length": cfg["chunk"], "num_proofs": proofs},
        "verify_key": VK.hex(),
        "sizes": s.__dict__,
        "reports": reports,
        **({"aggregate_share": res["agg"].hex()} if len(res["agg"]) <= 16000 else
           {"aggregate_share_sha256": hashlib.sha256(res["agg"]).hexdigest()}),
        "report_count": res["count"],
        "checksum": res["checksum"].hex(),
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{name}.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"{name}: {n} reports, verdicts={[r['verdict'] for r in reports]} -> {path}")


if __name__ == "__main__":
    O.build()
    only = set(sys.argv[1:])
    for name, cfg in CONFIGS.items():
        if not only or name in only:
            make(name, cfg)
