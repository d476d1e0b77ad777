#!/usr/bin/env python3
"""Throughput of Prio3SumVecField64MultiproofHmacSha256Aes128 helper prep + aggregate on one MI355X
(janus_amd/csrc/jx_mp64.hip).

Same measurement as bench.py, for the multiproof instance Janus builds at core/src/vdaf.rs:176-199:
a pool of K client reports (C-oracle client + leader prep_init, 1 % tampered) tiled on the device to
R reports, inputs resident in HBM; the timed region is `steps` fused prep_init + prep_next +
aggregate calls. The aggregate is verified against multiplicity x the oracle's output shares.
Prints one JSON line.

    python tools/bench_mp.py [--proofs 2 --bits 8 --length 1000 --chunk 88 --reports 1000000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

P64 = 2**64 - 2**32 + 1
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# Algorithmic int32 VALU instruction counts: one SHA-256 compression = 64 rounds x 14
# (6 v_alignbit, 2 xor3 + 2 v_bitop3 for ch/maj, 4 adds) + 48 schedule words x 10; one T-table AES-128
# block = 9 rounds x 24 (16 v_perm_b32 table addresses, 8 xor3) + 12 for the last round.
OPS_PER_SHA = 64 * 14 + 48 * 10
OPS_PER_AES = 9 * 24 + 12


def work(proofs, bits, length, chunk):
    M = bits * length
    calls = -(-M // chunk)
    P = 1
    while P < calls + 1:
        P <<= 1
    PL = 2 * chunk + 2 * P - 1
    sha = (26 + 8 * M + 9 + 63) // 64 + 8 + 4 * 6  # joint_rand_part stream + key pads/tags of ~6 HMACs
    aes = -(-8 * M // 16) + -(-8 * proofs * PL // 16) + 10
    return dict(sha=sha, aes=aes, ops_k1=sha * OPS_PER_SHA + aes * OPS_PER_AES,
                hbm_k1=8 * (M + proofs * PL + proofs * (5 + 2 * calls)) + 16 * length + 96 + 64 + 16,
                fmul_k3=2 * proofs * M)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proofs", type=int, default=2)
    ap.add_argument("--bits", type=int, default=8)
    ap.add_argument("--length", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=88)
    ap.add_argument("--reports", type=int, default=1_000_000)
    ap.add_argument("--pool", type=int, default=512)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    import torch

    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3
    from oracle import oracle as O  # input generation and the checker only

    vdaf = Prio3.sum_vec_field64_multiproof_hmacsha256_aes128(a.proofs, a.bits, a.length, a.chunk)
    orc = O.Prio3Oracle(O.SUMVEC_F64_MULTIPROOF, a.bits, a.length, a.chunk, a.proofs)
    vk = bytes(range(32))
    threads = min(16, os.cpu_count() or 1)
    rng = np.random.default_rng(0x5EED)
    K = a.pool
    meas = rng.integers(0, 1 << a.bits, size=(K, a.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
    t0 = time.perf_counter()
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=threads)
    for i in range(0, K, 100):
        j = int(rng.integers(0, lps.shape[1]))
        lps[i, j] ^= 1 << int(rng.integers(0, 8))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads, want_out_shares=True)
    t_pool = time.perf_counter() - t0
    print(f"pool of {K} generated + checked in {t_pool:.1f}s", file=sys.stderr, flush=True)

    R = a.reports
    reps = -(-R // K)
    dev = torch.device("cuda", 0)

    def tile(x):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev).repeat(reps, 1)[:R].contiguous()

    d_n, d_ps, d_his, d_lps = tile(nonces), tile(ps), tile(his), tile(lps)
    d_v = torch.empty(R, dtype=torch.uint8, device=dev)
    d_m = torch.empty((R, 32), dtype=torch.uint8, device=dev)
    with HelperEngine(vdaf, vk) as eng:
        def step():
            eng.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), R, 0,
                                          d_m.data_ptr(), d_v.data_ptr())
            eng.sync()

        for _ in range(a.warmup):
            step()
        eng.timing(True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        kt = eng.timing_read()
        agg, count, _ = eng.aggregate_share(0)
    # verification: aggregate == (steps + warmup) * sum_i mult_i * out_i
    total = a.steps + a.warmup
    mult = np.bincount(np.arange(R) % K, minlength=K)
    fin = want["verdicts"] == 0
    outs = want["out_shares"].reshape(K, a.length, 8).view("<u8").reshape(K, a.length).astype(object)
    acc = [0] * a.length
    for i in np.nonzero(fin)[0]:
        m = int(mult[i]) * total
        for j in range(a.length):
            acc[j] += m * int(outs[i, j])
    exp = b"".join((x % P64).to_bytes(8, "little") for x in acc)
    verified = agg == exp and count == total * int(mult[fin].sum()) and \
        bool(np.array_equal(d_v.cpu().numpy(), np.tile(want["verdicts"], reps)[:R]))
    w = work(a.proofs, a.bits, a.length, a.chunk)
    launches = max(1, kt["xof"]["launches"])
    per_launch = R / (launches / a.steps)
    k1_ms = kt["xof"]["ms"] / launches
    k3_ms = kt["flp"]["ms"] / max(1, kt["flp"]["launches"])
    k1_tops = w["ops_k1"] * per_launch / (k1_ms * 1e-3) / 1e12
    print(json.dumps({
        "metric": "helper reports/sec (prep_init+aggregate), Prio3SumVecField64MultiproofHmacSha256Aes128",
        "value": round(R * a.steps / dt, 1), "unit": "reports/s", "n_gpus": 1, "steps": a.steps,
        "config": {"proofs": a.proofs, "bits": a.bits, "length": a.length, "chunk_length": a.chunk,
                   "reports": R, "pool": K},
        "kernels": {"k1_ms_per_launch": round(k1_ms, 3), "k3_ms_per_launch": round(k3_ms, 3),
                    "k4_ms_per_launch": round(kt["accumulate"]["ms"] / max(1, kt["accumulate"]["launches"]), 3),
                    "slow_ms_per_launch": round(kt["slow"]["ms"] / max(1, kt["slow"]["launches"]), 3),
                    "reports_per_launch": int(per_launch)},
        "roofline": {"bound": "valu", "kernel": "K1 mp_xof_kernel", "achieved": round(k1_tops, 3),
                     "peak": round(VALU_PEAK_TOPS, 2), "frac": round(k1_tops / VALU_PEAK_TOPS, 4),
                     "unit": "TOP/s (algorithmic int32 VALU instructions: SHA-256 + T-table AES)",
                     "work_per_report": w},
        "verified": verified,
    }), flush=True)


if __name__ == "__main__":
    main()
