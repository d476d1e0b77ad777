#!/usr/bin/env python3
"""Throughput of batched HPKE open on one MI355X (janus_amd/csrc/jx_hpke.hip).

A pool of K report shares shaped like Janus's helper input shares (PlaintextInputShare with
a 48-byte Prio3 helper input share, InputShareAad with a 32-byte public share) is sealed by the
test oracle and tiled on the device to N ciphertexts; the timed region is one
jx_hpke_open_batch_device call over all N (inputs resident in HBM). Prints one JSON line.

    python tools/bench_hpke.py [--n 1048576] [--pool 256] [--reps 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--pool", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch

    from janus_amd import hpke
    from oracle import hpke_oracle as H

    rnd = random.Random(1)
    sk = rnd.randbytes(32)
    pk = H.x25519_base(sk)
    info = hpke.application_info()
    task = rnd.randbytes(32)
    encs, cts, aads, pts = [], [], [], []
    for i in range(a.pool):
        aad = hpke.input_share_aad(task, rnd.randbytes(16), 1_700_000_000 + i, rnd.randbytes(32))
        pt = (0).to_bytes(2, "big") + (48).to_bytes(4, "big") + rnd.randbytes(48)
        enc, ct = H.seal_base(pk, info, aad, pt, rnd.randbytes(32))
        encs.append(enc)
        cts.append(ct)
        aads.append(aad)
        pts.append(pt)
    reps = -(-a.n // a.pool)
    dev = torch.device("cuda", 0)
    tile = lambda xs: torch.from_numpy(np.frombuffer(b"".join(xs), np.uint8).copy()).to(dev).repeat(reps)[  # noqa: E731
        : a.n * len(xs[0])].contiguous()
    d_enc, d_ct, d_aad = tile(encs), tile(cts), tile(aads)
    cl, al = len(cts[0]), len(aads[0])
    d_co = torch.arange(a.n + 1, dtype=torch.int64, device=dev) * cl
    d_ao = torch.arange(a.n + 1, dtype=torch.int64, device=dev) * al
    d_pt = torch.empty(a.n * (cl - 16), dtype=torch.uint8, device=dev)
    d_ok = torch.empty(a.n, dtype=torch.uint8, device=dev)
    with hpke.HpkeOpener(sk, pk, info) as op:
        L = op._L

        def run():
            st = L.jx_hpke_open_batch_device(op._h, a.n, d_enc.data_ptr(), d_ct.data_ptr(), d_co.data_ptr(),
                                             d_aad.data_ptr(), d_ao.data_ptr(), d_pt.data_ptr(), d_ok.data_ptr())
            assert st == 0, st
            torch.cuda.synchronize()

        run()
        t = time.perf_counter()
        for _ in range(a.reps):
            run()
        dt = (time.perf_counter() - t) / a.reps
    ok = bool(d_ok.all().item())
    got = d_pt[: a.pool * (cl - 16)].cpu().numpy().tobytes()
    ok = ok and got == b"".join(pts)
    print(json.dumps({"metric": "HPKE opens/s (X25519 + HKDF-SHA256 + AES-128-GCM, RFC 9180 base)",
                      "value": round(a.n / dt, 1), "unit": "opens/s", "n": a.n, "ms_per_batch": round(dt * 1e3, 3),
                      "ciphertext_bytes": cl, "aad_bytes": al, "verified": ok}))


if __name__ == "__main__":
    main()
