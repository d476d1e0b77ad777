#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer fused path (jx_helper_prep_aggregate: the inputs in pageable host
memory, copied to HBM per launch, verdicts and prep messages copied back), against the device path with the
inputs already in HBM (bench.py's `value`). SumVec 8x1000/88, the bench's pool tiled on the host.

    python tools/bench_host_path.py --reports 1250000 --steps 3
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reports", type=int, default=1_250_000)
    ap.add_argument("--pool", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()

    import bench
    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3

    vdaf = Prio3.sum_vec(8, 1000, 88)
    vk = bytes(range(16))
    orc, nonces, ps, his, lps, want, how = bench.load_or_make_pool(vdaf, vk, a.pool, 16, 0)
    R, K = a.reports, a.pool
    idx = np.arange(R) % K
    h = [np.ascontiguousarray(x[idx]) for x in (nonces, ps, his, lps)]  # pageable host buffers
    in_bytes = sum(x.nbytes for x in h)
    with HelperEngine(vdaf, vk) as eng:
        eng.prep_and_aggregate(*h)  # warm-up (staging allocation)
        t = time.perf_counter()
        for _ in range(a.steps):
            verdicts, msgs = eng.prep_and_aggregate(*h)
        el = time.perf_counter() - t
        ok = bool(np.array_equal(verdicts, want["verdicts"][idx]))
        fin = verdicts == 0
        ok = ok and bool(np.array_equal(msgs[fin], want["prep_msgs"][idx][fin]))
        _, cnt, _ = eng.aggregate_share(0)
        ok = ok and cnt == int((want["verdicts"][idx] == 0).sum()) * (a.steps + 1)
    r = {"path": "jx_helper_prep_aggregate (host buffers, pageable)", "reports": R, "steps": a.steps,
         "reports_per_s": round(R * a.steps / el, 1), "ms_per_step": round(el / a.steps * 1e3, 2),
         "input_bytes_per_step": in_bytes, "input_GBps": round(in_bytes * a.steps / el / 1e9, 2),
         "verified": ok}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
