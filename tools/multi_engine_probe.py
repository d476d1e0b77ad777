#!/usr/bin/env python3
"""Probe: one process, E helper engines on one GPU, each preparing + aggregating its own part of the
SumVec bench workload on its own HIP stream (no ordering between the engines inside a step), against
E = 1. Reports/s over whole steps, per-engine HIP-event kernel times, and the merged aggregate checked
against the pool's block aggregates (bench.CyclicPool).

    python tools/multi_engine_probe.py --engines 1 2 3 --reports 1250000 --steps 5 --warmup 1
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
    ap.add_argument("--engines", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--reports", type=int, default=1_250_000)
    ap.add_argument("--pool", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()

    import torch

    import bench
    from janus_amd.distributed import merge_records, pack_record, shard_range
    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3

    vdaf = Prio3.sum_vec(8, 1000, 88)
    vk = bytes(range(16))
    orc, nonces, ps, his, lps, want, how = bench.load_or_make_pool(vdaf, vk, a.pool, 16, 0)
    dev = torch.device("cuda", 0)
    R, K = a.reports, a.pool
    idx = torch.from_numpy(np.arange(R) % K).to(dev)
    tile = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev).index_select(0, idx).contiguous()  # noqa: E731
    d_n, d_ps, d_his, d_lps = tile(nonces), tile(ps), tile(his), tile(lps)
    d_v = torch.empty(R, dtype=torch.uint8, device=dev)
    d_m = torch.empty((R, 16), dtype=torch.uint8, device=dev)

    def partial(x, y):
        h = orc.helper_prep_batch(vk, nonces[x:y], ps[x:y], his[x:y], lps[x:y], nthreads=16)
        return bench.field_elems(h["agg"], 16)

    cyc = bench.CyclicPool(want["verdicts"] == 0, [bench.field_elems(b.tobytes(), 16) for b in want["blocks"]],
                           bench.POOL_BLOCK, partial, bench.P128)
    out = []
    for E in a.engines:
        engs = [HelperEngine(vdaf, vk, device=0) for _ in range(E)]
        parts = [shard_range(R, k, E) for k in range(E)]
        torch.cuda.synchronize()

        def step():
            for eng, (x, y) in zip(engs, parts):
                eng.prep_and_aggregate_device(d_n[x:].data_ptr(), d_ps[x:].data_ptr(), d_his[x:].data_ptr(),
                                              d_lps[x:].data_ptr(), y - x, 0, d_m[x:].data_ptr(), d_v[x:].data_ptr(),
                                              stream=False)
            for eng in engs:
                eng.sync()

        for _ in range(a.warmup):
            step()
        for eng in engs:
            eng.timing(True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        kts = [eng.timing_read() for eng in engs]
        recs = [pack_record(*eng.aggregate_share(0)) for eng in engs]
        agg, cnt, _ = merge_records(recs, 16)
        exp_agg, exp_cnt = cyc.range(0, R, a.steps + a.warmup)
        ok = agg == b"".join(x.to_bytes(16, "little") for x in exp_agg) and cnt == exp_cnt
        ok = ok and bool(np.array_equal(d_v.cpu().numpy(), want["verdicts"][np.arange(R) % K]))
        k1 = sum(k["xof"]["ms"] for k in kts) / max(1, sum(k["xof"]["launches"] for k in kts))
        k3 = sum(k["flp"]["ms"] for k in kts) / max(1, sum(k["flp"]["launches"] for k in kts))
        r = {"engines": E, "reports_per_s": round(R * a.steps / el, 1), "ms_per_step": round(el / a.steps * 1e3, 3),
             "k1_ms_per_launch": round(k1, 3), "k3_ms_per_launch": round(k3, 3),
             "launches_per_engine_step": kts[0]["xof"]["launches"] // a.steps, "verified": ok}
        print(json.dumps(r), flush=True)
        out.append(r)
        for eng in engs:
            eng.close()
        del engs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
