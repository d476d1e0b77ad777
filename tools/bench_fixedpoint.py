#!/usr/bin/env python3
"""BASELINE configs[4]: Prio3FixedPointBoundedL2VecSum 16-bit length=10000, leader+helper ping-pong
prep with joint randomness, on one MI355X.

One step = one aggregation job of R reports taken through both roles with every input resident in
HBM (aggregation_job_driver.rs:259-436 + aggregator.rs:1712-2161, minus HTTP and the datastore):
  leader  jx_leader_prep_init_device   (leader_initialized: prepare_init agg_id 0, explicit shares)
  helper  jx_helper_prep_aggregate_device (helper_initialized + evaluate + accumulate)
  leader  jx_leader_prep_finish_device (leader_continued on the helper's Finish; helper rejects fail)
  leader  jx_accumulate_device
The two engines (one per role) share the GPU here; in a deployment they are two aggregators. The
helper-only rate (the north-star unit) and per-role kernel times are reported too. Inputs: a pool
of K distinct client reports (C-oracle shard; 1 in 6 claims a false norm and must be rejected)
tiled on the device. Verified: both aggregates add up to multiplicity x the sum of the accepted
entries' encodings, and every verdict matches the oracle. The C oracle (leader prep_init + helper
prep per report) and the C++ CPU engine's two roles (the baseline proper) are timed on the host
beside it (kind "port").

    python tools/bench_fixedpoint.py [--bits 16 --length 10000 --reports 8192 --pool 48]
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
P128 = 2**128 - 28 * 2**64 + 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=16)
    ap.add_argument("--length", type=int, default=10000)
    ap.add_argument("--reports", type=int, default=8192)
    ap.add_argument("--pool", type=int, default=48)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    a = ap.parse_args()

    import torch

    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3
    from oracle import oracle as O  # input generation, checker and CPU baseline only
    from tests.golden.make_golden import fixedpoint_measurements

    threads = min(16, os.cpu_count() or 1)
    vdaf = Prio3.fixedpoint_boundedl2_vec_sum(a.bits, a.length)
    orc = O.Prio3Oracle(O.FIXEDPOINT_L2, a.bits, a.length, 0)
    vk = bytes(range(16))
    K, R = a.pool, a.reports
    rng = np.random.default_rng(0x5EED)
    meas = fixedpoint_measurements(a.bits, a.length, rng, K)
    nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
    t0 = time.perf_counter()
    shards = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(K)]
    ps, lis, his = (np.frombuffer(b"".join(s[k] for s in shards), np.uint8).reshape(K, -1) for k in range(3))
    lps = np.stack([np.frombuffer(orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())[1],
                                  np.uint8) for i in range(K)])
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads)
    print(f"pool of {K} generated in {time.perf_counter() - t0:.1f}s; oracle verdicts {want['verdicts'].tolist()}",
          file=sys.stderr)

    reps = -(-R // K)
    dev = torch.device("cuda", 0)

    def tile(x):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev).repeat(reps, 1)[:R].contiguous()

    d_n, d_ps, d_lis, d_his = tile(nonces), tile(ps), tile(lis), tile(his)
    d_lps = torch.empty((R, vdaf.prep_share_len), dtype=torch.uint8, device=dev)
    d_msgs = torch.empty((R, 16), dtype=torch.uint8, device=dev)
    d_hv = torch.empty(R, dtype=torch.uint8, device=dev)
    d_lv = torch.empty(R, dtype=torch.uint8, device=dev)
    leader, helper = HelperEngine(vdaf, vk), HelperEngine(vdaf, vk)
    role_s = {"leader_init": 0.0, "helper": 0.0, "leader_finish_acc": 0.0}

    def step(timed):
        t = time.perf_counter()
        bid = leader.leader_init_device(R, d_n.data_ptr(), d_ps.data_ptr(), d_lis.data_ptr(), d_lps.data_ptr())
        leader.sync()
        t1 = time.perf_counter()
        helper.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), R, 0,
                                         d_msgs.data_ptr(), d_hv.data_ptr())
        helper.sync()
        t2 = time.perf_counter()
        leader.leader_finish_device(bid, R, d_msgs.data_ptr(), d_hv.data_ptr(), d_lv.data_ptr())
        leader.accumulate_device(bid, R)
        leader.sync()
        t3 = time.perf_counter()
        if timed:
            role_s["leader_init"] += t1 - t
            role_s["helper"] += t2 - t1
            role_s["leader_finish_acc"] += t3 - t2

    for _ in range(a.warmup):
        step(False)
    leader.timing(True)
    helper.timing(True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    kl, kh = leader.timing_read(), helper.timing_read()
    agg_l, cnt_l, cs_l = leader.aggregate_share(0)
    agg_h, cnt_h, cs_h = helper.aggregate_share(0)
    leader.close()
    helper.close()

    total = a.steps + a.warmup
    mult = np.bincount(np.arange(R) % K, minlength=K)
    fin = want["verdicts"] == 0
    enc = meas.astype(object) ^ (1 << (a.bits - 1))
    exp = [int((enc[fin, j] * mult[fin]).sum()) * total % P128 for j in range(a.length)]
    got = [(int.from_bytes(agg_l[16 * j:16 * j + 16], "little") + int.from_bytes(agg_h[16 * j:16 * j + 16], "little"))
           % P128 for j in range(a.length)]
    exp_count = total * int(mult[fin].sum())
    verified = got == exp and cnt_l == cnt_h == exp_count and cs_l == cs_h and \
        np.array_equal(d_hv.cpu().numpy(), np.tile(want["verdicts"], reps)[:R]) and \
        np.array_equal(d_lv.cpu().numpy() == 0, np.tile(fin, reps)[:R])

    # CPU baseline: the C++ CPU engine's leader prep_init -> helper prep + aggregate -> leader finish +
    # aggregate (cpu_baseline/jc_cpu_engine.cpp, byte-checked against the oracle) at 1 thread and at the
    # host's thread budget; the literal C oracle (leader prep_init + helper prep) per core beside it
    from bench import cpu_threads
    from cpu_baseline import cpu_engine as CE

    cpu = cpu_threads()

    def cpu_ping_pong(nth, m):
        idx = np.arange(m) % K
        t = time.perf_counter()
        ld = CE.leader_prep_init(5, a.bits, a.length, 0, vk, nonces[idx], ps[idx], lis[idx], vdaf.prep_share_len,
                                 nthreads=nth)
        hp = CE.helper_prep_aggregate(5, a.bits, a.length, 0, vk, nonces[idx], ps[idx], his[idx], ld["prep_shares"],
                                      nthreads=nth)
        fn = CE.leader_finish_aggregate(5, a.bits, a.length, 0, nonces[idx], lis[idx], ld["seeds"], ld["verdicts"],
                                        hp["prep_msgs"], hp["verdicts"], nthreads=nth)
        dt_ = time.perf_counter() - t
        assert np.array_equal(hp["verdicts"], want["verdicts"][idx]) and np.array_equal(fn["verdicts"] == 0, fin[idx])
        return m / dt_, dt_

    r1, d1 = cpu_ping_pong(1, min(K, 8))
    mN = max(cpu["threads"], int(a.cpu_seconds * r1 * cpu["threads"] * 0.8))
    rN, dN = cpu_ping_pong(cpu["threads"], mN)
    m = min(K, 2)
    t = time.perf_counter()
    for i in range(m):
        orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())
    th = time.perf_counter()
    orc.helper_prep_batch(vk, nonces[:m], ps[:m], his[:m], lps[:m], nthreads=1)
    per_l, per_h = (th - t) / m, (time.perf_counter() - th) / m

    def per_launch(kt, stage):
        return round(kt[stage]["ms"] / max(1, kt[stage]["launches"]), 3)

    print(json.dumps({
        "metric": "leader+helper ping-pong reports/sec (prep_init+prep_next+aggregate, both roles), "
                  f"Prio3FixedPointBoundedL2VecSum {a.bits}-bit length={a.length} (configs[4])",
        "value": round(R * a.steps / dt, 1), "unit": "reports/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
        "helper_reports_per_s": round(R * a.steps / role_s["helper"], 1),
        "role_ms_per_step": {k: round(v / a.steps * 1e3, 3) for k, v in role_s.items()},
        "config": {"workload": f"FixedPointBoundedL2VecSum bitsize={a.bits} length={a.length}", "reports": R,
                   "pool": K, "launches_per_step_helper": kh["xof"]["launches"] // a.steps},
        "kernels": {"helper": {s: per_launch(kh, s) for s in ("xof", "flp", "accumulate", "slow")},
                    "leader": {s: per_launch(kl, s) for s in ("xof", "flp", "accumulate")}},
        "verified": bool(verified),
        "cpu_baseline": {"value": round(rN, 2), "unit": "reports/s", "cores": cpu["threads"], "kind": "port",
                         "engine": "cpu_baseline/jc_cpu_engine.cpp (leader init + helper prep/aggregate + leader "
                                   "finish/aggregate, both roles)", "value_1_thread": round(r1, 2), **cpu,
                         "oracle_port_reports_per_s_1_core": round(1.0 / (per_l + per_h), 3),
                         "sample": f"{mN} reports at {cpu['threads']} threads ({dN:.1f} s), {min(K, 8)} at 1 thread "
                                   f"({d1:.1f} s); C oracle {m} reports ({per_l * 1e3:.0f} + {per_h * 1e3:.0f} ms "
                                   "per report)"},
        "data": f"synthetic: {K} distinct C-oracle client reports (1 in 6 with a false norm claim) tiled to {R}",
    }), flush=True)


if __name__ == "__main__":
    main()
