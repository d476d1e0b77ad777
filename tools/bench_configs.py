#!/usr/bin/env python3
"""Helper prep + aggregate throughput for the other BASELINE.json configs on one MI355X.

bench.py measures the headline config (Prio3SumVec 8x1000/88). This tool runs the same
measurement for configs[0..2] — Prio3Count, Prio3Sum{bits=32}, Prio3Histogram{256, 16} — at
the report counts BASELINE.json names (Count: 100k, the reference's CPU case, also run at 1M
here; Sum32 / Histogram: 1M reports). Per config: a pool of K distinct client reports (C-oracle
client + leader prep_init, 1 % tampered) tiled on the device, inputs resident in HBM; `steps`
fused jx_helper_prep_aggregate_device calls are timed between torch.cuda.synchronize(); the
aggregate share and count are verified against multiplicity x the oracle's output shares, and
every verdict against the oracle. The C++ CPU engine (cpu_baseline/jc_cpu_engine.cpp) is timed
beside it on the host's cores at 1 thread and at the affinity/cgroup thread budget (kind "port"),
with the literal C oracle port as a secondary figure. One JSON line per config.

    python tools/bench_configs.py [--only count,sum32,hist] [--cpu-seconds 3]
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
P128 = 2**128 - 28 * 2**64 + 1


def run(name, vdaf, meas_fn, R, K, steps, warmup, cpu_seconds, threads, cpu):
    import torch

    from janus_amd.engine import HelperEngine
    from oracle import oracle as O  # input generation and the checker only

    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    vk = bytes(range(16))
    rng = np.random.default_rng(0x5EED)
    meas = meas_fn(rng, K)
    nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=threads)
    for i in range(0, K, 100):  # 1 % invalid: one flipped bit in the leader prep share
        j = int(rng.integers(0, lps.shape[1]))
        lps[i, j] ^= 1 << int(rng.integers(0, 8))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads, want_out_shares=True)

    reps = -(-R // K)
    dev = torch.device("cuda", 0)

    def tile(x):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev).repeat(reps, 1)[:R].contiguous()

    d_n, d_his, d_lps = tile(nonces), tile(his), tile(lps)
    d_ps = tile(ps) if ps.shape[1] else None
    d_v = torch.empty(R, dtype=torch.uint8, device=dev)
    d_m = torch.empty((R, 16), dtype=torch.uint8, device=dev)
    with HelperEngine(vdaf, vk) as eng:
        # the inputs are resident and complete before the first step (torch.cuda.synchronize below) and every
        # step ends with eng.sync(), so the steps order themselves (stream=False): Count's 100k-report call
        # is ~0.13 ms, and bracketing it with stream waits would add ~20 us per call
        torch.cuda.synchronize()

        def step():
            eng.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr() if d_ps is not None else 0,
                                          d_his.data_ptr(), d_lps.data_ptr(), R, 0, d_m.data_ptr(), d_v.data_ptr(),
                                          stream=False)
            eng.sync()

        for _ in range(warmup):
            step()
        eng.timing(True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        kt = eng.timing_read()
        agg, count, _ = eng.aggregate_share(0)

    total = steps + warmup
    fb, OL = vdaf.field_bytes, vdaf.output_len
    p = P64 if fb == 8 else P128
    mult = np.bincount(np.arange(R) % K, minlength=K)
    fin = want["verdicts"] == 0
    outs = want["out_shares"].reshape(K, OL, fb)
    acc = [0] * OL
    for i in np.nonzero(fin)[0]:
        m = int(mult[i]) * total
        for j in range(OL):
            acc[j] += m * int.from_bytes(outs[i, j].tobytes(), "little")
    exp = b"".join((x % p).to_bytes(fb, "little") for x in acc)
    got_v = d_v.cpu().numpy()
    verdicts_ok = bool(np.array_equal(got_v, np.tile(want["verdicts"], reps)[:R]))
    msgs_ok = True
    if vdaf.prep_msg_len:  # every finished report's Finish{prep_msg} == the oracle's
        f = got_v == 0
        msgs_ok = bool(np.array_equal(d_m.cpu().numpy()[f], np.tile(want["prep_msgs"], (reps, 1))[:R][f]))
    agg_ok = agg == exp and count == total * int(mult[fin].sum())
    verified = agg_ok and verdicts_ok and msgs_ok

    # CPU baseline: the C++ CPU engine (cpu_baseline/jc_cpu_engine.cpp, byte-checked against the fixtures)
    # at 1 thread and at the host's thread budget on ~cpu_seconds of work each; the literal C oracle
    # port beside it as a secondary figure
    from cpu_baseline import cpu_engine as CE

    def engine_rate(nth, budget):
        m = min(K, max(64, 32 * nth))
        t = time.perf_counter()
        CE.helper_prep_aggregate(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length, vk, nonces[:m], ps[:m],
                                 his[:m], lps[:m], nthreads=nth)
        r0 = m / (time.perf_counter() - t)
        nn = max(m, int(budget * r0))
        idx = np.arange(nn) % K
        t = time.perf_counter()
        got = CE.helper_prep_aggregate(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length, vk, nonces[idx],
                                       ps[idx], his[idx], lps[idx], nthreads=nth)
        dt_ = time.perf_counter() - t
        assert np.array_equal(got["verdicts"], want["verdicts"][idx])
        return nn / dt_, nn, dt_

    r1, n1, d1 = engine_rate(1, cpu_seconds * 0.4)
    rN, nN, dN = engine_rate(cpu["threads"], cpu_seconds * 0.6)
    m = min(K, 512)
    t = time.perf_counter()
    orc.helper_prep_batch(vk, nonces[:m], ps[:m], his[:m], lps[:m], nthreads=cpu["threads"])
    r_oracle = m / (time.perf_counter() - t)

    def per_launch(stage):
        return round(kt[stage]["ms"] / max(1, kt[stage]["launches"]), 3)

    return {
        "metric": f"helper reports/sec (prep_init+aggregate), {name}",
        "value": round(R * steps / dt, 1), "unit": "reports/s", "n_gpus": 1, "steps": steps, "warmup": warmup,
        "ms_per_step": round(dt / steps * 1e3, 3), "higher_is_better": True,
        "config": {"workload": name, "reports": R, "pool": K},
        "kernels": {"k1_ms_per_launch": per_launch("xof"), "k3_ms_per_launch": per_launch("flp"),
                    "k4_ms_per_launch": per_launch("accumulate"), "launches_per_step": kt["xof"]["launches"] // steps,
                    "reports_per_launch": R * steps // max(1, kt["xof"]["launches"])},
        "verified": verified,
        "verification": {"aggregate_and_count": agg_ok, "verdicts": verdicts_ok, "prep_msgs_of_finished_reports": msgs_ok},
        "cpu_baseline": {"value": round(rN, 1), "unit": "reports/s", "cores": cpu["threads"], "kind": "port",
                         "engine": "cpu_baseline/jc_cpu_engine.cpp", "value_1_thread": round(r1, 1),
                         "oracle_port_reports_per_s": round(r_oracle, 1), **cpu,
                         "sample": f"{nN} reports at {cpu['threads']} threads ({dN:.1f} s) and {n1} at 1 thread "
                                   f"({d1:.1f} s), pool of {K} tiled, verdicts checked; C oracle on {m} reports"},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="count100k,count,sum32,hist")
    ap.add_argument("--pool", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    a = ap.parse_args()
    from janus_amd.vdaf import Prio3

    from bench import cpu_threads

    cpu = cpu_threads()
    threads = min(16, cpu["threads"])  # pool generation
    cfgs = {
        "count100k": ("Prio3Count (configs[0]: 100k reports)", Prio3.count(),
                      lambda rng, K: rng.integers(0, 2, size=(K, 1), dtype=np.uint64), 100_000),
        "count": ("Prio3Count", Prio3.count(),
                  lambda rng, K: rng.integers(0, 2, size=(K, 1), dtype=np.uint64), 1_000_000),
        "sum32": ("Prio3Sum bits=32 (configs[1])", Prio3.sum(32),
                  lambda rng, K: rng.integers(0, 1 << 32, size=(K, 1), dtype=np.uint64), 1_000_000),
        "hist": ("Prio3Histogram length=256 chunk_length=16 (configs[2])", Prio3.histogram(256, 16),
                 lambda rng, K: rng.integers(0, 256, size=(K, 1), dtype=np.uint64), 1_000_000),
    }
    for key in a.only.split(","):
        name, vdaf, fn, R = cfgs[key]
        print(json.dumps(run(name, vdaf, fn, R, a.pool, a.steps, a.warmup, a.cpu_seconds, threads, cpu)), flush=True)


if __name__ == "__main__":
    main()
