#!/usr/bin/env python3
"""BASELINE configs[4]: Prio3FixedPointBoundedL2VecSum 16-bit length=10000, leader+helper ping-pong
prep with joint randomness, on one MI355X.

One ping-pong step = one aggregation job of R reports taken through both roles with every input
resident in HBM (aggregation_job_driver.rs:259-436 + aggregator.rs:1712-2161, minus HTTP and the
datastore):
  leader  jx_leader_prep_init_device   (leader_initialized: prepare_init agg_id 0, explicit shares)
  helper  jx_helper_prep_aggregate_device (helper_initialized + evaluate + accumulate)
  leader  jx_leader_prep_finish_device (leader_continued on the helper's Finish; helper rejects fail)
  leader  jx_accumulate_device
The two engines (one per role) share the GPU here; in a deployment they are two aggregators on two
GPUs. So the tool also measures each role ALONE at its own full-device launch size (--role-reports):
  helper  prep + aggregate of R_h reports, one engine owning the GPU (its staging, 2.8 MB/report,
          sized to the launch instead of the shared 1/3-of-HBM budget);
  leader  prep_init + finish + aggregate of R_l reports (the leader reads its explicit 2.6 MB input
          share in place: HBM holds R_l input shares and ~0.2 MB/report of staging).
Inputs: a pool of K distinct client reports (C-oracle shard; 1 in 6 claims a false norm and must be
rejected) tiled on the device. Verified: aggregates add up to multiplicity x the sum of the accepted
entries' encodings, every verdict matches the oracle. The C++ CPU engine's two roles (the baseline
proper, kind "port") and the literal C oracle are timed on the host beside it.

    python tools/bench_fixedpoint.py [--bits 16 --length 10000 --reports 32768 --role-reports 65536]
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


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_pool(bits, length, K, vk, threads):
    """K distinct C-oracle client reports (shard + the leader's prepare_init) and the oracle's helper
    results; 1 in 6 measurements claims a false norm (tests/golden/make_golden.py)."""
    from oracle import oracle as O  # input generation and the checker only
    from tests.golden.make_golden import fixedpoint_measurements

    orc = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, length, 0)
    rng = np.random.default_rng(0x5EED)
    meas = fixedpoint_measurements(bits, length, rng, K)
    nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
    shards = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(K)]
    ps, lis, his = (np.frombuffer(b"".join(s[k] for s in shards), np.uint8).reshape(K, -1) for k in range(3))
    lps = np.stack([np.frombuffer(orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())[1],
                                  np.uint8) for i in range(K)])
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads)
    return orc, meas, nonces, ps, lis, his, lps, want


def run(bits=16, length=10000, reports=40960, role_reports=65536, pool=48, steps=3, warmup=1, cpu_seconds=10.0,
        skip=(), helper_staging_gb=-1, pad_lis=True, lanes_cap=None, helper_k1=None):
    """The configs[4] legs (ping-pong one job at a time, two jobs in flight, each role alone, CPU
    baseline); returns one JSON-able dict. Every leg is verified against the oracle."""
    import torch

    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3

    skip = set(skip)
    threads = min(16, os.cpu_count() or 1)
    vdaf = Prio3.fixedpoint_boundedl2_vec_sum(bits, length)
    vk = bytes(range(16))
    K = pool
    t0 = time.perf_counter()
    orc, meas, nonces, ps, lis, his, lps, want = make_pool(bits, length, K, vk, threads)
    pool_s = time.perf_counter() - t0
    fin = want["verdicts"] == 0
    enc = meas.astype(object) ^ (1 << (bits - 1))
    log(f"pool of {K} generated in {pool_s:.1f}s; oracle verdicts {want['verdicts'].tolist()}")
    dev = torch.device("cuda", 0)
    total = steps + warmup

    def tile(x, R):
        x = np.ascontiguousarray(x)
        x2 = x.reshape(K, -1)
        reps = -(-R // K)
        return torch.from_numpy(x2).to(dev).repeat(reps, 1)[:R].contiguous()

    # the leader's input-share rows padded to a multiple of 128 bytes (jx_leader_prep_init_device_ex): the
    # in-place FLP ring then reads whole cache lines (the leader assembles these rows after HPKE open, so the
    # padding is free at that copy)
    lis_stride = -(-lis.shape[1] // 128) * 128 if pad_lis else 0

    def tile_lis(R):
        if not lis_stride:
            return tile(lis, R)
        rows = np.zeros((K, lis_stride), np.uint8)
        rows[:, :lis.shape[1]] = lis
        return tile(rows, R)

    def tiled(x, R):  # host copy of tile(x, R): report g is pool report g % K
        return np.asarray(x)[np.arange(R) % K]

    def expected(R, jobs):
        mult = np.bincount(np.arange(R) % K, minlength=K)
        return ([int((enc[fin, j] * mult[fin]).sum()) * jobs % P128 for j in range(length)],
                jobs * int(mult[fin].sum()))

    def add_shares(*aggs):
        return [sum(int.from_bytes(g[16 * j:16 * j + 16], "little") for g in aggs) % P128 for j in range(length)]

    def per_launch(kt, stage):
        return round(kt[stage]["ms"] / max(1, kt[stage]["launches"]), 3)

    def msgs_ok(d_msgs, R):  # the helper's Finish{prep_msg} of every finished report == the oracle's
        f = tiled(fin, R)
        return bool(np.array_equal(d_msgs.cpu().numpy()[f], tiled(want["prep_msgs"], R)[f]))

    if helper_staging_gb < 0:  # the helper stages its measurement share (16 B per element) plus ~10 %
        helper_staging_gb = -(-int(reports * vdaf.meas_len * 16 * 1.15) // (1 << 30)) + 2

    def helper_engine():
        h = HelperEngine(vdaf, vk)
        if helper_staging_gb:  # one launch per job (staging comes from the device arena per launch)
            h.debug(5, reports)
        if lanes_cap is not None:  # lane-split K1 workgroups per CU (jx_engine_debug option 6)
            h.debug(6, lanes_cap)
        if helper_k1 is not None:  # helper K1 kernel (option 3)
            h.debug(3, helper_k1)
        return h

    def timed_steps(step, engines):
        for _ in range(warmup):
            step(False)
        for e in engines:
            e.timing(True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            step(True)
        torch.cuda.synchronize()
        return time.perf_counter() - t

    out = {
        "metric": "leader+helper ping-pong reports/sec (prep_init+prep_next+aggregate, both roles), "
                  f"Prio3FixedPointBoundedL2VecSum {bits}-bit length={length} (configs[4])",
        "unit": "reports/s", "n_gpus": 1, "steps": steps, "warmup": warmup, "higher_is_better": True,
        "data": f"synthetic: {K} distinct C-oracle client reports (1 in 6 with a false norm claim) tiled on device",
        "pool_seconds": round(pool_s, 1),
        "leader_input_row_stride": lis_stride or int(lis.shape[1]),
    }
    verified = True

    # ---------------------------------------------------------------- ping-pong, both roles on one GPU
    if "pingpong" not in skip:
        R = reports
        d_n, d_ps, d_lis, d_his = tile(nonces, R), tile(ps, R), tile_lis(R), tile(his, R)
        d_lps = torch.empty((R, vdaf.prep_share_len), dtype=torch.uint8, device=dev)
        d_msgs = torch.empty((R, 16), dtype=torch.uint8, device=dev)
        d_hv = torch.empty(R, dtype=torch.uint8, device=dev)
        d_lv = torch.empty(R, dtype=torch.uint8, device=dev)
        leader, helper = HelperEngine(vdaf, vk), helper_engine()
        role_s = {"leader_init": 0.0, "helper": 0.0, "leader_finish_acc": 0.0}

        def step(timed):
            t = time.perf_counter()
            bid = leader.leader_init_device(R, d_n.data_ptr(), d_ps.data_ptr(), d_lis.data_ptr(), d_lps.data_ptr(),
                                            lis_stride=lis_stride)
            leader.sync()
            t1 = time.perf_counter()
            helper.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), R,
                                             0, d_msgs.data_ptr(), d_hv.data_ptr())
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

        dt = timed_steps(step, (leader, helper))
        kl, kh = leader.timing_read(), helper.timing_read()
        agg_l, cnt_l, cs_l = leader.aggregate_share(0)
        agg_h, cnt_h, cs_h = helper.aggregate_share(0)
        exp, exp_count = expected(R, total)
        ok = add_shares(agg_l, agg_h) == exp and cnt_l == cnt_h == exp_count and cs_l == cs_h and \
            np.array_equal(d_hv.cpu().numpy(), tiled(want["verdicts"], R)) and \
            np.array_equal(d_lv.cpu().numpy() == 0, tiled(fin, R)) and msgs_ok(d_msgs, R)
        verified &= bool(ok)
        leader.close()
        helper.close()
        del d_n, d_ps, d_lis, d_his, d_lps, d_msgs, d_hv, d_lv
        torch.cuda.empty_cache()
        out.update({
            "value": round(R * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3),
            "helper_reports_per_s_in_pingpong": round(R * steps / role_s["helper"], 1),
            "role_ms_per_step": {k: round(v / steps * 1e3, 3) for k, v in role_s.items()},
            "config": {"workload": f"FixedPointBoundedL2VecSum bitsize={bits} length={length}", "reports": R,
                       "pool": K, "launches_per_step_helper": kh["xof"]["launches"] // steps},
            "kernels": {"helper": {s: per_launch(kh, s) for s in ("xof", "flp", "accumulate", "slow")},
                        "leader": {s: per_launch(kl, s) for s in ("xof", "flp", "accumulate")}},
            "pingpong_verified": bool(ok),
        })
        log(f"ping-pong: {out['value']} reports/s, verified {ok}")

    # ---------------------------------------------------------------- ping-pong, two jobs in flight
    # Janus steps several aggregation jobs at once (max_concurrent_job_workers, job_driver.rs:116-138), and
    # the two aggregators are independent processes: while the helper prepares job i-1 (helper engine,
    # its own stream), the leader initializes job i (leader engine, its own stream); then the leader
    # finishes job i-1. Each role alone leaves most SIMDs idle at these launch sizes (one report's sponge
    # chain is serial), so the two roles' kernels run side by side. The engines are ordered by hand
    # (stream=False): ordering both through torch's stream would serialize them. The inputs are resident
    # before the first step; job i-1's leader prep shares are complete (leader.sync) before its helper step.
    if "pipelined" not in skip:
        R = reports
        d_n, d_ps, d_lis, d_his = tile(nonces, R), tile(ps, R), tile_lis(R), tile(his, R)
        d_lps = [torch.empty((R, vdaf.prep_share_len), dtype=torch.uint8, device=dev) for _ in range(2)]
        d_msgs = torch.empty((R, 16), dtype=torch.uint8, device=dev)
        d_hv = torch.empty(R, dtype=torch.uint8, device=dev)
        d_lv = torch.empty(R, dtype=torch.uint8, device=dev)
        leader, helper = HelperEngine(vdaf, vk), helper_engine()
        torch.cuda.synchronize()
        state = {"i": 0, "prev": None, "done": 0}
        nf = False

        def pstep(timed):
            i = state["i"]
            bid = leader.leader_init_device(R, d_n.data_ptr(), d_ps.data_ptr(), d_lis.data_ptr(),
                                            d_lps[i % 2].data_ptr(), stream=nf, lis_stride=lis_stride)
            if state["prev"] is not None:
                helper.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(),
                                                 d_lps[(i - 1) % 2].data_ptr(), R, 0, d_msgs.data_ptr(),
                                                 d_hv.data_ptr(), stream=nf)
            helper.sync()
            if state["prev"] is not None:
                leader.leader_finish_device(state["prev"], R, d_msgs.data_ptr(), d_hv.data_ptr(), d_lv.data_ptr(),
                                            stream=nf)
                leader.accumulate_device(state["prev"], R, stream=nf)
                state["done"] += 1
            leader.sync()
            state["prev"] = bid
            state["i"] = i + 1

        pstep(False)  # fill the pipeline: job 0's leader init
        dt = timed_steps(pstep, (leader, helper))
        # drain: the last job's helper step and leader finish (untimed)
        helper.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(),
                                         d_lps[(state["i"] - 1) % 2].data_ptr(), R, 0, d_msgs.data_ptr(),
                                         d_hv.data_ptr(), stream=nf)
        helper.sync()
        leader.leader_finish_device(state["prev"], R, d_msgs.data_ptr(), d_hv.data_ptr(), d_lv.data_ptr(), stream=nf)
        leader.accumulate_device(state["prev"], R, stream=nf)
        leader.sync()
        jobs = state["done"] + 1
        kl, kh = leader.timing_read(), helper.timing_read()
        agg_l, cnt_l, cs_l = leader.aggregate_share(0)
        agg_h, cnt_h, cs_h = helper.aggregate_share(0)
        exp, exp_count = expected(R, jobs)
        ok = add_shares(agg_l, agg_h) == exp and cnt_l == cnt_h == exp_count and cs_l == cs_h and \
            np.array_equal(d_hv.cpu().numpy(), tiled(want["verdicts"], R)) and \
            np.array_equal(d_lv.cpu().numpy() == 0, tiled(fin, R)) and msgs_ok(d_msgs, R)
        verified &= bool(ok)
        leader.close()
        helper.close()
        del d_n, d_ps, d_lis, d_his, d_lps, d_msgs, d_hv, d_lv
        torch.cuda.empty_cache()
        out["pipelined"] = {"reports_per_s": round(R * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3),
                            "reports_per_job": R, "jobs_in_flight": 2, "verified": bool(ok),
                            "kernels": {"helper": {s: per_launch(kh, s) for s in ("xof", "flp", "accumulate")},
                                        "leader": {s: per_launch(kl, s) for s in ("xof", "flp", "accumulate")}}}
        log(f"pipelined ping-pong: {out['pipelined']}")

    # ---------------------------------------------------------------- each role alone, full-device launch
    roles = {}
    R = role_reports
    if "helper" not in skip:
        d_n, d_ps, d_his, d_lps = tile(nonces, R), tile(ps, R), tile(his, R), tile(lps, R)
        d_msgs = torch.empty((R, 16), dtype=torch.uint8, device=dev)
        d_hv = torch.empty(R, dtype=torch.uint8, device=dev)
        helper = HelperEngine(vdaf, vk)
        helper.debug(5, R)  # this engine owns the GPU: the whole step in one launch

        def hstep(timed):
            helper.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), R,
                                             0, d_msgs.data_ptr(), d_hv.data_ptr())
            helper.sync()

        dt = timed_steps(hstep, (helper,))
        kh = helper.timing_read()
        _, cnt_h, _ = helper.aggregate_share(0)
        _, exp_count = expected(R, total)
        ok = cnt_h == exp_count and np.array_equal(d_hv.cpu().numpy(), tiled(want["verdicts"], R)) and \
            msgs_ok(d_msgs, R)
        verified &= bool(ok)
        roles["helper"] = {"reports_per_s": round(R * steps / dt, 1), "reports": R,
                           "ms_per_step": round(dt / steps * 1e3, 3),
                           "launches_per_step": kh["xof"]["launches"] // steps,
                           "kernels_ms_per_launch": {s: per_launch(kh, s) for s in ("xof", "flp", "accumulate", "slow")},
                           "verified": bool(ok)}
        helper.close()
        del d_n, d_ps, d_his, d_lps, d_msgs, d_hv
        torch.cuda.empty_cache()
        log(f"helper alone: {roles['helper']}")
    if "leader" not in skip:
        d_n, d_ps, d_lis = tile(nonces, R), tile(ps, R), tile_lis(R)
        d_lps = torch.empty((R, vdaf.prep_share_len), dtype=torch.uint8, device=dev)
        d_msgs = tile(want["prep_msgs"], R)  # the helper's Finish messages (rejected reports: peer verdicts)
        d_hv = tile(want["verdicts"], R).reshape(R).contiguous()
        d_lv = torch.empty(R, dtype=torch.uint8, device=dev)
        leader = HelperEngine(vdaf, vk)

        def lstep(timed):
            bid = leader.leader_init_device(R, d_n.data_ptr(), d_ps.data_ptr(), d_lis.data_ptr(), d_lps.data_ptr(),
                                            lis_stride=lis_stride)
            leader.leader_finish_device(bid, R, d_msgs.data_ptr(), d_hv.data_ptr(), d_lv.data_ptr())
            leader.accumulate_device(bid, R)
            leader.sync()

        dt = timed_steps(lstep, (leader,))
        kl = leader.timing_read()
        _, cnt_l, _ = leader.aggregate_share(0)
        _, exp_count = expected(R, total)
        ok = cnt_l == exp_count and np.array_equal(d_lv.cpu().numpy() == 0, tiled(fin, R)) and \
            np.array_equal(d_lps[:K].cpu().numpy(), lps)  # prep shares == the oracle's prepare_init
        verified &= bool(ok)
        roles["leader"] = {"reports_per_s": round(R * steps / dt, 1), "reports": R,
                           "ms_per_step": round(dt / steps * 1e3, 3),
                           "kernels_ms_per_launch": {s: per_launch(kl, s) for s in ("xof", "flp", "accumulate")},
                           "verified": bool(ok)}
        leader.close()
        del d_n, d_ps, d_lis, d_lps, d_msgs, d_hv, d_lv
        torch.cuda.empty_cache()
        log(f"leader alone: {roles['leader']}")
    if roles:
        out["roles_alone"] = roles
        if len(roles) == 2:
            h, l_ = roles["helper"]["reports_per_s"], roles["leader"]["reports_per_s"]
            out["pingpong_from_roles_one_gpu"] = round(1.0 / (1.0 / h + 1.0 / l_), 1)
            out["pingpong_two_gpus"] = round(min(h, l_), 1)
    out["verified"] = bool(verified)

    # ---------------------------------------------------------------- CPU baseline
    if "cpu" not in skip:
        out["cpu_baseline"] = cpu_baseline(bits, length, vk, K, nonces, ps, lis, his, lps, want, orc, cpu_seconds,
                                           vdaf.prep_share_len)
    return out


def cpu_baseline(bits, length, vk, K, nonces, ps, lis, his, lps, want, orc, cpu_seconds, lps_len):
    """The C++ CPU engine's leader prep_init -> helper prep + aggregate -> leader finish + aggregate
    (cpu_baseline/jc_cpu_engine.cpp, byte-checked against the oracle) at 1 thread and at the host's
    thread budget; the literal C oracle (leader prep_init + helper prep) per core beside it."""
    from bench import cpu_threads
    from cpu_baseline import cpu_engine as CE

    cpu = cpu_threads()
    fin = want["verdicts"] == 0

    def cpu_ping_pong(nth, m):
        idx = np.arange(m) % K
        t = time.perf_counter()
        ld = CE.leader_prep_init(5, bits, length, 0, vk, nonces[idx], ps[idx], lis[idx], lps_len, nthreads=nth)
        hp = CE.helper_prep_aggregate(5, bits, length, 0, vk, nonces[idx], ps[idx], his[idx], ld["prep_shares"],
                                      nthreads=nth)
        fn = CE.leader_finish_aggregate(5, bits, length, 0, nonces[idx], lis[idx], ld["seeds"], ld["verdicts"],
                                        hp["prep_msgs"], hp["verdicts"], nthreads=nth)
        dt_ = time.perf_counter() - t
        assert np.array_equal(hp["verdicts"], want["verdicts"][idx]) and np.array_equal(fn["verdicts"] == 0, fin[idx])
        return m / dt_, dt_

    r1, d1 = cpu_ping_pong(1, min(K, 8))
    mN = max(cpu["threads"], int(cpu_seconds * r1 * cpu["threads"] * 0.8))
    rN, dN = cpu_ping_pong(cpu["threads"], mN)
    m = min(K, 2)
    t = time.perf_counter()
    for i in range(m):
        orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())
    th = time.perf_counter()
    orc.helper_prep_batch(vk, nonces[:m], ps[:m], his[:m], lps[:m], nthreads=1)
    per_l, per_h = (th - t) / m, (time.perf_counter() - th) / m
    return {
        "value": round(rN, 2), "unit": "reports/s", "cores": cpu["threads"], "kind": "port",
        "engine": "cpu_baseline/jc_cpu_engine.cpp (leader init + helper prep/aggregate + leader finish/aggregate, "
                  "both roles)", "value_1_thread": round(r1, 2), **cpu,
        "oracle_port_reports_per_s_1_core": round(1.0 / (per_l + per_h), 3),
        "sample": f"{mN} reports at {cpu['threads']} threads ({dN:.1f} s), {min(K, 8)} at 1 thread ({d1:.1f} s); "
                  f"C oracle {m} reports ({per_l * 1e3:.0f} + {per_h * 1e3:.0f} ms per report)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=16)
    ap.add_argument("--length", type=int, default=10000)
    ap.add_argument("--reports", type=int, default=40960, help="reports per ping-pong job (both roles on the GPU)")
    ap.add_argument("--role-reports", type=int, default=65536, help="reports per single-role step")
    ap.add_argument("--pool", type=int, default=48)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--skip", default="", help="comma list of legs to skip: pingpong,pipelined,helper,leader,cpu")
    ap.add_argument("--helper-staging-gb", type=int, default=-1,
                    help="staging budget of the helper engine in the two-role legs (default: sized so one launch "
                         "holds --reports; 0: the engine's own, 1/3 of HBM)")
    ap.add_argument("--packed-lis", action="store_true",
                    help="leader input shares in packed rows (no 128-byte padding of the row stride)")
    ap.add_argument("--lanes-cap", type=int, default=None, help="lane-split K1 workgroups per CU (debug option 6)")
    ap.add_argument("--helper-k1", type=int, default=None, help="helper K1 kernel (debug option 3: 3, 5, 6)")
    a = ap.parse_args()
    out = run(a.bits, a.length, a.reports, a.role_reports, a.pool, a.steps, a.warmup, a.cpu_seconds,
              set(filter(None, a.skip.split(","))), a.helper_staging_gb, pad_lis=not a.packed_lis,
              lanes_cap=a.lanes_cap, helper_k1=a.helper_k1)
    out["variant"] = {"packed_lis": a.packed_lis, "lanes_cap": a.lanes_cap, "helper_k1": a.helper_k1}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
