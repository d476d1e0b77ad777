#!/usr/bin/env python3
"""Helper throughput and latency at Janus's aggregation-job granularity on one MI355X.

Janus's helper handles one AggregationJobInitializeReq per HTTP request
(aggregator/src/aggregator.rs:1712-2013, per-report loop at :1763) and aggregation jobs hold
10-100 reports (docs/samples/basic_config/aggregation_job_creator.yaml:23-26); many requests are
in flight at once (tokio workers; the leader steps max_concurrent_job_workers jobs,
aggregator/src/binary_utils/job_driver.rs:116). This tool measures exactly that shape: T host
threads share ONE engine, every thread loops over jobs of n reports through the host-buffer ABI
(jx_helper_prep_batch -> jx_accumulate, the job's batch handle in between), and we report
reports/s over the wall time and the p50/p99 latency of the prepare call and of the whole job.

Inputs: a pool of K distinct C-oracle client reports (1 % tampered), tiled into jobs; every job's
verdicts and Finish{prep_msg}s are compared with the oracle's, and the engine's final aggregate
and count with the multiplicity-weighted oracle aggregate (verification, not timed).

    python tools/bench_jobs.py [--vdafs sumvec,count] [--sizes 10,100,1000,10000] [--threads 1,8,64]
                               [--seconds 2] [--mode direct|coalesce]
One JSON line per (vdaf, n, threads).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

P64 = 2**64 - 2**32 + 1
P128 = 2**128 - 28 * 2**64 + 1


def make_pool(vdaf, vk, K, threads):
    from oracle import oracle as O  # input generation and the checker only

    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    rng = np.random.default_rng(0x10B5)
    hi = 1 << vdaf.bits if vdaf.algo_id in (1, 2) else 2
    meas = rng.integers(0, hi, size=(K, max(1, vdaf.length)), dtype=np.uint64)
    if vdaf.algo_id == 0:
        meas = meas[:, :1]
    nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=threads)
    for i in range(0, K, 100):  # 1 % invalid: one flipped bit in the leader prep share
        j = int(rng.integers(0, lps.shape[1]))
        lps[i, j] ^= 1 << int(rng.integers(0, 8))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads, want_out_shares=True)
    return nonces, ps, his, lps, want


def make_enc_pool(vdaf, pool, seed=0x5EA1):
    """The pool's helper input shares sealed as DAP report shares (HPKE base mode, X25519 / HKDF-SHA256 /
    AES-128-GCM, the input-share application info and InputShareAad): every 50th ciphertext corrupted
    (HpkeDecryptError), every 97th report under an unknown HPKE config id (HpkeUnknownConfigId). Returns the
    pool with expected verdicts JX_OPEN_FAILURE (6) for those, and the encrypted-input extras."""
    import random

    from oracle import hpke_oracle as H  # input generation and the checker only

    nonces, ps, his, lps, want = pool
    K = nonces.shape[0]
    rnd = random.Random(seed)
    sk = rnd.randbytes(32)
    pk = H.x25519_base(sk)
    task_id = rnd.randbytes(32)
    info = H.dap_info()
    times = np.array([1_700_000_000 + i for i in range(K)], np.uint64)
    encs, cts, kidx = [], [], []
    status = np.zeros(K, np.uint8)
    for i in range(K):
        rid, pub = nonces[i].tobytes(), ps[i].tobytes()
        aad = task_id + rid + int(times[i]).to_bytes(8, "big") + len(pub).to_bytes(4, "big") + pub
        pt = (0).to_bytes(2, "big") + len(his[i]).to_bytes(4, "big") + his[i].tobytes()
        enc, ct = H.seal_base(pk, info, aad, pt, rnd.randbytes(32))
        k = (0, 0xFF)
        if i % 50 == 7:
            ct = ct[:5] + bytes([ct[5] ^ 0x10]) + ct[6:]
            status[i] = 1
        elif i % 97 == 11:
            k = (0xFF, 0xFF)
            status[i] = 7
        encs.append(enc)
        cts.append(ct)
        kidx.append(k)
    want = dict(want)
    want["verdicts"] = np.where(status != 0, 6, want["verdicts"]).astype(want["verdicts"].dtype)
    cto = np.zeros(K + 1, np.uint64)
    cto[1:] = np.cumsum([len(c) for c in cts])
    extra = {"sk": sk, "pk": pk, "task_id": task_id, "times": times,
             "encs": np.frombuffer(b"".join(encs), np.uint8), "cto": cto, "cts": b"".join(cts),
             "kidx": np.array(kidx, np.uint8), "status": status}
    return (nonces, ps, his, lps, want), extra


def make_leader_pool(vdaf, vk, K, seed=0x1EAD):
    """K leader jobs' inputs (C-oracle shards: nonce, public share, leader input share) and the oracle's
    leader prepare_init results (verdict, prep share)."""
    from oracle import oracle as O

    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    rng = np.random.default_rng(seed)
    hi = 1 << vdaf.bits if vdaf.algo_id in (1, 2) else 2
    meas = rng.integers(0, hi, size=(K, max(1, vdaf.length)), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
    ps, lis, verdicts, shares = [], [], np.zeros(K, np.uint8), []
    for i in range(K):
        a, b, _ = orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes())
        rc, share, _, _ = orc.prep_init(vk, 0, nonces[i].tobytes(), a, b)
        ps.append(a)
        lis.append(b)
        verdicts[i] = 1 if rc else 0
        shares.append(share if rc == 0 else bytes(orc.sizes.prep_share))
    return nonces, ps, lis, verdicts, shares


def weighted_aggregate(outs: np.ndarray, mult: np.ndarray, fb: int, p: int) -> bytes:
    """sum_i mult[i] * out_i mod p, by 32-bit limbs in int64 columns (mult < 2^20, K < 2^11)."""
    K, width = outs.shape
    ol = width // fb
    limbs = outs.reshape(K, ol, fb // 4, 4).astype(np.uint64)
    words = limbs[..., 0] | (limbs[..., 1] << 8) | (limbs[..., 2] << 16) | (limbs[..., 3] << 24)  # [K, ol, fb/4]
    sums = np.einsum("k,kew->ew", mult.astype(np.uint64), words)  # each < 2^63
    res = []
    for e in range(ol):
        v = sum(int(sums[e, w]) << (32 * w) for w in range(fb // 4)) % p
        res.append(v.to_bytes(fb, "little"))
    return b"".join(res)


def coalescer_phases(m0, m1):
    """Per-launch averages of the coalescer's phases over one case (jx_engine_memory deltas)."""
    d = {k: m1[k] - m0[k] for k in m1}
    la = d.get("coalesced_launches", 0)
    if not la:
        return None
    return {"launches": la, "jobs_per_launch": round(d["coalesced_jobs"] / la, 2),
            "reports_per_launch": round(d["coalesced_reports"] / la, 1),
            "gather_ms": round(d["coalesce_gather_us"] / la / 1e3, 3),
            "copy_ms": round(d["coalesce_copy_us"] / la / 1e3, 3),
            "enqueue_ms": round(d["coalesce_enqueue_us"] / la / 1e3, 3),
            "device_ms": round(d["coalesce_device_us"] / la / 1e3, 3),
            "arena_cross_stream_waits": d["arena_cross_stream_waits"], "arena_allocs": d["arena_allocs"],
            "window_us": m1["coalesce_window_us"]}


def run_case(eng, vdaf, pool, n, T, seconds, mode, max_jobs=None):
    nonces, ps, his, lps, want = pool
    K = nonces.shape[0]
    # per-thread job inputs: 4 distinct offsets per thread, contiguous copies made up front
    jobs = []
    for t in range(T):
        mine = []
        for j in range(4):
            off = ((t * 4 + j) * 7919 * n) % K
            idx = (off + np.arange(n)) % K
            mine.append((idx, np.ascontiguousarray(nonces[idx]), np.ascontiguousarray(ps[idx]),
                         np.ascontiguousarray(his[idx]), np.ascontiguousarray(lps[idx])))
        jobs.append(mine)
    mult = np.zeros(K, np.int64)
    lat_prep, lat_job = [], []
    errors = []
    bad = [0]
    lock = threading.Lock()
    barrier = threading.Barrier(T + 1)
    stop_at = [0.0]
    done_jobs = [0]
    t_end = []

    def worker(t):
        lp, lj, got = [], [], []
        k = 0
        barrier.wait()
        try:
            while time.perf_counter() < stop_at[0] and (max_jobs is None or k < max_jobs):
                _, nn, pp, hh, ll = jobs[t][k % 4]
                t0 = time.perf_counter()
                r = eng.helper_initialized_batch(nn, pp, hh, ll)
                t1 = time.perf_counter()
                eng.accumulate(n, batch_id=r.batch_id)
                t2 = time.perf_counter()
                lp.append(t1 - t0)
                lj.append(t2 - t0)
                got.append((k % 4, r.verdicts, r.prep_msgs))  # checked after the timed region
                k += 1
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            errors.append(repr(e))
        t_end.append(time.perf_counter())
        per_job = np.bincount([g[0] for g in got], minlength=4) if got else np.zeros(4, np.int64)
        local_mult = np.zeros(K, np.int64)
        nbad = 0
        for j in range(4):
            if per_job[j]:
                local_mult += np.bincount(jobs[t][j][0], minlength=K) * int(per_job[j])
        for j, v, m in got:
            idx = jobs[t][j][0]
            wv = want["verdicts"][idx]
            ok = np.array_equal(v, wv)
            if ok and vdaf.prep_msg_len:
                f = wv == 0
                ok = np.array_equal(m[f], want["prep_msgs"][idx][f])
            nbad += 0 if ok else 1
        with lock:
            bad[0] += nbad
            mult[:] += local_mult
            lat_prep.extend(lp)
            lat_job.extend(lj)
            done_jobs[0] += k

    eng.reset_aggregates()
    m0 = eng.memory()
    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    stop_at[0] = time.perf_counter() + seconds
    t_start = time.perf_counter()
    barrier.wait()
    for x in th:
        x.join()
    wall = max(t_end) - t_start  # the last job's end (the checks after it are not timed)
    m1 = eng.memory()
    agg, count, _ = eng.aggregate_share(0)
    fin = want["verdicts"] == 0
    m_fin = np.where(fin, mult, 0)
    p = P64 if vdaf.field_bytes == 8 else P128
    exp = weighted_aggregate(want["out_shares"].reshape(K, -1), m_fin, vdaf.field_bytes, p)
    agg_ok = agg == exp and count == int(m_fin.sum())
    reports = done_jobs[0] * n
    lp = np.array(lat_prep) * 1e3 if lat_prep else np.zeros(1)
    lj = np.array(lat_job) * 1e3 if lat_job else np.zeros(1)
    return {
        "vdaf": vdaf.name(), "mode": mode, "reports_per_job": n, "threads": T, "jobs": done_jobs[0],
        "reports": reports, "wall_s": round(wall, 3), "reports_per_s": round(reports / wall, 1),
        "prep_ms_p50": round(float(np.percentile(lp, 50)), 3), "prep_ms_p99": round(float(np.percentile(lp, 99)), 3),
        "job_ms_p50": round(float(np.percentile(lj, 50)), 3), "job_ms_p99": round(float(np.percentile(lj, 99)), 3),
        "coalescer": coalescer_phases(m0, m1),
        "verified": bool(agg_ok and bad[0] == 0 and not errors),
        "verification": {"aggregate_and_count": bool(agg_ok), "jobs_with_wrong_verdicts_or_msgs": bad[0],
                         "errors": errors[:3]},
    }


DRIVER = os.path.join(ROOT, "tools", "bin", "jobs_driver")


def build_driver() -> str:
    """tools/bin/jobs_driver: the native load generator (tools/jobs_driver.cpp) against the in-tree library."""
    import subprocess

    src = os.path.join(ROOT, "tools", "jobs_driver.cpp")
    lib = os.path.join(ROOT, "janus_amd", "lib", "libjanus_prio3.so")
    if os.path.exists(DRIVER) and os.path.getmtime(DRIVER) > max(os.path.getmtime(src), os.path.getmtime(lib)):
        return DRIVER
    os.makedirs(os.path.dirname(DRIVER), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", src, "-I" + os.path.join(ROOT, "include"),
                    "-L" + os.path.dirname(lib), "-ljanus_prio3", "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,$ORIGIN/../../janus_amd/lib", "-Wl,-rpath,/opt/rocm/lib", "-lpthread", "-o", DRIVER],
                   check=True)
    return DRIVER


def run_case_cpp(vdaf, vk, pool, n, T, seconds, mode, window_us, tmp, enc=None, leader=None, leader_threads=0):
    """One case through the native driver (no interpreter between the threads and the C ABI); the
    aggregate it read is checked here against the oracle. enc: the make_enc_pool extras (the jobs start from
    encrypted report shares); leader: (leader vk, make_leader_pool output) with leader_threads threads of
    leader prepare_init jobs beside the helper's."""
    import subprocess

    nonces, ps, his, lps, want = pool
    K = nonces.shape[0]
    pm = vdaf.prep_msg_len
    src = os.path.join(tmp, f"pool_{vdaf.algo_id}_{K}{'_enc' if enc else ''}.bin")
    if not os.path.exists(src):
        with open(src + ".tmp", "wb") as f:
            f.write(np.array([K, ps.shape[1], his.shape[1], lps.shape[1], pm, 1 if enc else 0,
                              len(enc["cts"]) if enc else 0, 0], np.uint64).tobytes())
            for a in (nonces, ps, his, lps, want["verdicts"].astype(np.uint8)):
                f.write(np.ascontiguousarray(a).tobytes())
            f.write(np.ascontiguousarray(want["prep_msgs"][:, :pm]).tobytes() if pm else b"")
            if enc:
                f.write(enc["sk"] + enc["pk"] + enc["task_id"])
                for a in (enc["times"], enc["encs"], enc["cto"]):
                    f.write(np.ascontiguousarray(a).tobytes())
                f.write(enc["cts"])
                f.write(np.ascontiguousarray(enc["kidx"]).tobytes())
                f.write(np.ascontiguousarray(enc["status"]).tobytes())
        os.replace(src + ".tmp", src)
    out = os.path.join(tmp, "jobs_out.bin")
    cmd = [DRIVER, src, out, str(vdaf.algo_id), str(vdaf.bits), str(vdaf.length), str(vdaf.chunk_length),
           str(vdaf.num_proofs), vk.hex(), str(n), str(T), str(seconds), str(int(mode == "coalesce")), str(window_us),
           "1"]
    if leader is not None and leader_threads:
        lvk, (ln, lps_, llis, lv, lsh) = leader
        lsrc = os.path.join(tmp, f"leader_{vdaf.algo_id}_{len(lv)}.bin")
        if not os.path.exists(lsrc):
            with open(lsrc + ".tmp", "wb") as f:
                f.write(np.array([len(lv), len(lps_[0]), len(llis[0]), len(lsh[0]), 0, 0, 0, 0], np.uint64).tobytes())
                f.write(np.ascontiguousarray(ln).tobytes() + b"".join(lps_) + b"".join(llis) + lv.tobytes() + b"".join(lsh))
            os.replace(lsrc + ".tmp", lsrc)
        cmd += ["1", lsrc, lvk.hex(), str(leader_threads)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120 + 4 * seconds)
    if r.returncode != 0:
        return {"vdaf": vdaf.name(), "mode": mode, "reports_per_job": n, "threads": T, "verified": False,
                "error": (r.stderr or "")[-400:]}
    line = json.loads(r.stdout.strip().splitlines()[-1])
    raw = open(out, "rb").read()
    head = np.frombuffer(raw[:32], np.uint64)
    ob = vdaf.output_len * vdaf.field_bytes
    agg = raw[32:32 + ob]
    mult = np.frombuffer(raw[32 + ob:32 + ob + 8 * K], np.uint64).astype(np.int64)
    fin = want["verdicts"] == 0
    m_fin = np.where(fin, mult, 0)
    p = P64 if vdaf.field_bytes == 8 else P128
    exp = weighted_aggregate(want["out_shares"].reshape(K, -1), m_fin, vdaf.field_bytes, p)
    agg_ok = agg == exp and int(head[3]) == int(m_fin.sum())
    res = {"vdaf": vdaf.name(), "mode": mode, "driver": "cpp", "reports_per_job": n, "threads": T}
    res.update(line)
    res["verified"] = bool(agg_ok and line["bad_jobs"] == 0 and line.get("leader_bad_jobs", 0) == 0)
    res["verification"] = {"aggregate_and_count": bool(agg_ok), "jobs_with_wrong_verdicts_or_msgs": line["bad_jobs"],
                           "leader_jobs_with_wrong_verdicts_or_prep_shares": line.get("leader_bad_jobs", 0)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vdafs", default="sumvec,count")
    ap.add_argument("--sizes", default="10,100,1000,10000")
    ap.add_argument("--threads", default="1,8,64")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--pool", type=int, default=2048)
    ap.add_argument("--mode", default="direct", choices=("direct", "coalesce"))
    ap.add_argument("--window-us", type=int, default=0, help="coalesce mode: the gathering window (0: engine default)")
    ap.add_argument("--out", default=None, help="also append the JSON lines to this file")
    ap.add_argument("--keep-pool", default=None,
                    help="cpp driver: write the pool file(s) into this directory and keep them (for running "
                         "tools/bin/jobs_driver directly, e.g. under rocprofv3)")
    ap.add_argument("--encrypted", action="store_true",
                    help="cpp driver: the jobs start from HPKE-encrypted report shares (jx_helper_prep_encrypted_batch)")
    ap.add_argument("--leader-threads", default="0",
                    help="cpp driver: comma list; L threads of 100-report leader prepare_init jobs of another task "
                         "beside the helper's (an aggregator that is leader for some tasks and helper for others)")
    ap.add_argument("--driver", default="cpp", choices=("cpp", "python"),
                    help="cpp: native threads (tools/jobs_driver.cpp) call the C ABI; python: Python threads "
                         "through janus_amd.engine (the interpreter's lock serialises their host work)")
    a = ap.parse_args()

    from bench import cpu_threads
    from janus_amd.vdaf import Prio3

    threads_gen = min(16, cpu_threads()["threads"])
    vdafs = {"sumvec": Prio3.sum_vec(8, 1000, 88), "count": Prio3.count(), "sum32": Prio3.sum(32),
             "hist": Prio3.histogram(256, 16)}
    vk = bytes(range(16))
    out = open(a.out, "a") if a.out else None
    for key in a.vdafs.split(","):
        vdaf = vdafs[key]
        t0 = time.perf_counter()
        pool = make_pool(vdaf, vk, a.pool, threads_gen)
        print(f"# {key}: pool of {a.pool} in {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
        if a.driver == "cpp":  # this process never touches the GPU: the driver child does
            import tempfile

            build_driver()
            enc = None
            if a.encrypted:
                t0 = time.perf_counter()
                pool, enc = make_enc_pool(vdaf, pool)
                print(f"# sealed {a.pool} report shares in {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
            lts = [int(x) for x in a.leader_threads.split(",")]
            leader = None
            if any(lts):
                lvk = bytes(range(100, 116))
                leader = (lvk, make_leader_pool(vdaf, lvk, min(a.pool, 512)))
            with tempfile.TemporaryDirectory() as tmp:
                if a.keep_pool:
                    os.makedirs(a.keep_pool, exist_ok=True)
                    tmp = a.keep_pool
                for n in [int(x) for x in a.sizes.split(",") if int(x) > 0]:
                    for T in [int(x) for x in a.threads.split(",")]:
                        for L in lts:
                            r = run_case_cpp(vdaf, vk, pool, n, T, a.seconds, a.mode, a.window_us, tmp, enc=enc,
                                             leader=leader, leader_threads=L)
                            line = json.dumps(r)
                            print(line, flush=True)
                            if out:
                                out.write(line + "\n")
                                out.flush()
            continue
        import torch  # noqa: F401  (one HIP runtime: torch first, see janus_amd/_lib.py)

        from janus_amd.engine import HelperEngine
        with HelperEngine(vdaf, vk) as eng:
            if a.mode == "coalesce":
                eng.coalesce(True, window_us=a.window_us)
            # warm-up: first-touch allocations and kernel loads
            run_case(eng, vdaf, pool, 64, 1, 0.2, a.mode, max_jobs=2)
            for n in [int(x) for x in a.sizes.split(",")]:
                for T in [int(x) for x in a.threads.split(",")]:
                    r = run_case(eng, vdaf, pool, n, T, a.seconds, a.mode)
                    line = json.dumps(r)
                    print(line, flush=True)
                    if out:
                        out.write(line + "\n")
                        out.flush()
    if out:
        out.close()


if __name__ == "__main__":
    main()
