#!/usr/bin/env python3
"""Benchmark: helper reports/s for Prio3 prep_init + prep_next + aggregate on MI355X.

Metric (BASELINE.json): "helper reports/sec (prep_init+aggregate), Prio3SumVec len=1000 @1/2/4/8 GPU".
Workload: Prio3SumVec{bits=8, length=1000, chunk_length=88} (BASELINE configs[3]); one step =
every GPU prepares and aggregates R reports (default R = 10M / 8 = 1.25M, so the 8-GPU step is the
10M-report target) and, for N > 1, the partial aggregate shares are combined with an RCCL
all-gather + on-device mod-p add (compute_aggregate_share, aggregate_share.rs:55-96).
Scaling is weak (fixed reports per GPU). Inputs are resident in HBM before the timed region.

Synthetic data: a pool of K distinct reports (client shard + leader prep_init produced by the
C oracle, the same role prio's client/leader play in Janus's own tests, core/src/test_util/
mod.rs:86-237; 1 in 100 with a tampered leader prep share) is tiled on the device to R reports.
Every report is fully recomputed by the kernels; the final aggregate is checked against
multiplicity * the oracle's pool aggregate.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 via torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "helper reports/sec (prep_init+aggregate), Prio3SumVec len=1000 @1/2/4/8 GPU"
P128 = 2**128 - 28 * 2**64 + 1
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 256 CUs x 4 SIMD32 x 32 lanes x 2.4 GHz = 78.6 int32 Top/s
HBM_PEAK_GBPS = 8000.0
# Algorithmic int32 VALU work: one Keccak-p[1600,12] permutation = 190 instructions/round
# x 12 rounds on gfx950 (theta 20 v_bitop3 + 10 v_alignbit + 60 xor, rho 48 v_alignbit, chi 50 v_bitop3,
# iota 2); one Field128 Montgomery product (K1 coefficients / inversion) = 56; one Field128 product in the
# FLP wire sums (K3, 2 per measurement element) = 16 32x32->64 partial products.
OPS_PER_PERM = 190 * 12
OPS_PER_MONT = 56
OPS_PER_FMUL = 16
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_v3_pmc_summary.json")


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def sumvec_work(bits, length, chunk):
    """Per-report algorithmic work (perms, Montgomery products) of each stage."""
    M = bits * length
    MB = M * 16
    calls = -(-M // chunk)
    P = 1
    while P < calls + 1:
        P <<= 1
    A = 2 * chunk
    proof_len = A + 2 * P - 1
    perms_meas = -(-MB // 168)
    perms_part = (42 + MB) // 168 + 1
    perms_proof = -(-(proof_len * 16) // 168)
    perms_tail = 4  # corrected seed, joint rands, query rands (+1 prep msg only when parts differ)
    perms = perms_meas + perms_part + perms_proof + perms_tail
    # K1 tail: t^P, L, batch inversion (3 per call) + ~143 for the inversion chain, d_k
    mont_k1 = 6 + 3 * (calls + 1) + 143 + 2 * calls + 8
    # K3: two products per measurement element (wire sums), wire finish ~8 per slot, v and G(t) 2 per coeff
    fmul_k3 = 2 * M
    mont_k3 = 8 * chunk + 2 * (2 * P - 1) + 20
    return dict(perms=perms, mont_k1=mont_k1, fmul_k3=fmul_k3, mont_k3=mont_k3,
                ops_k1=perms * OPS_PER_PERM + mont_k1 * OPS_PER_MONT,
                ops_k3=fmul_k3 * OPS_PER_FMUL + mont_k3 * OPS_PER_MONT,
                hbm_k1=16 * (M + proof_len + 6 + 2 * calls) + 16 * length + 16 + 48 + 32 + 16,
                hbm_k3=16 * (M + proof_len + 6 + 2 * calls) + 16 * (A + 3) + 1)


def pmc_traffic(kernel: str, reports_per_launch: float):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (separate
    FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled per the gfx950 correction), scaled to this
    run's reports per launch. None if the summary or kernel is missing."""
    try:
        d = json.load(open(PMC_SUMMARY))
        names = [k for k in d["kernels"] if k == kernel] or \
            [k for k in d["kernels"] if k.startswith(kernel) and "<true" not in k and "true>" not in k]
        e = d["kernels"][names[0]]
        per_report = (e["hbm_read_bytes"] + e["hbm_write_bytes"]) / d["workload"]["reports_per_launch"]
        return int(per_report * reports_per_launch), os.path.relpath(PMC_SUMMARY, ROOT)
    except (OSError, KeyError, ValueError, IndexError):
        return None, None


def make_pool(vdaf, vk, K, seed=0x5EED, threads=16):
    from oracle import oracle as O  # input generation (client + leader), see module docstring
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    rng = np.random.default_rng(seed)
    meas = rng.integers(0, 1 << vdaf.bits, size=(K, vdaf.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=threads)
    for i in range(0, K, 100):  # 1% invalid: one flipped bit in the leader prep share
        j = int(rng.integers(0, lps.shape[1]))
        lps[i, j] ^= 1 << int(rng.integers(0, 8))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads)
    return orc, nonces, ps, his, lps, want


def cpu_baseline(orc, vk, nonces, ps, his, lps, seconds, threads):
    """The C oracle (a literal port of the reference algorithm) timed on this host's cores."""
    K = nonces.shape[0]
    n = K
    t = time.perf_counter()
    orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads)
    dt = time.perf_counter() - t
    rate = n / dt
    # scale the sample to ~`seconds` of CPU work
    reps = max(1, int(seconds * rate / K))
    tile = lambda a: np.ascontiguousarray(np.tile(a, (reps, 1)))  # noqa: E731
    t = time.perf_counter()
    orc.helper_prep_batch(vk, tile(nonces), tile(ps), tile(his), tile(lps), nthreads=threads)
    dt = time.perf_counter() - t
    return {"value": round(reps * K / dt, 2), "unit": "reports/s", "cores": threads, "kind": "port",
            "sample": f"{reps * K} Prio3SumVec(8x1000/88) helper prep_init+prep_next+aggregate reports "
                      f"({K} distinct x {reps}), C oracle oracle/prio3_oracle.c, {threads} threads, {dt:.1f} s"}


def _free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def ensure_world(gpus: int) -> None:
    """`--gpus N` means N ranks, one per GPU. Without a torch.distributed launcher in the
    environment, start one (torch.distributed.run as a child process, before this process touches
    the GPU) and exit with its status; refuse N beyond the visible GPUs or a launcher world of
    another size, instead of silently measuring one GPU."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            sys.exit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}")
        return
    if gpus == 1:
        return
    import subprocess

    import torch  # device_count() does not initialise the HIP runtime on this image

    have = torch.cuda.device_count()
    if gpus > have:
        sys.exit(f"bench.py: --gpus {gpus} but only {have} GPU(s) visible")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *sys.argv[1:]]
    sys.exit(subprocess.run(cmd).returncode)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reports-per-gpu", type=int, default=1_250_000)
    ap.add_argument("--pool", type=int, default=2048)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bits", type=int, default=8)
    ap.add_argument("--length", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=88)
    args = ap.parse_args()
    ensure_world(args.gpus)

    import torch
    import torch.distributed as dist

    from janus_amd.distributed import ShardCombiner
    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus  # ensure_world
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    vdaf = Prio3.sum_vec(args.bits, args.length, args.chunk)
    vk = bytes(range(16))
    threads = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    orc, nonces, ps, his, lps, want = make_pool(vdaf, vk, args.pool, threads=threads)
    log(f"pool of {args.pool} reports generated in {time.perf_counter() - t0:.1f}s; "
        f"{int(want['count'])} valid")

    R = args.reports_per_gpu
    reps = -(-R // args.pool)

    def dev_tile(a):
        t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        return t.repeat(reps, 1)[:R].contiguous()

    d_n, d_ps, d_his, d_lps = dev_tile(nonces), dev_tile(ps), dev_tile(his), dev_tile(lps)
    d_verdicts = torch.empty(R, dtype=torch.uint8, device=dev)
    d_msgs = torch.empty((R, 16), dtype=torch.uint8, device=dev)
    eng = HelperEngine(vdaf, vk, device=local_rank)
    combiner = ShardCombiner(eng) if world > 1 else None

    def step():
        eng.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), R,
                                      0, d_msgs.data_ptr(), d_verdicts.data_ptr())
        if combiner is not None:  # shard records: RCCL all-gather + device mod-p merge
            combiner.combine(0)
        eng.sync()

    for _ in range(args.warmup):
        step()
    eng.timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t
    kt = eng.timing_read()
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    # ---- verification: aggregate == (steps + warmup) * multiplicity * pool aggregate
    agg, count, _ = eng.aggregate_share(0)
    total_steps = args.steps + args.warmup
    mult = np.bincount(np.arange(R) % args.pool, minlength=args.pool)
    fin = want["verdicts"] == 0
    exp_count = total_steps * int(mult[fin].sum())
    # expected aggregate = total_steps * sum_i mult_i * out_i ; recompute from per-report out shares
    res = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads, want_out_shares=True)
    outs = res["out_shares"].reshape(args.pool, vdaf.output_len, 16)
    vals = [int.from_bytes(bytes(b), "little") for b in outs.reshape(-1, 16)]
    acc = [0] * vdaf.output_len
    for i in range(args.pool):
        if res["verdicts"][i] == 0:
            m = int(mult[i]) * total_steps
            for j in range(vdaf.output_len):
                acc[j] += m * vals[i * vdaf.output_len + j]
    exp = b"".join((x % P128).to_bytes(16, "little") for x in acc)
    verified = agg == exp and count == exp_count
    verdict_ok = bool(np.array_equal(d_verdicts.cpu().numpy(), np.tile(want["verdicts"], reps)[:R]))
    if world > 1:
        c_agg, c_count, _ = combiner.result()
        exp_c = b"".join(((x * world) % P128).to_bytes(16, "little") for x in acc)
        verified = verified and c_agg == exp_c and c_count == world * exp_count

    total_reports = R * world * args.steps
    value = total_reports / elapsed
    work = sumvec_work(args.bits, args.length, args.chunk)
    launches = max(1, kt["xof"]["launches"])
    chunk_reports = R / (launches / args.steps)  # reports per K1 launch
    k1_ms = kt["xof"]["ms"] / launches
    k3_ms = kt["flp"]["ms"] / max(1, kt["flp"]["launches"])
    k1_tops = work["ops_k1"] * chunk_reports / (k1_ms * 1e-3) / 1e12
    k3_tops = work["ops_k3"] * chunk_reports / (k3_ms * 1e-3) / 1e12
    dominant = "K1 xof_kernel" if kt["xof"]["ms"] >= kt["flp"]["ms"] else "K3 flp_psum_part_kernel"
    ach = k1_tops if dominant.startswith("K1") else k3_tops
    traffic, traffic_src = pmc_traffic("jx::xof_kernel" if dominant.startswith("K1") else
                                       "jx::flp_psum_part_kernel", chunk_reports)
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "reports/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (Field128 mod-p integer arithmetic, Keccak-p[1600,12])",
        "data": f"synthetic: {args.pool} distinct client reports (C-oracle client+leader, 1% tampered) "
                f"tiled on device to {R} reports/GPU; inputs resident in HBM",
        "config": {"workload": f"Prio3SumVec bits={args.bits} length={args.length} chunk_length={args.chunk}: "
                               "helper prep_init + prep_shares_to_prep + prep_next + aggregate",
                   "reports_per_gpu": R, "global_reports_per_step": R * world,
                   "parallelism": f"report-sharded x{world} (RCCL all-gather + device mod-p combine)"},
        "roofline": {"bound": "valu", "kernel": dominant, "achieved": round(ach, 3), "peak": round(VALU_PEAK_TOPS, 2),
                     "unit": "TOP/s (int32 VALU instructions/s, algorithmic count: DESIGN.md §5)",
                     "frac": round(ach / VALU_PEAK_TOPS, 4),
                     "traffic": traffic, "traffic_unit": "HBM bytes per launch (rocprofv3 2*FETCH_SIZE + WRITE_SIZE)",
                     "traffic_source": traffic_src,
                     "algorithmic_bytes": int(work["hbm_k1"] * chunk_reports),
                     "hbm_GBps": round(work["hbm_k1"] * chunk_reports / (k1_ms * 1e-3) / 1e9, 1),
                     "hbm_peak_GBps": HBM_PEAK_GBPS},
        "kernels": {"k1_xof_ms_per_launch": round(k1_ms, 3), "k3_flp_ms_per_launch": round(k3_ms, 3),
                    "k4_acc_ms_per_launch": round(kt["accumulate"]["ms"] / max(1, kt["accumulate"]["launches"]), 3),
                    "slow_ms_per_launch": round(kt["slow"]["ms"] / max(1, kt["slow"]["launches"]), 3),
                    "reports_per_launch": int(chunk_reports),
                    "k1_tops": round(k1_tops, 3), "k3_tops": round(k3_tops, 3),
                    "k1_hbm_GBps": round(work["hbm_k1"] * chunk_reports / (k1_ms * 1e-3) / 1e9, 1),
                    "k3_hbm_GBps": round(work["hbm_k3"] * chunk_reports / (k3_ms * 1e-3) / 1e9, 1),
                    "work_per_report": work},
        "verified": bool(verified and verdict_ok),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(orc, vk, nonces, ps, his, lps, args.cpu_seconds, threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
