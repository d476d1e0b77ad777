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
# K1 roofline, two counts:
#  (a) instruction issue: the gfx950 instructions this Keccak needs per round (theta 20 v_bitop3 +
#      10 v_alignbit + 60 xor, rho 48 v_alignbit, chi 50 v_bitop3, iota 2 = 190) x 12 rounds = 2280
#      per permutation; 56 per Field128 Montgomery product; 16 per lazy FLP product. frac_issue says
#      how busy the SIMDs' issue slots are. (Its ceiling is ~0.66: alignbit issues at half rate.)
#  (b) algorithmic, kernel-independent: the spec's 64-bit operations of Keccak-p[1600] (theta 50,
#      rho 24 rotations, chi 75, iota 1 = 155 per round; 1860 per 12-round permutation) counted as
#      32-bit operations (x2: 3720) and 160 per Field128 product (16 32x32->64
#      products at ~10 ops each). SURVEY.md priced these against a 39.3 T peak (256 CU x 64 lanes x
#      2.4 GHz, 1 op per lane-cycle), which undercounts gfx950's 4 SIMD-32 per CU by 2x; here the
#      peak is the 78.6 T int32 lane-op rate for both counts.
OPS_PER_PERM = 190 * 12
# Instruction-mix ceiling of the Keccak round: gfx950 does not issue every instruction at the flat
# 78.6 T rate. Measured rates at 8 waves/SIMD on independent chains (profiles/r01_microbench_valu.jsonl,
# tools/microbench_valu.hip), as fractions of 78.6 T: v_bitop3_b32 0.70, v_alignbit_b32 0.465;
# v_xor_b32 is taken at 1.0 (its microbench reads 1.13: the compiler fuses xor pairs into v_bitop3).
# A round (62 xor + 70 bitop3 + 58 alignbit) therefore issues at most 190 / (62 + 70/0.70 + 58/0.465)
# = 0.663 of 78.6 T = 52.1 T, at the nominal 2.4 GHz; the PMC clock under K1 is lower (power).
KECCAK_ROUND_MIX = {"v_xor_b32": (62, 1.0), "v_bitop3_b32": (70, 0.70), "v_alignbit_b32": (58, 0.465)}
OPS_PER_MONT = 56
OPS_PER_FMUL = 16
ALG_OPS_PER_PERM = 3720
ALG_OPS_PER_FMUL = 160
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06_pmc_summary.json")
K1_KERNEL = "jx::xof_kernel<false, 0>"  # rocprofv3 name of the helper K1 (jx_kernels.hip)
KERNEL_SOURCES = ["janus_amd/csrc/jx_kernels.hip", "janus_amd/csrc/jx_engine.cpp", "janus_amd/csrc/jx_kernels.h",
                  "janus_amd/csrc/jx_field.h", "janus_amd/csrc/jx_keccak.h", "janus_amd/csrc/jx_sha256.h"]


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def sources_digest() -> str:
    """sha256 over the engine's kernel sources: ties a PMC summary to the kernels it measured."""
    import hashlib

    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    return h.hexdigest()[:16]


def sumvec_work(bits, length, chunk):
    """Per-report work of each stage (permutations, field products) and its instruction /
    algorithmic op counts and HBM bytes."""
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
                alg_ops_k1=perms * ALG_OPS_PER_PERM + mont_k1 * ALG_OPS_PER_FMUL,
                alg_ops_k3=(fmul_k3 + mont_k3) * ALG_OPS_PER_FMUL,
                hbm_k1=16 * (M + proof_len + 6 + 2 * calls) + 16 * length + 16 + 48 + 32 + 16,
                hbm_k3=16 * (M + proof_len + 6 + 2 * calls) + 16 * (A + 3) + 1)


def keccak_mix_ceiling_tops() -> float:
    n = sum(c for c, _ in KECCAK_ROUND_MIX.values())
    return VALU_PEAK_TOPS * n / sum(c / r for c, r in KECCAK_ROUND_MIX.values())


def pmc_clock(kernel: str):
    """Shader clock under `kernel` from the committed PMC summary (GRBM_GUI_ACTIVE / 8 XCDs / duration),
    or None when the summary was taken on other kernel sources."""
    try:
        d = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None
    if d.get("workload", {}).get("sources_digest") != sources_digest():
        return None
    return d.get("kernels", {}).get(kernel, {}).get("clock_GHz")


def pmc_kernel(kernel: str):
    """(entry, reports per launch) of `kernel` in the committed PMC summary when it was taken on these
    kernel sources, else (None, None)."""
    try:
        d = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None, None
    wl = d.get("workload", {})
    if wl.get("sources_digest") != sources_digest() or not wl.get("reports_per_launch"):
        return None, None
    return d.get("kernels", {}).get(kernel), wl["reports_per_launch"]


def pmc_traffic(kernel: str, reports_per_launch: float):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (separate
    FETCH_SIZE / WRITE_SIZE passes over uniform launches; FETCH_SIZE doubled per the gfx950
    correction), scaled to this run's reports per launch. Refused (None + reason) when the summary
    was taken on other kernel sources, lacks the kernel, or has no launch size."""
    try:
        d = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError) as e:
        return None, None, f"no PMC summary: {e}"
    src = os.path.relpath(PMC_SUMMARY, ROOT)
    wl = d.get("workload", {})
    if wl.get("sources_digest") != sources_digest():
        return None, src, "PMC summary was taken on other kernel sources"
    e = d.get("kernels", {}).get(kernel)
    if not e or "hbm_read_bytes" not in e or "hbm_write_bytes" not in e or not wl.get("reports_per_launch"):
        return None, src, f"PMC summary lacks {kernel} bytes or its launch size"
    per_report = (e["hbm_read_bytes"] + e["hbm_write_bytes"]) / wl["reports_per_launch"]
    return int(per_report * reports_per_launch), src, f"{per_report:.0f} B/report over " \
        f"{wl['reports_per_launch']}-report launches"


# PMC summaries of the secondary configs (scripts/gpu_pmc_r06_configs.sh): one rocprofv3 kernel trace and
# separate --pmc passes over tools/bench_configs.py steps of that config
CONFIG_PMC_SUMMARIES = {"configs[1]": os.path.join(ROOT, "profiles", "r06_sum32_pmc_summary.json"),
                        "configs[2]": os.path.join(ROOT, "profiles", "r06_hist_pmc_summary.json")}


def stage_roofline(summary_path: str, prefix: str, ms_per_launch: float, reports_per_launch: float, stage: str) -> dict:
    """A stage's own VALU-issue roofline from a committed PMC summary: the instructions of the stage's kernels
    (names starting with `prefix`: jx::xof for K1, jx::flp for K3) per report (SQ_INSTS_VALU x 64 lanes /
    the summary's reports per launch) x this run's reports per launch / this run's HIP-event stage time per
    launch, over the 78.6 T int32 issue peak; frac_pmc_run is the summary's own instructions / rocprof durations.
    None (with a reason) when the summary is missing or was taken on other kernel sources."""
    try:
        d = json.load(open(summary_path))
    except (OSError, ValueError) as e:
        return {"frac": None, "note": f"no PMC summary: {e}"}
    src = os.path.relpath(summary_path, ROOT)
    wl = d.get("workload", {})
    if wl.get("sources_digest") != sources_digest() or not wl.get("reports_per_launch"):
        return {"frac": None, "source": src, "note": "PMC summary was taken on other kernel sources"}
    ks = {k: e for k, e in d.get("kernels", {}).items() if k.startswith(prefix) and "SQ_INSTS_VALU" in e.get("pmc", {})}
    if not ks or not ms_per_launch:
        return {"frac": None, "source": src, "note": f"no {prefix}* kernel with SQ_INSTS_VALU in the summary"}
    rpl = wl["reports_per_launch"]
    # per launch: every kernel of the stage runs once per launch (per-dispatch averages)
    insts = sum(e["pmc"]["SQ_INSTS_VALU"] for e in ks.values())
    ns = sum(e["avg_ns"] for e in ks.values())
    lane_ops_per_report = insts * 64 / rpl
    ach = lane_ops_per_report * reports_per_launch / (ms_per_launch * 1e-3) / 1e12
    run = insts * 64 / (ns * 1e-9) / 1e12
    clk = [e.get("clock_GHz") for e in ks.values() if e.get("clock_GHz")]
    return {"bound": "valu", "stage": stage, "kernels": sorted(ks), "achieved": round(ach, 3),
            "peak": round(VALU_PEAK_TOPS, 2), "unit": "TOP/s int32 lane-op issue", "frac": round(ach / VALU_PEAK_TOPS, 4),
            "frac_pmc_run": round(run / VALU_PEAK_TOPS, 4), "ms_per_launch": ms_per_launch,
            "pmc_ms_per_launch": round(ns / 1e6, 3), "reports_per_launch": reports_per_launch,
            "lane_ops_per_report": round(lane_ops_per_report, 1), "clock_GHz_pmc": round(max(clk), 3) if clk else None,
            "valu_util_pmc": round(max(e.get("valu_util", 0) for e in ks.values()), 3),
            "hbm_bytes_per_report": round(sum(e.get("hbm_bytes_per_report", 0) for e in ks.values()), 1),
            "source": src, "note": "PMC SQ_INSTS_VALU x 64 per report (source) x reports / this run's HIP-event stage "
                                   "time per launch; frac_pmc_run: the summary's instructions / its rocprof durations"}


POOL_BLOCK = 256  # pool reports per stored block aggregate (CyclicPool prefix sums)


def make_pool(vdaf, vk, K, seed=0x5EED, threads=16):
    """K distinct client reports and the oracle's helper results: verdicts, prep messages, the pool
    aggregate and the aggregate of every POOL_BLOCK-report block (for expectations over any range of
    the cyclic tiling, CyclicPool)."""
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
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=threads, want_out_shares=True)
    outs, fin = want.pop("out_shares"), want["verdicts"] == 0
    nb = -(-K // POOL_BLOCK)
    want["blocks"] = np.stack([np.frombuffer(orc.aggregate(
        [outs[i].tobytes() for i in range(b * POOL_BLOCK, min(K, (b + 1) * POOL_BLOCK)) if fin[i]]), np.uint8)
        for b in range(nb)])
    return orc, nonces, ps, his, lps, want


class CyclicPool:
    """Expected aggregates over any range of the cyclic tiling report g -> pool[g % K] (each rank's
    shard [start, start + R) of the global report index, and the merged range of all ranks).

    With F(g) = the aggregate of reports [0, g): F(g) = (g // K) * pool total + prefix(g % K), and the
    aggregate of [lo, hi) is F(hi) - F(lo) mod p. prefix(r) adds the stored block aggregates below r
    and `partial(a, r)` (the aggregate of pool[a:r], fewer than `block` reports) above them. Counts
    the same way from the per-report finished flags."""

    def __init__(self, fin, block_aggs, block: int, partial, p: int):
        self.K, self.block, self.partial, self.p = len(fin), block, partial, p
        width = len(block_aggs[0])
        self.cum = [[0] * width]
        for b in block_aggs:
            self.cum.append([(x + y) % p for x, y in zip(self.cum[-1], b)])
        self.fin_cum = np.concatenate([[0], np.cumsum(np.asarray(fin, dtype=np.int64))])

    def prefix(self, r: int):
        b, t = divmod(r, self.block)
        vec = list(self.cum[b])
        if t:
            vec = [(x + y) % self.p for x, y in zip(vec, self.partial(b * self.block, r))]
        return vec, int(self.fin_cum[r])

    def F(self, g: int):
        q, r = divmod(g, self.K)
        vec, c = self.prefix(r)
        tot = self.cum[-1]
        return [(q * t + x) % self.p for t, x in zip(tot, vec)], q * int(self.fin_cum[-1]) + c

    def range(self, lo: int, hi: int, times: int = 1):
        """(aggregate as field elements, count) of reports [lo, hi), accumulated `times` times."""
        (a, ca), (b, cb) = self.F(lo), self.F(hi)
        return [(y - x) * times % self.p for x, y in zip(a, b)], (cb - ca) * times


def field_elems(b: bytes, fb: int) -> list[int]:
    return [int.from_bytes(b[i:i + fb], "little") for i in range(0, len(b), fb)]


def prio3_work(v, role: str = "helper") -> dict:
    """Instruction model of one report's K1 (XOF stage) and K3 (FLP stage) for any TurboSHAKE Prio3
    instance (the SumVec numbers of sumvec_work, generalised): Keccak-p[1600,12] permutations at
    OPS_PER_PERM, Montgomery products at OPS_PER_MONT, lazy FLP products at OPS_PER_FMUL. The helper
    squeezes its measurement and proof shares and absorbs the joint-rand part; the leader absorbs
    only (its shares are explicit)."""
    fb = v.field_bytes
    MB = v.meas_len * fb
    jr = v.joint_rand_len > 0
    helper = role == "helper"
    perms = (-(-MB // 168) if helper else 0) + ((42 + MB) // 168 + 1 if jr else 0) + \
        (-(-(v.proof_len * fb) // 168) if helper else 0) + 4
    calls, chunk = v.calls, max(1, v.gadget_chunk)
    mont_k1 = 6 + 3 * (calls + 1) + 143 + 2 * calls + 8 + chunk + -(-chunk // 2)
    if v.algo_id == 5:  # FixedPointBoundedL2VecSum's second gadget
        mont_k1 += 3 * (v.norm_calls + 1) + 143 + 2 * v.norm_calls
    fmul_k3 = 2 * v.meas_len + (2 * v.length if v.algo_id == 5 else 0)
    mont_k3 = 8 * chunk + 2 * (2 * v.P - 1) + 20
    return dict(perms=perms, mont_k1=mont_k1, fmul_k3=fmul_k3, mont_k3=mont_k3,
                ops_k1=perms * OPS_PER_PERM + mont_k1 * OPS_PER_MONT,
                ops_k3=fmul_k3 * OPS_PER_FMUL + mont_k3 * OPS_PER_MONT)


def pool_cache_path(vdaf, vk, K, seed=0x5EED) -> str:
    import hashlib

    key = hashlib.sha256(f"{vdaf.algo_id}/{vdaf.bits}/{vdaf.length}/{vdaf.chunk_length}/{K}/{seed}/{vk.hex()}/"
                         f"pool-v2/{POOL_BLOCK}".encode()).hexdigest()[:16]
    return os.path.join(os.environ.get("JX_POOL_CACHE", "/tmp"), f"janus_amd_bench_pool_{key}.npz")


def load_or_make_pool(vdaf, vk, K, threads, local_rank: int, wait_s: float = 900.0):
    """The synthetic pool, generated once per node: local rank 0 runs the C oracle and writes the pool
    (inputs + the oracle's verdicts and aggregate) atomically to a cache file; the other ranks wait for
    the file and read it. An 8-rank start therefore costs one generation, not eight."""
    from oracle import oracle as O

    path = pool_cache_path(vdaf, vk, K)
    if not os.path.exists(path):
        if local_rank == 0:
            orc, nonces, ps, his, lps, want = make_pool(vdaf, vk, K, threads=threads)
            tmp = f"{path}.{os.getpid()}.tmp.npz"
            np.savez(tmp, nonces=nonces, ps=ps, his=his, lps=lps, verdicts=want["verdicts"],
                     prep_msgs=want["prep_msgs"], blocks=want["blocks"],
                     agg=np.frombuffer(want["agg"], np.uint8), count=np.array([want["count"]], np.int64))
            os.replace(tmp, path)
            return orc, nonces, ps, his, lps, want, "generated"
        t0 = time.perf_counter()
        while not os.path.exists(path):
            if time.perf_counter() - t0 > wait_s:
                sys.exit(f"bench.py: rank {local_rank} waited {wait_s:.0f}s for the pool file {path}")
            time.sleep(0.5)
    d = np.load(path)  # allow_pickle=False: plain arrays this script wrote
    orc = O.Prio3Oracle(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length)
    want = {"verdicts": d["verdicts"], "prep_msgs": d["prep_msgs"], "blocks": d["blocks"], "agg": d["agg"].tobytes(),
            "count": int(d["count"][0])}
    return orc, d["nonces"], d["ps"], d["his"], d["lps"], want, "cached"


def cpu_threads() -> dict:
    """Host threads for the CPU baseline: the CPUs this process may run on (affinity), capped by the
    cgroup CPU quota when one is set (a GPU box's share of a larger machine)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    use = min(aff, quota) if quota else aff
    return {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "threads": use}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(orc, vdaf, vk, nonces, ps, his, lps, seconds, threads):
    """The CPU engine (cpu_baseline/jc_cpu_engine.cpp: the same barycentric FLP, word-wise sponges and
    lazy field sums as the GPU path, report-parallel) timed on this host's cores at 1 thread and at
    `threads` threads on a bounded sample, plus the literal C oracle port as a secondary figure."""
    from cpu_baseline import cpu_engine as CE

    K = nonces.shape[0]

    def rate(threads_, budget):
        m = min(K, max(16, threads_ * 8))
        t = time.perf_counter()
        CE.helper_prep_aggregate(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length, vk, nonces[:m], ps[:m],
                                 his[:m], lps[:m], nthreads=threads_)
        r0 = m / (time.perf_counter() - t)
        n = max(m, int(budget * r0))  # the pool tiled to ~budget seconds
        idx = np.arange(n) % K
        t = time.perf_counter()
        CE.helper_prep_aggregate(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length, vk, nonces[idx], ps[idx],
                                 his[idx], lps[idx], nthreads=threads_)
        dt = time.perf_counter() - t
        return n / dt, n, dt

    r1, n1, d1 = rate(1, seconds * 0.3)
    rN, nN, dN = rate(threads, seconds * 0.5)
    m = min(K, 256)
    t = time.perf_counter()
    orc.helper_prep_batch(vk, nonces[:m], ps[:m], his[:m], lps[:m], nthreads=threads)
    r_oracle = m / (time.perf_counter() - t)
    return {"value": round(rN, 1), "unit": "reports/s", "cores": threads, "kind": "port",
            "value_1_thread": round(r1, 1), "cpu_model": cpu_model(),
            "oracle_port_reports_per_s": round(r_oracle, 1),
            "sample": f"{nN} Prio3SumVec({vdaf.bits}x{vdaf.length}/{vdaf.chunk_length}) helper prep_init+prep_next+"
                      f"aggregate reports at {threads} threads ({dN:.1f} s) and {n1} at 1 thread ({d1:.1f} s): "
                      "C++ CPU engine cpu_baseline/jc_cpu_engine.cpp (byte-checked against the fixtures); "
                      f"the literal C oracle (oracle/prio3_oracle.c) does {r_oracle:.0f}/s at {threads} threads"}


def _free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _visible_filter(n: int) -> int:
    """GPUs left after the HIP/ROCr visibility variables (comma lists of indices or UUIDs)."""
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def count_gpus(sysfs_root: str = "/sys/class/kfd/kfd/topology/nodes") -> int | None:
    """GPUs on this node without starting a GPU runtime: amdsmi (the management library; no HIP) or,
    failing that, the KFD topology in sysfs (nodes with SIMDs are GPUs). None when neither answers.
    Never torch.cuda: its fallback (_cuda_getDeviceCount) initialises HIP, and a launcher started after
    that would be a process that touched the GPU handing over to others."""
    try:
        import amdsmi

        amdsmi.amdsmi_init()
        try:
            n = len(amdsmi.amdsmi_get_processor_handles())
        finally:
            amdsmi.amdsmi_shut_down()
        if n > 0:
            return _visible_filter(n)
    except Exception:  # noqa: BLE001 - missing module or library, no permission: try sysfs
        pass
    try:
        n = 0
        for node in os.listdir(sysfs_root):
            props = os.path.join(sysfs_root, node, "properties")
            try:
                with open(props) as f:
                    kv = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if int(kv.get("simd_count", "0")) > 0:
                n += 1
        if n > 0:
            return _visible_filter(n)
    except (OSError, ValueError):
        pass
    return None


def ensure_world(gpus: int, sysfs_root: str = "/sys/class/kfd/kfd/topology/nodes") -> None:
    """`--gpus N` means N ranks, one per GPU. Without a torch.distributed launcher in the
    environment, start one (torch.distributed.run as a child process, before this process touches
    the GPU) and exit with its status; refuse N beyond the GPUs that amdsmi / the KFD topology report
    (or when neither can count them), or a launcher world of another size, instead of silently measuring
    one GPU. Nothing here imports torch or starts HIP."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            sys.exit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}")
        return
    if gpus == 1:
        return
    import subprocess

    have = count_gpus(sysfs_root)
    if have is None:
        sys.exit(f"bench.py: --gpus {gpus}: cannot count the node's GPUs (amdsmi and the KFD topology both "
                 "unavailable); refusing to start a launcher")
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
    ap.add_argument("--pool", type=int, default=32768)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bits", type=int, default=8)
    ap.add_argument("--length", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=88)
    ap.add_argument("--no-secondary", dest="secondary", action="store_false",
                    help="skip the other BASELINE configs (configs[0-2], configs[4]) that the N=1 run measures after "
                         "the headline")
    ap.add_argument("--no-dist", dest="dist", action="store_false",
                    help="at N=1, skip the RCCL (nccl) process group and the shard-record all-gather + device merge "
                         "that every step otherwise ends with (by default the N=1 step carries the N>1 step's work)")
    ap.add_argument("--pipes", type=int, default=0,
                    help="engine pipelines of the fused device path (0: the engine's choice, 2 for a multi-launch step; "
                         "1: one stream)")
    ap.add_argument("--alone-steps", type=int, default=2,
                    help="with pipelines: after the timed steps, this many single-stream steps time each kernel "
                         "alone (roofline.alone); they count in the verified aggregate")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal of the N>1 path on a 1-GPU box: every rank runs on cuda:0 and the shard records "
                         "go over gloo (launch under torch.distributed.run; the numbers are not a scaling result)")
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
    gpu = 0 if args.share_gpu else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    use_dist = world > 1 or args.dist
    if use_dist:
        if args.share_gpu:
            dist.init_process_group("gloo")
        elif world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
        else:
            dist.init_process_group("nccl", device_id=dev)
    # the world the collective actually formed: a launcher world that RCCL silently shrank would
    # otherwise report one GPU's work as N GPUs'
    rccl_world = dist.get_world_size() if use_dist else 1
    if rccl_world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the process group has {rccl_world} ranks")

    vdaf = Prio3.sum_vec(args.bits, args.length, args.chunk)
    vk = bytes(range(16))
    cpu = cpu_threads()
    threads = min(16, cpu["threads"])  # pool generation (the oracle) per node
    t0 = time.perf_counter()
    orc, nonces, ps, his, lps, want, how = load_or_make_pool(vdaf, vk, args.pool, threads, local_rank)
    startup_s = time.perf_counter() - t0
    log(f"pool of {args.pool} reports {how} in {startup_s:.1f}s; {int(want['count'])} valid")

    R = args.reports_per_gpu
    K = args.pool
    # Rank r prepares the global reports [r R, (r + 1) R) of the cyclic tiling g -> pool[g % K]: ranks hold
    # different reports (shard_range over world R reports), and the expected results follow from the
    # offsets (CyclicPool), so a rank that merged a duplicate or a neighbour's record fails verification.
    from janus_amd.distributed import shard_range

    start, stop = shard_range(R * world, rank, world)
    assert stop - start == R
    idx = (start + np.arange(R)) % K
    d_idx = torch.from_numpy(idx).to(dev)

    def dev_tile(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev).index_select(0, d_idx).contiguous()

    d_n, d_ps, d_his, d_lps = dev_tile(nonces), dev_tile(ps), dev_tile(his), dev_tile(lps)
    del d_idx
    d_verdicts = torch.empty(R, dtype=torch.uint8, device=dev)
    d_msgs = torch.empty((R, 16), dtype=torch.uint8, device=dev)
    eng = HelperEngine(vdaf, vk, device=gpu)
    if args.pipes:
        eng.debug(4, args.pipes)
    combiner = ShardCombiner(eng) if use_dist else None

    def step():
        eng.prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(), R,
                                      0, d_msgs.data_ptr(), d_verdicts.data_ptr())
        if combiner is not None:  # shard records: RCCL all-gather + device mod-p merge
            combiner.combine(0)
        eng.sync()

    for _ in range(args.warmup):
        step()
    eng.timing(True)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t
    kt = eng.timing_read()
    elapsed_min = elapsed
    if use_dist:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.share_gpu else dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        e2 = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.share_gpu else dev)
        dist.all_reduce(e2, op=dist.ReduceOp.MIN)
        elapsed, elapsed_min = float(e.item()), float(e2.item())
    # pipelines (jx_engine.cpp pipes_for): the launches of a step alternate over concurrent streams, so a
    # kernel's HIP-event duration includes the device time it shared with another launch's kernels. A few
    # single-stream steps after the timed region time every kernel alone (roofline.alone).
    pipes = eng.memory()["last_pipelines"]  # what the engine ran (fewer than asked if the arena was short)
    kt_alone = None
    if pipes > 1 and args.alone_steps > 0:
        eng.debug(4, 1)
        eng.timing(True)
        for _ in range(args.alone_steps):
            step()
        kt_alone = eng.timing_read()
        eng.debug(4, args.pipes)

    # ---- verification against the oracle, from the pool's block aggregates (CyclicPool): this rank's
    # aggregate == (steps + warmup) x the aggregate of its global range; the merged record == the same
    # over every rank's range; every verdict and every finished report's Finish{prep_msg} == the oracle's
    agg, count, _ = eng.aggregate_share(0)
    total_steps = args.steps + args.warmup + (args.alone_steps if kt_alone else 0)

    def partial(a, r):
        h = orc.helper_prep_batch(vk, nonces[a:r], ps[a:r], his[a:r], lps[a:r], nthreads=threads)
        return field_elems(h["agg"], 16)

    cyc = CyclicPool(want["verdicts"] == 0, [field_elems(b.tobytes(), 16) for b in want["blocks"]], POOL_BLOCK,
                     partial, P128)
    enc = lambda v: b"".join(x.to_bytes(16, "little") for x in v)  # noqa: E731
    exp_agg, exp_count = cyc.range(start, stop, total_steps)
    verified = agg == enc(exp_agg) and count == exp_count
    got_v = d_verdicts.cpu().numpy()
    verdict_ok = bool(np.array_equal(got_v, want["verdicts"][idx]))
    fin_rows = got_v == 0
    msgs_ok = bool(np.array_equal(d_msgs.cpu().numpy()[fin_rows], want["prep_msgs"][idx][fin_rows]))
    if combiner is not None:
        c_agg, c_count, _ = combiner.result()
        all_agg, all_count = cyc.range(0, R * world, total_steps)
        verified = verified and c_agg == enc(all_agg) and c_count == all_count

    rank_ok = bool(verified and verdict_ok and msgs_ok)
    all_ok = rank_ok
    ranks_verified = int(rank_ok)
    if use_dist:  # every rank checked its own range: the line reports the AND over ranks
        f = torch.tensor([int(rank_ok)], dtype=torch.int32, device="cpu" if args.share_gpu else dev)
        dist.all_reduce(f, op=dist.ReduceOp.SUM)
        ranks_verified = int(f.item())
        all_ok = ranks_verified == world

    total_reports = R * world * args.steps
    value = total_reports / elapsed
    work = sumvec_work(args.bits, args.length, args.chunk)
    launches = max(1, kt["xof"]["launches"])
    per_rank = R * args.steps               # reports this rank prepared in the timed region
    chunk_reports = per_rank / launches     # average reports per K1 launch
    k1_ms = kt["xof"]["ms"] / launches
    k3_ms = kt["flp"]["ms"] / max(1, kt["flp"]["launches"])
    # achieved rates from total kernel time over total reports (exact for unequal launches)
    k1_tops = work["ops_k1"] * per_rank / (kt["xof"]["ms"] * 1e-3) / 1e12
    k3_tops = work["ops_k3"] * per_rank / (kt["flp"]["ms"] * 1e-3) / 1e12
    # K1 (the XOF stage) is the dominant kernel: 4.7x K3's time per report
    ach = k1_tops
    k1_clock = pmc_clock(K1_KERNEL)
    k1_clock = round(k1_clock, 3) if k1_clock else None
    # the device over whole steps, and the kernels alone (single-stream steps after the timed region)
    ms_all = sum(kt[k]["ms"] for k in ("xof", "flp", "accumulate", "slow"))
    concurrency = ms_all / (elapsed * 1e3)  # kernels in flight on average (this rank's streams)
    dev_tops = (work["ops_k1"] + work["ops_k3"]) * per_rank / elapsed / 1e12
    alone = None
    # K1's own rate: its launches on one stream (the alone steps after the timed region when pipelines
    # overlap the timed launches, else the timed launches themselves)
    ka, steps_a = (kt_alone, args.alone_steps) if kt_alone else (kt, args.steps)
    la = max(1, ka["xof"]["launches"])
    a_tops = work["ops_k1"] * R * steps_a / (ka["xof"]["ms"] * 1e-3) / 1e12
    if kt_alone:
        alone = {"steps": args.alone_steps, "k1_xof_ms_per_launch": round(kt_alone["xof"]["ms"] / la, 3),
                 "k3_flp_ms_per_launch": round(kt_alone["flp"]["ms"] / max(1, kt_alone["flp"]["launches"]), 3),
                 "k4_acc_ms_per_launch": round(kt_alone["accumulate"]["ms"] / max(1, kt_alone["accumulate"]["launches"]), 3),
                 "kernel": "K1 xof_kernel", "achieved_model": round(a_tops, 3),
                 "frac_model": round(a_tops / VALU_PEAK_TOPS, 4),
                 "note": "the same step on one stream (debug option 4 = 1), untimed for `value`: each kernel's own "
                         "rate"}
    # instructions per report: counted by the PMC pass (SQ_INSTS_VALU x 64 lanes, committed summary on these
    # sources) when there is one, else the issue model (work_per_report)
    pmc_k1, pmc_rpl = pmc_kernel(K1_KERNEL)
    if pmc_k1 and "SQ_INSTS_VALU" in pmc_k1.get("pmc", {}):
        lane_ops = pmc_k1["pmc"]["SQ_INSTS_VALU"] * 64 / pmc_rpl
        frac_src = "PMC SQ_INSTS_VALU x 64 per report (" + os.path.relpath(PMC_SUMMARY, ROOT) + ") / K1 HIP-event " \
                   "duration of its single-stream launches"
        frac_pmc = pmc_k1["pmc"]["SQ_INSTS_VALU"] * 64 / (pmc_k1["avg_ns"] * 1e-9) / 1e12 / VALU_PEAK_TOPS
    else:
        lane_ops = work["ops_k1"]
        frac_src = "issue model (2280 per Keccak-p[1600,12], bench.py sumvec_work) / K1 HIP-event duration of its " \
                   "single-stream launches (no PMC summary on these sources)"
        frac_pmc = None
    own_tops = lane_ops * R * steps_a / (ka["xof"]["ms"] * 1e-3) / 1e12
    alg_alone = work["alg_ops_k1"] * R * steps_a / (ka["xof"]["ms"] * 1e-3) / 1e12
    rpl_alone = R * steps_a / la
    k1_ms_alone = ka["xof"]["ms"] / la
    traffic, traffic_src, traffic_note = pmc_traffic(K1_KERNEL, rpl_alone)
    alg_bytes = work["hbm_k1"] * rpl_alone
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
                   "parallelism": f"report-sharded x{world} (RCCL all-gather + device mod-p combine)",
                   "combine_timed": combiner is not None,
                   "combine_note": "every step ends with the shard-record RCCL all-gather + device merge"
                   if combiner is not None else "N=1 with --no-dist: no combine in the step"},
        "startup": {"pool": how, "seconds": round(startup_s, 1)},
        "roofline": {"bound": "valu", "kernel": "K1 xof_kernel (helper XOF stage)", "achieved": round(own_tops, 3),
                     "peak": round(VALU_PEAK_TOPS, 2),
                     "unit": "TOP/s int32 lane-op issue (256 CU x 4 SIMD32 x 32 lanes x 2.4 GHz)",
                     "frac": round(own_tops / VALU_PEAK_TOPS, 4),
                     "frac_source": frac_src,
                     "frac_pmc_run": round(frac_pmc, 4) if frac_pmc else None,
                     "k1_ms_per_launch_alone": round(ka["xof"]["ms"] / la, 3),
                     "reports_per_launch_alone": round(R * steps_a / la, 1),
                     "frac_in_pipeline": round(ach / VALU_PEAK_TOPS, 4),
                     "frac_device_step": round(dev_tops / VALU_PEAK_TOPS, 4),
                     "kernel_concurrency": round(concurrency, 3),
                     "frac_model_alone": round(a_tops / VALU_PEAK_TOPS, 4),
                     "mix_ceiling": round(keccak_mix_ceiling_tops(), 2),
                     "frac_of_mix_ceiling": round(a_tops / keccak_mix_ceiling_tops(), 4),
                     "clock_GHz_pmc": k1_clock,
                     "frac_of_mix_ceiling_at_clock": round(a_tops / (keccak_mix_ceiling_tops() * k1_clock / 2.4), 4)
                     if k1_clock else None,
                     "mix_note": "mix_ceiling = the Keccak round's issue ceiling at the measured per-instruction "
                                 "rates (bench.py KECCAK_ROUND_MIX, DESIGN.md §5), nominal 2.4 GHz; "
                                 "_at_clock scales it to the PMC shader clock under K1; both over K1 alone (model count)",
                     "achieved_algorithmic": round(alg_alone, 3),
                     "frac_algorithmic": round(alg_alone / VALU_PEAK_TOPS, 4),
                     "algorithmic_unit": "TOP/s of the spec's 32-bit ops (3720 per Keccak-p[1600,12], 160 per "
                                         "Field128 product), kernel-independent, K1 alone",
                     "traffic": traffic, "traffic_unit": "HBM bytes per average launch (rocprofv3 2*FETCH_SIZE + "
                                                         "WRITE_SIZE)",
                     "traffic_source": traffic_src, "traffic_note": traffic_note,
                     "algorithmic_bytes": int(alg_bytes), "reports_per_launch": round(rpl_alone, 1),
                     "hbm_GBps": round(alg_bytes / (k1_ms_alone * 1e-3) / 1e9, 1),
                     "hbm_peak_GBps": HBM_PEAK_GBPS,
                     "pipelines": pipes, "kernel_concurrency": round(concurrency, 3),
                     "device_step": {"achieved": round(dev_tops, 3), "frac": round(dev_tops / VALU_PEAK_TOPS, 4),
                                     "note": "(K1 + K3 issue-model instructions per report) x this rank's reports / "
                                             "the timed wall time: the whole device over whole steps"},
                     "alone": alone,
                     "frac_note": "frac: K1's own issue rate, its instructions per report (PMC-counted when the "
                                  "committed summary matches these sources) x reports / its HIP-event duration on one "
                                  "stream; frac_pmc_run: the same from the PMC run alone (rocprof duration). "
                                  "frac_in_pipeline: K1's issue-model work over its HIP-event duration inside the "
                                  "timed pipelined steps, where a launch shares the device with the other pipeline "
                                  "(kernel_concurrency = summed kernel durations / wall time); frac_device_step: "
                                  "(K1 + K3 issue-model instructions) x reports / timed wall time"},
        "kernels": {"pipelines": pipes, "k1_xof_ms_per_launch": round(k1_ms, 3), "k3_flp_ms_per_launch": round(k3_ms, 3),
                    "k4_acc_ms_per_launch": round(kt["accumulate"]["ms"] / max(1, kt["accumulate"]["launches"]), 3),
                    "slow_ms_per_launch": round(kt["slow"]["ms"] / max(1, kt["slow"]["launches"]), 3),
                    "reports_per_launch": int(chunk_reports),
                    "k1_tops": round(k1_tops, 3), "k3_tops": round(k3_tops, 3),
                    "k1_hbm_GBps": round(work["hbm_k1"] * chunk_reports / (k1_ms * 1e-3) / 1e9, 1),
                    "k3_hbm_GBps": round(work["hbm_k3"] * chunk_reports / (k3_ms * 1e-3) / 1e9, 1),
                    "work_per_report": work},
        "verified": all_ok,
        "rccl_world": rccl_world, "ranks_verified": ranks_verified,
        "collective": ("gloo (--share-gpu rehearsal)" if args.share_gpu else "nccl (RCCL)") if use_dist else None,
        "elapsed_spread": round(elapsed / elapsed_min, 4) if elapsed_min > 0 else None,
        "verification": {"all_ranks": all_ok, "aggregate_and_count": bool(verified), "verdicts": verdict_ok,
                         "prep_msgs_of_finished_reports": msgs_ok,
                         "rank_range": [start, stop], "note": "rank r holds global reports [r R, (r+1) R) of the "
                         "cyclic pool tiling; expected aggregates from the pool's block aggregates (CyclicPool); all_ranks = "
                         "every rank's own check (ranks_verified of rccl_world ranks), the other fields are rank 0's; "
                         "elapsed_spread = max / min per-rank timed seconds"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(orc, vdaf, vk, nonces, ps, his, lps, args.cpu_seconds, cpu["threads"])
        out["cpu_baseline"].update(cpu)
    eng.close()
    del d_n, d_ps, d_his, d_lps, d_verdicts, d_msgs
    if combiner is not None:
        del combiner
    torch.cuda.empty_cache()
    if world == 1 and args.secondary:
        t_sec = time.perf_counter()
        out["secondary"] = secondary_configs(cpu, threads)
        out["secondary_seconds"] = round(time.perf_counter() - t_sec, 1)
        out["verified_all_configs"] = bool(out["verified"] and all(v["verified"] for v in out["secondary"].values()))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


def secondary_configs(cpu: dict, threads: int) -> dict:
    """The other BASELINE.json configs, measured after the headline with the SumVec engine freed
    (tools/bench_configs.py, tools/bench_fixedpoint.py): Prio3Count at 100k
    reports (configs[0]), Prio3Sum bits=32 at 1M (configs[1]), Prio3Histogram 256/16 at 1M (configs[2]),
    Prio3FixedPointBoundedL2VecSum 16-bit x 10000 leader+helper ping-pong (configs[4]: two 40,960-report
    jobs in flight, and one job at a time). Each entry: reports/s, kernel ms, the issue-roofline
    fraction of its dominant kernel (prio3_work), a CPU baseline at 1 and N threads, and verification
    against the oracle (verdicts, prep messages of finished reports, aggregate and count)."""
    from janus_amd.vdaf import Prio3
    from tools import bench_configs as BC
    from tools import bench_fixedpoint as BF

    t0 = time.perf_counter()
    sec = {}
    specs = [
        # timed steps: Count's 100k-report call takes ~0.13 ms, so 200 of them (~30 ms) get above timer noise
        ("configs[0]", "Prio3Count (configs[0]: 100k reports)", Prio3.count(),
         lambda rng, K: rng.integers(0, 2, size=(K, 1), dtype=np.uint64), 100_000, 200),
        ("configs[1]", "Prio3Sum bits=32 (configs[1])", Prio3.sum(32),
         lambda rng, K: rng.integers(0, 1 << 32, size=(K, 1), dtype=np.uint64), 1_000_000, 10),
        ("configs[2]", "Prio3Histogram length=256 chunk_length=16 (configs[2])", Prio3.histogram(256, 16),
         lambda rng, K: rng.integers(0, 256, size=(K, 1), dtype=np.uint64), 1_000_000, 10),
    ]
    for key, name, v, fn, R, nsteps in specs:
        t = time.perf_counter()
        r = BC.run(name, v, fn, R, 4096, nsteps, 1, 3.0, threads, cpu)
        r["roofline"] = issue_roofline(v, "helper", R, r["kernels"])
        if key in CONFIG_PMC_SUMMARIES:  # each stage's own PMC-counted issue rate (K1 and K3)
            kk = r["kernels"]
            r["k1_roofline"] = stage_roofline(CONFIG_PMC_SUMMARIES[key], "jx::xof", kk["k1_ms_per_launch"],
                                              kk["reports_per_launch"], "K1 (XOF)")
            r["k3_roofline"] = stage_roofline(CONFIG_PMC_SUMMARIES[key], "jx::flp", kk["k3_ms_per_launch"],
                                              kk["reports_per_launch"], "K3 (FLP)")
        r["driver_seconds"] = round(time.perf_counter() - t, 1)
        sec[key] = r
        log(f"{key}: {r['value']:.0f} reports/s verified={r['verified']} ({r['driver_seconds']} s)")
    t = time.perf_counter()
    v = Prio3.fixedpoint_boundedl2_vec_sum(16, 10000)
    fp = BF.run(16, 10000, reports=40960, pool=48, steps=3, warmup=1, cpu_seconds=6.0,
                skip=("helper", "leader"))
    fp["serial"] = {"reports_per_s": fp.pop("value"), "ms_per_step": fp.pop("ms_per_step"),
                    "kernels": fp.pop("kernels"), "role_ms_per_step": fp.pop("role_ms_per_step")}
    fp["value"] = fp["pipelined"]["reports_per_s"]
    fp["value_note"] = "two 40,960-report aggregation jobs in flight (leader init of job i beside the helper of " \
                       "job i-1); 'serial' = one job at a time through leader init, helper, leader finish"
    fp["roofline"] = issue_roofline(v, "helper", 40960, {"k1_ms_per_launch": fp["pipelined"]["kernels"]["helper"]["xof"]},
                                    kernel="K1 helper xof_lanes_kernel (two-jobs shape)")
    fp["roofline_leader"] = issue_roofline(v, "leader", 40960,
                                           {"k1_ms_per_launch": fp["pipelined"]["kernels"]["leader"]["xof"]},
                                           kernel="K1 leader xof_leader_kernel (two-jobs shape)")
    fp["driver_seconds"] = round(time.perf_counter() - t, 1)
    sec["configs[4]"] = fp
    sec["jobs"] = job_granularity(threads)
    log(f"configs[4]: {fp['value']:.0f} reports/s (two jobs), verified={fp['verified']} ({fp['driver_seconds']} s); "
        f"secondary configs {time.perf_counter() - t0:.1f} s")
    return sec


def job_granularity(threads: int) -> dict:
    """The headline VDAF at Janus's aggregation-job size: native threads submit 100-report
    SumVec 8x1000/88 jobs to ONE engine through the host-buffer ABI (jx_helper_prep_batch -> jx_accumulate per
    job; tools/jobs_driver.cpp in a child process), with the device coalescer on and off; every job's verdicts
    and prep messages and the final aggregate verified against the oracle (tools/bench_jobs.py). Two shapes:
    64 threads (value), and 10 = max_concurrent_job_workers of the reference's sample job driver
    (docs/samples/basic_config/aggregation_job_driver.yaml:16)."""
    import tempfile

    from janus_amd.vdaf import Prio3
    from tools import bench_jobs as BJ

    t = time.perf_counter()
    v = Prio3.sum_vec(8, 1000, 88)
    vk = bytes(range(16))
    pool = BJ.make_pool(v, vk, 2048, threads)
    # the same jobs from HPKE-sealed report shares (1,024 of the pool; 2 % corrupted ciphertexts, 1 % unknown config)
    K = 1024
    sub = tuple(a[:K] for a in pool[:4]) + ({k: x[:K] for k, x in pool[4].items() if isinstance(x, np.ndarray)},)
    epool, enc = BJ.make_enc_pool(v, sub)
    BJ.build_driver()
    keys = ("reports_per_s", "prep_ms_p50", "prep_ms_p99", "jobs", "jobs_per_launch", "device_ms", "verified", "error")
    shapes = {}
    with tempfile.TemporaryDirectory() as tmp:
        for T in (64, 10):
            shapes[T] = {}
            for mode in ("coalesce", "direct"):
                r = BJ.run_case_cpp(v, vk, pool, 100, T, 2.0, mode, 0, tmp)
                shapes[T][mode] = {k: r.get(k) for k in keys if k in r}
            r = BJ.run_case_cpp(v, vk, epool, 100, T, 2.0, "coalesce", 0, tmp, enc=enc)
            shapes[T]["encrypted"] = {k: r.get(k) for k in keys if k in r}
            base = shapes[T]["coalesce"].get("reports_per_s") or 0
            shapes[T]["encrypted"]["ratio_to_prepare_only"] = \
                round((r.get("reports_per_s") or 0) / base, 3) if base else None
    ok = all(x.get("verified") for sh in shapes.values() for x in sh.values())
    res = {"metric": "helper reports/sec at Janus's job size: 100-report Prio3SumVec 8x1000/88 jobs from 64 threads on "
                     "one engine (prep_init+prep_next+aggregate per job)",
           "value": shapes[64]["coalesce"].get("reports_per_s"), "unit": "reports/s", "coalesced": shapes[64]["coalesce"],
           "one_call_at_a_time": shapes[64]["direct"],
           "encrypted": shapes[64]["encrypted"],
           "ten_workers": {"threads": 10, "coalesced": shapes[10]["coalesce"], "one_call_at_a_time": shapes[10]["direct"],
                           "encrypted": shapes[10]["encrypted"]},
           "encrypted_note": "the same jobs from HPKE-sealed report shares (jx_helper_prep_encrypted_batch: X25519 "
                             "decap, key schedule, AES-128-GCM open, PlaintextInputShare decode inside the coalesced "
                             "launch; 2 % corrupted ciphertexts, 1 % unknown config ids), every job's verdicts, prep "
                             "messages and open statuses and the aggregate verified",
           "verified": ok, "driver_seconds": round(time.perf_counter() - t, 1)}
    log(f"jobs: 64 threads coalesced {res['value']} reports/s (one call at a time {shapes[64]['direct'].get('reports_per_s')}, "
        f"encrypted {shapes[64]['encrypted'].get('reports_per_s')}); 10 threads {shapes[10]['coalesce'].get('reports_per_s')} "
        f"/ {shapes[10]['direct'].get('reports_per_s')} / encrypted {shapes[10]['encrypted'].get('reports_per_s')}; "
        f"verified={ok} ({res['driver_seconds']} s)")
    return res


def issue_roofline(v, role: str, reports: int, kernels: dict, kernel: str | None = None) -> dict:
    """Instruction-issue fraction of the dominant kernel of one launch of `reports` reports, from the
    prio3_work model and the HIP-event kernel time."""
    w = prio3_work(v, role)
    k1 = kernels.get("k1_ms_per_launch") or 0.0
    k3 = kernels.get("k3_ms_per_launch") or 0.0
    reports = min(reports, kernels.get("reports_per_launch", reports))
    k1_dom = k1 >= k3
    ms = k1 if k1_dom else k3
    ops = w["ops_k1"] if k1_dom else w["ops_k3"]
    ach = ops * reports / (ms * 1e-3) / 1e12 if ms else 0.0
    return {"bound": "valu", "kernel": kernel or ("K1 (XOF)" if k1_dom else "K3 (FLP)"), "achieved": round(ach, 3),
            "peak": round(VALU_PEAK_TOPS, 2), "unit": "TOP/s int32 instruction issue (model: bench.py prio3_work)",
            "frac": round(ach / VALU_PEAK_TOPS, 4), "ms_per_launch": ms, "reports_per_launch": reports,
            "ops_per_report": ops}


if __name__ == "__main__":
    main()
