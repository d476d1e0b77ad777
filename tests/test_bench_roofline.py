"""bench.py's roofline bookkeeping on the CPU: the Keccak instruction-mix ceiling, and the PMC
summary it reads being refused when it was taken on other kernel sources."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_keccak_mix_ceiling():
    # 190 instructions per round at the measured per-instruction rates
    n = sum(c for c, _ in bench.KECCAK_ROUND_MIX.values())
    assert n == 190 == bench.OPS_PER_PERM // 12
    assert abs(bench.keccak_mix_ceiling_tops() - 52.11) < 0.05
    assert bench.keccak_mix_ceiling_tops() < bench.VALU_PEAK_TOPS


def test_pmc_summary_refused_on_other_sources(tmp_path, monkeypatch):
    summary = {"workload": {"reports_per_launch": 1000, "sources_digest": "not-these-sources"},
               "kernels": {"jx::xof_kernel<0, false>": {"hbm_read_bytes": 1e9, "hbm_write_bytes": 1e9,
                                                       "clock_GHz": 2.1}}}
    p = tmp_path / "s.json"
    p.write_text(json.dumps(summary))
    monkeypatch.setattr(bench, "PMC_SUMMARY", str(p))
    traffic, _, note = bench.pmc_traffic("jx::xof_kernel<0, false>", 500)
    assert traffic is None and "other kernel sources" in note
    assert bench.pmc_clock("jx::xof_kernel<0, false>") is None
    summary["workload"]["sources_digest"] = bench.sources_digest()
    p.write_text(json.dumps(summary))
    traffic, _, _ = bench.pmc_traffic("jx::xof_kernel<0, false>", 500)
    assert traffic == 1_000_000_000  # 2e9 bytes over 1000 reports, scaled to 500
    assert bench.pmc_clock("jx::xof_kernel<0, false>") == 2.1


def test_prio3_work_matches_sumvec_model_and_roofline_picks_dominant():
    from janus_amd.vdaf import Prio3

    g, s = bench.prio3_work(Prio3.sum_vec(8, 1000, 88)), bench.sumvec_work(8, 1000, 88)
    assert g["perms"] == s["perms"] and abs(g["ops_k1"] - s["ops_k1"]) / s["ops_k1"] < 0.01
    fp_h, fp_l = bench.prio3_work(Prio3.fixedpoint_boundedl2_vec_sum(16, 10000)), \
        bench.prio3_work(Prio3.fixedpoint_boundedl2_vec_sum(16, 10000), "leader")
    assert 30000 < fp_h["perms"] < 31000 and 15000 < fp_l["perms"] < 16000  # two sponges vs the absorb only
    r = bench.issue_roofline(Prio3.sum(32), "helper", 1000, {"k1_ms_per_launch": 1.0, "k3_ms_per_launch": 2.0})
    assert r["kernel"] == "K3 (FLP)" and 0 < r["frac"] < 1
    r = bench.issue_roofline(Prio3.count(), "helper", 1000, {"k1_ms_per_launch": 1.0, "k3_ms_per_launch": 0.0})
    assert r["kernel"] == "K1 (XOF)"
    json.dumps(r)  # the bench line is JSON


def test_pmc_kernel_instruction_count_only_on_these_sources(tmp_path, monkeypatch):
    """roofline.frac takes K1's instructions per report from the committed PMC summary only when that
    summary was taken on these kernel sources (bench.pmc_kernel)."""
    k = bench.K1_KERNEL
    summary = {"workload": {"reports_per_launch": 262144, "sources_digest": "other"},
               "kernels": {k: {"avg_ns": 26.0e6, "pmc": {"SQ_INSTS_VALU": 16.0e9}}}}
    p = tmp_path / "s.json"
    p.write_text(json.dumps(summary))
    monkeypatch.setattr(bench, "PMC_SUMMARY", str(p))
    assert bench.pmc_kernel(k) == (None, None)
    summary["workload"]["sources_digest"] = bench.sources_digest()
    p.write_text(json.dumps(summary))
    ent, rpl = bench.pmc_kernel(k)
    assert rpl == 262144 and ent["pmc"]["SQ_INSTS_VALU"] == 16.0e9
    # the PMC run's own issue fraction: instructions x 64 lanes / duration / 78.6 T
    frac = ent["pmc"]["SQ_INSTS_VALU"] * 64 / (ent["avg_ns"] * 1e-9) / 1e12 / bench.VALU_PEAK_TOPS
    assert 0.4 < frac < 0.6
