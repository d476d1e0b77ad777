#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel-trace stats + PMC passes) into one JSON per run.

    python tools/prof_summary.py <prof_dir> [--reports-per-launch N] > profiles/<name>.json

<prof_dir> holds `trace/run_kernel_stats.csv` and any `pmc_*/run_counter_collection.csv`.
Derived per kernel (MI355X_MICROARCH.md, HBM/rocprofv3 section):
  hbm_read_bytes  = 2 x FETCH_SIZE x 1024  (FETCH_SIZE is in KiB and counts half the bytes of
                    wide coalesced reads on gfx950)
  hbm_write_bytes = WRITE_SIZE x 1024
  clock_GHz       = GRBM_GUI_ACTIVE / 8 XCDs / duration
  valu_util       = SQ_INSTS_VALU / (256 CU x 4 SIMD x cycles / 2)  (wave64 VALU op = 2 cycles on a SIMD-32)
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import sys


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--reports-per-launch", type=int, default=0)
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    out = {"workload": {"reports_per_launch": a.reports_per_launch, "sources_digest": bench.sources_digest(),
                        "command": a.command,
                        "counters": "separate rocprofv3 --pmc passes; hbm_read_bytes = 2 x FETCH_SIZE x 1024 "
                                    "(gfx950 correction), hbm_write_bytes = WRITE_SIZE x 1024"},
           "kernels": {}}
    stats = os.path.join(a.prof_dir, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            out["kernels"].setdefault(short(r["Name"]), {}).update(
                calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), total_ns=float(r["TotalDurationNs"]),
                pct=float(r["Percentage"]))
    for f in sorted(glob.glob(os.path.join(a.prof_dir, "pmc_*", "run_counter_collection.csv"))):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        n = collections.Counter()
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            acc[k]["_vgpr"] = float(r["VGPR_Count"])
            acc[k]["_scratch"] = float(r["Scratch_Size"])
            n[(k, r["Counter_Name"])] += 1
        for k, d in acc.items():
            ent = out["kernels"].setdefault(k, {})
            for c, v in d.items():
                if c.startswith("_"):
                    ent[c[1:]] = v
                else:
                    ent.setdefault("pmc", {})[c] = v / max(1, n[(k, c)])  # per dispatch
    for k, e in out["kernels"].items():
        p = e.get("pmc", {})
        dur = e.get("avg_ns")
        if "FETCH_SIZE" in p:
            e["hbm_read_bytes"] = 2 * p["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in p:
            e["hbm_write_bytes"] = p["WRITE_SIZE"] * 1024
        if dur and "GRBM_GUI_ACTIVE" in p:
            cyc = p["GRBM_GUI_ACTIVE"] / 8
            e["clock_GHz"] = cyc / dur
            if "SQ_INSTS_VALU" in p:
                e["valu_util"] = p["SQ_INSTS_VALU"] / (256 * 4 * cyc / 2)
        if a.reports_per_launch and "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes_per_report"] = (e["hbm_read_bytes"] + e["hbm_write_bytes"]) / a.reports_per_launch
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
