"""CPU: the trace analysis tools behind DESIGN.md §5.5 and §7.3 (tools/launch_anatomy.py, tools/stream_gaps.py)
on small synthetic rocprofv3 CSVs with known answers."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KHDR = "Kernel_Name,Start_Timestamp,End_Timestamp,Stream_Id\n"
CHDR = "Kind,Direction,Stream_Id,Start_Timestamp,End_Timestamp\n"


def _run(tool, *args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool), *args], capture_output=True, text=True,
                         check=True)
    return json.loads(out.stdout)


def test_launch_anatomy_phases(tmp_path):
    """Two launches on one lane stream: upload = first H2D -> K1 start, tail = K1 end -> scatter end, down =
    scatter end -> last D2H end, turn = the next launch's first H2D - the previous launch's last D2H end."""
    k = tmp_path / "k.csv"
    c = tmp_path / "c.csv"
    ms = 1_000_000
    k.write_text(KHDR + "".join([
        f"jx::xof_pairs_kernel<true>(x),{1 * ms},{5 * ms},2\n",
        f"jx::flp_psum_final_kernel(x),{5 * ms},{5 * ms + ms // 5},2\n",
        f"jx::scatter_jobs_kernel(x),{5 * ms + ms // 5},{5 * ms + ms // 4},2\n",
        f"jx::xof_pairs_kernel<true>(x),{8 * ms},{12 * ms},2\n",
        f"jx::scatter_jobs_kernel(x),{12 * ms},{12 * ms + ms // 2},2\n",
    ]))
    c.write_text(CHDR + "".join([
        f"MEMORY_COPY,MEMORY_COPY_HOST_TO_DEVICE,2,{ms // 2},{ms // 2 + 10}\n",
        f"MEMORY_COPY,MEMORY_COPY_DEVICE_TO_HOST,2,{5 * ms + ms // 4},{5 * ms + ms // 2}\n",
        f"MEMORY_COPY,MEMORY_COPY_HOST_TO_DEVICE,2,{7 * ms},{7 * ms + 10}\n",
        f"MEMORY_COPY,MEMORY_COPY_DEVICE_TO_HOST,2,{12 * ms + ms // 2},{13 * ms}\n",
    ]))
    d = _run("launch_anatomy.py", str(k), "--copies", str(c))
    assert d["launches"] == 2
    assert d["k1"]["mean_ms"] == 4.0
    assert abs(d["tail"]["mean_ms"] - (0.25 + 0.5) / 2) < 1e-9
    assert abs(d["upload"]["mean_ms"] - (0.5 + 1.0) / 2) < 1e-9
    assert abs(d["down"]["mean_ms"] - (0.25 + 0.5) / 2) < 1e-9
    assert d["turn"]["n"] == 1 and abs(d["turn"]["mean_ms"] - 1.5) < 1e-9


def test_stream_gaps_and_trim_attribution(tmp_path):
    """Per-stream gaps over 1 ms, which of them overlap a hipFree interval of the trim log, and how many kernels
    each stream started while a free ran."""
    k = tmp_path / "k.csv"
    ms = 1_000_000
    base = 10_000 * ms
    rows = []
    for i in range(25):  # stream 1: back to back, one 3 ms hole at 10 ms
        t = base + i * ms + (3 * ms if i >= 10 else 0)
        rows.append(f"a(x),{t},{t + ms},1\n")
    for i in range(40):  # stream 2: keeps launching every 0.5 ms
        t = base + i * ms // 2
        rows.append(f"b(x),{t},{t + ms // 4},2\n")
    k.write_text(KHDR + "".join(rows))
    trims = tmp_path / "t.log"
    # the free covers stream 1's hole; the boottime column is off the trace's clock
    trims.write_text(f"monotonic {base + 10 * ms} {base + 12 * ms} boottime 5 6 1048576 100\n")
    d = _run("stream_gaps.py", str(k), "--trims", str(trims))
    assert d["trims"] == 1 and d["trim_clock"] == "monotonic"
    s1, s2 = d["streams"]["1"], d["streams"]["2"]
    assert s1["gaps_over_1ms"] == 1 and s1["gaps_over_1ms_overlapping_a_trim"] == 1
    assert abs(s1["max_gap_ms"] - 3.0) < 1e-9
    assert s2["gaps_over_1ms"] == 0 and s2["kernels_started_during_a_free"] == 5
    assert s1["longest"][0]["overlapping_trims_ms"] == [2.0]
