#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / scratch / occupancy of a HIP source for gfx950 (compiler remarks).

    python tools/kernel_resources.py janus_amd/csrc/jx_kernels.hip [name-filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip", "-c", src,
                      "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
dem = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.splitlines()
for (k, v), d in zip(rows.items(), dem):
    if flt in d:
        print(f"{d[:70]:70s} vgpr {v.get('VGPRs', '?'):>4} agpr {v.get('AGPRs', '?'):>4} "
              f"scratch {v.get('ScratchSize', '?'):>5} occ {v.get('Occupancy', '?')}")
