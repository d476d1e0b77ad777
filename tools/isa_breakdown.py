#!/usr/bin/env python3
"""Static ISA breakdown of one kernel's hot loop and tail (gfx950 assembly from hipcc -S).

For the K3 ring kernel (flp_psum_part_glds_kernel) the hot loop is the one holding the s_barrier; its
body is one call (one coefficient pair, PPW measurement elements). The once-every-512-calls column
normalisation sits inside the loop behind a branch: its instructions (the run of v_lshrrev_b64 26 /
v_lshl_add_u64 / v_and / v_mov that ends the loop body) are reported apart, so `per_call` is what a call
executes. Everything after the loop is the group finish (`tail`, static: its inner loops are counted
once).

    python tools/isa_breakdown.py [kernel-substring] > profiles/r04_k3_isa_breakdown.json
"""
from __future__ import annotations

import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "janus_amd", "csrc", "jx_kernels.hip")


def asm() -> list[str]:
    out = "/tmp/_isa_breakdown.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip",
                    "--cuda-device-only", "-S", SRC, "-o", out], check=True, capture_output=True)
    return open(out).read().split("\n")


def ops(lines):
    body = [x.strip() for x in lines if x.strip() and not x.strip().startswith((".", ";"))]
    return collections.Counter(x.split()[0] for x in body)


def summary(c: collections.Counter) -> dict:
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    return {"valu": valu, "v_mad_u64_u32": c.get("v_mad_u64_u32", 0),
            "lds_reads": sum(v for k, v in c.items() if k.startswith("ds_read")),
            "global_load_lds": sum(v for k, v in c.items() if k.startswith("global_load_lds")),
            "global_loads": sum(v for k, v in c.items() if k.startswith("global_load") and "lds" not in k),
            "scratch": sum(v for k, v in c.items() if k.startswith("scratch_")),
            "top": dict(c.most_common(12))}


def main():
    want = sys.argv[1] if len(sys.argv) > 1 else "flp_psum_part_glds_kernelILi2ELb0ELb0E"
    s = asm()
    start = next(i for i, l in enumerate(s) if re.match(r"^_Z\S*%s\S*:" % re.escape(want), l))
    end = next(i for i in range(start, len(s)) if s[i].strip().startswith(".Lfunc_end"))
    body = s[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    bar = next(i for i, l in enumerate(body) if "s_barrier" in l)
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_(?:c)?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and labels.get(m.group(1), 1 << 30) <= bar < i:
            loops.append((labels[m.group(1)], i))
    lo, hi = min(loops, key=lambda t: t[1] - t[0])  # the innermost loop around the barrier
    loop = body[lo:hi + 1]
    # the normalisation block: from the first 64-bit shift by 26 to the end of the loop body
    norm_at = next((i for i, l in enumerate(loop) if re.search(r"v_lshrrev_b64 \S+, 26,", l)), len(loop))
    hot, norm = loop[:norm_at], loop[norm_at:]
    tail = body[hi + 1:]
    out = {"kernel": body[0].rstrip(":"), "source": os.path.relpath(SRC, ROOT),
           "per_call": summary(ops(hot)), "normalize_every_512_calls": summary(ops(norm)),
           "tail_static": summary(ops(tail)),
           "note": "static counts from hipcc -S (gfx950); per_call = one iteration of the ring loop without the "
                   "rarely-taken normalisation block; tail_static counts each inner loop of the group finish once"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
