"""Build the gfx950 engine library in-tree: janus_amd/lib/libjanus_prio3.so.

hipcc cross-compiles for gfx950 without a GPU. Run: ``python -m janus_amd.build``.
"""
from __future__ import annotations

import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = [os.path.join(_HERE, "csrc", f) for f in ("jx_kernels.hip", "jx_engine.cpp", "jx_arena.cpp", "jx_coalesce.cpp",
                                                  "jx_hpke.hip", "jx_mp64.hip")]
HEADERS = [os.path.join(_HERE, "csrc", f) for f in ("jx_field.h", "jx_keccak.h", "jx_sha256.h", "jx_kernels.h",
                                                  "jx_hpke.h", "jx_sha_aes.h", "jx_engine_internal.h")]
OUT = os.path.join(_HERE, "lib", "libjanus_prio3.so")
# jx_mp64.hip: keep the LDS for the AES table (the AMDGPU backend would otherwise move a small private
# array of the out-of-line helpers into LDS, +16 KiB per workgroup, one workgroup less per CU)
EXTRA_FLAGS = {"jx_mp64.hip": ["-mllvm", "-disable-promote-alloca-to-lds"]}
ARCH = os.environ.get("JX_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SOURCES + HEADERS + [os.path.join(_HERE, "..", "include", h) for h in ("jx_prio3.h", "jx_hpke.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    """Build the library (measurement variants live in tools/kernel_probe.hip, not here)."""
    out = OUT
    if not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    # compile the translation units in parallel
    procs = []
    for src in SOURCES:
        obj = os.path.join(os.path.dirname(out), os.path.basename(src) + ".o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-x", "hip", "-c", src, "-o", obj]
        cmd += EXTRA_FLAGS.get(os.path.basename(src), [])
        procs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), cmd))
        objs.append(obj)
    for p, cmd in procs:
        log, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(log.decode())
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}")
        if verbose and log:
            sys.stderr.write(log.decode())
    tmp = f"{out}.{os.getpid()}.tmp"  # link aside, then rename: a reader never sees a partial library
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    for o in objs:
        os.remove(o)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
