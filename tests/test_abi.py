"""The C-ABI library loads and exports every symbol include/jx_prio3.h declares (no GPU calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from janus_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols(header="jx_prio3.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|void|const char\*)\s+(jx_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        from janus_amd import build
        build.build()
    return _lib.load()


def test_header_lists_match(lib):
    assert header_symbols() == sorted(_lib.EXPORTED_SYMBOLS)


def test_all_symbols_exported(lib):
    from janus_amd import hpke
    assert header_symbols("jx_hpke.h") == sorted(hpke.EXPORTED_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (jx_\w+)", out))
    for header in ("jx_prio3.h", "jx_hpke.h"):
        missing = set(header_symbols(header)) - exported
        assert not missing, missing
        for s in header_symbols(header):
            assert getattr(lib, s) is not None


def test_status_strings(lib):
    assert lib.jx_status_str(0) == b"ok"
    assert lib.jx_status_str(-2) == b"unsupported Prio3 parameters"


def test_gpu_code_object_is_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle id of the embedded code object


def test_create_without_device_fails_loudly(lib):
    """No GPU in this container: engine creation must fail with an error, never fall back."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = _lib.JxParams(2, 8, 1000, 88, 1)
    h = ctypes.c_void_p()
    vk = (ctypes.c_uint8 * 16)()
    st = lib.jx_engine_create(ctypes.byref(p), ctypes.cast(vk, ctypes.c_void_p), 0, ctypes.byref(h))
    assert st != 0
    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3
    with pytest.raises(_lib.EngineError):
        HelperEngine(Prio3.sum_vec(8, 1000, 88), bytes(16))
