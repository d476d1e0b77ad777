"""janus_amd — MI355X-native batched Prio3 helper prepare + aggregate for Janus.

The one hot path of cjpatton/janus (helper aggregate-init: prio `helper_initialized` +
`evaluate` per report, then batch accumulation) as hand-written gfx950 HIP kernels behind
the C ABI in include/jx_prio3.h. See DESIGN.md.
"""
from .vdaf import Prio3  # noqa: F401

__all__ = ["Prio3", "HelperEngine"]


def __getattr__(name):
    if name == "HelperEngine":
        from .engine import HelperEngine
        return HelperEngine
    raise AttributeError(name)
