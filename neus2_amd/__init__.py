"""neus2_amd — MI355X (gfx950) NeuS2 training hot path.

Product path: libneus2_hip.so (hand-written HIP kernels + C++ Testbed + C-ABI, include/neus2_hip.h),
driven through the pyngp mirror in neus2_amd.pyngp. There is no CPU fallback.
"""
from . import config, pyngp, scenes  # noqa: F401
from ._lib import LIB_PATH, NeusError, lib  # noqa: F401

__all__ = ["config", "scenes", "lib", "LIB_PATH", "NeusError", "pyngp"]
