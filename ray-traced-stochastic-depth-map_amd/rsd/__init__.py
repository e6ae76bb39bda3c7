"""rsd -- Python host binding of librsd, the MI355X-native Ray-SD + SVAO hot path.

    abi     ctypes mirror of include/rsd.h (the drop-in C ABI)
    scenes  seeded procedural stand-ins for the reference's benchmark scenes
    frame   one-GPU frame driver issuing SVAO::execute's dispatch sequence
"""
from . import abi, scenes  # noqa: F401
from .frame import CONFIGS, FrameConfig, Renderer  # noqa: F401
