import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "ray-traced-stochastic-depth-map_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

# The parity tests compare the SVAO passes with the oracle bit for bit: they run the exact numerics
# (rsd.h RSD_NUMERICS_EXACT).  The product default, fast numerics, is graded by tolerance in
# tests/test_gpu_numerics.py, which asks for it explicitly (FrameConfig(numerics="fast")).
os.environ.setdefault("RSD_NUMERICS", "exact")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librsd's HIP kernels)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O
