"""div_rcp (csrc/svao_math.h): the five-operation RN(a / b) from y = RN(1 / b) that replaces the
IEEE division by the per-direction constants pdf and sphereHeight in SVAO pass 1 / pass 2.  Checked
bit-for-bit against binary32 `/` by a C program (tests/native/check_div_rcp.c, same FMA steps):
the SVAO divisors at radius 0.2 / 0.5 and divisors across [2^-30, 2^30] (incl. all-ones and
power-of-two significands), over numerators spanning the precondition range.  The full
exhaustive run (all numerators in [2^-60, 2^31], 68 divisors) passed when div_rcp was added; the
GPU parity tests cover the kernels end to end."""
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

HERE = Path(__file__).resolve().parent


def _divisors():
    f = np.float32
    r8 = [0.917883, 0.564429, 0.734504, 0.359545, 0.820004, 0.470149, 0.650919, 0.205215]  # Common.slang:53
    out = []
    for R in (f(0.2), f(0.5)):
        for sr in r8:
            rad = f(sr) * R
            h = np.sqrt(f(R * R) - f(rad * rad))
            out += [h, f(2) * h]
    out += [f(np.ldexp(f(1.99999988), k)) for k in (-30, 0, 29)] + [f(2.0 ** k) for k in (-30, 0, 29)]
    return [repr(float(x)) for x in out]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_div_rcp_matches_ieee_division(tmp_path):
    exe = tmp_path / "check_div_rcp"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(HERE / "native" / "check_div_rcp.c"),
                    "-lm", "-lpthread"], check=True)
    # the lowest 3 binades of the precondition range, where residual exactness is tightest, plus
    # a sample binade of typical numerators, for every divisor
    for env in ({"LIMIT_BINADES": "3"}, {"LIMIT_BINADES": "2", "START_EXP": "-4"}):
        out = subprocess.run([str(exe)] + _divisors(), check=True, capture_output=True, text=True, env=env).stdout
        assert "total bad 0" in out, (env, out)
