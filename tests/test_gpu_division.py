"""The exact unscaled division of pass 1 (svao_math.h div_unscaled / rcp_refined) against the GPU's IEEE
binary32 division, bit for bit, over 2^28 random operand pairs inside its precondition range
(tests/native/check_div_unscaled.hip, built by __graft_entry__.build())."""
import ctypes as C
from pathlib import Path

import pytest

LIB = Path(__file__).resolve().parent / "native" / "_build" / "libcheck_div.so"


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_div_unscaled_matches_ieee_division(seed):
    import torch
    assert torch.cuda.is_available()
    assert LIB.exists(), "tests/native/_build/libcheck_div.so missing: run __graft_entry__.build()"
    lib = C.CDLL(str(LIB))
    bad = C.c_ulonglong(0)
    ex = (C.c_uint32 * 4)()
    assert lib.check_div_unscaled(C.c_uint64(1 << 28), C.c_uint64(seed), C.byref(bad), ex) == 0
    assert bad.value == 0, f"{bad.value} mismatches, e.g. a, b, a/b, got = {[hex(x) for x in ex]}"
