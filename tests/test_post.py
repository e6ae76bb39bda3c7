"""CPU tests of the post-SVAO image passes: the ImageEquation formula
compiler of librsd (host-only entry points, no GPU needed) and the oracles' own sanity."""
import ctypes as C

import numpy as np
import pytest

F = np.float32

REFERENCE_FORMULAS = ["I0[xy].rrra", "I0[xy].r * I1[xy]", "I0[xy].xxxx", "I0[xy].gggg",
                      "1.0 - max(I0[xy].x-I0[xy].y, 0.05)", "I0[xy]", "I0[xy]/1000.0"]  # scripts/*.py


def _compile(abi, formula):
    h = C.c_void_p()
    st = abi.lib().rsd_image_equation_compile(formula.encode(), C.byref(h))
    return st, h


@pytest.mark.parametrize("formula", REFERENCE_FORMULAS + [
    "saturate(I0[xy] * 2.0f - 0.5)", "float4(I0[xy].rgb, 1.0)", "lerp(I0[xy], I1[xy], 0.25)",
    "dot(I0[xy].xyz, I1[xy].xyz)", "pow(abs(I2[xy]), 2.2) + -I3[xy]", "clamp(I0[xy], 0.1, 0.9).wzyx",
    "float4(float2(I0[xy].x, 1), I1[xy].xy)", "step(0.5, I0[xy].r)", "exp2(-I0[xy].r * I0[xy].r)"])
def test_formulas_compile(formula):
    from rsd import abi
    st, h = _compile(abi, formula)
    assert st == abi.RSD_OK, abi.lib().rsd_last_error()
    n, mask = C.c_uint32(), C.c_uint32()
    assert abi.lib().rsd_image_equation_info(h, C.byref(n), C.byref(mask)) == abi.RSD_OK
    assert 1 <= n.value <= 64
    assert mask.value == sum(1 << k for k in range(4) if f"I{k}[" in formula)
    abi.lib().rsd_image_equation_release(h)


@pytest.mark.parametrize("formula,why", [
    ("I0[xy].rgb", "result must be a scalar or a float4"), ("I4[xy]", "unknown identifier"),
    ("I0[uv]", "indexed by [xy]"), ("I0[xy].q", "bad swizzle"), ("max(I0[xy])", "takes 2 arguments"),
    ("(I0[xy]", "expected ')'"), ("I0[xy] +", "unexpected end"), ("I0[xy].x.y", "past the value's width"),
    ("float4(I0[xy].xy, 1.0)", "do not add up"), ("I0[xy] $ 2", "trailing")])
def test_formula_errors(formula, why):
    from rsd import abi
    st, h = _compile(abi, formula)
    assert abi.STATUS_NAMES[st] == "RSD_ERR_INVALID_ARG" and not h.value
    assert why in abi.lib().rsd_last_error().decode()


def test_image_eq_oracle_semantics():
    from oracle import image_eq as IE
    H, W = 3, 5
    a = np.arange(H * W, dtype=np.uint8).reshape(H, W) * 17
    rgba = np.random.default_rng(0).random((H, W, 4)).astype(F)
    r = IE.evaluate("I0[xy].rrra", [(a, IE.FMT_R8UNORM), (None, 0), (None, 0), (None, 0)], W, H)
    v = a.astype(F) / F(255)
    assert np.array_equal(r[..., 0], v) and np.array_equal(r[..., 2], v) and (r[..., 3] == 1).all()
    r = IE.evaluate("I0[xy].r * I1[xy]", [(a, IE.FMT_R8UNORM), (rgba, IE.FMT_RGBA32F), (None, 0), (None, 0)], W, H)
    assert np.array_equal(r, v[..., None] * rgba)
    # unbound inputs read 0, a smaller input reads 0 outside its extent
    r = IE.evaluate("I2[xy] + I1[xy]", [(None, 0), (rgba[:2, :3], IE.FMT_RGBA32F), (None, 0), (None, 0)], W, H)
    assert np.array_equal(r[:2, :3], rgba[:2, :3]) and (r[2:] == 0).all() and (r[:, 3:] == 0).all()
    out = IE.store(np.full((1, 1, 4), F(0.5)), IE.FMT_R8UNORM)
    assert out[0, 0] == 128


def test_blur_oracle_properties(oracle):
    """A constant image stays constant (the weights are normalised); pixels outside the guard
    band are not written; a depth edge stops the blur."""
    H, W, g = 40, 56, 6
    z = np.full((H, W), 5.0, F)
    src = np.full((H, W), 100, np.uint8)
    out, _ = oracle.cross_bilateral_blur(src, z, g)
    assert (out[g:-g, g:-g] == 100).all() and (out[:g] == 0).all() and (out[:, -g:] == 0).all()
    src = np.zeros((H, W), np.uint8)
    src[:, W // 2:] = 255
    z[:, W // 2:] = 50.0  # the bright half is far behind: no bleeding across the edge
    out, _ = oracle.cross_bilateral_blur(src, z, g)
    assert (out[g:-g, g:W // 2 - 1] == 0).all() and (out[g:-g, W // 2 + 1:-g] == 255).all()
    z[:] = 5.0  # same depth: the edge is smoothed
    out, _ = oracle.cross_bilateral_blur(src, z, g)
    assert 0 < out[H // 2, W // 2 - 1] < 255
