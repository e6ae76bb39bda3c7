"""GPU parity of the post-SVAO image passes through the C ABI:
rsd_cross_bilateral_blur vs oracle.cross_bilateral_blur, rsd_image_equation_run vs the
numpy restatement oracle/image_eq.py.  Bit-exact."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _stream(torch):
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("radius,better,guard", [(4, 1, 16), (1, 1, 0), (7, 0, 8), (20, 1, 3)])
def test_blur_parity(torch, oracle, radius, better, guard):
    from rsd import abi
    rng = np.random.default_rng(radius)
    H, W = 67, 131
    yy, xx = np.mgrid[0:H, 0:W]
    z = (5.0 + 3.0 * np.sin(xx / 9.0) + (xx > 70) * 20.0 + 0.01 * yy).astype(F)  # smooth + one depth edge
    src = rng.integers(0, 256, (H, W)).astype(np.uint8)
    dz, ds = torch.from_numpy(z).cuda(), torch.from_numpy(src).cuda()
    pp = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
    out = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
    st = abi.lib().rsd_cross_bilateral_blur(C.c_void_p(ds.data_ptr()), C.c_void_p(dz.data_ptr()), W, H,
                                            C.c_void_p(pp.data_ptr()), C.c_void_p(out.data_ptr()), W, H, guard,
                                            radius, better, _stream(torch))
    abi.check(st, "rsd_cross_bilateral_blur")
    torch.cuda.synchronize()
    want, _ = oracle.cross_bilateral_blur(src, z, guard, radius, bool(better))
    assert np.array_equal(out.cpu().numpy(), want)


FORMULAS = ["I0[xy].rrra", "I0[xy].r * I1[xy]", "I0[xy].xxxx", "I0[xy].gggg", "1.0 - max(I0[xy].x-I0[xy].y, 0.05)",
            "I0[xy]", "I0[xy]/1000.0", "saturate(I1[xy] * 2.0f - 0.5)", "float4(I1[xy].bgr, 1.0)",
            "lerp(I1[xy], I2[xy], 0.25)", "dot(I1[xy].xyz, I2[xy].xyz)", "pow(abs(I1[xy]), 2.2) + -I3[xy]",
            "clamp(I1[xy], 0.1, 0.9).wzyx", "float4(float2(I0[xy].x, 1), I2[xy].xy)", "step(0.5, I1[xy].r)",
            "exp2(-I1[xy].r * I2[xy].g) + sqrt(abs(I3[xy])) * frac(I1[xy] * 7.0)", "min(I1[xy], I2[xy]) / I3[xy]",
            "sin(I1[xy]) * cos(I2[xy].x) + log2(abs(I3[xy]) + 1.0)"]


@pytest.mark.parametrize("out_fmt", [2, 0, 5, 1])  # RGBA32F, R32F, R8Unorm, RG32F
def test_image_equation_parity(torch, out_fmt):
    from oracle import image_eq as IE
    from rsd import abi
    rng = np.random.default_rng(out_fmt)
    H, W = 37, 70
    imgs = [rng.integers(0, 256, (H, W)).astype(np.uint8),                     # R8Unorm
            (rng.random((H, W, 4)) * 3 - 1).astype(F),                         # RGBA32F
            rng.random((H - 5, W - 9, 2)).astype(F),                           # RG32F, smaller
            (rng.random((H, W)) * 4 - 2).astype(F)]                            # R32F
    fmts = [IE.FMT_R8UNORM, IE.FMT_RGBA32F, IE.FMT_RG32F, IE.FMT_R32F]
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in imgs]
    tex = (abi.Texture * 4)()
    for k, (a, t) in enumerate(zip(imgs, dev)):
        tex[k] = abi.Texture(t.data_ptr(), a.shape[1], a.shape[0], 1, fmts[k], t.numel() * t.element_size())
    ch = {2: 4, 1: 2, 0: 1, 5: 1}[out_fmt]
    dt = torch.uint8 if out_fmt == 5 else torch.float32
    for formula in FORMULAS:
        h = C.c_void_p()
        abi.check(abi.lib().rsd_image_equation_compile(formula.encode(), C.byref(h)), formula)
        out = torch.zeros((H, W, ch), dtype=dt, device="cuda")
        ot = abi.Texture(out.data_ptr(), W, H, 1, out_fmt, out.numel() * out.element_size())
        abi.check(abi.lib().rsd_image_equation_run(h, tex, C.byref(ot), _stream(torch)), formula)
        torch.cuda.synchronize()
        abi.lib().rsd_image_equation_release(h)
        want = IE.store(IE.evaluate(formula, list(zip(imgs, fmts)), W, H), out_fmt)
        got = out.cpu().numpy().reshape(want.shape)
        if got.dtype == np.uint8:
            assert np.array_equal(got, want), formula
        else:  # bit-exact, NaNs (of either sign / payload) compare equal
            nan = np.isnan(want)
            assert np.array_equal(np.isnan(got), nan), formula
            assert np.array_equal(got[~nan].view(np.uint32), want[~nan].view(np.uint32)), formula


def test_image_equation_ieee_special_values(torch):
    """Division by +-0, 0/0, inf/inf, inf - inf and 0 * inf: the kernel's IEEE binary32 results,
    pinned as bit patterns (not via numpy), and their R8Unorm stores (NaN -> 0, D3D11 3.2.3.6)."""
    from rsd import abi
    num = np.array([1.0, -1.0, 1.0, 0.0, np.inf, np.inf, 0.0, 2.0], F)
    den = np.array([0.0, 0.0, -0.0, 0.0, np.inf, -np.inf, np.inf, 4.0], F)
    want_div = np.array([0x7F800000, 0xFF800000, 0xFF800000, None, None, None, 0x00000000, 0x3F000000], object)
    want_sub = np.array([0x3F800000, 0xBF800000, 0x3F800000, 0x00000000, None, 0x7F800000, 0xFF800000,
                         0xC0000000], object)   # num - den
    want_mul = np.array([0x00000000, 0x80000000, 0x80000000, 0x00000000, 0x7F800000, 0xFF800000, None,
                         0x41000000], object)   # num * den
    W, H = 8, 1
    a = torch.from_numpy(num.reshape(H, W)).cuda()
    b = torch.from_numpy(den.reshape(H, W)).cuda()
    tex = (abi.Texture * 4)()
    tex[0] = abi.Texture(a.data_ptr(), W, H, 1, abi.FMT_R32F, a.numel() * 4)
    tex[1] = abi.Texture(b.data_ptr(), W, H, 1, abi.FMT_R32F, b.numel() * 4)
    for formula, want in (("I0[xy].r / I1[xy].r", want_div), ("I0[xy].r - I1[xy].r", want_sub), ("I0[xy].r * I1[xy].r", want_mul)):
        h = C.c_void_p()
        abi.check(abi.lib().rsd_image_equation_compile(formula.encode(), C.byref(h)), formula)
        out = torch.zeros((H, W), dtype=torch.float32, device="cuda")
        out8 = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
        ot = abi.Texture(out.data_ptr(), W, H, 1, abi.FMT_R32F, out.numel() * 4)
        ot8 = abi.Texture(out8.data_ptr(), W, H, 1, abi.FMT_R8UNORM, out8.numel())
        abi.check(abi.lib().rsd_image_equation_run(h, tex, C.byref(ot), _stream(torch)), formula)
        abi.check(abi.lib().rsd_image_equation_run(h, tex, C.byref(ot8), _stream(torch)), formula)
        torch.cuda.synchronize()
        abi.lib().rsd_image_equation_release(h)
        bits = out.cpu().numpy().reshape(-1).view(np.uint32)
        got8 = out8.cpu().numpy().reshape(-1)
        for k, w in enumerate(want):
            if w is None:  # NaN (any payload)
                assert np.isnan(bits[k:k + 1].view(F))[0], (formula, k, hex(bits[k]))
                assert got8[k] == 0, (formula, k)  # NaN -> 0 in a UNORM store
            else:
                assert bits[k] == w, (formula, k, hex(bits[k]), hex(w))
                v = np.array([w], np.uint32).view(F)[0]
                assert got8[k] == (255 if v >= 1 else 0 if not v > 0 else int(np.floor(v * 255 + 0.5))), (formula, k)


@pytest.mark.parametrize("shape,dtype", [((37, 70), np.float32), ((64, 40, 4), np.float32), ((21, 33), np.uint8),
                                         ((18, 18, 2), np.float32)])
def test_deinterleave_interleave_parity(torch, shape, dtype):
    from oracle.texops import deinterleave, interleave
    from rsd import abi
    rng = np.random.default_rng(sum(shape))
    a = (rng.random(shape) * 255).astype(dtype)
    H, W = shape[:2]
    texel = a.itemsize * (shape[2] if len(shape) == 3 else 1)
    src = torch.from_numpy(a).cuda()
    want = deinterleave(a)
    dst = torch.full(want.shape, 7, dtype=src.dtype, device="cuda")
    abi.check(abi.lib().rsd_deinterleave(C.c_void_p(src.data_ptr()), W, H, texel, C.c_void_p(dst.data_ptr()),
                                         _stream(torch)), "rsd_deinterleave")
    back = torch.full_like(src, 9)
    abi.check(abi.lib().rsd_interleave(C.c_void_p(dst.data_ptr()), W, H, texel, C.c_void_p(back.data_ptr()),
                                       _stream(torch)), "rsd_interleave")
    torch.cuda.synchronize()
    assert np.array_equal(dst.cpu().numpy(), want)
    assert np.array_equal(back.cpu().numpy(), interleave(want, H, W))
    assert np.array_equal(back.cpu().numpy(), a)


def test_ray_min_max_length_parity(torch):
    """rsd_ray_min_max_length over random interval words plus the special cases: rayMax == 0,
    inverted intervals, +-inf and NaN bit patterns."""
    from oracle.texops import ray_min_max_length
    from rsd import abi
    rng = np.random.default_rng(5)
    H, W = 45, 77
    mn = (rng.random((H, W)) * 50).astype(F)
    mx = (mn + (rng.random((H, W)) * 10 - 2)).astype(F)
    mnu, mxu = mn.view(np.uint32).copy(), mx.view(np.uint32).copy()
    mxu[rng.random((H, W)) < 0.2] = 0
    special = np.array([0x7F800000, 0xFF800000, 0x7FC00000, 0x00000001, 0x80000000], np.uint32)
    mnu[0, :25] = np.repeat(special, 5)
    mxu[0, :25] = np.tile(special, 5)
    dmn, dmx = torch.from_numpy(mnu.view(np.int32)).cuda(), torch.from_numpy(mxu.view(np.int32)).cuda()
    out = torch.full((H, W), 7.0, dtype=torch.float32, device="cuda")
    abi.check(abi.lib().rsd_ray_min_max_length(C.c_void_p(dmn.data_ptr()), C.c_void_p(dmx.data_ptr()), W, H,
                                               C.c_void_p(out.data_ptr()), _stream(torch)), "rsd_ray_min_max_length")
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    want = ray_min_max_length(mnu, mxu)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert (got > 0).mean() > 0.4 and (got[mxu == 0] == 0).all()
