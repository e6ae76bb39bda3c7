"""CPU tests of the alpha test in the oracle, and of librsd's host side.

The reference holds no fixtures for its alpha test (it runs inside Falcor's material system,
MaterialFactory.slang:124-151), so the texture sampling is librsd's own definition
(DESIGN.md "Alpha test") and is pinned here by independent restatements: numpy's float16 for
the MaterialHeader threshold, a numpy float32 bilinear sampler and box mip chain, and
scene-level identities (a card that always fails the test is the same as no card; a card
that always passes is the same as an opaque one)."""
import dataclasses
import math

import numpy as np
import pytest

F = np.float32


def _tri_scene(oracle, materials, textures, uv=None, n=None):
    """n alpha-masked unit triangles (one per material unless n is given) side by side."""
    from rsd.scenes import AlphaMaterials
    n = len(materials) if n is None else n
    pos, ind = [], []
    for i in range(n):
        pos += [[2.0 * i, 0, 0], [2.0 * i + 1, 0, 0], [2.0 * i, 1, 0]]
        ind.append([3 * i, 3 * i + 1, 3 * i + 2])
    pos, ind = np.array(pos, F), np.array(ind, np.uint32)
    uv = np.tile(np.array([[0, 0], [1, 0], [0, 1]], F), (n, 1)) if uv is None else np.asarray(uv, F)
    m = np.array([mm[:2] for mm in materials], F)
    am = AlphaMaterials(uv, np.arange(n, dtype=np.uint32) % len(materials), m[:, 0].copy(), m[:, 1].copy(),
                        np.array([mm[2] for mm in materials], np.uint32), textures)
    return oracle.Scene(pos, ind, np.full(n, 5, np.uint32), am), am


def test_threshold_is_float16(oracle):
    """MaterialHeader keeps the alpha threshold as float16 (MaterialData.slang:99): the test
    passes at exactly float16(threshold) and fails one float32 ulp below it."""
    from rsd.scenes import NO_TEXTURE
    thr = [0.33, 0.1, 0.7777, 0.5, 1e-5, 0.999]
    mats = []
    for t in thr:
        h = F(np.float16(t))
        mats += [(t, float(h), NO_TEXTURE), (t, float(np.nextafter(h, F(-1))), NO_TEXTURE)]
    sc, _ = _tri_scene(oracle, mats, [])
    for i, t in enumerate(thr):
        assert sc.alpha_threshold(2 * i) == F(np.float16(t))
        assert not sc.alpha_fails(2 * i, 0.2, 0.2)
        assert sc.alpha_fails(2 * i + 1, 0.2, 0.2)


def _np_texel(tex, x, y):
    h, w = tex.shape
    return F(tex[y % h, x % w]) / F(255.0)


def _np_bilinear(tex, u, v):
    h, w = tex.shape
    x, y = F(u) * F(w) - F(0.5), F(v) * F(h) - F(0.5)
    x0, y0 = np.floor(x), np.floor(y)
    qx, qy = np.floor((x - x0) * F(256.0) + F(0.5)), np.floor((y - y0) * F(256.0) + F(0.5))
    ix, iy = int(x0), int(y0)
    if qx >= 256:
        qx, ix = F(0), ix + 1
    if qy >= 256:
        qy, iy = F(0), iy + 1
    wx, wy = qx * F(1 / 256), qy * F(1 / 256)
    r0 = _np_texel(tex, ix, iy) * (F(1) - wx) + _np_texel(tex, ix + 1, iy) * wx
    r1 = _np_texel(tex, ix, iy + 1) * (F(1) - wx) + _np_texel(tex, ix + 1, iy + 1) * wx
    return r0 * (F(1) - wy) + r1 * wy


def _np_mips(tex):
    chain = [tex.astype(np.int64)]
    while chain[-1].shape != (1, 1):
        a = chain[-1]
        h, w = a.shape
        nh, nw = max(1, h // 2), max(1, w // 2)
        ys, xs = np.arange(nh), np.arange(nw)
        y0, y1 = np.minimum(2 * ys, h - 1), np.minimum(2 * ys + 1, h - 1)
        x0, x1 = np.minimum(2 * xs, w - 1), np.minimum(2 * xs + 1, w - 1)
        s = a[y0][:, x0] + a[y0][:, x1] + a[y1][:, x0] + a[y1][:, x1]
        chain.append((s + 2) // 4)
    return [c.astype(np.uint8) for c in chain]


@pytest.mark.parametrize("shape", [(8, 8), (5, 7), (1, 9), (16, 3)])
def test_lod0_bilinear_matches_numpy(oracle, shape):
    """LOD 0 (G-buffer, Raytraced AO): one bilinear tap, wrap addressing, 1/256 weights, on a
    texture coordinate interpolated with the DXR barycentrics (b0 = 1 - u - v)."""
    rng = np.random.default_rng(sum(shape))
    tex = rng.integers(0, 256, shape).astype(np.uint8)
    uv = np.array([[-1.3, 0.4], [2.7, -0.6], [0.2, 3.1]], F)
    sc, _ = _tri_scene(oracle, [(0.5, 1.0, 0)], [tex], uv=uv)
    for bu, bv in rng.random((300, 2)).astype(F):
        if bu + bv > 1:
            continue
        w0 = F(1) - bu - bv
        tu = uv[0, 0] * w0 + uv[1, 0] * bu + uv[2, 0] * bv
        tv = uv[0, 1] * w0 + uv[1, 1] * bu + uv[2, 1] * bv
        assert sc.alpha_value(0, float(bu), float(bv)) == _np_bilinear(tex, tu, tv)


def test_mip_chain_and_lod_clamp(oracle):
    """A far hit clamps to the last mip (1 x 1): the (a+b+c+d+2)/4 box chain's single texel."""
    rng = np.random.default_rng(3)
    for shape in [(64, 64), (5, 3), (32, 8), (1, 1), (7, 1)]:
        tex = rng.integers(0, 256, shape).astype(np.uint8)
        sc, _ = _tri_scene(oracle, [(0.5, 1.0, 0)], [tex])
        last = _np_mips(tex)[-1]
        # spread * t huge -> level far above the chain
        a = sc.alpha_value(0, 0.3, 0.3, lod_ray_cone=True, t=1e6, d=(0.0, 0.0, -1.0), spread=0.01)
        bu = bv = F(0.3)
        w0 = F(1) - bu - bv
        assert a == _np_bilinear(last, F(0) * w0 + F(1) * bu + F(0) * bv, F(0) * w0 + F(0) * bu + F(1) * bv), shape
        assert abs(a - last[0, 0] / 255.0) < 1e-6


def test_ray_cone_lod_trilinear(oracle):
    """Between two mips the sample is the LOD-fraction (8 bits) blend of two bilinear taps;
    level = 0.5 log2(w h) + log2(spread t / |d.n|) (TexLODHelpers.slang:122-129)."""
    rng = np.random.default_rng(11)
    tex = rng.integers(0, 256, (16, 16)).astype(np.uint8)
    mips = _np_mips(tex)
    sc, _ = _tri_scene(oracle, [(0.5, 1.0, 0)], [tex])
    spread = F(0.003)
    for t in [F(10.0), F(37.5), F(80.0), F(150.0), F(5.0)]:
        bu, bv = F(0.21), F(0.33)
        w0 = F(1) - bu - bv
        tu, tv = F(0) * w0 + F(1) * bu + F(0) * bv, F(0) * w0 + F(0) * bu + F(1) * bv
        lam = F(0) + F(math.log2(float(abs(spread * t + F(0)) / abs(F(-1.0)))))
        level = F(0.5) * F(math.log2(float(F(256)))) + lam
        lod = min(max(level, F(0)), F(len(mips) - 1))
        l0 = int(np.floor(lod))
        qf = np.floor((lod - F(l0)) * F(256) + F(0.5))
        if qf >= 256:
            l0, qf = l0 + 1, F(0)
        s0 = _np_bilinear(mips[l0], tu, tv)
        want = s0 if qf == 0 or l0 + 1 >= len(mips) else \
            s0 * (F(1) - qf * F(1 / 256)) + _np_bilinear(mips[l0 + 1], tu, tv) * (qf * F(1 / 256))
        got = sc.alpha_value(0, float(bu), float(bv), lod_ray_cone=True, t=float(t), d=(0.0, 0.0, -1.0),
                             spread=float(spread))
        assert got == want, t


def test_ray_cone_spread(oracle):
    """RAY_CONE_SPREAD = the "%f" text of atan(2 tan(fovY/2) / height); librsd's host helper
    (no GPU needed) and the oracle agree, and the value is the 6-decimal rounding."""
    from rsd import abi
    for f, h in [(21.0, 270), (21.0, 1080), (35.0, 512), (10.0, 77), (21.0, 302)]:
        fov = 2 * math.atan(0.5 * 24.0 / f)
        exact = math.atan(2 * math.tan(fov / 2) / h)
        o = oracle.ray_cone_spread(f, h)
        assert abs(o - exact) <= 6e-7
        assert o == F(float("%f" % o))
        assert abi.lib().rsd_ray_cone_spread(f, h) == o


def _frame_inputs(oracle, scene, vis=(120, 72), g=16):
    W, H = vis[0] + 2 * g, vis[1] + 2 * g
    cam = oracle.camera_look_at(scene.camera["pos"], scene.camera["target"], scene.camera["up"],
                                aspect=float(F(W) / F(H)))
    return cam, W, H


def _variant(scene, alpha, keep_cards=True):
    """The scene with card materials forced to constant `alpha` (or the cards removed)."""
    from rsd.scenes import NO_TEXTURE, Scene
    am = scene.alpha
    if not keep_cards:
        keep = am.tri_material == 0
        return Scene(scene.name, scene.positions, scene.indices[keep], scene.flags[keep], scene.camera,
                     dataclasses.replace(am, tri_material=am.tri_material[keep]))
    n = len(am.thresholds)
    al = np.full(n, alpha, F)
    al[0] = 1.0
    return Scene(scene.name, scene.positions, scene.indices, scene.flags, scene.camera,
                 dataclasses.replace(am, alphas=al, material_textures=np.full(n, NO_TEXTURE, np.uint32)))


def _osc(oracle, s):
    return oracle.Scene(s.positions, s.indices, s.flags, s.alpha)


def test_invisible_cards_equal_no_cards(oracle):
    """Cards whose alpha always fails: G-buffer, CoverageMask SD map and Raytraced AO are
    bit-identical to the scene without them (the test ignores the hit entirely)."""
    from helpers import oracle_vao
    from rsd.scenes import make_scene
    s = make_scene("foliage_small")
    a, b = _osc(oracle, _variant(s, 0.0)), _osc(oracle, _variant(s, 0.0, keep_cards=False))
    cam, W, H = _frame_inputs(oracle, s)
    za, na = oracle.gbuffer(a, cam, W, H, 1)
    zb, nb = oracle.gbuffer(b, cam, W, H, 1)
    assert np.array_equal(za.view(np.uint32), zb.view(np.uint32)) and np.array_equal(na, nb)
    p = oracle.SDParams(4, 1, 8, 0, 1, 1, 0, 1, 1, 0.375)
    sa, _ = oracle.sd_trace(a, cam, p, za, None, None, W, H)
    sb, _ = oracle.sd_trace(b, cam, p, za, None, None, W, H)
    assert np.array_equal(sa.view(np.uint32), sb.view(np.uint32))
    vao, sdW, sdH = oracle_vao(oracle, W, H, 1, sd_guard_px=0, radius=1.5)
    sp = oracle.SVAOParams(8, 4, 3, 1, 1, 16)
    ao1, st, _, _ = oracle.svao_pass1(cam, vao, sp, za, na, sdW, sdH)
    assert (st != 0).sum() > 50
    assert np.array_equal(oracle.svao_pass2_raytraced(a, cam, vao, sp, za, na, st, ao1),
                          oracle.svao_pass2_raytraced(b, cam, vao, sp, za, na, st, ao1))


def test_opaque_cards_equal_opaque_scene(oracle):
    """Cards whose alpha always passes behave like the opaque scene (every SD implementation)."""
    from rsd.scenes import make_scene
    s = make_scene("foliage_small")
    a, b = _osc(oracle, _variant(s, 1.0)), oracle.Scene(s.positions, s.indices, s.flags)  # no alpha data
    cam, W, H = _frame_inputs(oracle, s)
    za, _ = oracle.gbuffer(a, cam, W, H, 1)
    zb, _ = oracle.gbuffer(b, cam, W, H, 1)
    assert np.array_equal(za, zb)
    for impl, N in [(0, 4), (3, 4), (1, 4)]:
        p = oracle.SDParams(N, impl, 8, 0, 1, 1, 0, 1, 1, 0.375)
        sa, _ = oracle.sd_trace(a, cam, p, za, None, None, W, H)
        sb, _ = oracle.sd_trace(b, cam, p, za, None, None, W, H)
        assert np.array_equal(sa.view(np.uint32), sb.view(np.uint32)), impl


def test_alpha_changes_the_frame(oracle):
    """With the textured cards the alpha test is not a no-op (holes in the leaves)."""
    from rsd.scenes import make_scene
    s = make_scene("foliage_small")
    a, b = _osc(oracle, s), _osc(oracle, _variant(s, 1.0))
    cam, W, H = _frame_inputs(oracle, s)
    za, _ = oracle.gbuffer(a, cam, W, H, 1)
    zb, _ = oracle.gbuffer(b, cam, W, H, 1)
    assert (za != zb).sum() > 100
    p = oracle.SDParams(4, 0, 8, 0, 1, 1, 0, 1, 1, 0.375)
    sa, _ = oracle.sd_trace(a, cam, p, za, None, None, W, H)
    p.alpha_test = 0
    s0, _ = oracle.sd_trace(a, cam, p, za, None, None, W, H)
    assert (sa != s0).sum() > 100


def test_default_reservoir_counts_failed_hits(oracle):
    """Default implementation: a hit failing the alpha test still takes a reservoir count
    (Common.slangh:136-175 increments before the test), so MaxCount = 1 behind an invisible
    card yields the cleared depth, not the surface behind it."""
    from rsd.scenes import NO_TEXTURE, AlphaMaterials
    pos = np.array([[-50, -50, 0], [50, -50, 0], [0, 50, 0], [-50, -50, -1], [50, -50, -1], [0, 50, -1]], F)
    ind = np.array([[0, 1, 2], [3, 4, 5]], np.uint32)
    am = AlphaMaterials(np.zeros((6, 2), F), np.array([1, 0], np.uint32), np.array([0.5, 0.5], F),
                        np.array([1.0, 0.0], F), np.array([NO_TEXTURE, NO_TEXTURE], np.uint32), [])
    sc = oracle.Scene(pos, ind, np.array([5, 0], np.uint32), am)
    cam = oracle.camera_look_at([0, 0, 3], [0, 0, 0], [0, 1, 0], aspect=1.0)
    z = np.full((8, 8), 1.0, F)
    for mc, want_hit in [(1, False), (2, True)]:
        p = oracle.SDParams(2, 0, mc, 0, 0, 1, 0, 0, 1, 0.375)
        sd, _ = oracle.sd_trace(sc, cam, p, z, None, None, 8, 8)
        assert (sd[..., 0] == 1.0).all()  # slot 0: the invisible card's (ignored) sample
        assert (sd[..., 1] < 1.0).all() == want_hit and (sd[..., 1] == 1.0).all() != want_hit, mc
