"""TemporalAO (enabled) and motion vectors: properties of the oracle restatement
(oracle/rsd_oracle.c ocpu_temporal_ao / ocpu_motion_vectors, TemporalAO.ps.slang:55-101) on CPU,
and the host-side prevViewToCurView.  The reference holds no TemporalAO fixtures, so the pass is
pinned by its defining behaviour: a static camera accumulates up to 30 frames, a stable-mask
pixel, an off-screen motion vector or a > 10 % depth change resets the history to 1."""
import numpy as np
import pytest

F = np.float32


def _cam(oracle, pos=(0.0, 2.0, 8.0), target=(0.0, 1.0, 0.0)):
    return oracle.camera_look_at(pos, target, (0.0, 1.0, 0.0), aspect=96 / 64)


def _m(cam, prev):
    from rsd.temporal import prev_view_to_cur_view
    return prev_view_to_cur_view(cam, prev)


def test_prev_view_to_cur_view_identity_and_translation(oracle):
    c0 = _cam(oracle)
    assert np.allclose(_m(c0, c0), np.eye(4), atol=1e-6)
    c1 = _cam(oracle, pos=(0.0, 2.0, 7.0), target=(0.0, 1.0, -1.0))  # moved 1 m along -z, same orientation
    m = _m(c1, c0)
    assert np.allclose(m[:3, :3], np.eye(3), atol=1e-6)
    # a point 5 m in front of c0 is 4 m in front of c1 (view space looks down -z)
    p = m @ np.array([0.0, 0.0, -5.0, 1.0])
    assert abs(-p[2] - 5.0 * np.cos(np.arctan(1 / 8)) + 1.0 * np.cos(np.arctan(1 / 8))) < 0.2


def test_motion_vectors_static_camera_are_zero(oracle):
    c = _cam(oracle)
    z = np.linspace(1.0, 30.0, 64 * 96, dtype=F).reshape(64, 96)
    mv = oracle.motion_vectors(c, c, z)
    assert np.abs(mv).max() < 2e-5


def test_motion_vectors_follow_the_camera(oracle):
    """Camera moved to the right: scene points move left on screen -> prevUV - uv > 0 in x."""
    c0 = _cam(oracle, pos=(0.0, 2.0, 8.0), target=(0.0, 1.0, 0.0))
    c1 = _cam(oracle, pos=(0.3, 2.0, 8.0), target=(0.3, 1.0, 0.0))
    z = np.full((64, 96), 8.0, F)
    mv = oracle.motion_vectors(c1, c0, z)
    assert (mv[..., 0] > 0).all() and np.abs(mv[..., 1]).max() < 0.01
    behind = oracle.motion_vectors(c1, _cam(oracle, pos=(0.0, 2.0, -30.0), target=(0.0, 1.0, -40.0)), z)
    assert (behind == 2.0).all()  # every hit is behind that previous camera: off screen


def test_motion_vectors_background_is_zero(oracle):
    """Sky / background pixels (linear depth >= farZ: rsd_gbuffer's miss value, or a linearized
    cleared raster depth 1.0) keep the cleared mvec (0, 0) under a moving camera, like
    GBufferRaster (GBufferRaster.cpp:176 clear, GBufferRaster.3d.slang:117 geometry only)."""
    c0 = _cam(oracle, pos=(0.0, 2.0, 8.0), target=(0.0, 1.0, 0.0))
    c1 = _cam(oracle, pos=(0.5, 2.3, 7.0), target=(0.2, 1.0, 0.0))
    z = np.full((64, 96), 8.0, F)
    z[:20] = c1.farZ                                        # rsd_gbuffer miss
    z[20:24] = np.float32(c1.farZ) * np.float32(1.0001)     # linearized raster depth 1.0 (> farZ)
    mv = oracle.motion_vectors(c1, c0, z)
    assert (mv[:24] == 0.0).all()
    assert (np.abs(mv[24:]).max(axis=-1) > 0).all()        # geometry still moves


def test_temporal_accumulates_to_thirty_and_resets(oracle):
    H, W, g = 64, 96, 4
    c = _cam(oracle)
    rng = np.random.default_rng(3)
    ao = rng.integers(0, 256, (H, W)).astype(np.uint8)
    z = (5.0 + rng.random((H, W))).astype(F)
    mv = np.zeros((H, W, 2), F)
    m = _m(c, c)
    prev_z, prev_ao, prev_n = np.zeros_like(z), np.zeros_like(ao), np.zeros_like(ao)
    for frame in range(35):
        out, n = oracle.temporal_ao(ao, z, mv, prev_z, prev_ao, prev_n, c, m, g)
        prev_z, prev_ao, prev_n = z, out, n
        inner = (slice(g, H - g), slice(g, W - g))
        want = 1 if frame == 0 else min(frame + 1, 30)
        assert (n[inner] == want).all(), frame
        assert np.array_equal(out[inner], ao[inner])  # a constant signal stays itself
        assert (n[:g] == 0).all() and (out[:, :g] == 0).all()  # scissor
    # stable mask, off-screen motion, depth change: history back to 1, AO = the new AO
    mask = np.zeros_like(ao)
    mask[10:20, 10:20] = 1
    mv2 = mv.copy()
    mv2[30:40, 30:40] = 0.9
    z2 = z.copy()
    z2[50:55, 50:60] *= 1.2
    ao2 = (255 - ao).astype(np.uint8)
    out, n = oracle.temporal_ao(ao2, z2, mv2, prev_z, prev_ao, prev_n, c, m, g, stable_mask=mask)
    for sl in ((slice(10, 20), slice(10, 20)), (slice(30, 40), slice(30, 40)), (slice(50, 55), slice(50, 60))):
        assert (n[sl] == 1).all() and np.array_equal(out[sl], ao2[sl])
    assert (n[25:28, 70:80] == 30).all()
    # elsewhere the 30-frame history dominates: (30 * old + new) / 31
    exp = np.floor((30 * int(ao[25, 70]) / 255 + int(ao2[25, 70]) / 255) / 31 * 255 + 0.5)
    assert abs(int(out[25, 70]) - exp) <= 1


def test_temporal_ao_host_mirror_refuses_bad_shapes():
    pytest.importorskip("torch")
    import torch

    from rsd.temporal import TemporalAO
    t = TemporalAO(enabled=True)
    ao = torch.zeros((8, 8), dtype=torch.uint8)
    with pytest.raises(ValueError):
        t.execute(ao, torch.zeros((8, 8), dtype=torch.float64), torch.zeros((8, 8, 2)), None, None)
    d = TemporalAO(enabled=False)  # disabled: a copy, no librsd call
    src = torch.arange(64, dtype=torch.uint8).reshape(8, 8)
    assert torch.equal(d.execute(src, None, None, None, None), src)


def test_taa_static_history_is_identity_without_clamp(oracle):
    """Catmull-Rom at texel centres reproduces the history; with a wide colour box and no
    anti-flicker a static frame blended with itself stays itself (TAA.ps.slang:44-150)."""
    rng = np.random.default_rng(4)
    H, W = 24, 40
    c = rng.random((H, W, 4)).astype(F)
    out = oracle.taa(c, np.zeros((H, W, 2), F), c, color_box_sigma=100.0, anti_flicker=False)
    assert np.abs(out[..., :3] - c[..., :3]).max() < 1e-6 and (out[..., 3] == 1.0).all()


def test_taa_first_frame_and_clamp(oracle):
    """First frame (zero history): the history is clamped into the colour box, then blended by
    alpha; a constant image stays constant whatever the history (box of zero width)."""
    H, W = 16, 16
    const = np.full((H, W, 4), 0.5, F)
    out = oracle.taa(const, np.zeros((H, W, 2), F), np.zeros_like(const))
    inner = out[1:-1, 1:-1, :3]  # border pixels see zero neighbours (Load outside = 0)
    assert np.allclose(inner, 0.5, atol=1e-6)
    # the longest 3x3 motion vector steers the history fetch: a history shifted by one texel
    # and a matching motion vector give the same result as no shift
    rng = np.random.default_rng(5)
    c = rng.random((H, W, 4)).astype(F)
    prev = np.roll(c, 1, axis=1)  # prev[x] = c[x - 1]
    mv = np.zeros((H, W, 2), F)
    mv[..., 0] = 1.0 / W  # history at x + 1 px
    a = oracle.taa(c, mv, prev, color_box_sigma=100.0, anti_flicker=False)
    b = oracle.taa(c, np.zeros_like(mv), c, color_box_sigma=100.0, anti_flicker=False)
    assert np.abs(a - b).max() < 1e-5


def test_flicker_mask_plane_and_edge(oracle):
    """A fronto-parallel plane is stable everywhere inside; a depth step makes the pixels next to
    it unstable only where neither neighbour of an axis lies in the plane."""
    H, W = 32, 48
    c = oracle.camera_look_at((0.0, 0.0, 0.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), aspect=W / H)
    z = np.full((H, W), 5.0, F)
    n = np.zeros((H, W, 4), F)
    n[..., 2] = 1.0  # world +z = towards the camera (view space +z)
    m = oracle.ao_flicker_mask(z, n, c)
    assert (m[1:-1, 1:-1] == 1).all()
    z2 = z.copy()
    z2[:, 24:] = 9.0
    m2 = oracle.ao_flicker_mask(z2, n, c)
    assert (m2[1:-1, 1:23] == 1).all() and (m2[1:-1, 25:-1] == 1).all()  # one in-plane neighbour suffices
    z3 = z.copy()
    z3[:, ::2] = 9.0  # alternating columns: no in-plane neighbour in x
    assert (oracle.ao_flicker_mask(z3, n, c)[1:-1, 1:-1] == 0).all()


def test_binary_dilation_ring(oracle):
    """min spreads a single 0 over the gather footprints around it; max spreads a single 1; a
    uniform mask is unchanged; wrap addressing at the border."""
    H, W = 20, 20
    ones = np.ones((H, W), np.uint8)
    assert (oracle.binary_dilation(ones, "min") == 1).all()
    hole = ones.copy()
    hole[10, 10] = 0
    d = oracle.binary_dilation(hole, "min")
    assert d[10, 10] == 0 and 4 <= (d == 0).sum() <= 25 and d[0, 0] == 1
    dot = np.zeros((H, W), np.uint8)
    dot[0, 0] = 1
    dm = oracle.binary_dilation(dot, "max")
    assert dm[0, 0] == 1 and dm[H - 1, W - 1] == 1  # wraps around the corner


def test_deinterleave_interleave_oracle():
    """DeinterleaveTexture / InterleaveTexture restated in numpy: layer contents, zero padding of
    ragged sizes, and the round trip."""
    from oracle.texops import deinterleave, interleave
    rng = np.random.default_rng(7)
    for H, W in ((8, 12), (13, 9), (1, 1)):
        a = rng.random((H, W)).astype(F)
        d = deinterleave(a)
        assert d.shape == (16, (H + 3) // 4, (W + 3) // 4)
        assert d[5, 0, 0] == (a[1, 1] if H > 1 and W > 1 else 0.0)
        assert np.array_equal(interleave(d, H, W), a)
        if H % 4:
            assert (d[12:, -1, :] == 0).all()  # rows beyond the source read 0


def test_ray_min_max_length_oracle():
    """RayMinMaxLength.ps.slang:4-16 known answers: rayMax word 0 -> 0, inverted -> 0, NaN -> 0."""
    from oracle.texops import ray_min_max_length
    f = lambda *v: np.array(v, np.float32).view(np.uint32)  # noqa: E731
    mn = f(1.0, 2.0, 5.0, 0.0, np.inf, 1.0)
    mx = f(33.0, 0.0, 3.0, 0.0, np.inf, np.nan)
    mx[1] = 0
    got = ray_min_max_length(mn, mx)
    assert got.tolist() == [1.0, 0.0, 0.0, 0.0, 0.0, 0.0]


def test_motion_vectors_raster_near_far_ten(oracle):
    """The raster variant classifies the cleared depth 1.0 as background on the raw value: with near
    0.1 / far 10 its linearisation (9.99996) is below farZ and the linear-depth variant would move it."""
    c0 = _cam(oracle, pos=(0.0, 2.0, 8.0), target=(0.0, 1.0, 0.0))
    c1 = _cam(oracle, pos=(0.5, 2.3, 7.0), target=(0.2, 1.0, 0.0))
    c0.nearZ, c0.farZ, c1.nearZ, c1.farZ = 0.1, 10.0, 0.1, 10.0
    d = np.full((64, 96), 0.9, F)
    d[:20] = 1.0
    mv = oracle.motion_vectors_raster(c1, c0, d)
    assert (mv[:20] == 0.0).all() and (np.abs(mv[20:]).max(axis=-1) > 0).all()
    lin = oracle.linearize_depth(d, 0.1, 10.0)
    assert (lin[:20] < 10.0).all()  # the linear depth alone cannot tell the cleared depth from geometry
