"""GPU parity of the traversal-order any-hit streams (rsd.h RSD_HIT_ORDER_TRAVERSAL, the depth-first order, and
RSD_HIT_ORDER_WAVEFRONT, the row walk's 8-wide order) and of the Use16Bit SD map (StochasticDepthMapRT.cpp:192-198).

The traversal order depends on the BVH, so the oracle walks librsd's own tree: the GPU scene's
rsd_scene_export_bvh bytes (ocpu_sd_trace_ordered).  Bit-exact, like test_gpu_parity.py."""
import numpy as np
import pytest

from helpers import small_frame_config, to_oracle

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _run(scene_name, cfg, oracle, band=(0, 1), consume=False):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    scene = make_scene(scene_name)
    r = Renderer(scene, cfg)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    torch.cuda.synchronize()
    g0 = r.numpy()  # the interval maps the trace reads (consume resets them)
    r.sd.zero_()
    r.sd_trace(band=band, consume=consume)
    g = r.numpy()
    bvh, off = r.gscene.export_bvh()
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags, scene.alpha)
    cam, sdp = to_oracle(r.cam, oracle.Camera), to_oracle(r.sdp, oracle.SDParams)
    if cfg.hit_order == 2:  # the wavefront order: librsd's pool bound from the tree depth (rsd.h)
        soft = min(208 - 3 * int(r.gscene.info.wide_depth), 160)
        sd, stats = oracle.sd_trace_wavefront(osc, bvh, off, soft, cam, sdp, g0["depth"], g0["ray_min"], g0["ray_max"],
                                              r.sd_w, r.sd_h, band=band)
    else:
        sd, stats = oracle.sd_trace_ordered(osc, bvh, off, cam, sdp, g0["depth"], g0["ray_min"], g0["ray_max"], r.sd_w,
                                            r.sd_h, band=band)
    r.close()
    return g, g0, sd, stats


@pytest.mark.parametrize("N,impl,max_count", [(1, 0, 8), (2, 0, 8), (4, 0, 8), (8, 0, 8), (16, 0, 16),
                                              (4, 3, 8), (8, 3, 8), (4, 1, 8), (8, 1, 8), (4, 0, 2), (4, 0, 32)])
def test_traversal_order_parity(oracle, N, impl, max_count):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=N, max_count=max_count, impl=impl)
    cfg.hit_order = 1
    g, _, sd, stats = _run("arcade_tiny", cfg, oracle)
    assert stats[0] > 100
    assert bits_equal(g["sd"], sd)


@pytest.mark.parametrize("cull", [0, 2])
def test_traversal_order_cull_and_no_interval(oracle, cull):
    cfg = small_frame_config(visible=(160, 96), guard=0, divisor=1, N=4)
    cfg.hit_order, cfg.cull_mode, cfg.ray_interval, cfg.sd_guard_px = 1, cull, False, 0
    g, _, sd, stats = _run("arcade_tiny", cfg, oracle)
    assert stats[0] > 0.5 * g["sd"].shape[1] * g["sd"].shape[2]  # no interval: every ray with TMin <= TMax
    assert bits_equal(g["sd"], sd)


def test_traversal_order_alpha_scene(oracle):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=4)
    cfg.hit_order = 1
    g, _, sd, _ = _run("foliage_small", cfg, oracle)
    assert bits_equal(g["sd"], sd)


def test_traversal_order_band_consume(oracle):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=4)
    cfg.hit_order = 1
    g, g0, sd, _ = _run("arcade_tiny", cfg, oracle, band=(1, 3), consume=True)
    rows = np.array([y for y in range(g["sd"].shape[1]) if (y // 8) % 3 == 1])
    assert bits_equal(g["sd"][:, rows], sd[:, rows])
    assert (g["ray_max"] == 0).all()  # consumed


def test_traversal_default_differs_from_kbuffer():
    """On the GPU: under the traversal order the Default reservoir is not the K-buffer."""
    import torch
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS["suntemple_1080p_q"]
    scene = make_scene(name)
    out = {}
    for impl in (0, 3):
        for order in (0, 1):
            r = Renderer(scene, FrameConfig(**kw, implementation=impl, hit_order=order))
            r.gbuffer()
            r.frame()
            out[impl, order] = r.numpy()["sd"]
            r.close()
    torch.cuda.synchronize()
    assert bits_equal(out[0, 0], out[3, 0])  # canonical: the collapse
    assert not bits_equal(out[0, 1], out[3, 1])  # traversal: the reservoir samples
    assert not bits_equal(out[0, 1], out[0, 0])


@pytest.mark.timeout(600)
def test_traversal_order_config1_whole_map(oracle):
    from rsd.frame import CONFIGS, FrameConfig
    kw, name = CONFIGS["suntemple_1080p_q"]
    cfg = FrameConfig(**kw, hit_order=1)
    g, _, sd, stats = _run(name, cfg, oracle)
    assert stats[0] > 10000
    assert bits_equal(g["sd"], sd)


@pytest.mark.parametrize("N", [1, 2, 4])
def test_use16bit_parity(oracle, N):
    """Use16Bit: the R16F / RG16F / RGBA16F map is the f32 map rounded to binary16 (nearest even)."""
    import torch
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=N)
    scene = make_scene("arcade_tiny")
    r32 = Renderer(scene, cfg)
    r32.gbuffer()
    r32.frame()
    g32 = r32.numpy()
    cfg16 = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=N)
    cfg16.use_16bit = True
    r16 = Renderer(scene, cfg16, dev=r32.dev, gpu_scene=r32.gscene)
    # the same trace inputs: G-buffer and the interval maps of r32's pass 1 (its trace did not consume them)
    r16.depth.copy_(r32.depth)
    r16.normals.copy_(r32.normals)
    r16.ray_minmax.copy_(r32.ray_minmax)
    r16.sd_trace()
    torch.cuda.synchronize()
    assert r16.sd.dtype == torch.float16
    got = r16.sd.cpu().numpy()
    want = g32["sd"].astype(np.float16)
    assert np.array_equal(got.view(np.uint16), want.view(np.uint16))
    # and the oracle's f32 map rounds to the same bits
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    sd, _ = oracle.sd_trace(osc, to_oracle(r32.cam, oracle.Camera), to_oracle(r32.sdp, oracle.SDParams), g32["depth"],
                            g32["ray_min"], g32["ray_max"], r32.sd_w, r32.sd_h)
    assert np.array_equal(sd.astype(np.float16).view(np.uint16), got.view(np.uint16))
    with pytest.raises(ValueError):
        r16.pass2()
    r32.close()


def test_use16bit_refuses_n8():
    import ctypes as C

    from rsd import abi
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    cfg = small_frame_config(visible=(64, 64), guard=0, divisor=1, N=8)
    r = Renderer(make_scene("arcade_tiny"), cfg)
    r.sdp.use_16bit = 1
    st = abi.lib().rsd_sd_trace(r.gscene.h, C.byref(r.cam), C.byref(r.sdp), C.c_void_p(r.depth.data_ptr()),
                                cfg.fb_w, cfg.fb_h, None, None, C.c_void_p(r.sd.data_ptr()), r.sd_w, r.sd_h, None,
                                None)
    assert st == abi.ERR_UNSUPPORTED
    r.close()


# ---- the wavefront order (RSD_HIT_ORDER_WAVEFRONT, sd_trace_wavefront_kernel vs oracle o_wavefront_walk)
@pytest.mark.parametrize("N,impl,max_count", [(1, 0, 8), (4, 0, 8), (8, 0, 8), (16, 0, 16), (4, 3, 8), (4, 1, 8),
                                              (4, 0, 2), (4, 0, 32)])
def test_wavefront_order_parity(oracle, N, impl, max_count):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=N, max_count=max_count, impl=impl)
    cfg.hit_order = 2
    g, _, sd, stats = _run("arcade_tiny", cfg, oracle)
    assert stats[0] > 100
    assert bits_equal(g["sd"], sd)


def test_wavefront_order_alpha_cull_band(oracle):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=4)
    cfg.hit_order = 2
    g, _, sd, _ = _run("foliage_small", cfg, oracle)
    assert bits_equal(g["sd"], sd)
    cfg = small_frame_config(visible=(160, 96), guard=0, divisor=1, N=4)
    cfg.hit_order, cfg.cull_mode, cfg.ray_interval, cfg.sd_guard_px = 2, 2, False, 0
    g, _, sd, _ = _run("arcade_tiny", cfg, oracle)
    assert bits_equal(g["sd"], sd)
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=4)
    cfg.hit_order = 2
    g, g0, sd, _ = _run("arcade_tiny", cfg, oracle, band=(1, 3), consume=True)
    rows = np.array([y for y in range(g["sd"].shape[1]) if (y // 8) % 3 == 1])
    assert bits_equal(g["sd"][:, rows], sd[:, rows])
    assert (g["ray_max"] == 0).all()


@pytest.mark.timeout(600)
def test_wavefront_order_config1_whole_map(oracle):
    """configs[1]: the whole SD map bit for bit, and the stream is its own (not the depth-first order's map)."""
    from rsd.frame import CONFIGS, FrameConfig
    kw, name = CONFIGS["suntemple_1080p_q"]
    g, _, sd, stats = _run(name, FrameConfig(**kw, hit_order=2), oracle)
    assert stats[0] > 10000
    assert bits_equal(g["sd"], sd)
    g1, _, _, _ = _run(name, FrameConfig(**kw, hit_order=1), oracle)
    assert not bits_equal(g["sd"], g1["sd"])
