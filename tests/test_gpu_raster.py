"""GPU parity of the raster SD walk (RSD_WALK_RASTER: triangles projected onto the SD texel grid,
exact watertight tests, per-texel K nearest (t, prim) keys by 64-bit atomicMin chains, then the
split walk's resolve kernel).  The canonical any-hit result does not depend on how the hits are
found, so the raster walk must give the oracle's bits exactly, like the BVH walks."""
import os

import numpy as np
import pytest

from helpers import small_frame_config, to_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture
def raster_walk(monkeypatch):
    monkeypatch.setenv("RSD_TRACE_WALK", "raster")  # librsd reads it per trace call
    yield
    monkeypatch.delenv("RSD_TRACE_WALK", raising=False)


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _trace_vs_oracle(oracle, scene_name, cfg, rows=None, consume=False):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd import abi
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    scene = make_scene(scene_name)
    r = Renderer(scene, cfg)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    g0 = r.numpy()
    r.sd.zero_()
    cnt = r.sd_trace(counters=True)
    assert cnt.walk == abi.WALK_RASTER
    g_cnt = r.numpy()
    r.sd.zero_()
    r.sd_trace(consume=consume)
    g = r.numpy()
    assert bits_equal(g["sd"], g_cnt["sd"])  # the instrumented launch gives the same bits
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags, scene.alpha)
    sd, stats = oracle.sd_trace(osc, to_oracle(r.cam, oracle.Camera), to_oracle(r.sdp, oracle.SDParams), g0["depth"],
                                g0["ray_min"], g0["ray_max"], r.sd_w, r.sd_h, rows=rows)
    r.close()
    return g, sd, stats, cnt


@pytest.mark.parametrize("N,impl,max_count,divisor", [(1, 0, 8, 2), (2, 0, 8, 2), (4, 0, 8, 4), (8, 0, 8, 1),
                                                      (16, 0, 16, 1), (4, 3, 8, 2), (8, 3, 4, 2), (4, 0, 2, 2),
                                                      (4, 0, 16, 2)])
def test_raster_parity_small(oracle, raster_walk, N, impl, max_count, divisor):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=divisor, N=N, max_count=max_count, impl=impl)
    g, sd, stats, cnt = _trace_vs_oracle(oracle, "arcade_tiny", cfg)
    assert stats[0] > 100 and cnt.rays_active == stats[0]
    assert bits_equal(g["sd"], sd)


@pytest.mark.parametrize("cull", [0, 2])
def test_raster_no_interval_and_cull(oracle, raster_walk, cull):
    cfg = small_frame_config(visible=(160, 96), guard=0, divisor=1, N=4)
    cfg.cull_mode, cfg.ray_interval, cfg.sd_guard_px = cull, False, 0
    g, sd, stats, _ = _trace_vs_oracle(oracle, "arcade_tiny", cfg)
    assert bits_equal(g["sd"], sd)


def test_raster_alpha_scene(oracle, raster_walk):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=4)
    g, sd, _, _ = _trace_vs_oracle(oracle, "foliage_small", cfg)
    assert bits_equal(g["sd"], sd)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config", ["suntemple_1080p_q", "bistro_1080p_full"])
def test_raster_fullsize(oracle, raster_walk, config):
    from rsd.frame import CONFIGS, FrameConfig
    kw, name = CONFIGS[config]
    cfg = FrameConfig(**kw)
    g, sd, stats, _ = _trace_vs_oracle(oracle, name, cfg, consume=True)
    assert stats[0] > 10000
    assert bits_equal(g["sd"], sd), config
    assert (g["ray_max"] == 0).all()  # consumed


def test_raster_band_rows(oracle, raster_walk):
    """Band / row-range traces with the raster walk: each band's rows equal the full trace."""
    import torch
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=4)
    r = Renderer(make_scene("arcade_tiny"), cfg)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    r.sd_trace()
    full = r.numpy()["sd"]
    r.sd.zero_()
    for b in range(3):
        r.sd_trace(band=(b, 3))
    assert bits_equal(r.numpy()["sd"], full)
    r.sd.zero_()
    r.sd_trace_rows((0, 48))
    r.sd_trace_rows((48, r.sd_h))
    torch.cuda.synchronize()
    assert bits_equal(r.numpy()["sd"], full)
    r.close()
