"""The two-pass SD setup (csrc/sd_trace.hip sd_classify_kernel + sd_live_kernel, RSD_SETUP_TWOPASS): pass A streams over
the map and lists the texels pass 1 touched, pass B evaluates only those.  It is the default for the full-resolution
maps (configs[2]-[4], whose whole-map parity tests in test_gpu_fullsize.py / test_gpu_configs.py run it); here it is
forced on small frames and compared with the CPU oracle bit for bit, with the one-pass setup along a camera path with
clean tiles (the tile stamps differ -- a tile with touched but dead texels is stamped unknown -- the maps may not), and
inside the consuming band frames (intervals reset by the trace)."""
import os

import numpy as np
import pytest

from helpers import oracle_frame, small_frame_config, to_oracle

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.fixture
def twopass():
    os.environ["RSD_SETUP_TWOPASS"] = "on"
    yield
    os.environ.pop("RSD_SETUP_TWOPASS", None)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("N,impl,max_count,divisor", [(4, 0, 8, 2), (8, 0, 8, 1), (16, 0, 16, 1), (4, 1, 8, 2),
                                                      (4, 3, 8, 2), (1, 0, 1, 1)])
def test_twopass_setup_equals_oracle(oracle, twopass, N, impl, max_count, divisor):
    import torch
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    s = make_scene("arcade_tiny")
    cfg = small_frame_config(visible=(256, 160), guard=32, divisor=divisor, N=N, max_count=max_count, impl=impl)
    r = Renderer(s, cfg)
    r.gbuffer()
    r.frame()
    torch.cuda.synchronize()
    g = r.numpy()
    osc = oracle.Scene(s.positions, s.indices, s.flags, s.alpha)
    o = oracle_frame(oracle, osc, to_oracle(r.cam, oracle.Camera), to_oracle(r.vao, oracle.VAOData),
                     to_oracle(r.sdp, oracle.SDParams), to_oracle(r.svp, oracle.SVAOParams), cfg.fb_w, cfg.fb_h,
                     r.sd_w, r.sd_h)
    assert (o["ray_min"] != 0x7F7FFFFF).any()
    assert np.array_equal(bits(g["sd"]), bits(o["sd"]))
    assert np.array_equal(g["ao"], o["ao"])
    r.close()


@pytest.mark.timeout(600)
def test_twopass_setup_equals_onepass_along_camera_path():
    """configs[1]'s map (one-pass by default) forced two-pass along the orbit with clean tiles, against the one-pass
    setup on its own frame slot: every pose's SD map and AO equal."""
    import torch
    from rsd.frame import CONFIGS, FrameConfig, Renderer, camera_path
    from rsd.scenes import make_scene
    kw, name = CONFIGS["suntemple_1080p_q"]
    r = Renderer(make_scene(name), FrameConfig(**kw))
    one = r.frame_slot(own_gbuffer=True)
    two = r.frame_slot(own_gbuffer=True)
    one.keep_clean_tiles()
    two.keep_clean_tiles()
    try:
        for p in camera_path("orbit120")[::15]:
            for slot, mode in ((one, "off"), (two, "on")):
                os.environ["RSD_SETUP_TWOPASS"] = mode
                slot.set_pose(*p)
                slot.gbuffer()
                slot.frame()
            torch.cuda.synchronize()
            assert np.array_equal(bits(one.sd.cpu().numpy()), bits(two.sd.cpu().numpy()))
            assert np.array_equal(one.ao.cpu().numpy(), two.ao.cpu().numpy())
    finally:
        os.environ.pop("RSD_SETUP_TWOPASS", None)
    r.close()


@pytest.mark.timeout(300)
def test_twopass_setup_in_consuming_band_frames(oracle, twopass):
    """BandFrame's consuming traces (the setup resets the intervals it read): three bands of one frame, then the
    next frames, equal the explicit-clear frame bit for bit, and the interval maps end cleared."""
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    from rsd.shard import BandFrame
    cfg = small_frame_config(visible=(224, 136), guard=16, divisor=2, N=4)
    r = Renderer(make_scene("arcade_tiny"), cfg)
    r.gbuffer()
    os.environ["RSD_SETUP_TWOPASS"] = "off"
    r.frame()
    want = r.numpy()
    os.environ["RSD_SETUP_TWOPASS"] = "on"
    bf = BandFrame(r, 0, 1)
    for k in range(3):
        bf.frame()
        g = r.numpy()
        assert (g["ray_min"] == 0x7F7FFFFF).all() and (g["ray_max"] == 0).all(), k
        assert np.array_equal(bits(g["sd"]), bits(want["sd"])) and np.array_equal(g["ao"], want["ao"]), k
    r.close()
