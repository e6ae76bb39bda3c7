"""GPU parity at every BASELINE.json config as stated (VERDICT r1 "configs untested"):

  configs[0]  Arcade 256 x 256, SD N = 1, divisor 1, GuardBand 0 -- the SD pass driven directly
              (no ray interval) and the whole SVAO frame at that size, against the oracle's own
              G-buffer -> pass 1 -> SD trace -> pass 2.
  configs[1]  Sun Temple 1080p, 1/4-res SD, N = 4 -- the WHOLE SD map, the whole pass 1 and pass 2
              against the oracle on the GPU's G-buffer (bench.py's default frame).
  configs[4]  Bistro 4K full-res N = 16 along the 120-pose orbit camera (rsd.frame.camera_path):
              several poses, each with its own G-buffer; pass 1, the whole SD map and pass 2 over
              the whole frame.  Plus the frames-in-flight schedule on a path
              (every slot renders its own pose) equal to the sequential frames.

Bit-exact, like test_gpu_parity.py."""
import numpy as np
import pytest

from helpers import oracle_frame, to_oracle

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _structs(r, O):
    return (to_oracle(r.cam, O.Camera), to_oracle(r.vao, O.VAOData), to_oracle(r.sdp, O.SDParams),
            to_oracle(r.svp, O.SVAOParams))


@pytest.mark.timeout(300)
def test_config0_arcade_256(oracle):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import ARCADE_CONFIG, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = ARCADE_CONFIG
    scene = make_scene(name)
    cfg = FrameConfig(**kw)
    r = Renderer(scene, cfg)
    assert (cfg.fb_w, cfg.fb_h, r.sd_w, r.sd_h, r.sdp.guard_band) == (256, 256, 256, 256, 0)
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    cam, vao, sdp, svp = _structs(r, oracle)
    r.gbuffer()
    # the SD pass driven directly: StochasticDepthMapRT without the optional rayMin / rayMax
    # inputs (StochasticDepthMapRT.cpp:212-213) -- every one of the 65,536 rays is live
    r.sdp.ray_interval = 0
    r.sd_trace()
    g = r.numpy()
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, sdp.cull_mode)
    assert bits_equal(g["depth"], z) and np.array_equal(g["normals"], n)
    sdp_direct = to_oracle(r.sdp, oracle.SDParams)
    sd, stats = oracle.sd_trace(osc, cam, sdp_direct, z, None, None, r.sd_w, r.sd_h)
    assert stats[0] == 65536
    assert bits_equal(g["sd"], sd)
    # the SVAO frame at the same size (ray intervals on, SD guard band 0)
    r.sdp.ray_interval = 1
    r.frame()
    g = r.numpy()
    o = oracle_frame(oracle, osc, cam, vao, sdp, svp, cfg.fb_w, cfg.fb_h, r.sd_w, r.sd_h)
    for k in ("stencil", "ao"):
        assert np.array_equal(g[k], o[k]), k
    assert bits_equal(g["sd"], o["sd"])
    assert (o["ray_max"] != 0).any()
    r.close()


@pytest.mark.timeout(600)
def test_config1_whole_frame(oracle):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS["suntemple_1080p_q"]
    scene = make_scene(name)
    cfg = FrameConfig(**kw)
    r = Renderer(scene, cfg)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = _structs(r, oracle)
    ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, g["depth"], g["normals"], r.sd_w, r.sd_h)
    assert np.array_equal(g["stencil"], st)
    assert np.array_equal(g["ray_min"], rmin) and np.array_equal(g["ray_max"], rmax)
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    sd, stats = oracle.sd_trace(osc, cam, sdp, g["depth"], rmin, rmax, r.sd_w, r.sd_h)
    assert stats[0] > 10000
    assert bits_equal(g["sd"], sd), "whole configs[1] SD map"
    ao = oracle.svao_pass2(cam, vao, svp, g["depth"], g["normals"], st, sd, ao1)
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    assert np.array_equal(g["ao"][gv], ao[gv])
    r.close()


@pytest.mark.timeout(1200)
def test_config4_camera_path_poses(oracle):
    """configs[4]: Bistro-like 4K full-res N = 16 at poses 0, 41, 83 of the orbit120 path."""
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import CONFIGS, DEFAULT_CAMERA_PATH, FrameConfig, Renderer, camera_path
    from rsd.scenes import make_scene
    kw, name = CONFIGS["bistro_4k_full_n16"]
    poses = camera_path(DEFAULT_CAMERA_PATH["bistro_4k_full_n16"])
    scene = make_scene(name)
    cfg = FrameConfig(**kw)
    r = Renderer(scene, cfg)
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    for k, i in enumerate((0, 41, 83)):
        r.set_pose(*poses[i])
        r.gbuffer()
        r.frame()
        g = r.numpy()
        cam, vao, sdp, svp = _structs(r, oracle)
        if k == 0:  # the G-buffer of a moved camera (whole 4K frame, once)
            z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, sdp.cull_mode)
            assert bits_equal(g["depth"], z) and np.array_equal(g["normals"], n)
        ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, g["depth"], g["normals"], r.sd_w, r.sd_h)
        assert np.array_equal(g["stencil"], st), i
        assert np.array_equal(g["ray_min"], rmin) and np.array_equal(g["ray_max"], rmax), i
        assert (rmax != 0).sum() > 1000, "no SD rays requested at this pose"
        sd, _ = oracle.sd_trace(osc, cam, sdp, g["depth"], rmin, rmax, r.sd_w, r.sd_h)  # the whole map
        assert bits_equal(sd, g["sd"]), i
        ao = oracle.svao_pass2(cam, vao, svp, g["depth"], g["normals"], st, g["sd"], ao1)
        gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
        assert np.array_equal(g["ao"][gv], ao[gv]), i
    r.close()


@pytest.mark.timeout(300)
def test_camera_path_frames_in_flight():
    """bench.py's throughput region on a camera path: 3 slots with their own camera and G-buffer
    on 3 streams, frame i at pose i, equal to the sequential frames bit for bit."""
    import torch
    from rsd.frame import CONFIGS, FrameConfig, Renderer, camera_path
    from rsd.scenes import make_scene
    from rsd.shard import BandFrame
    kw, name = CONFIGS["suntemple_1080p_q"]
    r = Renderer(make_scene(name), FrameConfig(**kw))
    poses = camera_path("orbit12", seed=7)
    ref = []
    for p in poses[:6]:
        r.set_pose(*p)
        r.gbuffer()
        r.frame()
        ref.append(r.numpy())
    F = 3
    slots = [r] + [r.frame_slot(own_gbuffer=True) for _ in range(F - 1)]
    frames = [BandFrame(s, throughput=True) for s in slots]
    streams = [torch.cuda.Stream() for _ in range(F)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    out = {}
    for group in (range(0, 3), range(3, 6)):  # 3 frames in flight, then read them back
        for i in group:
            with torch.cuda.stream(streams[i % F]):
                slots[i % F].set_pose(*poses[i])
                slots[i % F].gbuffer()
                frames[i % F].frame()
        torch.cuda.synchronize()
        for i in group:
            out[i] = slots[i % F].numpy()
    for i in range(6):
        for key in ("ao", "stencil", "depth"):
            assert np.array_equal(out[i][key], ref[i][key]), (i, key)
        assert bits_equal(out[i]["sd"], ref[i]["sd"]), i
    assert not np.array_equal(ref[0]["ao"], ref[3]["ao"])  # the poses differ
    r.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("walk", ["fused", "quad"])
def test_longest_first_queue_same_bits(monkeypatch, walk):
    """The longest-first live-ray queue (default) only reorders the work: the SD map equals the
    single-ended queue's (RSD_TRACE_LPT=off) and an absolute-threshold split's, bit for bit."""
    import torch
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS["suntemple_1080p_q"]
    r = Renderer(make_scene(name), FrameConfig(**kw))
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    torch.cuda.synchronize()
    iv = r.ray_minmax.clone()
    maps = []
    for lpt in ("off", None, "2.0", "-0.5"):
        monkeypatch.setenv("RSD_TRACE_WALK", walk)
        if lpt is None:
            monkeypatch.delenv("RSD_TRACE_LPT", raising=False)
        else:
            monkeypatch.setenv("RSD_TRACE_LPT", lpt)
        r.ray_minmax.copy_(iv)
        r.sd.zero_()
        r.sd_trace()
        torch.cuda.synchronize()
        maps.append(r.sd.cpu().numpy().view(np.uint32).copy())
    for m in maps[1:]:
        assert np.array_equal(m, maps[0])
    r.close()
