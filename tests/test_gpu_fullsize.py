"""GPU parity at the BASELINE configs' full sizes (configs[2..4]: 1080p full-res N = 8 on a
2.8 M-triangle scene, 4K 1/4-res on 10 M triangles, 4K full-res N = 16).

Each stage is checked on the GPU's own inputs (the stages are deterministic functions of them):
pass 1 over the full frame, the SD trace over the WHOLE SD map (the oracle on every host CPU it
may use: only the live texels cost a traversal, ~0.2 M at configs[2]), and pass 2 over the full
frame.  Bit-exact, like test_gpu_parity.py.  (configs[1]: tests/test_gpu_configs.py and every
bench.py run, cpu_baseline.bit_identical_to_gpu.)"""
import numpy as np
import pytest

from helpers import to_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
@pytest.mark.parametrize("config", ["bistro_1080p_full", "emerald_4k_q", "bistro_4k_full_n16"])
def test_fullsize_config_parity(oracle, config):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, scene_name = CONFIGS[config]
    scene = make_scene(scene_name)
    cfg = FrameConfig(**kw)
    r = Renderer(scene, cfg)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao = to_oracle(r.cam, oracle.Camera), to_oracle(r.vao, oracle.VAOData)
    sdp, svp = to_oracle(r.sdp, oracle.SDParams), to_oracle(r.svp, oracle.SVAOParams)

    # pass 1 ("AO 1") over the whole frame, on the GPU's G-buffer
    ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, g["depth"], g["normals"], r.sd_w, r.sd_h)
    assert np.array_equal(g["stencil"], st)
    assert np.array_equal(g["ray_min"], rmin) and np.array_equal(g["ray_max"], rmax)
    assert (rmax != 0).sum() > 1000, "no SD rays requested: degenerate frame"

    # SD trace: the whole map, every texel's bits
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags, scene.alpha)
    sd, stats = oracle.sd_trace(osc, cam, sdp, g["depth"], rmin, rmax, r.sd_w, r.sd_h)
    assert stats[0] > 1000, "no live SD rays: degenerate frame"
    diff = (sd.view(np.uint32) != g["sd"].view(np.uint32)).any(axis=(0, 3))
    assert not diff.any(), (config, int(diff.sum()), np.argwhere(diff)[:5].tolist())

    # pass 2 ("AO 2") over the whole frame, on the GPU's SD map
    ao = oracle.svao_pass2(cam, vao, svp, g["depth"], g["normals"], st, g["sd"], ao1)
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    assert np.array_equal(g["ao"][gv], ao[gv])
    r.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("config,flight,walk", [("suntemple_1080p_q", 2, None), ("suntemple_1080p_q", 3, "quad"),
                                                ("suntemple_1080p_q", 4, None), ("emerald_4k_q", 2, None)])
def test_frames_in_flight_equal_sequential(monkeypatch, config, flight, walk):
    """bench.py's frames in flight: F frame slots on F streams, frames overlapping across slots
    (each slot consuming its own interval maps), give the sequential frame bit-for-bit in every
    slot -- librsd's SD-trace scratch is per (scene, stream), so concurrent traces of one scene
    never share it.  The sequential frame itself is pinned against the oracle above / by bench.py."""
    import torch
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    from rsd.shard import BandFrame
    kw, scene_name = CONFIGS[config]
    r = Renderer(make_scene(scene_name), FrameConfig(**kw))
    r.gbuffer()
    r.frame()
    ref = r.numpy()
    slots = [r] + [r.frame_slot() for _ in range(flight - 1)]
    for s in slots:
        s.sd.zero_()
        s.ao.zero_()
    if walk:  # the depth-first quad walk (the default is the row walk, with or without RSD_SD_THROUGHPUT)
        monkeypatch.setenv("RSD_TRACE_WALK", walk)
    frames = [BandFrame(s, throughput=True) for s in slots]
    streams = [torch.cuda.Stream() for _ in slots]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    for i in range(4 * flight):
        with torch.cuda.stream(streams[i % flight]):
            frames[i % flight].frame()
    torch.cuda.synchronize()
    for k, s in enumerate(slots):
        g = s.numpy()
        for key in ("ao", "stencil"):
            assert np.array_equal(g[key], ref[key]), (k, key)
        assert np.array_equal(g["sd"].view(np.uint32), ref["sd"].view(np.uint32)), k
        # the last trace of every slot consumed (reset) its intervals for the next frame
        assert (g["ray_max"] == 0).all() and (g["ray_min"] == np.uint32(0x7F7FFFFF)).all(), k
    r.close()

