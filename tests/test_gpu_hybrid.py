"""The hybrid SD walk (rsd.h RSD_WALK_HYBRID, csrc/sd_trace.hip walk 6): with one frame in flight the longest-first rays
take the row walk and the others the quad walk, in one launch (K = 16, an A/B option since round 6: 8-lane rows holding
two keys per lane).  Canonical hit stream, so the bits must be the single
walk's (and the oracle's, which the parity / configs tests check at every config)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(t):
    return np.ascontiguousarray(t.cpu().numpy()).view(np.uint32)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config,alone", [("emerald_4k_q", "quad"), ("bistro_1080p_full", "quad"),
                                          ("suntemple_1080p_q", "fused"),
                                          ("bistro_4k_full_n16", "quad")])  # K = 16: two keys per row lane
def test_hybrid_walk_equals_quad_walk(config, alone):
    import torch
    from rsd import abi
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS[config]
    if kw.get("sd_samples") == 16:  # K = 16: the two-keys-per-lane rows, an A/B option (sd_trace.hip hybridK)
        os.environ["RSD_TRACE_HYBRID16"] = "on"
    r = Renderer(make_scene(name), FrameConfig(**kw))
    r.keep_clean_tiles()
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    torch.cuda.synchronize()
    saved = r.ray_minmax.clone()
    maps = {}
    try:
        for mode in ("off", "on"):
            os.environ["RSD_TRACE_HYBRID"] = mode
            for rep in range(2):  # the second trace of the map runs over clean tiles
                r.ray_minmax.copy_(saved)
                r.sd_trace()
            torch.cuda.synchronize()
            maps[mode] = bits(r.sd)
            c = r.sd_trace(counters=True)
            single = abi.WALK_QUAD if alone == "quad" else abi.WALK_FUSED
            assert int(c.walk) == (abi.WALK_HYBRID if mode == "on" else single), (mode, int(c.walk))
            # with frames in flight (RSD_SD_THROUGHPUT) the quad walk of the full-resolution maps runs alone; the
            # fused row walk of the small maps is replaced by the hybrid there too (round 6, sd_trace.hip hybridOk)
            c = r.sd_trace(counters=True, throughput=True)
            assert int(c.walk) == (abi.WALK_HYBRID if mode == "on" and alone == "fused" else single), (mode, int(c.walk))
        # band split by SD rows (the band frame's full-resolution split): the same rows, the same bits
        r.ray_minmax.copy_(saved)
        r.invalidate_sd_tiles()
        r.sd.zero_()
        h = r.sd_h // 16 * 8  # a multiple of 8 rows
        r.sd_trace_rows((0, h))
        torch.cuda.synchronize()
        half = bits(r.sd)[:, :h]
    finally:
        os.environ.pop("RSD_TRACE_HYBRID", None)
        os.environ.pop("RSD_TRACE_HYBRID16", None)
    assert np.array_equal(maps["on"], maps["off"])
    assert np.array_equal(half, maps["off"][:, :h])
    r.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("scene,N,max_count", [("arcade_tiny", 16, 16), ("arcade_tiny", 8, 16), ("arcade_tiny", 16, 12),
                                               ("suntemple", 16, 16)])
def test_two_keys_per_lane_rows_equal_oracle(oracle, scene, N, max_count):
    """K = 16 on 8-lane rows (row_insert2 / sd_algorithm_row2: lane l holds keys 2l and 2l + 1), the hybrid's row blocks
    with RSD_TRACE_HYBRID16=on: the SD map of an uninstrumented trace equals the oracle's bit for bit."""
    import torch
    from helpers import small_frame_config, to_oracle
    from rsd import abi
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    s = make_scene(scene, target_tris=60_000 if scene == "suntemple" else None)
    cfg = small_frame_config(visible=(320, 192), guard=32, divisor=1, N=N, max_count=max_count)
    r = Renderer(s, cfg)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    os.environ["RSD_TRACE_HYBRID16"] = "on"
    try:
        assert int(r.sd_trace(counters=True).walk) == abi.WALK_HYBRID
        r.sd_trace()
        torch.cuda.synchronize()
    finally:
        os.environ.pop("RSD_TRACE_HYBRID16", None)
    g = r.numpy()
    osc = oracle.Scene(s.positions, s.indices, s.flags, s.alpha)
    sd, stats = oracle.sd_trace(osc, to_oracle(r.cam, oracle.Camera), to_oracle(r.sdp, oracle.SDParams), g["depth"],
                                g["ray_min"], g["ray_max"], r.sd_w, r.sd_h)
    assert stats[0] > 0
    assert np.array_equal(np.ascontiguousarray(g["sd"]).view(np.uint32), np.ascontiguousarray(sd).view(np.uint32))
    r.close()
