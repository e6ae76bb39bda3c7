"""GPU: the segment entry grid (csrc/entry_grid.h) changes where a canonical walk starts, never
what it finds.  Every walk (fused row, split row, quad) with the grid on must give the SD map of
the same walk from the root (RSD_TRACE_ENTRY=off) bit for bit, and the oracle's; the grid must
cut the node visits; a scene uploaded without a grid (RSD_ENTRY_CELLS=0) traces the same bits."""
import numpy as np
import pytest

from helpers import small_frame_config, to_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def device():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import Device
    d = Device(0)
    yield d
    d.close()


_scenes = {}


def gpu_scene(name, device, cells=None, monkeypatch=None):
    key = (name, cells)
    if key not in _scenes:
        from rsd.frame import GpuScene
        from rsd.scenes import make_scene
        s = make_scene(name) if name != "suntemple_small" else make_scene("suntemple", target_tris=120_000)
        if cells is not None:
            monkeypatch.setenv("RSD_ENTRY_CELLS", str(cells))
        _scenes[key] = (s, GpuScene(device, s))
        if cells is not None:
            monkeypatch.delenv("RSD_ENTRY_CELLS")
    return _scenes[key]


def trace(r, monkeypatch, entry, walk, throughput=False):
    monkeypatch.setenv("RSD_TRACE_ENTRY", entry)
    if walk:
        monkeypatch.setenv("RSD_TRACE_WALK", walk)
    else:
        monkeypatch.delenv("RSD_TRACE_WALK", raising=False)
    cnt = r.sd_trace(counters=True, throughput=throughput)
    return r.numpy()["sd"].view(np.uint32).copy(), cnt


@pytest.mark.parametrize("scene", ["arcade_tiny", "suntemple_small"])
@pytest.mark.parametrize("walk", ["fused", "split", "quad"])
@pytest.mark.parametrize("N,impl,max_count", [(4, 0, 8), (4, 1, 8), (8, 3, 8), (16, 0, 16), (2, 0, 32)])
def test_entry_grid_same_bits(device, oracle, monkeypatch, scene, walk, N, impl, max_count):
    from rsd.frame import Renderer
    if walk == "split" and (impl == 1 or max_count > 16):
        pytest.skip("the split walk needs MaxCount <= K (the trace falls back to the fused walk)")
    s, gs = gpu_scene(scene, device)
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=N, max_count=max_count, impl=impl)
    r = Renderer(s, cfg, dev=device, gpu_scene=gs)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    on, c_on = trace(r, monkeypatch, "on", walk)
    off, c_off = trace(r, monkeypatch, "off", walk)
    assert np.array_equal(on, off)
    assert c_on.rays_active == c_off.rays_active > 0
    if scene == "arcade_tiny":
        g = r.numpy()
        cam = to_oracle(r.cam, oracle.Camera)
        sdp = to_oracle(r.sdp, oracle.SDParams)
        osc = oracle.Scene(s.positions, s.indices, s.flags)
        sd, _ = oracle.sd_trace(osc, cam, sdp, g["depth"], g["ray_min"], g["ray_max"], r.sd_w, r.sd_h)
        assert np.array_equal(on, np.ascontiguousarray(sd).view(np.uint32))


def test_entry_grid_cuts_node_visits(device, monkeypatch):
    """configs[1]-like frame of a 120 K-triangle stand-in: the walks start below the tree top."""
    from rsd.frame import Renderer
    s, gs = gpu_scene("suntemple_small", device)
    assert gs.info.entry_cells > 0
    cfg = small_frame_config(visible=(480, 272), guard=32, divisor=4, N=4, max_count=8)
    r = Renderer(s, cfg, dev=device, gpu_scene=gs)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    on, c_on = trace(r, monkeypatch, "on", "fused")
    off, c_off = trace(r, monkeypatch, "off", "fused")
    assert np.array_equal(on, off)
    assert c_on.nodes_visited < 0.8 * c_off.nodes_visited, (c_on.nodes_visited, c_off.nodes_visited)


def test_entry_grid_no_interval_and_throughput(device, monkeypatch):
    """Without ray intervals every segment runs to farZ: longer than the scene, the walk starts at
    the root; the depth-first quad walk (RSD_SD_THROUGHPUT) gives the same bits as the row walk."""
    from rsd.frame import Renderer
    s, gs = gpu_scene("arcade_tiny", device)
    cfg = small_frame_config(visible=(128, 128), guard=0, divisor=1, N=4, max_count=8)
    cfg.ray_interval = False
    cfg.sd_guard_px = 0
    r = Renderer(s, cfg, dev=device, gpu_scene=gs)
    r.gbuffer()
    a, _ = trace(r, monkeypatch, "on", None)
    b, _ = trace(r, monkeypatch, "off", None)
    c, _ = trace(r, monkeypatch, "on", "quad", throughput=True)
    assert np.array_equal(a, b) and np.array_equal(a, c)


def test_scene_without_entry_grid(device, monkeypatch):
    from rsd.frame import Renderer
    s, gs = gpu_scene("arcade_tiny", device)
    s0, gs0 = gpu_scene("arcade_tiny", device, cells=0, monkeypatch=monkeypatch)
    assert gs0.info.entry_cells == 0 and gs.info.entry_cells > 0
    cfg = small_frame_config(visible=(192, 112), guard=32, divisor=2, N=4, max_count=8)
    maps = []
    for g in (gs, gs0):
        r = Renderer(s, cfg, dev=device, gpu_scene=g)
        r.gbuffer()
        r.clear_intervals()
        r.pass1()
        maps.append(trace(r, monkeypatch, "on", None)[0])
    assert np.array_equal(maps[0], maps[1])



@pytest.mark.parametrize("offset", [(3000.0, -500.0, 7000.0), (-40000.0, 0.0, 25000.0)])
def test_entry_grid_far_from_origin(device, oracle, monkeypatch, offset):
    """The scene and camera translated far from the origin: coarser float spacing in the setup's
    lookup (segment box pad, cell index) must still only change where the walk starts."""
    import dataclasses
    from rsd.frame import GpuScene, Renderer
    from rsd.scenes import make_scene
    s0 = make_scene("arcade_tiny")
    off = np.asarray(offset, np.float32)
    cam = dict(s0.camera)
    cam["pos"] = [float(a + b) for a, b in zip(cam["pos"], off)]
    cam["target"] = [float(a + b) for a, b in zip(cam["target"], off)]
    s = dataclasses.replace(s0, name="arcade_far", positions=(s0.positions + off).astype(np.float32), camera=cam)
    gs = GpuScene(device, s)
    assert gs.info.entry_cells > 0
    cfg = small_frame_config(visible=(192, 112), guard=32, divisor=2, N=4, max_count=8)
    r = Renderer(s, cfg, dev=device, gpu_scene=gs)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    on, c_on = trace(r, monkeypatch, "on", None)
    off_, _ = trace(r, monkeypatch, "off", None)
    q, _ = trace(r, monkeypatch, "on", "quad")
    assert np.array_equal(on, off_) and np.array_equal(on, q)
    assert c_on.rays_active > 0
    g = r.numpy()
    osc = oracle.Scene(s.positions, s.indices, s.flags)
    sd, _ = oracle.sd_trace(osc, to_oracle(r.cam, oracle.Camera), to_oracle(r.sdp, oracle.SDParams), g["depth"],
                            g["ray_min"], g["ray_max"], r.sd_w, r.sd_h)
    assert np.array_equal(on, np.ascontiguousarray(sd).view(np.uint32))
    gs.release()
