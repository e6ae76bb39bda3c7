"""GPU parity: librsd's HIP kernels vs the CPU oracle on identical inputs.

Bar (DESIGN.md "Parity"): bit-exact.  Depth maps, SD maps and ray intervals are
compared as raw bits; AO and stencil are integer images.  The any-hit stream is
canonical, so the product's SAH BVH and the oracle's median BVH must produce the
same bits.  All inputs are seeded and deterministic."""
import ctypes as C

import numpy as np
import pytest

from helpers import oracle_frame, small_frame_config, to_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.fixture(scope="module")
def device(torch_dev):
    from rsd.frame import Device
    d = Device(0)
    yield d
    d.close()


_scene_cache = {}


def scenes(name, device, oracle):
    if name not in _scene_cache:
        from rsd.frame import GpuScene
        from rsd.scenes import make_scene
        s = make_scene(name)
        _scene_cache[name] = (s, GpuScene(device, s), oracle.Scene(s.positions, s.indices, s.flags, s.alpha))
    return _scene_cache[name]


def renderer(name, cfg, device, oracle):
    from rsd.frame import Renderer
    s, gs, os_ = scenes(name, device, oracle)
    return Renderer(s, cfg, dev=device, gpu_scene=gs), os_


def oracle_structs(r, oracle):
    return (to_oracle(r.cam, oracle.Camera), to_oracle(r.vao, oracle.VAOData), to_oracle(r.sdp, oracle.SDParams),
            to_oracle(r.svp, oracle.SVAOParams))


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


@pytest.mark.parametrize("cull", [0, 1, 2])
def test_gbuffer_parity(device, oracle, cull):
    cfg = small_frame_config(visible=(200, 120), guard=16)
    cfg.cull_mode = cull
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    g = r.numpy()
    cam, _, _, _ = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cull)
    assert bits_equal(g["depth"], z)
    assert np.array_equal(g["normals"], n)


@pytest.mark.parametrize("divisor", [1, 2, 4])
def test_pass1_parity(device, oracle, divisor):
    cfg = small_frame_config(visible=(224, 128), guard=32, divisor=divisor)
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    ao, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, g["depth"], g["normals"], r.sd_w, r.sd_h)
    assert np.array_equal(g["stencil"], st)
    assert np.array_equal(g["ao"], ao)
    assert np.array_equal(g["ray_min"], rmin)
    assert np.array_equal(g["ray_max"], rmax)


@pytest.mark.parametrize("N,impl,max_count", [(1, 0, 1), (2, 0, 8), (4, 0, 8), (8, 0, 8), (16, 0, 16),
                                              (4, 3, 8), (8, 3, 8), (4, 1, 8), (2, 1, 8), (4, 0, 32)])
def test_sd_trace_parity(device, oracle, N, impl, max_count):
    cfg = small_frame_config(visible=(192, 112), guard=32, divisor=2, N=N, max_count=max_count, impl=impl)
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    cnt = r.sd_trace(counters=True)
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    sd, stats = oracle.sd_trace(osc, cam, sdp, g["depth"], g["ray_min"], g["ray_max"], r.sd_w, r.sd_h)
    assert cnt.rays_dispatched == r.sd_w * r.sd_h
    assert cnt.rays_active == stats[0] and cnt.rays_active > 0
    assert bits_equal(g["sd"], sd)


@pytest.mark.parametrize("N", [1, 4, 8])
def test_sd_trace_no_interval_parity(device, oracle, N):
    """SD pass driven directly (config-1 style): no ray interval, guard band 0."""
    cfg = small_frame_config(visible=(128, 128), guard=0, divisor=1, N=N, max_count=8)
    cfg.ray_interval = False
    cfg.sd_guard_px = 0
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.sd_trace()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    sd, stats = oracle.sd_trace(osc, cam, sdp, g["depth"], None, None, r.sd_w, r.sd_h)
    assert stats[0] == r.sd_w * r.sd_h
    assert bits_equal(g["sd"], sd)


@pytest.mark.parametrize("N,divisor", [(4, 4), (8, 1), (1, 2)])
def test_full_frame_parity(device, oracle, N, divisor):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=divisor, N=N)
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    o = oracle_frame(oracle, osc, cam, vao, sdp, svp, cfg.fb_w, cfg.fb_h, r.sd_w, r.sd_h)
    assert bits_equal(g["depth"], o["depth"])
    assert np.array_equal(g["stencil"], o["stencil"])
    assert bits_equal(g["sd"], o["sd"])
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    assert np.array_equal(g["ao"][gv], o["ao"][gv])


def _tiny_scene(kind):
    from rsd.scenes import Scene
    cam = {"pos": [0.0, 0.0, 3.0], "target": [0.0, 0.0, 0.0], "up": [0.0, 1.0, 0.0]}
    if kind == "empty":
        return Scene("empty", np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint32), np.zeros(0, np.uint32), cam)
    pos = np.array([[-1, -1, 0], [1, -1, 0], [0, 1, 0], [-1, -1, -1], [1, -1, -1], [0, 1, -1]], np.float32)
    ind = np.array([[0, 1, 2], [3, 4, 5]], np.uint32)
    if kind == "one":
        ind = ind[:1]
    return Scene(kind, pos, ind, np.zeros(len(ind), np.uint32), cam)


@pytest.mark.parametrize("kind", ["empty", "one", "two"])
def test_degenerate_scenes(device, oracle, kind):
    from rsd.frame import GpuScene, Renderer
    s = _tiny_scene(kind)
    cfg = small_frame_config(visible=(64, 48), guard=8, divisor=1, N=4)
    cfg.ray_interval = False
    cfg.sd_guard_px = 0
    gs = GpuScene(device, s)
    r = Renderer(s, cfg, dev=device, gpu_scene=gs)
    r.gbuffer()
    r.sd_trace()
    g = r.numpy()
    osc = oracle.Scene(s.positions, s.indices, s.flags)
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cfg.cull_mode)
    assert bits_equal(g["depth"], z) and np.array_equal(g["normals"], n)
    sd, stats = oracle.sd_trace(osc, cam, sdp, z, None, None, r.sd_w, r.sd_h)
    assert bits_equal(g["sd"], sd)
    gs.release()


@pytest.mark.parametrize("world", [2, 3])
def test_band_union_equals_full_frame(device, oracle, world):
    """Running every band of a B-way screen-band split covers exactly the full frame."""
    cfg = small_frame_config(visible=(224, 136), guard=16, divisor=2, N=4)
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    full = r.numpy()
    r.ao.zero_()
    r.stencil.zero_()
    r.sd.zero_()
    r.clear_intervals()
    for b in range(world):
        r.pass1(band=(b, world))
    for b in range(world):
        r.sd_trace(band=(b, world))
    for b in range(world):
        r.pass2(band=(b, world))
    g = r.numpy()
    for k in ("ao", "stencil", "ray_min", "ray_max"):
        assert np.array_equal(g[k], full[k]), k
    assert bits_equal(g["sd"], full["sd"])


@pytest.mark.parametrize("ray_pipeline,cull", [(1, 1), (0, 1), (1, 0), (0, 2)])
def test_raytraced_svao_parity(device, oracle, ray_pipeline, cull):
    """SVAO secondaryDepthMode Raytraced: pass 1 with TRACE_OUT_OF_SCREEN
    and the aoAnyHit pass 2, both extents (rayPipeline), all cull modes."""
    from rsd import abi
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=1)
    cfg.secondary = abi.DEPTH_RAYTRACED
    cfg.ray_pipeline = bool(ray_pipeline)
    cfg.cull_mode = cull
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    assert vao.sdGuard == 0
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cull)
    ao1, st, _, _ = oracle.svao_pass1(cam, vao, svp, z, n, r.sd_w, r.sd_h)
    assert np.array_equal(g["stencil"], st)
    assert (st != 0).sum() > 100, "no refined directions: the test frame is degenerate"
    ao = oracle.svao_pass2_raytraced(osc, cam, vao, svp, z, n, st, ao1, cull=cull, ray_pipeline=ray_pipeline)
    assert np.array_equal(g["ao"], ao)
    assert not np.array_equal(ao, ao1)  # the refinement changed something


def test_raytraced_band_union_equals_full_frame(device, oracle):
    from rsd import abi
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=1)
    cfg.secondary = abi.DEPTH_RAYTRACED
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    full = r.numpy()
    r.ao.zero_()
    r.stencil.zero_()
    for b in range(3):
        r.pass1(band=(b, 3))
    for b in range(3):
        r.pass2_raytraced(band=(b, 3))
    g = r.numpy()
    assert np.array_equal(g["stencil"], full["stencil"]) and np.array_equal(g["ao"], full["ao"])


# ---- alpha-masked materials ------------------------------------------

@pytest.mark.parametrize("cull", [0, 1])
def test_gbuffer_alpha_parity(device, oracle, cull):
    """Primary visibility skips alpha-masked hits failing the alpha test at LOD 0."""
    cfg = small_frame_config(visible=(200, 120), guard=16)
    cfg.cull_mode = cull
    r, osc = renderer("foliage_small", cfg, device, oracle)
    r.gbuffer()
    g = r.numpy()
    cam, _, _, _ = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cull)
    assert bits_equal(g["depth"], z)
    assert np.array_equal(g["normals"], n)
    # the cards do cut holes: the opaque variant of the scene sees different depths
    from rsd.scenes import make_scene
    s = make_scene("foliage_small", alpha=False)
    zo, _ = oracle.gbuffer(oracle.Scene(s.positions, s.indices, s.flags), cam, cfg.fb_w, cfg.fb_h, cull)
    assert (zo != z).sum() > 200


@pytest.mark.parametrize("walk", ["split", "fused", "quad"])
@pytest.mark.parametrize("N,impl,max_count", [(4, 0, 8), (8, 3, 8), (4, 1, 8), (2, 0, 1)])
def test_sd_trace_alpha_parity(device, oracle, walk, N, impl, max_count, monkeypatch):
    """SD any-hit with USE_ALPHA_TEST at the ray-cone LOD, every traversal walk."""
    monkeypatch.setenv("RSD_TRACE_WALK", walk)
    cfg = small_frame_config(visible=(192, 112), guard=32, divisor=2, N=N, max_count=max_count, impl=impl)
    r, osc = renderer("foliage_small", cfg, device, oracle)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    r.sd_trace()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    assert sdp.alpha_test == 1
    sd, stats = oracle.sd_trace(osc, cam, sdp, g["depth"], g["ray_min"], g["ray_max"], r.sd_w, r.sd_h)
    assert stats[0] > 0
    assert bits_equal(g["sd"], sd)
    # AlphaTest off: the cards are opaque to the SD rays
    sdp.alpha_test = 0
    sd0, _ = oracle.sd_trace(osc, cam, sdp, g["depth"], g["ray_min"], g["ray_max"], r.sd_w, r.sd_h)
    r.sdp.alpha_test = 0
    r.sd_trace()
    g0 = r.numpy()
    assert bits_equal(g0["sd"], sd0)
    assert not bits_equal(sd0, sd)


@pytest.mark.parametrize("alpha_test", [1, 0])
def test_raytraced_svao_alpha_parity(device, oracle, alpha_test):
    from rsd import abi
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=1)
    cfg.secondary = abi.DEPTH_RAYTRACED
    cfg.alpha_test = bool(alpha_test)
    r, osc = renderer("foliage_small", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cfg.cull_mode)
    assert bits_equal(g["depth"], z)
    ao1, st, _, _ = oracle.svao_pass1(cam, vao, svp, z, n, r.sd_w, r.sd_h)
    assert np.array_equal(g["stencil"], st)
    ao = oracle.svao_pass2_raytraced(osc, cam, vao, svp, z, n, st, ao1, cull=cfg.cull_mode,
                                     ray_pipeline=int(cfg.ray_pipeline), alpha_test=alpha_test)
    assert np.array_equal(g["ao"], ao)


def test_full_frame_alpha_parity(device, oracle):
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=4, N=4)
    r, osc = renderer("foliage_small", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    o = oracle_frame(oracle, osc, cam, vao, sdp, svp, cfg.fb_w, cfg.fb_h, r.sd_w, r.sd_h)
    assert bits_equal(g["depth"], o["depth"])
    assert bits_equal(g["sd"], o["sd"])
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    assert np.array_equal(g["ao"][gv], o["ao"][gv])


def test_ray_cone_spread_matches_oracle(oracle):
    from rsd import abi
    for f, h in [(21.0, 270), (21.0, 1080), (35.0, 512), (10.0, 77)]:
        assert abi.lib().rsd_ray_cone_spread(f, h) == oracle.ray_cone_spread(f, h)


def test_obj_ingest_frame_parity(device, oracle, tmp_path):
    """An OBJ scene with an alpha-textured (map_d) double-sided card, loaded by rsd.ingest and
    uploaded with rsd_scene_upload_alpha: G-buffer and SD map bit-exact vs the oracle."""
    from test_ingest import _foliage_obj
    from rsd.frame import GpuScene, Renderer
    from rsd.ingest import load_obj
    _foliage_obj(tmp_path)
    B = load_obj(tmp_path / "scene.obj", double_sided={"leaf"})
    B.set_camera((0.5, 0.3, 9.0), (0, 0, 0))
    s = B.build("obj_foliage")
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=1, N=4)
    cfg.ray_interval = False
    cfg.sd_guard_px = 0
    gs = GpuScene(device, s)
    r = Renderer(s, cfg, dev=device, gpu_scene=gs)
    r.gbuffer()
    r.sd_trace()
    g = r.numpy()
    osc = oracle.Scene(s.positions, s.indices, s.flags, s.alpha)
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cfg.cull_mode)
    assert bits_equal(g["depth"], z) and np.array_equal(g["normals"], n)
    sd, _ = oracle.sd_trace(osc, cam, sdp, z, None, None, r.sd_w, r.sd_h)
    assert bits_equal(g["sd"], sd)
    gs.release()


def test_pyscene_ingest_frame_parity(device, oracle):
    """A .pyscene scene (built-in meshes under a node hierarchy, a mirrored instance, an imported
    OBJ, an alpha-masked pane) loaded by rsd.pyscene: G-buffer, SD map and AO bit-exact vs the
    oracle."""
    from conftest import ROOT
    from rsd.frame import GpuScene, Renderer
    from rsd.pyscene import load_pyscene
    s = load_pyscene(ROOT / "tests" / "fixtures" / "courtyard.pyscene").build("courtyard")
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=2, N=4)
    gs = GpuScene(device, s)
    r = Renderer(s, cfg, dev=device, gpu_scene=gs)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    osc = oracle.Scene(s.positions, s.indices, s.flags, s.alpha)
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cfg.cull_mode)
    assert bits_equal(g["depth"], z) and np.array_equal(g["normals"], n)
    ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, z, n, r.sd_w, r.sd_h)
    sd, _ = oracle.sd_trace(osc, cam, sdp, z, rmin, rmax, r.sd_w, r.sd_h)
    assert bits_equal(g["sd"], sd)
    assert np.array_equal(g["ao"], oracle.svao_pass2(cam, vao, svp, z, n, st, sd, ao1))
    assert (rmax != 0).sum() > 0
    gs.release()


def test_fbx_ingest_frame_parity(device, oracle):
    """The reference's binary FBX fixture (data/framework/meshes/sphere.fbx) loaded by rsd.fbx -- twice, once
    through a scaled, rotated and translated instance -- on a floor: G-buffer, pass-1 intervals, SD map and AO
    bit-exact vs the oracle."""
    from conftest import ROOT
    from rsd.fbx import euler, load_fbx
    from rsd.frame import GpuScene, Renderer
    from rsd.ingest import Mesh
    fx = ROOT / "tests" / "fixtures" / "sphere.fbx"
    B = load_fbx(fx)
    T = euler((0.0, 30.0, 10.0))
    T[:3, :3] *= 0.6
    T[:3, 3] = (1.4, 0.6, -0.5)
    load_fbx(fx, transform=T, builder=B)
    floor = Mesh(np.array([[-4, -1, 4], [4, -1, 4], [4, -1, -4], [-4, -1, -4]], np.float32),
                 np.array([[0, 1, 2], [0, 2, 3]], np.uint32))
    B.add_instance(B.add_mesh(floor))
    B.set_camera((0.3, 1.2, 4.5), (0.4, -0.2, 0.0))
    s = B.build("fbx_spheres")
    assert len(s.indices) == 2 * 760 + 2
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=2, N=4)
    gs = GpuScene(device, s)
    r = Renderer(s, cfg, dev=device, gpu_scene=gs)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    osc = oracle.Scene(s.positions, s.indices, s.flags, s.alpha)
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cfg.cull_mode)
    assert bits_equal(g["depth"], z) and np.array_equal(g["normals"], n)
    ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, z, n, r.sd_w, r.sd_h)
    sd, _ = oracle.sd_trace(osc, cam, sdp, z, rmin, rmax, r.sd_w, r.sd_h)
    assert (rmax != 0).sum() > 0
    assert bits_equal(g["sd"], sd)
    assert np.array_equal(g["ao"], oracle.svao_pass2(cam, vao, svp, z, n, st, sd, ao1))
    gs.release()


def test_consumed_intervals_frames_match_fresh_frames(device, oracle):
    """BandFrame folds the interval clear into the trace (RSD_SD_CONSUME_INTERVALS): after
    a consuming trace the maps are exactly the cleared state, and consecutive frames stay
    bit-identical to a frame with an explicit clear."""
    from rsd.shard import BandFrame
    cfg = small_frame_config(visible=(224, 136), guard=16, divisor=2, N=4)
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    want = r.numpy()
    bf = BandFrame(r, 0, 1)
    for k in range(3):
        bf.frame()
        g = r.numpy()
        assert (g["ray_min"] == 0x7F7FFFFF).all() and (g["ray_max"] == 0).all(), k
        assert bits_equal(g["sd"], want["sd"]) and np.array_equal(g["ao"], want["ao"]), k
        assert np.array_equal(g["stencil"], want["stencil"]), k


def test_sd_trace_on_many_streams(device, oracle):
    """librsd keeps the SD-trace scratch per (scene, stream) and recycles it past 16 streams:
    traces on 20 fresh streams (both walks) all give the default-stream SD map."""
    import torch
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=2, N=4)
    r, _ = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    r.sd_trace()
    ref = r.numpy()["sd"].view(np.uint32).copy()
    for k in range(20):
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            r.sd.zero_()
            r.sd_trace(throughput=bool(k % 2))
        torch.cuda.current_stream().wait_stream(st)
        assert np.array_equal(r.numpy()["sd"].view(np.uint32), ref), k


# ---- NUM_DIRECTIONS 16 / 32 (Common.slang:51-58; R16Uint / R32Uint stencils, SVAO.cpp:132-134) ----

@pytest.mark.parametrize("nd", [16, 32])
@pytest.mark.parametrize("N,divisor", [(4, 2), (8, 1)])
def test_directions_full_frame_parity(device, oracle, nd, N, divisor):
    cfg = small_frame_config(visible=(224, 128), guard=32, divisor=divisor, N=N)
    cfg.num_directions = nd
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    assert svp.num_directions == nd
    o = oracle_frame(oracle, osc, cam, vao, sdp, svp, cfg.fb_w, cfg.fb_h, r.sd_w, r.sd_h)
    assert g["stencil"].dtype == o["stencil"].dtype == {16: np.uint16, 32: np.uint32}[nd]
    assert np.array_equal(g["stencil"], o["stencil"])
    assert (o["stencil"] >> 8 != 0).sum() > 50, "no direction above 8 refined: the frame is degenerate"
    assert np.array_equal(g["ray_min"], o["ray_min"]) and np.array_equal(g["ray_max"], o["ray_max"])
    assert bits_equal(g["sd"], o["sd"])
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    assert np.array_equal(g["ao"][gv], o["ao"][gv])


@pytest.mark.parametrize("nd", [16, 32])
def test_directions_raytraced_parity(device, oracle, nd):
    from rsd import abi
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=1)
    cfg.secondary = abi.DEPTH_RAYTRACED
    cfg.num_directions = nd
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cfg.cull_mode)
    ao1, st, _, _ = oracle.svao_pass1(cam, vao, svp, z, n, r.sd_w, r.sd_h)
    assert np.array_equal(g["stencil"], st)
    ao = oracle.svao_pass2_raytraced(osc, cam, vao, svp, z, n, st, ao1, cull=cfg.cull_mode, ray_pipeline=1)
    assert np.array_equal(g["ao"], ao)


def test_directions_unsupported(device, oracle):
    """Common.slang:51-58 has sample radii for 8, 16 and 32 directions only: librsd refuses others."""
    cfg = small_frame_config(visible=(96, 64), guard=16, divisor=2)
    r, _ = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.svp.num_directions = 12
    with pytest.raises(Exception, match="NUM_DIRECTIONS"):
        r.pass1()


# ---- dualAO (SVAO.cpp:129-131: RG8Unorm bright / dark; SVAORaster.ps.slang:101-104, SVAORaster2.ps.slang:60-64) ----

@pytest.mark.parametrize("nd", [8, 16])
def test_dual_ao_full_frame_parity(device, oracle, nd):
    cfg = small_frame_config(visible=(224, 128), guard=32, divisor=2, N=4)
    cfg.dual_ao = True
    cfg.num_directions = nd
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    assert svp.dual_ao == 1
    o = oracle_frame(oracle, osc, cam, vao, sdp, svp, cfg.fb_w, cfg.fb_h, r.sd_w, r.sd_h)
    assert g["ao"].shape == o["ao"].shape == (cfg.fb_h, cfg.fb_w, 2)
    assert np.array_equal(g["stencil"], o["stencil"])
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    assert np.array_equal(g["ao"][gv], o["ao"][gv])
    assert (o["ao"][gv][..., 1] < o["ao"][gv][..., 0]).any()  # the dark channel differs somewhere


def test_dual_ao_raytraced_parity(device, oracle):
    from rsd import abi
    cfg = small_frame_config(visible=(160, 96), guard=16, divisor=1)
    cfg.secondary = abi.DEPTH_RAYTRACED
    cfg.dual_ao = True
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.frame()
    g = r.numpy()
    cam, vao, sdp, svp = oracle_structs(r, oracle)
    z, n = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, cfg.cull_mode)
    ao1, st, _, _ = oracle.svao_pass1(cam, vao, svp, z, n, r.sd_w, r.sd_h)
    assert np.array_equal(g["stencil"], st)
    ao = oracle.svao_pass2_raytraced(osc, cam, vao, svp, z, n, st, ao1, cull=cfg.cull_mode, ray_pipeline=1)
    assert np.array_equal(g["ao"], ao)


@pytest.mark.parametrize("nd,visible", [(8, (224, 128)), (16, (224, 128)), (8, (200, 120)), (8, (1000, 72))])
def test_busy_tile_flags(device, oracle, torch_dev, nd, visible):
    """rsd_svao_params.tile_flags (ABI v4): pass 1 flags exactly the 16x16 tiles of the visible region
    that hold a stencilled VISIBLE pixel; pass 2 visits only those and clears them; the AO equals a
    frame without flags (every tile visited) and the oracle.  Widths 200 and 1000 (width % 32 in
    [1, 16]): pass 1's padded dispatch runs 16 columns right of the last tile, whose pixels must not
    vote (they would flag the next row's first tile, or write past the buffer on the last row)."""
    cfg = small_frame_config(visible=visible, guard=32, divisor=2)
    cfg.num_directions = nd
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    r.clear_intervals()
    r.pass1()
    g = r.numpy()
    buf = r.tile_flags.cpu().numpy().view(np.uint32)
    g_, vw, vh = cfg.guard_band, cfg.visible_w, cfg.visible_h
    tx, ty = (vw + 15) // 16, (vh + 31) // 32 * 32 // 16
    T = tx * ty
    assert buf.size == 2 * T + 4  # T flag words, {count[2], -, -}, T list entries (ABI v5)
    # frames alternate between the two counts; pass 1 zeroes the one it does not append to
    assert buf[T] == 0 or buf[T + 1] == 0
    count = int(buf[T]) + int(buf[T + 1])
    flags, lst = buf[:T], buf[T + 4:T + 4 + count]
    # the list holds every flagged tile once
    assert count == int(flags.sum()) and sorted(lst.tolist()) == np.flatnonzero(flags).tolist()
    st = np.zeros((ty * 16, tx * 16), g["stencil"].dtype)
    st[:vh, :vw] = g["stencil"][g_:g_ + vh, g_:g_ + vw]  # visible pixels only
    want = np.zeros((ty, tx), np.uint8)
    for j in range(ty):
        for i in range(tx):
            want[j, i] = (st[16 * j:16 * j + 16, 16 * i:16 * i + 16] != 0).any()
    assert want.any() and not want.all()
    assert np.array_equal(flags.reshape(ty, tx), want)
    r.sd_trace()
    r.pass2()
    with_flags = r.numpy()["ao"]
    assert not r.tile_flags.cpu().numpy().view(np.uint32)[:T].any()  # flags consumed
    # the same frame without flags
    from rsd import abi
    svp = abi.SVAOParams.from_buffer_copy(r.svp)
    svp.tile_flags = None
    r.svp, keep = svp, r.svp
    r.ao.zero_()
    r.clear_intervals()
    r.pass1()
    r.sd_trace()
    r.pass2()
    assert np.array_equal(r.numpy()["ao"], with_flags)
    r.svp = keep
    cam, vao, sdp, svp_o = oracle_structs(r, oracle)
    o = oracle_frame(oracle, osc, cam, vao, sdp, svp_o, cfg.fb_w, cfg.fb_h, r.sd_w, r.sd_h)
    assert np.array_equal(with_flags, o["ao"])


def test_busy_tile_list_and_flag_grid_agree(device, oracle, torch_dev):
    """The whole-frame pass 2 walks pass 1's busy-tile list; a row-range pass 2 (HaloFrame's bands)
    visits the flagged tiles of its rows.  Both give the same AO and consume every flag; any sequence
    of the two keeps the alternating list counts consistent (svao.hip tile_gen), including two pass 1
    runs before one pass 2 (the flags OR, the list holds each tile once)."""
    cfg = small_frame_config(visible=(224, 128), guard=32, divisor=2)
    r, osc = renderer("arcade_tiny", cfg, device, oracle)
    r.gbuffer()
    vw, vh = cfg.visible_w, cfg.visible_h
    T = ((vw + 15) // 16) * ((vh + 31) // 32 * 2)
    out = []
    for mode in ("list", "rows", "rows", "list", "list", "twice", "rows", "list"):
        r.ao.zero_()
        r.clear_intervals()
        r.pass1()
        if mode == "twice":
            r.clear_intervals()
            r.pass1()
        r.sd_trace()
        if mode == "rows":
            r.pass2_rows((0, 64))
            r.pass2_rows((64, vh))
        else:
            r.pass2()
        out.append(r.numpy()["ao"])
        assert not r.tile_flags.cpu().numpy().view(np.uint32)[:T].any(), mode
    for mode, ao in zip(("list", "rows", "rows", "list", "list", "twice", "rows", "list"), out):
        assert np.array_equal(out[0], ao), mode


def test_busy_tile_loop_matches_one_workgroup_per_tile(monkeypatch, torch_dev):
    """At 1080p the specialised pass 2 strides the resident workgroups over the busy-tile list
    (svao_pass2_loop_kernel, ~1.3 busy tiles per workgroup at configs[1]); RSD_PASS2_LOOP=off gives every
    list entry its own workgroup.  Same AO bits, every flag consumed, over frames of a camera path."""
    from rsd.frame import CONFIGS, FrameConfig, Renderer, camera_path
    from rsd.scenes import make_scene
    kw, sc = CONFIGS["suntemple_1080p_q"]
    r = Renderer(make_scene(sc), FrameConfig(**kw))
    vw, vh = r.cfg.visible_w, r.cfg.visible_h
    T = ((vw + 15) // 16) * ((vh + 31) // 32 * 2)  # the flags; the list and its counts follow them
    poses = [None] + camera_path("orbit120")[::50]
    for frame, pose in enumerate(poses):
        if pose is not None:
            r.set_pose(*pose)
        r.gbuffer()
        aos = []
        for loop in ("on", "off"):
            monkeypatch.setenv("RSD_PASS2_LOOP", loop)
            r.ao.zero_()
            r.clear_intervals()
            r.pass1()
            r.sd_trace()
            r.pass2()
            aos.append(r.numpy()["ao"])
            assert not r.tile_flags.cpu().numpy().view(np.uint32)[:T].any(), (frame, loop)
        assert np.array_equal(aos[0], aos[1]), frame
        assert (aos[0] != aos[0].flat[0]).any()  # a non-trivial AO image


def test_stale_tile_flags_do_not_hide_tiles(device):
    """a pass 1 over some rows whose busy tiles no pass 2 consumed (a pass 2 over OTHER rows) leaves
    their flags set; the next whole frame must still list those tiles (pass 1 stamps a flag with the buffer's
    generation, svao.hip tile_gen_pass1) and equal a clean frame bit for bit."""
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS["suntemple_1080p_q"]
    r = Renderer(make_scene(name), FrameConfig(**kw))
    r.gbuffer()
    r.frame()
    ref = r.numpy()["ao"]
    r.clear_intervals()
    r.pass1_rows((0, 320))
    r.sd_trace()
    r.pass2_rows((640, 960))  # consumes only its own rows' flags
    torch_ao = r.ao
    torch_ao.zero_()
    r.frame()
    assert np.array_equal(r.numpy()["ao"], ref)
    r.close()
