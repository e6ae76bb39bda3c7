"""GPU: an SVAO render graph executed by the C++ graph host (include/rsd_graph.h) vs the
oracle chain GBufferRaster -> LinearizeDepth -> CompressNormals -> SVAO (AO 1, SD trace,
AO 2).  Bit-exact, like test_gpu_parity.py."""
import numpy as np
import pytest

from conftest import ROOT
from helpers import small_frame_config, to_oracle

pytestmark = pytest.mark.gpu

SCRIPT = ROOT / "tests" / "graphs" / "svao_hotpath.py"


@pytest.fixture(scope="module")
def setup(oracle):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd import graph as rg
    from rsd.frame import Device, GpuScene, make_camera, make_vao, sd_params, svao_params
    from rsd.scenes import make_scene
    cfg = small_frame_config()  # 160 x 96 visible, guard 16, divisor 2, N = 4, radius 1, 64 px SD guard
    scene = make_scene("arcade_tiny")
    dev = Device(0)
    gs = GpuScene(dev, scene)
    cam = make_camera(scene, cfg)
    g = rg.load_script(SCRIPT)["SVAOHotPath"]
    g.set_scene(gs.h, cam)
    g.compile(cfg.fb_w, cfg.fb_h)
    g.execute()
    torch.cuda.synchronize()
    vao, sd_w, sd_h = make_vao(cfg)
    yield dict(g=g, cfg=cfg, scene=scene, cam=cam, vao=vao, sd_w=sd_w, sd_h=sd_h, sdp=sd_params(cfg, vao.sdGuard),
               svp=svao_params(cfg), torch=torch)
    g.close()
    gs.release()
    dev.close()


def _np(t):
    return t.cpu().numpy()


@pytest.fixture(scope="module")
def expected(setup, oracle):
    s = setup
    O = oracle
    cfg = s["cfg"]
    ocam = to_oracle(s["cam"], O.Camera)
    oscene = O.Scene(s["scene"].positions, s["scene"].indices, s["scene"].flags)
    d, nw = O.gbuffer_raster(oscene, ocam, cfg.fb_w, cfg.fb_h, 1)
    z = O.linearize_depth(d, ocam.nearZ, ocam.farZ)
    n = O.compress_normals(nw, ocam)
    vao = to_oracle(s["vao"], O.VAOData)
    svp = to_oracle(s["svp"], O.SVAOParams)
    sdp = to_oracle(s["sdp"], O.SDParams)
    ao1, st, rmin, rmax = O.svao_pass1(ocam, vao, svp, z, n, s["sd_w"], s["sd_h"])
    sd, _ = O.sd_trace(oscene, ocam, sdp, z, rmin, rmax, s["sd_w"], s["sd_h"])
    ao = O.svao_pass2(ocam, vao, svp, z, n, st, sd, ao1)
    return dict(depth=d, normal_w=nw, linear_z=z, normals=n, stencil=st, ray_min=rmin, ray_max=rmax, sd=sd, ao=ao)


def test_graph_execution_order(setup):
    g = setup["g"]
    assert g.execution_order() == ["GuardBand", "GBufferRaster", "LinearizeDepth", "CompressNormals", "SVAO",
                                   "Blur"]
    assert g.dict_int("guardBand") == 16
    t = g.pass_times()
    assert set(t) == set(g.execution_order()) and t["SVAO"] > 0.0


def test_graph_gbuffer_chain(setup, expected):
    g = setup["g"]
    np.testing.assert_array_equal(_np(g.output_tensor("GBufferRaster.depth")).view(np.uint32),
                                  expected["depth"].view(np.uint32))
    np.testing.assert_array_equal(_np(g.output_tensor("GBufferRaster.faceNormalW")).view(np.uint32),
                                  expected["normal_w"].view(np.uint32))
    np.testing.assert_array_equal(_np(g.output_tensor("LinearizeDepth.linearDepth")).view(np.uint32),
                                  expected["linear_z"].view(np.uint32))
    np.testing.assert_array_equal(_np(g.output_tensor("CompressNormals.normalOut")).view(np.uint16),
                                  expected["normals"])


def test_graph_svao(setup, expected):
    g = setup["g"]
    rmax = _np(g.output_tensor("SVAO.internalRayMax")).view(np.uint32)
    assert (rmax != 0).sum() > 0, "no SD rays requested: the test frame is degenerate"
    np.testing.assert_array_equal(_np(g.output_tensor("SVAO.stencil")), expected["stencil"])
    np.testing.assert_array_equal(_np(g.output_tensor("SVAO.internalRayMin")).view(np.uint32), expected["ray_min"])
    np.testing.assert_array_equal(rmax, expected["ray_max"])
    np.testing.assert_array_equal(_np(g.output_tensor("SVAO.ao")), expected["ao"])


def test_graph_reexecute_is_stable(setup, expected):
    g, torch = setup["g"], setup["torch"]
    g.execute()
    g.execute()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(g.output_tensor("SVAO.ao")), expected["ao"])


def test_graph_blur(setup, expected, oracle):
    """Blur = CrossBilateralBlur of SVAO.ao over the linear depth, inside the 16 px guard band."""
    g = setup["g"]
    want, _ = oracle.cross_bilateral_blur(expected["ao"], expected["linear_z"], 16)
    got = _np(g.output_tensor("Blur.colorOut"))
    np.testing.assert_array_equal(got, want)
    assert not np.array_equal(got[16:-16, 16:-16], expected["ao"][16:-16, 16:-16])


def test_graph_ao_post_chain(setup, expected, oracle):
    """scripts/SVAO.py's chain to the marked output AmbientRef.out (blur -> disabled TemporalAO
    -> Switch -> ImageEquation 'I0[xy].rrra') and two SAVO_record.py formulas, bit-exact."""
    from oracle import image_eq as IE
    from rsd import graph as rg
    s = setup
    cfg = s["cfg"]
    from rsd.frame import Device, GpuScene
    dev = Device(0)
    gs = GpuScene(dev, s["scene"])
    g = rg.load_script(ROOT / "tests" / "graphs" / "svao_post.py")["SVAOPost"]
    g.set_scene(gs.h, s["cam"])
    g.compile(cfg.fb_w, cfg.fb_h)
    g.execute()
    s["torch"].cuda.synchronize()
    blurred, _ = oracle.cross_bilateral_blur(expected["ao"], expected["linear_z"], 16)
    W, H = cfg.fb_w, cfg.fb_h
    amb = IE.store(IE.evaluate("I0[xy].rrra", [(blurred, IE.FMT_R8UNORM), (None, 0), (None, 0), (None, 0)], W, H),
                   IE.FMT_RGBA32F)
    got = _np(g.output_tensor("AmbientRef.out"))
    np.testing.assert_array_equal(got.view(np.uint32).reshape(-1), amb.view(np.uint32).reshape(-1))
    e1 = IE.store(IE.evaluate("1.0 - max(I0[xy].x-I0[xy].y, 0.05)", [(amb, IE.FMT_RGBA32F)] + [(None, 0)] * 3, W, H),
                  IE.FMT_R8UNORM)
    np.testing.assert_array_equal(_np(g.output_tensor("ImageEquation1.out")).reshape(H, W), e1)
    lz = IE.store(IE.evaluate("I0[xy]/1000.0", [(expected["linear_z"], IE.FMT_R32F)] + [(None, 0)] * 3, W, H),
                  IE.FMT_R32F)
    np.testing.assert_array_equal(_np(g.output_tensor("ImageEquationLinearDepth.out")).view(np.uint32).reshape(-1),
                                  lz.view(np.uint32).reshape(-1))
    g.close()
    gs.release()
    dev.close()


def test_graph_ray_min_max_length(setup, expected):
    """RayMinMaxLength fed by SVAO's internal interval maps (scripts/SVAO.py:70-71) in the C++
    graph host: the lengths of the frame's SD ray intervals."""
    from oracle.texops import ray_min_max_length
    from rsd import graph as rg
    torch, cfg = setup["torch"], setup["cfg"]
    g = rg.load_script(SCRIPT)["SVAOHotPath"]
    g.create_pass("RayMinMaxLength", "RayMinMaxLength", {})
    g.add_edge("SVAO.internalRayMin", "RayMinMaxLength.kRayMin")
    g.add_edge("SVAO.internalRayMax", "RayMinMaxLength.kRayMax")
    g.mark_output("RayMinMaxLength.len")
    from rsd.frame import Device, GpuScene
    dev = Device(0)
    gs = GpuScene(dev, setup["scene"])
    g.set_scene(gs.h, setup["cam"])
    g.compile(cfg.fb_w, cfg.fb_h)
    g.execute()
    torch.cuda.synchronize()
    got = _np(g.output_tensor("RayMinMaxLength.len")).reshape(setup["sd_h"], setup["sd_w"])
    want = ray_min_max_length(expected["ray_min"], expected["ray_max"])
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    assert (got > 0).sum() > 0
    g.close()
    gs.release()
    dev.close()
