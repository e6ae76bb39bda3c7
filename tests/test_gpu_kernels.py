"""GPU parity of the SVAO AO-kernel and depth-mode variants (exact numerics, bit-identical to the oracle):

  * the HBAO kernel (rsd_svao_params.ao_kernel, SVAO.cpp:233 AO_KERNEL; Common.slang:60-66 radii,
    :362-365 pdf, :421-430 HBAOKernel, :455-461 requireRay, :477-488 addSample / resetSample, :326-330
    finalize; SVAORaster.ps.slang:57, :91, :108) with 8 / 16 / 32 directions, SingleDepth and
    StochasticDepth secondary modes, dualAO;
  * the DualDepth primary mode (rsd_svao_params.primary_depth_mode / d_depth2; SVAORaster.ps.slang:69-70,
    Common.slang:498-505 evalDualVisibility, :555-558 in calcAO2) with a second depth layer behind the
    first, for both kernels;
  * the DualDepth secondary mode (calcAO2 has no branch for it: the raster visibility is subtracted and
    added back, Common.slang:553-663);
  * the Raytraced secondary mode (calcAO2 DEPTH_MODE_RAYTRACING, Common.slang:598-651) with both kernels
    and both primary modes: the HBAO ray's committed closest hit over [sphereStart, sphereEnd]
    (:622-628, 646-650; SVAORaster2.ps.slang:12-15, 42-45; Ray.rt.slang:37-43) and evalDualVisibility
    before the ray (:555-558), both extents (rayPipeline), and the band union."""
import numpy as np
import pytest

from helpers import small_frame_config, to_oracle

pytestmark = pytest.mark.gpu


def _structs(r, O):
    return (to_oracle(r.cam, O.Camera), to_oracle(r.vao, O.VAOData), to_oracle(r.sdp, O.SDParams),
            to_oracle(r.svp, O.SVAOParams))


def _bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _frame(oracle, kernel="vao", primary=0, secondary=2, nd=8, dual_ao=False, N=4, ray_pipeline=True, cull=1,
           bands=1):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    cfg = small_frame_config(visible=(224, 128), guard=32, divisor=1 if secondary == 3 else 2, N=N)
    cfg.ao_kernel, cfg.primary, cfg.secondary, cfg.num_directions, cfg.dual_ao = kernel, primary, secondary, nd, dual_ao
    cfg.ray_pipeline, cfg.cull_mode = bool(ray_pipeline), cull
    cfg.numerics = "exact"
    scene = make_scene("arcade_tiny")
    r = Renderer(scene, cfg)
    r.gbuffer()
    if primary == 1:  # a second layer behind the first (DepthPeeling's role in scripts/SVAO_depth.py)
        r.depth2.copy_(r.depth * 1.1 + 0.25)
    r.clear_intervals()
    r.pass1()
    g1 = r.numpy()
    r.frame()
    g = r.numpy()
    if bands > 1:  # the band union (multi-GPU split of the Raytraced pass) equals the whole frame
        r.ao.zero_()
        r.stencil.zero_()
        for b in range(bands):
            r.pass1(band=(b, bands))
        for b in range(bands):
            r.pass2_raytraced(band=(b, bands))
        gb = r.numpy()
        assert np.array_equal(gb["stencil"], g["stencil"]) and np.array_equal(gb["ao"], g["ao"]), "band union"
    cam, vao, sdp, svp = _structs(r, oracle)
    d2 = g1["depth"] * np.float32(1.1) + np.float32(0.25) if primary == 1 else None
    if d2 is not None:
        assert _bits_equal(r.depth2.cpu().numpy(), d2)
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, g1["depth"], g1["normals"], r.sd_w, r.sd_h, depth2=d2)
    assert np.array_equal(g1["stencil"], st), "stencil"
    assert np.array_equal(g1["ao"], ao1), "pass-1 AO"
    if secondary == 2:
        assert np.array_equal(g1["ray_min"], rmin) and np.array_equal(g1["ray_max"], rmax), "intervals"
        sd, _ = oracle.sd_trace(osc, cam, sdp, g1["depth"], rmin, rmax, r.sd_w, r.sd_h)
        assert _bits_equal(g["sd"], sd)
    else:
        sd = np.zeros((1, 1, 1, min(N, 4)), np.float32)
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    if secondary in (1, 2):
        ao = oracle.svao_pass2(cam, vao, svp, g1["depth"], g1["normals"], st, sd, ao1, depth2=d2)
        assert np.array_equal(g["ao"][gv], ao[gv]), "frame AO"
    elif secondary == 3:
        ao = oracle.svao_pass2_raytraced(osc, cam, vao, svp, g1["depth"], g1["normals"], st, ao1, cull=cull,
                                         ray_pipeline=int(ray_pipeline), depth2=d2)
        assert np.array_equal(g["ao"], ao), "Raytraced frame AO"
    else:
        ao = ao1
        assert np.array_equal(g["ao"], ao1), "SingleDepth frame = pass 1"
    r.close()
    return dict(ao1=ao1, st=st, ao=ao, gv=gv)


@pytest.mark.parametrize("nd,secondary,dual_ao", [(8, 2, False), (16, 2, False), (32, 2, True), (8, 0, False),
                                                  (8, 2, True)])
def test_hbao_parity(oracle, nd, secondary, dual_ao):
    o = _frame(oracle, kernel="hbao", secondary=secondary, nd=nd, dual_ao=dual_ao)
    assert (o["st"] != 0).any() or secondary == 0
    v = _frame(oracle, kernel="vao", secondary=secondary, nd=nd, dual_ao=dual_ao)
    assert not np.array_equal(o["ao"][o["gv"]], v["ao"][v["gv"]])  # a different kernel


@pytest.mark.parametrize("kernel,secondary", [("vao", 0), ("vao", 2), ("hbao", 2), ("hbao", 0)])
def test_dual_depth_primary_parity(oracle, kernel, secondary):
    o = _frame(oracle, kernel=kernel, primary=1, secondary=secondary)
    s = _frame(oracle, kernel=kernel, primary=0, secondary=secondary)
    assert not np.array_equal(o["ao1"], s["ao1"])  # the second layer changed some raster samples


@pytest.mark.parametrize("kernel", ["vao", "hbao"])
def test_dual_depth_secondary_parity(oracle, kernel):
    o = _frame(oracle, kernel=kernel, secondary=1)
    assert (o["st"] != 0).any()


@pytest.mark.parametrize("kernel,primary,ray_pipeline,cull,bands", [
    ("hbao", 0, True, 1, 1), ("hbao", 0, False, 0, 3), ("hbao", 1, True, 1, 1), ("vao", 1, True, 1, 3),
    ("vao", 1, False, 2, 1), ("hbao", 1, False, 1, 2)])
def test_raytraced_kernels_and_depth_modes(oracle, kernel, primary, ray_pipeline, cull, bands):
    """{VAO, HBAO} x {SingleDepth, DualDepth} in the Raytraced secondary mode (VAO / SingleDepth is
    test_gpu_parity.py's test_raytraced_svao_parity), against the oracle's literal replay of the hit stream."""
    o = _frame(oracle, kernel=kernel, primary=primary, secondary=3, ray_pipeline=ray_pipeline, cull=cull, bands=bands)
    assert (o["st"] != 0).sum() > 50, "no refined directions: the test frame is degenerate"
    assert not np.array_equal(o["ao"], o["ao1"])  # the rays changed something
    if kernel == "hbao" and primary == 0 and cull == 1:
        v = _frame(oracle, kernel="vao", secondary=3, ray_pipeline=ray_pipeline, cull=cull)
        assert not np.array_equal(o["ao"], v["ao"])  # a different kernel


def test_raytraced_refuses_bad_modes(oracle):
    """An AO kernel / primary depth mode librsd does not define, or DualDepth without its layer, is refused."""
    from rsd import abi
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    cfg = small_frame_config(visible=(96, 64), guard=16, divisor=1)
    cfg.secondary, cfg.numerics = abi.DEPTH_RAYTRACED, "exact"
    r = Renderer(make_scene("arcade_tiny"), cfg)
    r.gbuffer()
    r.pass1()
    svp = abi.SVAOParams.from_buffer_copy(r.svp)
    svp.ao_kernel = 2
    r.svp = svp
    with pytest.raises(abi.RsdError) as e:
        r.pass2_raytraced()
    assert e.value.status == abi.ERR_INVALID_ARG
    svp.ao_kernel, svp.primary_depth_mode, svp.d_depth2 = 0, 1, None
    with pytest.raises(abi.RsdError, match="d_depth2"):
        r.pass2_raytraced()
    r.close()
