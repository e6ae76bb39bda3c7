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
  * the Raytraced pass 2 refuses HBAO / DualDepth (RSD_ERR_UNSUPPORTED)."""
import numpy as np
import pytest

from helpers import small_frame_config, to_oracle

pytestmark = pytest.mark.gpu


def _structs(r, O):
    return (to_oracle(r.cam, O.Camera), to_oracle(r.vao, O.VAOData), to_oracle(r.sdp, O.SDParams),
            to_oracle(r.svp, O.SVAOParams))


def _bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _frame(oracle, kernel="vao", primary=0, secondary=2, nd=8, dual_ao=False, N=4):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    cfg = small_frame_config(visible=(224, 128), guard=32, divisor=2, N=N)
    cfg.ao_kernel, cfg.primary, cfg.secondary, cfg.num_directions, cfg.dual_ao = kernel, primary, secondary, nd, dual_ao
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


def test_raytraced_refuses_hbao(oracle):
    from rsd import abi
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    cfg = small_frame_config(visible=(96, 64), guard=16, divisor=1)
    cfg.secondary, cfg.ao_kernel, cfg.numerics = abi.DEPTH_RAYTRACED, "hbao", "exact"
    r = Renderer(make_scene("arcade_tiny"), cfg)
    r.gbuffer()
    r.pass1()
    with pytest.raises(abi.RsdError) as e:
        r.pass2_raytraced()
    assert e.value.status == abi.ERR_UNSUPPORTED
    r.close()
