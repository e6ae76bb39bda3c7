"""GPU parity of TemporalAO (enabled) and the motion vectors through the C ABI
(rsd_temporal_ao, rsd_motion_vectors) against the oracle (ocpu_temporal_ao,
ocpu_motion_vectors): synthetic inputs with every branch of TemporalAO.ps.slang:55-101, and a
rendered camera sequence (G-buffer -> SVAO -> motion vectors -> TemporalAO) whose history must
grow where the reprojection holds.  Bit-exact."""
import ctypes as C

import numpy as np
import pytest

from helpers import small_frame_config, to_oracle

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


@pytest.mark.parametrize("guard,use_mask", [(0, False), (16, True), (5, False)])
def test_temporal_ao_synthetic_parity(torch, oracle, guard, use_mask):
    from rsd import abi
    from rsd.frame import FrameConfig, look_at
    from rsd.temporal import prev_view_to_cur_view
    rng = np.random.default_rng(guard)
    H, W = 90, 150
    cfg = FrameConfig(visible_w=W, visible_h=H, guard_band=0)
    c0 = look_at([0.0, 2.0, 8.0], [0.0, 1.0, 0.0], [0.0, 1.0, 0.0], cfg)
    c1 = look_at([0.2, 2.1, 7.7], [0.1, 1.0, 0.0], [0.0, 1.0, 0.0], cfg)
    m = np.ascontiguousarray(prev_view_to_cur_view(c1, c0), F)
    ao = rng.integers(0, 256, (H, W)).astype(np.uint8)
    z = (2.0 + 10.0 * rng.random((H, W))).astype(F)
    mv = (rng.normal(0.0, 0.01, (H, W, 2))).astype(F)
    mv[rng.random((H, W)) < 0.1] = 0.7  # off screen
    mv[rng.random((H, W)) < 0.1] = 0.0
    # previous depth: the current depth give or take up to 20 % (both sides of the 10 % test)
    prev_z = (z * (1.0 + rng.uniform(-0.2, 0.2, (H, W)))).astype(F)
    prev_z[rng.random((H, W)) < 0.02] = 0.0
    prev_ao = rng.integers(0, 256, (H, W)).astype(np.uint8)
    prev_n = rng.integers(0, 31, (H, W)).astype(np.uint8)
    mask = (rng.random((H, W)) < 0.2).astype(np.uint8) if use_mask else None
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in
         dict(ao=ao, z=z, mv=mv, pz=prev_z, pa=prev_ao, pn=prev_n).items()}
    dm = torch.from_numpy(mask).cuda() if use_mask else None
    out = torch.full((H, W), 7, dtype=torch.uint8, device="cuda")
    hist = torch.full((H, W), 9, dtype=torch.uint8, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    abi.check(abi.lib().rsd_temporal_ao(_p(d["ao"]), _p(d["z"]), _p(d["mv"]), _p(d["pz"]), _p(d["pa"]), _p(d["pn"]),
                                        _p(dm), W, H, guard, C.byref(c1), m.ctypes.data_as(C.c_void_p), _p(out),
                                        _p(hist), s), "rsd_temporal_ao")
    torch.cuda.synchronize()
    want, want_n = oracle.temporal_ao(ao, z, mv, prev_z, prev_ao, prev_n, to_oracle(c1, oracle.Camera), m, guard,
                                      stable_mask=mask, ao_dst=np.full((H, W), 7, np.uint8),
                                      history_dst=np.full((H, W), 9, np.uint8))
    got_n = hist.cpu().numpy()
    assert np.array_equal(out.cpu().numpy(), want)
    assert np.array_equal(got_n, want_n)
    inner = got_n[guard:H - guard, guard:W - guard]
    assert (inner == 1).mean() > 0.1 and (inner > 1).mean() > 0.1  # both branches exercised


def test_temporal_ao_rejects_bad_arguments(torch):
    from rsd import abi
    from rsd.frame import FrameConfig, look_at
    cfg = FrameConfig(visible_w=64, visible_h=64, guard_band=0)
    c = look_at([0.0, 2.0, 8.0], [0.0, 1.0, 0.0], [0.0, 1.0, 0.0], cfg)
    m = np.eye(4, dtype=F)
    t = torch.zeros((64, 64), dtype=torch.float32, device="cuda")
    st = abi.lib().rsd_temporal_ao(_p(t), _p(t), _p(t), _p(t), _p(t), _p(t), None, 64, 64, 32, C.byref(c),
                                   m.ctypes.data_as(C.c_void_p), _p(t), _p(t), None)
    assert st == abi.ERR_INVALID_ARG  # 2 * guard >= size
    st = abi.lib().rsd_temporal_ao(None, _p(t), _p(t), _p(t), _p(t), _p(t), None, 64, 64, 0, C.byref(c),
                                   m.ctypes.data_as(C.c_void_p), _p(t), _p(t), None)
    assert st == abi.ERR_INVALID_ARG


def test_motion_vectors_background_zero(torch, oracle):
    """Background pixels (linear depth >= farZ) get mvec (0, 0) under a moving camera, on the GPU
    and in the oracle (GBufferRaster.cpp:176 clears mvec; GBufferRaster.3d.slang:117 writes it for
    geometry only); geometry pixels are bit-identical to the oracle."""
    from rsd.frame import FrameConfig, look_at
    from rsd.temporal import motion_vectors
    cfg = FrameConfig(visible_w=160, visible_h=96, guard_band=16)
    c0 = look_at((0.0, 2.0, 8.0), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0), cfg)
    c1 = look_at((0.6, 2.2, 7.5), (0.1, 1.0, 0.0), (0.0, 1.0, 0.0), cfg)
    rng = np.random.default_rng(11)
    z = (4.0 + 20.0 * rng.random((cfg.fb_h, cfg.fb_w))).astype(np.float32)
    z[: cfg.fb_h // 3] = c1.farZ                                    # rsd_gbuffer miss value
    z[cfg.fb_h // 3: cfg.fb_h // 3 + 8] = np.float32(1000.2441)     # linearized raster depth 1.0
    zt = torch.from_numpy(z).cuda()
    mv = motion_vectors(c1, c0, zt).cpu().numpy()
    want = oracle.motion_vectors(to_oracle(c1, oracle.Camera), to_oracle(c0, oracle.Camera), z)
    assert np.array_equal(mv.view(np.uint32), want.view(np.uint32))
    bg = z >= c1.farZ
    assert (mv[bg] == 0.0).all() and (np.abs(mv[~bg]).max(axis=-1) > 0).all()


@pytest.mark.parametrize("near,far", [(0.1, 1000.0), (0.1, 10.0)])
def test_motion_vectors_raster_background_from_raw_depth(torch, oracle, near, far):
    """rsd_motion_vectors_raster (the GBufferRaster pass's mvec): background is the cleared raster depth
    1.0 decided on the raw value, so it stays (0, 0) even where its linearisation lands below farZ
    (near 0.1 / far 10: 9.99996 -- ADVICE r3); geometry bit-identical to the oracle."""
    from rsd import abi
    from rsd.frame import FrameConfig, look_at
    cfg = FrameConfig(visible_w=160, visible_h=96, guard_band=16, near=near, far=far)
    c0 = look_at((0.0, 2.0, 8.0), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0), cfg)
    c1 = look_at((0.6, 2.2, 7.5), (0.1, 1.0, 0.0), (0.0, 1.0, 0.0), cfg)
    rng = np.random.default_rng(12)
    d = rng.uniform(0.5, 0.99, (cfg.fb_h, cfg.fb_w)).astype(np.float32)  # non-linear depth of geometry
    d[: cfg.fb_h // 3] = 1.0  # cleared
    lin = (np.float32(near) * np.float32(far) / (np.float32(far) + np.float32(1.0) * (np.float32(near) -
                                                                                       np.float32(far))))
    if far == 10.0:
        assert lin < np.float32(far)  # the case the linear-depth classification gets wrong
    dt = torch.from_numpy(d).cuda()
    mv = torch.zeros((cfg.fb_h, cfg.fb_w, 2), dtype=torch.float32, device="cuda")
    abi.check(abi.lib().rsd_motion_vectors_raster(C.byref(c1), C.byref(c0), _p(dt), cfg.fb_w, cfg.fb_h, _p(mv),
                                                  C.c_void_p(torch.cuda.current_stream().cuda_stream)),
              "rsd_motion_vectors_raster")
    got = mv.cpu().numpy()
    want = oracle.motion_vectors_raster(to_oracle(c1, oracle.Camera), to_oracle(c0, oracle.Camera), d)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert (got[: cfg.fb_h // 3] == 0.0).all() and (np.abs(got[cfg.fb_h // 3:]).max(axis=-1) > 0).all()


def test_temporal_sequence_parity_and_accumulation(torch, oracle):
    """Four poses of a slowly moving camera: each frame's motion vectors and TemporalAO output
    equal the oracle's, and the history grows where the reprojection holds."""
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    from rsd.temporal import TemporalAO, motion_vectors, prev_view_to_cur_view
    cfg = small_frame_config(visible=(256, 144), guard=32, divisor=2, N=4)
    scene = make_scene("arcade_tiny")
    r = Renderer(scene, cfg)
    pos0, tgt0, up = (np.array(scene.camera[k], np.float64) for k in ("pos", "target", "up"))
    tao = TemporalAO(enabled=True)
    prev_cam, o_prev = None, None
    g = cfg.guard_band
    for i in range(4):
        step = np.array([0.02, 0.0, 0.01]) * i
        r.set_pose((pos0 + step).tolist(), (tgt0 + step).tolist(), up.tolist())
        r.gbuffer()
        r.ao.zero_()
        r.frame()
        prev_cam = prev_cam or r.cam
        mv = motion_vectors(r.cam, prev_cam, r.depth)
        out = tao.execute(r.ao, r.depth, mv, r.cam, prev_cam, g)
        torch.cuda.synchronize()
        z, ao_in = r.depth.cpu().numpy(), r.ao.cpu().numpy()
        oc, op = to_oracle(r.cam, oracle.Camera), to_oracle(prev_cam, oracle.Camera)
        want_mv = oracle.motion_vectors(oc, op, z)
        assert np.array_equal(mv.cpu().numpy().view(np.uint32), want_mv.view(np.uint32)), i
        assert (want_mv[z >= oc.farZ] == 0.0).all()  # background keeps the cleared mvec
        if o_prev is None:
            H, W = z.shape
            o_prev = (np.zeros_like(z), np.zeros_like(ao_in), np.zeros_like(ao_in))
        m = prev_view_to_cur_view(r.cam, prev_cam)
        want, want_n = oracle.temporal_ao(ao_in, z, want_mv, *o_prev, oc, m, g)
        assert np.array_equal(out.cpu().numpy(), want), i
        assert np.array_equal(tao.history.cpu().numpy(), want_n), i
        o_prev = (z, want, want_n)
        prev_cam = r.cam
    inner = want_n[g:-g, g:-g]
    assert (inner == 4).mean() > 0.8, np.bincount(inner.ravel())
    r.close()


def test_graph_temporal_ao_enabled(torch, oracle):
    """scripts/SVAO.py's chain with TemporalAO enabled, run by the C++ graph host over three
    camera poses: GBufferRaster.mvec and TemporalAO.aoOut equal the oracle's every frame."""
    from conftest import ROOT
    from rsd import graph as rg
    from rsd.frame import Device, GpuScene, look_at
    from rsd.scenes import make_scene
    from rsd.temporal import prev_view_to_cur_view
    cfg = small_frame_config()
    scene = make_scene("arcade_tiny")
    dev = Device(0)
    gs = GpuScene(dev, scene)
    g = rg.load_script(ROOT / "tests" / "graphs" / "svao_temporal.py")["SVAOTemporal"]
    pos0, tgt0 = np.array(scene.camera["pos"]), np.array(scene.camera["target"])
    prev_cam, o_prev = None, None
    G = 16  # svao_temporal.py GuardBand
    for i in range(3):
        step = np.array([0.03, 0.0, 0.0]) * i
        cam = look_at((pos0 + step).tolist(), (tgt0 + step).tolist(), scene.camera["up"], cfg)
        g.set_scene(gs.h, cam)
        if i == 0:
            g.compile(cfg.fb_w, cfg.fb_h)
        g.execute()
        torch.cuda.synchronize()
        z = g.output_tensor("LinearizeDepth.linearDepth").cpu().numpy().reshape(cfg.fb_h, cfg.fb_w)
        blurred = g.output_tensor("CrossBilateralBlur0.colorOut").cpu().numpy().reshape(cfg.fb_h, cfg.fb_w)
        mv = g.output_tensor("GBufferRaster.mvec").cpu().numpy().reshape(cfg.fb_h, cfg.fb_w, 2)
        ao = g.output_tensor("TemporalAO.aoOut").cpu().numpy().reshape(cfg.fb_h, cfg.fb_w)
        oc = to_oracle(cam, oracle.Camera)
        op = to_oracle(prev_cam or cam, oracle.Camera)
        want_mv = oracle.motion_vectors(oc, op, z)
        assert np.array_equal(mv.view(np.uint32), want_mv.view(np.uint32)), i
        if o_prev is None:
            o_prev = (np.zeros_like(z), np.zeros_like(blurred), np.zeros_like(blurred))
        want, want_n = oracle.temporal_ao(blurred, z, want_mv, *o_prev, oc, prev_view_to_cur_view(cam, prev_cam or cam),
                                          G)
        assert np.array_equal(ao[G:-G, G:-G], want[G:-G, G:-G]), i
        o_prev = (z, want, want_n)
        prev_cam = cam
    assert (want_n[G:-G, G:-G] == 3).mean() > 0.8
    g.close()
    gs.release()
    dev.close()


@pytest.mark.parametrize("sigma,anti", [(1.0, True), (0.5, False), (4.0, True)])
def test_taa_parity(torch, oracle, sigma, anti):
    """rsd_taa vs ocpu_taa on random colours / motion (some pointing off the image: wrap taps)."""
    from rsd.temporal import TAA
    rng = np.random.default_rng(int(sigma * 10))
    H, W = 45, 77
    frames = [(rng.random((H, W, 4)) * 2).astype(F) for _ in range(3)]
    mvs = [rng.normal(0.0, 0.02, (H, W, 2)).astype(F) for _ in range(3)]
    mvs[1][:5] = 0.6  # far off the image: wrap addressing
    t = TAA(alpha=0.1, color_box_sigma=sigma, anti_flicker=anti)
    prev = np.zeros((H, W, 4), F)
    for c, mv in zip(frames, mvs):
        out = t.execute(torch.from_numpy(c).cuda(), torch.from_numpy(mv).cuda())
        torch.cuda.synchronize()
        want = oracle.taa(c, mv, prev, alpha=0.1, color_box_sigma=sigma, anti_flicker=anti)
        got = out.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
        prev = want


def test_graph_taa_after_temporal_chain(torch, oracle):
    """scripts/SVAO.py's AmbientTAA: ImageEquation 'I0[xy].rrra' -> TAA with GBufferRaster.mvec,
    two camera poses, bit-exact against ocpu_taa on the graph's own inputs."""
    from conftest import ROOT
    from rsd import graph as rg
    from rsd.frame import Device, GpuScene, look_at
    from rsd.scenes import make_scene
    cfg = small_frame_config()
    scene = make_scene("arcade_tiny")
    dev = Device(0)
    gs = GpuScene(dev, scene)
    g = rg.load_script(ROOT / "tests" / "graphs" / "svao_temporal.py")["SVAOTemporal"]
    pos0, tgt0 = np.array(scene.camera["pos"]), np.array(scene.camera["target"])
    prev = None
    for i in range(2):
        step = np.array([0.0, 0.02, 0.03]) * i
        cam = look_at((pos0 + step).tolist(), (tgt0 + step).tolist(), scene.camera["up"], cfg)
        g.set_scene(gs.h, cam)
        if i == 0:
            g.compile(cfg.fb_w, cfg.fb_h)
        g.execute()
        torch.cuda.synchronize()
        amb = g.output_tensor("AmbientRef.out").cpu().numpy().reshape(cfg.fb_h, cfg.fb_w, 4)
        mv = g.output_tensor("GBufferRaster.mvec").cpu().numpy().reshape(cfg.fb_h, cfg.fb_w, 2)
        got = g.output_tensor("AmbientTAA.colorOut").cpu().numpy().reshape(cfg.fb_h, cfg.fb_w, 4)
        prev = np.zeros_like(amb) if prev is None else prev
        want = oracle.taa(amb, mv, prev, alpha=0.1, color_box_sigma=1.0, anti_flicker=True)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), i
        prev = want
    g.close()
    gs.release()
    dev.close()


def test_flicker_mask_and_dilation_parity(torch, oracle):
    from rsd import abi
    from rsd.frame import FrameConfig, look_at
    rng = np.random.default_rng(11)
    H, W = 70, 110
    cfg = FrameConfig(visible_w=W, visible_h=H, guard_band=0)
    cam = look_at([0.3, 2.0, 8.0], [0.0, 1.0, 0.0], [0.0, 1.0, 0.0], cfg)
    z = (4.0 + np.cumsum(rng.normal(0, 0.05, (H, W)), axis=1)).astype(F)
    z[:, 40:] += 3.0  # a depth step
    z[5:9, 5:9] = z[5:9, 5:9][::-1]  # a flipped patch
    n = rng.normal(0, 1, (H, W, 4)).astype(F)
    n[..., :3] /= np.linalg.norm(n[..., :3], axis=-1, keepdims=True)
    n[::3, ::3, :3] = [0.0, 0.0, 1.0]
    dz, dn = torch.from_numpy(z).cuda(), torch.from_numpy(n).cuda()
    mask = torch.full((H, W), 7, dtype=torch.uint8, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    abi.check(abi.lib().rsd_ao_flicker_mask(_p(dz), _p(dn), W, H, C.byref(cam), _p(mask), s), "rsd_ao_flicker_mask")
    torch.cuda.synchronize()
    want = oracle.ao_flicker_mask(z, n, to_oracle(cam, oracle.Camera))
    got = mask.cpu().numpy()
    assert np.array_equal(got, want)
    assert 0 < got.sum() < got.size
    for op in (0, 1):
        out = torch.zeros_like(mask)
        abi.check(abi.lib().rsd_binary_dilation(_p(mask), W, H, op, _p(out), s), "rsd_binary_dilation")
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), oracle.binary_dilation(want, "max" if op else "min")), op
    assert abi.lib().rsd_binary_dilation(_p(mask), W, H, 0, _p(mask), s) == abi.ERR_INVALID_ARG  # no in-place


def test_graph_temporal_ao_with_stable_mask(torch, oracle):
    """scripts/SVAO.py's stable mask: AOFlickerMask -> BinaryDilation(min) -> TemporalAO.stableMask
    (useStableMask), three poses, bit-exact against the oracle chain on the graph's own inputs."""
    from conftest import ROOT
    from rsd import graph as rg
    from rsd.frame import Device, GpuScene, look_at
    from rsd.scenes import make_scene
    from rsd.temporal import prev_view_to_cur_view
    cfg = small_frame_config()
    scene = make_scene("arcade_tiny")
    dev = Device(0)
    gs = GpuScene(dev, scene)
    g = rg.load_script(ROOT / "tests" / "graphs" / "svao_temporal_mask.py")["SVAOTemporalMask"]
    pos0, tgt0 = np.array(scene.camera["pos"]), np.array(scene.camera["target"])
    prev_cam, o_prev = None, None
    G = 16
    hw = (cfg.fb_h, cfg.fb_w)
    for i in range(3):
        step = np.array([0.03, 0.0, 0.0]) * i
        cam = look_at((pos0 + step).tolist(), (tgt0 + step).tolist(), scene.camera["up"], cfg)
        g.set_scene(gs.h, cam)
        if i == 0:
            g.compile(cfg.fb_w, cfg.fb_h)
        g.execute()
        torch.cuda.synchronize()
        z = g.output_tensor("LinearizeDepth.linearDepth").cpu().numpy().reshape(hw)
        blurred = g.output_tensor("CrossBilateralBlur0.colorOut").cpu().numpy().reshape(hw)
        mv = g.output_tensor("GBufferRaster.mvec").cpu().numpy().reshape(hw + (2,))
        mask = g.output_tensor("AOFlickerMask.mask").cpu().numpy().reshape(hw)
        dil = g.output_tensor("BinaryDilation.output").cpu().numpy().reshape(hw)
        ao = g.output_tensor("TemporalAO.aoOut").cpu().numpy().reshape(hw)
        oc = to_oracle(cam, oracle.Camera)
        nrm = g.output_tensor("GBufferRaster.faceNormalW").cpu().numpy().reshape(hw + (4,))
        assert np.array_equal(mask, oracle.ao_flicker_mask(z, nrm, oc)), i
        assert np.array_equal(dil, oracle.binary_dilation(mask, "min")), i
        assert 0 < dil.sum() < dil.size
        if o_prev is None:
            o_prev = (np.zeros_like(z), np.zeros_like(blurred), np.zeros_like(blurred))
        want, want_n = oracle.temporal_ao(blurred, z, mv, *o_prev, oc, prev_view_to_cur_view(cam, prev_cam or cam), G,
                                          stable_mask=dil)
        assert np.array_equal(ao[G:-G, G:-G], want[G:-G, G:-G]), i
        o_prev = (z, want, want_n)
        prev_cam = cam
    g.close()
    gs.release()
    dev.close()


def test_graph_deinterleave_roundtrip(torch, oracle):
    """DeinterleaveTexture -> InterleaveTexture in the C++ graph host: the 16 layers equal the
    numpy restatement (oracle/texops.py) and the round trip gives the linear depth back."""
    from oracle.texops import deinterleave
    from rsd import graph as rg
    from rsd.frame import Device, GpuScene, make_camera
    from rsd.scenes import make_scene
    cfg = small_frame_config()
    scene = make_scene("arcade_tiny")
    dev = Device(0)
    gs = GpuScene(dev, scene)
    g = rg.RenderGraph("dei")
    g.create_pass("GBufferRaster", "GBufferRaster", {})
    g.create_pass("LinearizeDepth", "LinearizeDepth", {})
    g.create_pass("Dei", "DeinterleaveTexture", {})
    g.create_pass("Int", "InterleaveTexture", {})
    g.add_edge("GBufferRaster.depth", "LinearizeDepth.depth")
    g.add_edge("LinearizeDepth.linearDepth", "Dei.texIn")
    g.add_edge("Dei.texOut", "Int.texIn")
    for o in ("Int.texOut", "Dei.texOut", "LinearizeDepth.linearDepth"):
        g.mark_output(o)
    g.set_scene(gs.h, make_camera(scene, cfg))
    g.compile(cfg.fb_w, cfg.fb_h)
    g.execute()
    torch.cuda.synchronize()
    H, W = cfg.fb_h, cfg.fb_w
    z = g.output_tensor("LinearizeDepth.linearDepth").cpu().numpy().reshape(H, W)
    layers = g.output_tensor("Dei.texOut").cpu().numpy().reshape(16, (H + 3) // 4, (W + 3) // 4)
    assert np.array_equal(layers.view(np.uint32), deinterleave(z).view(np.uint32))
    back = g.output_tensor("Int.texOut").cpu().numpy().reshape(H, W)
    assert np.array_equal(back.view(np.uint32), z.view(np.uint32))
    g.close()
    gs.release()
    dev.close()
