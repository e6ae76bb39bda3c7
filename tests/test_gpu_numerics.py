"""Fast numerics (rsd.h RSD_NUMERICS_FAST, the product default) graded against the exact oracle.

The SVAO passes built with FMA contraction, v_rcp_f32 division and hardware sqrt / rsq
(csrc/svao_fast.hip) are not bit-identical to the oracle; they are graded by BASELINE.md
section 4's AO tolerance, at every BASELINE config:

  * AO of the whole fast frame vs the oracle's exact frame on the same G-buffer (oracle pass 1 ->
    oracle SD trace -> oracle pass 2): mean absolute error <= 1/255 over the visible pixels and
    |diff| <= 2/255 on >= 99.5 % of them (the tolerance is written below: AO_MAE, AO_P2, AO_P2_FRAC);
  * the pass-1 decisions: stencil pixels and touched SD texels (an interval requested or not) that
    differ from the oracle's, as fractions (reported, bounded by DECISION_FRAC);
  * the SD trace stays exact: the GPU's SD map equals the oracle's trace of the GPU's OWN intervals
    bit for bit (the trace kernels are not built with fast numerics);
  * pass 2 on the GPU's own inputs (stencil, pass-1 AO, SD map) vs the oracle's pass 2 on them:
    the same AO tolerance.

RSD_NUMERICS_REPORT=<path>: the measured fractions of every case are appended there as JSON lines
(DESIGN.md section 2 quotes them)."""
import json
import os

import numpy as np
import pytest

from helpers import to_oracle

pytestmark = pytest.mark.gpu

AO_MAE = 1.0 / 255.0   # mean absolute AO error over the visible pixels
AO_P2 = 2              # ... and |diff| <= 2/255 ...
AO_P2_FRAC = 0.995     # ... on at least 99.5 % of them
DECISION_FRAC = 0.01   # stencil pixels / touched SD texels allowed to flip (reported; measured far below)


def _bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _ao_stats(a, b, gv):
    """AO difference in 1/255 units over the visible pixels (both channels with dualAO)."""
    d = np.abs(a[gv].astype(np.int32) - b[gv].astype(np.int32))
    return {"mae": float(d.mean()) / 255.0, "frac_le2": float((d <= AO_P2).mean()), "max": int(d.max()),
            "frac_exact": float((d == 0).mean())}


def _check_ao(s, what):
    assert s["mae"] <= AO_MAE, (what, s)
    assert s["frac_le2"] >= AO_P2_FRAC, (what, s)


def _report(case, **kw):
    path = os.environ.get("RSD_NUMERICS_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(dict(case=case, **kw)) + "\n")


def _grade(oracle, r, scene, case):
    """One fast frame of renderer r (G-buffer already rendered) graded against the oracle."""
    import torch
    cfg = r.cfg
    assert r.svp.numerics == 0, "the renderer must run the fast numerics"
    r.clear_intervals()
    r.pass1()
    torch.cuda.synchronize()
    ao1_g = r.ao.cpu().numpy().copy()
    r.sd_trace()
    r.pass2()
    g = r.numpy()
    cam, vao = to_oracle(r.cam, oracle.Camera), to_oracle(r.vao, oracle.VAOData)
    sdp, svp = to_oracle(r.sdp, oracle.SDParams), to_oracle(r.svp, oracle.SVAOParams)
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags, scene.alpha)
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)

    # the exact frame of the oracle on the same G-buffer
    ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, g["depth"], g["normals"], r.sd_w, r.sd_h)
    sd, _ = oracle.sd_trace(osc, cam, sdp, g["depth"], rmin, rmax, r.sd_w, r.sd_h)
    ao = oracle.svao_pass2(cam, vao, svp, g["depth"], g["normals"], st, sd, ao1)
    frame = _ao_stats(g["ao"], ao, gv)

    # pass-1 decisions
    stencil_flip = float((g["stencil"][gv] != st[gv]).mean())
    touched_g = (g["ray_max"] != 0)
    touched_o = (rmax != 0)
    touched_flip = float((touched_g != touched_o).sum() / max(1, touched_o.sum()))
    both = touched_g & touched_o
    iv_differ = float(((g["ray_min"] != rmin) | (g["ray_max"] != rmax))[both].mean()) if both.any() else 0.0
    pass1 = _ao_stats(ao1_g, ao1, gv)

    # the SD trace of the GPU's own intervals: exact
    sd_own, stats = oracle.sd_trace(osc, cam, sdp, g["depth"], g["ray_min"], g["ray_max"], r.sd_w, r.sd_h)
    assert stats[0] > 0, "no live SD rays: degenerate frame"
    sd_exact = _bits_equal(g["sd"], sd_own)

    # pass 2 on the GPU's own inputs
    ao_own = oracle.svao_pass2(cam, vao, svp, g["depth"], g["normals"], g["stencil"], g["sd"], ao1_g)
    pass2 = _ao_stats(g["ao"], ao_own, gv)

    _report(case, frame_ao=frame, pass1_ao=pass1, pass2_ao_own_inputs=pass2, stencil_flip_frac=stencil_flip,
            touched_texel_flip_frac=touched_flip, interval_bits_differ_frac=iv_differ, sd_map_exact=sd_exact,
            live_texels=int(touched_o.sum()), stencilled_px=int((st[gv] != 0).sum()))
    assert sd_exact, (case, "SD map differs from the oracle's trace of the GPU's own intervals")
    _check_ao(frame, (case, "frame"))
    _check_ao(pass2, (case, "pass 2 on own inputs"))
    assert stencil_flip <= DECISION_FRAC, (case, stencil_flip)
    assert touched_flip <= DECISION_FRAC, (case, touched_flip)
    return frame


@pytest.mark.timeout(900)
@pytest.mark.parametrize("config", ["arcade_256", "suntemple_1080p_q", "bistro_1080p_full", "emerald_4k_q",
                                    "bistro_4k_full_n16"])
def test_fast_numerics_config(oracle, config):
    """configs[0]..[4] (configs[4] at pose 41 of its orbit120 camera path)."""
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import ARCADE_CONFIG, CONFIGS, DEFAULT_CAMERA_PATH, FrameConfig, Renderer, camera_path
    from rsd.scenes import make_scene
    kw, name = ARCADE_CONFIG if config == "arcade_256" else CONFIGS[config]
    scene = make_scene(name)
    r = Renderer(scene, FrameConfig(**kw, numerics="fast"))
    if config in DEFAULT_CAMERA_PATH:
        r.set_pose(*camera_path(DEFAULT_CAMERA_PATH[config])[41])
    r.gbuffer()
    _grade(oracle, r, scene, config)
    r.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("directions,dual,N", [(8, False, 1), (8, False, 8), (16, False, 4), (32, False, 2),
                                               (8, True, 4), (16, True, 16)])
def test_fast_numerics_small(oracle, directions, dual, N):
    """The generic kernels (16 / 32 directions), dualAO and every N, on a small frame."""
    import dataclasses
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    from helpers import small_frame_config
    cfg = dataclasses.replace(small_frame_config(visible=(320, 192), N=N, max_count=max(8, N)),
                              num_directions=directions, dual_ao=dual, numerics="fast")
    scene = make_scene("arcade_tiny")
    r = Renderer(scene, cfg)
    r.gbuffer()
    _grade(oracle, r, scene, f"small_d{directions}_dual{int(dual)}_n{N}")
    r.close()


@pytest.mark.timeout(300)
def test_exact_numerics_still_bit_identical(oracle):
    """RSD_NUMERICS_EXACT next to the fast default in one process: the exact frame is the oracle's
    bit for bit, and the fast frame of the same inputs differs from it only within the tolerance."""
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS["suntemple_1080p_q"]
    scene = make_scene(name)
    ex = Renderer(scene, FrameConfig(**kw, numerics="exact"))
    fa = Renderer(scene, FrameConfig(**kw, numerics="fast"), gpu_scene=ex.gscene, dev=ex.dev)
    for r in (ex, fa):
        r.gbuffer()
        r.frame()
    ge, gf = ex.numpy(), fa.numpy()
    cam, vao = to_oracle(ex.cam, oracle.Camera), to_oracle(ex.vao, oracle.VAOData)
    sdp, svp = to_oracle(ex.sdp, oracle.SDParams), to_oracle(ex.svp, oracle.SVAOParams)
    ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, ge["depth"], ge["normals"], ex.sd_w, ex.sd_h)
    assert np.array_equal(ge["stencil"], st) and np.array_equal(ge["ray_min"], rmin)
    cfg = ex.cfg
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    _check_ao(_ao_stats(gf["ao"], ge["ao"], gv), "fast vs exact frame")
    assert not np.array_equal(gf["ray_min"], ge["ray_min"]), "the fast kernels ran the exact arithmetic"
    fa.close()
    ex.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kernel,primary", [("vao", 0), ("hbao", 0), ("vao", 1), ("hbao", 1)])
def test_fast_numerics_degenerate_inputs(oracle, kernel, primary):
    """The fast build assumes no NaN operands (-fno-honor-nans): inputs that produce NaN / inf
    inside the SVAO arithmetic must still give AO within the tolerance of the exact oracle frame.  The
    G-buffer gets patches of background depth exactly at farZ, zero depth (a pixel at the camera: posV = 0,
    zero-length view vectors), +inf, NaN and negative depth; with DualDepth the second layer is left at its
    zero initialisation (Common.slang:285-330 Init / finalize; :498-505 evalDualVisibility)."""
    import dataclasses

    import torch
    from rsd.frame import Renderer
    from rsd.scenes import make_scene
    from helpers import small_frame_config
    cfg = dataclasses.replace(small_frame_config(visible=(320, 192)), numerics="fast", ao_kernel=kernel,
                              primary=primary)
    scene = make_scene("arcade_tiny")
    r = Renderer(scene, cfg)
    r.gbuffer()
    g0 = cfg.guard_band
    d = r.depth
    d[g0 + 20:g0 + 40, g0 + 30:g0 + 90] = cfg.far                 # background at exactly farZ
    d[g0 + 60:g0 + 70, g0 + 120:g0 + 170] = 0.0                    # at the camera
    d[g0 + 90:g0 + 100, g0 + 20:g0 + 40] = float("inf")
    d[g0 + 110:g0 + 112, g0 + 200:g0 + 260] = float("nan")
    d[g0 + 130:g0 + 140, g0 + 60:g0 + 80] = -1.0
    torch.cuda.synchronize()
    r.clear_intervals()
    r.pass1()
    r.sd_trace()
    r.pass2()
    g = r.numpy()
    d2 = np.zeros_like(g["depth"]) if primary == 1 else None
    cam, vao = to_oracle(r.cam, oracle.Camera), to_oracle(r.vao, oracle.VAOData)
    sdp, svp = to_oracle(r.sdp, oracle.SDParams), to_oracle(r.svp, oracle.SVAOParams)
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags, scene.alpha)
    ao1, st, rmin, rmax = oracle.svao_pass1(cam, vao, svp, g["depth"], g["normals"], r.sd_w, r.sd_h, depth2=d2)
    sd, _ = oracle.sd_trace(osc, cam, sdp, g["depth"], rmin, rmax, r.sd_w, r.sd_h)
    ao = oracle.svao_pass2(cam, vao, svp, g["depth"], g["normals"], st, sd, ao1, depth2=d2)
    gv = slice(cfg.guard_band, cfg.fb_h - cfg.guard_band), slice(cfg.guard_band, cfg.fb_w - cfg.guard_band)
    s = _ao_stats(g["ao"], ao, gv)
    bad = ~np.isfinite(g["depth"][gv]) | (g["depth"][gv] <= 0.0) | (g["depth"][gv] >= cfg.far)
    dp = np.abs(g["ao"][gv].astype(np.int32) - ao[gv].astype(np.int32))[bad]
    _report(f"degenerate_{kernel}_p{primary}", frame_ao=s, degenerate_px=int(bad.sum()),
            degenerate_px_max_diff=int(dp.max()), degenerate_px_exact=float((dp == 0).mean()))
    assert bad.sum() > 2000
    _check_ao(s, ("degenerate inputs", kernel, primary))
    assert int(dp.max()) <= AO_P2, ("the degenerate pixels themselves", int(dp.max()))
    r.close()
