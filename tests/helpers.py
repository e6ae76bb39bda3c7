"""Shared test helpers: struct conversion between librsd and the oracle, and the oracle
side of a whole frame (G-buffer -> pass 1 -> SD trace -> pass 2)."""
from __future__ import annotations

import ctypes as C

import numpy as np


def to_oracle(struct, oracle_cls):
    """Byte-copy a librsd ctypes struct into the oracle's struct of identical layout.  The oracle's
    struct may be a prefix of librsd's (device-only trailing fields such as rsd_svao_params.tile_flags)."""
    out = oracle_cls()
    names = [f[0] for f in type(struct)._fields_]
    # a field the oracle does not use keeps librsd's name with an "_unused" suffix
    onames = [f[0].removesuffix("_unused") for f in oracle_cls._fields_]
    names = [n.removeprefix("d_") for n in names]  # librsd's device pointers vs the oracle's host pointers
    assert names[:len(onames)] == onames, (oracle_cls, onames, names)
    assert C.sizeof(out) <= C.sizeof(struct), (oracle_cls, C.sizeof(out), C.sizeof(struct))
    C.memmove(C.byref(out), C.byref(struct), C.sizeof(out))
    return out


def oracle_vao(O, fb_w, fb_h, divisor, sd_guard_px=512, radius=0.2, exponent=2.0, thickness=0.0):
    """SVAO::compile restated independently (SVAO.cpp:143-150, 700-723)."""
    v = O.VAOData()
    v.resolution[:] = [fb_w, fb_h]
    v.invResolution[0] = float(np.float32(1.0) / np.float32(fb_w))
    v.invResolution[1] = float(np.float32(1.0) / np.float32(fb_h))
    v.sdGuard = sd_guard_px // divisor
    low = ((fb_w + divisor - 1) // divisor, (fb_h + divisor - 1) // divisor) if divisor > 1 else (fb_w, fb_h)
    v.lowResolution[:] = low
    v.noiseScale[:] = [float(np.float32(fb_w) / np.float32(4)), float(np.float32(fb_h) / np.float32(4))]
    v.radius, v.exponent, v.thickness = radius, exponent, thickness
    v.ssRadiusCutoff, v.ssMaxRadius = 6.0, 512.0
    return v, low[0] + 2 * v.sdGuard, low[1] + 2 * v.sdGuard


def oracle_frame(O, oscene, cam, vao, sdp, svp, fb_w, fb_h, sd_w, sd_h, threads=None):
    z, n = O.gbuffer(oscene, cam, fb_w, fb_h, sdp.cull_mode, threads=threads)
    ao1, st, rmin, rmax = O.svao_pass1(cam, vao, svp, z, n, sd_w, sd_h)
    sd, stats = O.sd_trace(oscene, cam, sdp, z, rmin, rmax, sd_w, sd_h, threads=threads)
    ao2 = O.svao_pass2(cam, vao, svp, z, n, st, sd, ao1, threads=threads)
    return dict(depth=z, normals=n, ao1=ao1, stencil=st, ray_min=rmin, ray_max=rmax, sd=sd, ao=ao2, stats=stats)


def small_frame_config(visible=(160, 96), guard=16, divisor=2, N=4, max_count=8, impl=0, radius=1.0):
    """A small frame; the AO radius is scaled up so that, at this resolution, the sample
    radius exceeds ssRadiusCutoff (6 px) and pass 1 actually requests SD rays."""
    from rsd.frame import FrameConfig
    return FrameConfig(visible_w=visible[0], visible_h=visible[1], guard_band=guard, divisor=divisor,
                       sd_samples=N, max_count=max_count, implementation=impl, sd_guard_px=64, radius=radius)
