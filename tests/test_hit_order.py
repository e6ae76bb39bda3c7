"""Any-hit order (rsd.h rsd_hit_order) on the CPU: librsd's host BVH build (rsd_bvh_build, no GPU)
and the oracle's traversal-order walk over it (ocpu_sd_trace_ordered).

Under the canonical order (ascending (t, prim)) the Default reservoir never replaces a slot on
opaque geometry, so it equals the KBuffer.  Under the traversal order (the DXR-like
order: nearest-child-first depth-first walk, commit = TMax <- t) the reservoir samples
(Common.slangh:136-153).  These tests pin the properties that do not depend on the tree shape; the
GPU walk is checked bit for bit against the same oracle in test_gpu_hit_order.py."""
import numpy as np
import pytest

from helpers import to_oracle


@pytest.fixture(scope="module")
def frame(oracle):
    """A small arcade frame: the oracle's G-buffer, the SD pass driven directly (no interval)."""
    from rsd import abi
    from rsd.frame import FrameConfig, host_bvh, make_camera, make_vao, sd_params
    from rsd.scenes import make_scene
    scene = make_scene("arcade_tiny")
    cfg = FrameConfig(visible_w=128, visible_h=96, guard_band=0, divisor=1, sd_guard_px=0, ray_interval=False)
    cam = to_oracle(make_camera(scene, cfg), oracle.Camera)
    vao, sd_w, sd_h = make_vao(cfg)
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    z, _ = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, 1, threads=8)
    bvh, off = host_bvh(scene)

    def params(**kw):
        c = FrameConfig(**{**cfg.__dict__, **kw})
        return to_oracle(sd_params(c, vao.sdGuard), oracle.SDParams)

    def ordered(**kw):
        return oracle.sd_trace_ordered(osc, bvh, off, cam, params(hit_order=abi.HIT_ORDER_TRAVERSAL, **kw), z, None,
                                       None, sd_w, sd_h, threads=8)[0]

    def canonical(**kw):
        return oracle.sd_trace(osc, cam, params(**kw), z, None, None, sd_w, sd_h, threads=8)[0]

    soft = min(208 - 3 * wide_depth(bvh), 160)  # librsd's pool bound for the wavefront order (rsd.h)

    def wavefront(**kw):
        return oracle.sd_trace_wavefront(osc, bvh, off, soft, cam, params(hit_order=abi.HIT_ORDER_WAVEFRONT, **kw), z,
                                         None, None, sd_w, sd_h, threads=8)[0]

    return dict(scene=scene, bvh=bvh, off=off, ordered=ordered, canonical=canonical, wavefront=wavefront,
                sd=(sd_w, sd_h))


def wide_depth(bvh):
    """Inner 4-wide nodes on the longest root-to-leaf path of librsd's exported BVH (rsd_scene_info.wide_depth)."""
    u = bvh.view(np.uint32)

    def depth(node):
        nb = u[32 * node: 32 * node + 32]
        d = 0
        for c in range(4):
            ref, cnt = int(nb[24 + c]), int(nb[28 + c])
            if ref != 0xFFFFFFFF and cnt == 0:
                d = max(d, depth(ref))
        return 1 + d

    return depth(0)


def test_host_bvh_layout(frame):
    bvh, off = frame["bvh"], frame["off"]
    scene = frame["scene"]
    nt = scene.indices.shape[0]
    # nodes (32 floats each), then one 48-B record per triangle, then 12 x 16 B of padding
    assert off % 8 == 0 and bvh.size == 4 * off + 12 * nt + 48
    tris = bvh[4 * off: 4 * off + 12 * nt].reshape(nt, 12)
    prims = np.sort(tris[:, 3].view(np.uint32))
    assert np.array_equal(prims, np.arange(nt, dtype=np.uint32))  # every triangle exactly once
    from rsd.frame import host_bvh
    b2, o2 = host_bvh(scene)
    assert o2 == off and np.array_equal(b2.view(np.uint32), bvh.view(np.uint32))  # deterministic build


def test_canonical_default_equals_kbuffer(frame):
    """The collapse the traversal order exists for: canonical Default == KBuffer (opaque scene)."""
    from rsd import abi
    for N in (1, 4):
        d = frame["canonical"](sd_samples=N, implementation=abi.SD_DEFAULT)
        k = frame["canonical"](sd_samples=N, implementation=abi.SD_KBUFFER)
        assert np.array_equal(d.view(np.uint32), k.view(np.uint32)), N


def test_traversal_default_samples_stochastically(frame):
    from rsd import abi
    d = frame["ordered"](sd_samples=4, implementation=abi.SD_DEFAULT)
    k = frame["ordered"](sd_samples=4, implementation=abi.SD_KBUFFER)
    c = frame["canonical"](sd_samples=4, implementation=abi.SD_DEFAULT)
    differ = (d.view(np.uint32) != k.view(np.uint32)).any(axis=-1).mean()
    assert differ > 0.005, differ  # the reservoir replaced slots (texels with more than N hits)
    assert not np.array_equal(d.view(np.uint32), c.view(np.uint32))
    # the first layer sample is still a surface: every texel that saw geometry keeps a depth < 1
    hit = c[0, :, :, 0] < 1.0
    assert (d[0][hit] < 1.0).any(axis=-1).all()


def test_traversal_nearest_hit_is_order_independent(frame):
    """KBuffer with N = 1 keeps the nearest hit in ANY order (each commit shrinks TMax to the hit,
    every nearer hit is still delivered and replaces it) -- so both orders agree exactly."""
    from rsd import abi
    for impl in (abi.SD_KBUFFER,):
        o = frame["ordered"](sd_samples=1, implementation=impl, max_count=64)
        c = frame["canonical"](sd_samples=1, implementation=impl, max_count=64)
        assert np.array_equal(o.view(np.uint32), c.view(np.uint32))


def test_traversal_coverage_mask_runs(frame):
    from rsd import abi
    m = frame["ordered"](sd_samples=4, implementation=abi.SD_COVERAGE_MASK)
    assert np.isfinite(m).all() and (m <= 1.0).all() and (m < 1.0).any()


def test_oracle_refuses_silent_canonical(frame, oracle):
    from rsd import abi
    p = oracle.SDParams()
    p.hit_order = abi.HIT_ORDER_TRAVERSAL
    with pytest.raises(ValueError):
        oracle.sd_trace(None, None, p, np.zeros((1, 1), np.float32), None, None, 1, 1)


def test_wavefront_nearest_hit_is_order_independent(frame):
    """The wavefront order (rsd.h RSD_HIT_ORDER_WAVEFRONT) delivers every hit nearer than the committed one too:
    KBuffer with N = 1 keeps the nearest hit, equal to both other orders."""
    from rsd import abi
    w = frame["wavefront"](sd_samples=1, implementation=abi.SD_KBUFFER, max_count=64)
    c = frame["canonical"](sd_samples=1, implementation=abi.SD_KBUFFER, max_count=64)
    assert np.array_equal(w.view(np.uint32), c.view(np.uint32))


def test_wavefront_default_samples_its_own_order(frame):
    """Under the wavefront order the Default reservoir samples (slots replaced) and the stream is not the
    depth-first one: the maps differ from the KBuffer's and from the depth-first order's."""
    from rsd import abi
    w = frame["wavefront"](sd_samples=4, implementation=abi.SD_DEFAULT)
    k = frame["wavefront"](sd_samples=4, implementation=abi.SD_KBUFFER)
    o = frame["ordered"](sd_samples=4, implementation=abi.SD_DEFAULT)
    assert (w.view(np.uint32) != k.view(np.uint32)).any(axis=-1).mean() > 0.005
    assert not np.array_equal(w.view(np.uint32), o.view(np.uint32))
    c = frame["canonical"](sd_samples=4, implementation=abi.SD_DEFAULT)
    hit = c[0, :, :, 0] < 1.0
    assert (w[0][hit] < 1.0).any(axis=-1).all()
