"""CPU tests of the oracle itself: intersection / culling conventions, normal packing,
and the any-hit-stream semantics of the SD trace against a brute-force restatement
(every triangle tested, hits sorted by (t, prim), algorithm replayed in numpy float32)."""
import math

import numpy as np
import pytest

from helpers import oracle_vao

F = np.float32


def test_watertight_facing_convention(oracle):
    # ray down -z onto a triangle that is counter-clockwise seen from the origin
    o, d = [0.25, 0.25, 10.0], [0.0, 0.0, -1.0]
    v0, v1, v2 = [0, 0, 0], [1, 0, 0], [0, 1, 0]
    hit, t, u, v, det = oracle.intersect(o, d, v0, v1, v2)
    assert hit and t == 10.0 and det > 0
    assert (u, v) == (0.25, 0.25)  # DXR barycentrics = weights of v1, v2
    hit, t, u, v, det = oracle.intersect(o, d, v0, v2, v1)
    assert hit and det < 0
    assert not oracle.intersect([2.0, 2.0, 10.0], d, v0, v1, v2)[0]


def test_watertight_shared_edge(oracle):
    # rays through the diagonal shared by two triangles of a quad never fall through
    rng = np.random.default_rng(5)
    a, b, c, e = [0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]
    for s in rng.random(500):
        p = [float(F(s)), float(F(s)), 3.0]
        h1 = oracle.intersect(p, [0, 0, -1], a, b, c)[0]
        h2 = oracle.intersect(p, [0, 0, -1], a, c, e)[0]
        assert h1 or h2


def test_normal_packing_roundtrip(oracle):
    rng = np.random.default_rng(1)
    for n in rng.normal(size=(300, 3)):
        n = (n / np.linalg.norm(n)).astype(np.float32)
        d = oracle.decode_normal(oracle.encode_normal(n))
        assert np.linalg.norm(d - n) < 0.03
    assert oracle.encode_normal([0, 0, 1]) == 0
    assert oracle.encode_normal([1, 0, 0]) == 127
    assert oracle.encode_normal([0, 1, 0]) == 127 << 8
    assert np.allclose(oracle.decode_normal(0), [0, 0, 1])


def _layered_scene(n_planes=12, seed=3, jitter=0.0):
    """Stacked, slightly tilted quads in front of the camera (many hits per ray)."""
    rng = np.random.default_rng(seed)
    pos, ind = [], []
    for k in range(n_planes):
        z = -2.0 - 0.7 * k + jitter * rng.random()
        tilt = 0.05 * rng.standard_normal()
        q = np.array([[-3, -3, z], [3, -3, z + tilt], [3, 3, z + 2 * tilt], [-3, 3, z + tilt]], np.float32)
        base = len(pos) * 4
        pos.append(q)
        # alternate winding so that back-face culling removes some planes
        if k % 3 == 2:
            ind += [[base, base + 2, base + 1], [base, base + 3, base + 2]]
        else:
            ind += [[base, base + 1, base + 2], [base, base + 2, base + 3]]
    return np.concatenate(pos), np.array(ind, np.uint32)


def _replay(hits, N, impl, max_count, cosT, near, far, alpha):
    """Common.slangh:102-254 over the sorted hit stream, numpy float32."""
    depths = [F(1.0)] * N
    count = 0
    idx = lut = None
    if impl == 1:
        idx = [sum(math.comb(N, j) for j in range(i)) for i in range(N + 1)]
        lut = [0] + sorted(range(1, 1 << N), key=lambda m: (bin(m).count("1"), m))
    for t, u, v in hits:
        rng = F(hash_(u, v))
        z = F(F(t) * F(cosT))
        z = F(min(max(F(F(z - F(near)) / F(F(far) - F(near))), F(0)), F(1)))
        if impl == 1:
            R = int(math.floor(F(F(F(alpha) * F(N)) + rng)))
            mask = 0
            if R >= N:
                mask = 0xFFFF
            elif R != 0:
                r2 = F(hash_(rng, z))
                lo, hi = F(idx[R]), F(idx[R + 1])
                mask = lut[int(F(lo + F(r2 * F(hi - lo))))]
            maxT = F(0)
            for i in range(N):
                if (mask >> i) & 1 and z < depths[i]:
                    depths[i] = z
                maxT = max(maxT, depths[i])
            if not z < maxT:
                break
        elif impl == 3:
            if z >= depths[N - 1]:
                break
            count += 1
            rayT = z
            for i in range(N):
                if z < depths[i]:
                    depths[i], z = z, depths[i]
            if depths[N - 1] == rayT or count >= max_count:
                break
        else:
            slot = count
            count += 1
            if count > N:
                slot = int(F(rng * F(count)))
            if slot < N and not depths[slot] <= z:
                depths[slot] = z
            if count >= max_count:
                break
    return depths


hash_ = None


@pytest.mark.parametrize("impl,N,max_count,cull", [(0, 4, 8, 1), (0, 1, 1, 1), (0, 8, 8, 0), (0, 2, 5, 2),
                                                   (3, 4, 8, 1), (3, 2, 3, 0), (1, 4, 8, 1), (1, 8, 8, 0),
                                                   (0, 16, 16, 0)])
def test_sd_trace_equals_bruteforce_sorted_stream(oracle, impl, N, max_count, cull):
    global hash_
    hash_ = oracle.hash2
    pos, ind = _layered_scene()
    flags = np.zeros(len(ind), np.uint32)
    flags[::5] = 1  # some double-sided triangles
    sc = oracle.Scene(pos, ind, flags)
    W = H = 12
    cam = oracle.camera_look_at([0.1, 0.2, 1.0], [0.0, 0.0, -5.0], [0, 1, 0], aspect=1.0)
    lz = np.zeros((H, W), np.float32)  # TMin = 0.1 * near
    p = oracle.SDParams(N, impl, max_count, 0, 1, 1, 0, cull, 0, float(F(1.5 / N)))
    sd, stats = oracle.sd_trace(sc, cam, p, lz, None, None, W, H, threads=2)
    tris = pos[ind]
    for y in range(H):
        for x in range(W):
            o, d, tmin, tmax, cosT = oracle.sd_ray(cam, p, lz, None, None, W, H, x, y)
            hits = []
            for prim, (v0, v1, v2) in enumerate(tris):
                hit, t, u, v, det = oracle.intersect(o, d, v0, v1, v2)
                if not hit or not (tmin <= t <= tmax):
                    continue
                if cull and not flags[prim] & 1:
                    front = det > 0
                    if (cull == 1 and not front) or (cull == 2 and front):
                        continue
                hits.append((t, prim, u, v))
            hits.sort(key=lambda h: (h[0], h[1]))
            want = _replay([(t, u, v) for t, _, u, v in hits], N, impl, max_count, cosT, cam.nearZ, cam.farZ,
                           float(F(1.5 / N)))
            got = [sd[k // 4, y, x, k % 4] for k in range(N)] if N >= 4 else list(sd[0, y, x, :N])
            assert [F(g) for g in got] == want, (x, y, hits[:10])


def test_sd_result_depends_only_on_max_count_nearest_hits(oracle):
    """Default reservoir commits at the MAX_COUNT-th hit: planes behind it are irrelevant."""
    pos, ind = _layered_scene(n_planes=14)
    W = H = 16
    cam = oracle.camera_look_at([0.0, 0.0, 1.0], [0.0, 0.0, -5.0], [0, 1, 0], aspect=1.0)
    lz = np.zeros((H, W), np.float32)
    p = oracle.SDParams(4, 0, 8, 0, 1, 1, 0, 0, 0, 0.375)
    full, _ = oracle.sd_trace(oracle.Scene(pos, ind), cam, p, lz, None, None, W, H)
    # keep the 8 nearest planes (16 triangles) only
    cut, _ = oracle.sd_trace(oracle.Scene(pos, ind[:16]), cam, p, lz, None, None, W, H)
    assert np.array_equal(full, cut)


def test_sd_empty_interval_keeps_default_depth(oracle):
    pos, ind = _layered_scene()
    sc = oracle.Scene(pos, ind)
    W = H = 8
    cam = oracle.camera_look_at([0.0, 0.0, 1.0], [0.0, 0.0, -5.0], [0, 1, 0], aspect=1.0)
    lz = np.zeros((H, W), np.float32)
    rmin = np.full((H, W), np.float32(3.4028235e38).view(np.uint32), np.uint32)  # cleared (SVAO.cpp:339)
    rmax = np.zeros((H, W), np.uint32)
    p = oracle.SDParams(4, 0, 8, 0, 1, 1, 1, 1, 0, 0.375)
    sd, stats = oracle.sd_trace(sc, cam, p, lz, rmin, rmax, W, H)
    assert stats[0] == 0 and np.all(sd == 1.0)


def test_svao_pass1_interval_invariants(oracle):
    from rsd.scenes import make_scene
    s = make_scene("arcade_tiny")
    sc = oracle.Scene(s.positions, s.indices, s.flags)
    g, vis = 16, (96, 64)
    W, H = vis[0] + 2 * g, vis[1] + 2 * g
    cam = oracle.camera_look_at(s.camera["pos"], s.camera["target"], s.camera["up"], aspect=float(F(W) / F(H)))
    z, n = oracle.gbuffer(sc, cam, W, H)
    vao, sdW, sdH = oracle_vao(oracle, W, H, 2, sd_guard_px=64, radius=1.5)
    p = oracle.SVAOParams(8, 4, 2, 1, 1, g)
    ao, st, rmin, rmax = oracle.svao_pass1(cam, vao, p, z, n, sdW, sdH)
    touched = rmax != 0
    assert touched.any() and (st != 0).any()
    assert np.all(rmin[~touched] == np.float32(3.4028235e38).view(np.uint32))
    assert np.all(rmin[touched].view(np.float32) <= rmax[touched].view(np.float32))
    # pass 2 only rewrites stencilled pixels
    N = 4
    sd = np.ones((1, sdH, sdW, N), np.float32)
    ao2 = oracle.svao_pass2(cam, vao, p, z, n, st, sd, ao)
    assert np.array_equal(ao2[st == 0], ao[st == 0])


def test_raster_gbuffer_chain_matches_linear_gbuffer(oracle):
    """GBufferRaster.depth -> LinearizeDepth and .faceNormalW -> CompressNormals restate the
    same closest hits as the direct linear G-buffer: identical misses, normals bit-equal,
    depth equal up to the float round trip through the non-linear depth."""
    from rsd.scenes import make_scene
    s = make_scene("arcade_tiny")
    os_ = oracle.Scene(s.positions, s.indices, s.flags)
    cam = oracle.camera_look_at([0, 1.7, 3.0], [0, 1.2, -2.0], [0, 1, 0], aspect=96 / 64)
    z, n = oracle.gbuffer(os_, cam, 96, 64, 1)
    d, nw = oracle.gbuffer_raster(os_, cam, 96, 64, 1)
    miss = d == 1.0
    assert miss.sum() < miss.size and np.all(nw[miss] == 0)
    assert np.all(z[miss] == np.float32(cam.farZ))
    np.testing.assert_array_equal(oracle.compress_normals(nw, cam)[~miss], n[~miss])
    zl = oracle.linearize_depth(d, cam.nearZ, cam.farZ)
    np.testing.assert_allclose(zl[~miss], z[~miss], rtol=2e-3)
    # Linearize.ps.slang formula, evaluated in float32 by numpy
    zn, zf = np.float32(cam.nearZ), np.float32(cam.farZ)
    np.testing.assert_array_equal(zl, zn * zf / (zf + d * (zn - zf)))


def test_raytraced_ao_independent_of_bvh(oracle):
    """The Raytraced pass 2 depends on hit distances only: permuting the triangles (another
    BVH, other primitive ids) leaves the AO image bit-identical; the refinement is not a no-op."""
    from rsd.scenes import make_scene
    s = make_scene("arcade_tiny")
    g, vis = 16, (96, 64)
    W, H = vis[0] + 2 * g, vis[1] + 2 * g
    cam = oracle.camera_look_at(s.camera["pos"], s.camera["target"], s.camera["up"], aspect=float(F(W) / F(H)))
    sc = oracle.Scene(s.positions, s.indices, s.flags)
    z, n = oracle.gbuffer(sc, cam, W, H)
    vao, sdW, sdH = oracle_vao(oracle, W, H, 1, sd_guard_px=0, radius=1.5)
    p = oracle.SVAOParams(8, 4, 3, 1, 1, g)
    ao1, st, _, _ = oracle.svao_pass1(cam, vao, p, z, n, sdW, sdH)
    assert (st != 0).sum() > 50
    ao = oracle.svao_pass2_raytraced(sc, cam, vao, p, z, n, st, ao1)
    perm = np.random.default_rng(7).permutation(len(s.indices))
    sc2 = oracle.Scene(s.positions, s.indices[perm], s.flags[perm])
    ao2 = oracle.svao_pass2_raytraced(sc2, cam, vao, p, z, n, st, ao1)
    assert np.array_equal(ao, ao2)
    assert not np.array_equal(ao, ao1)
    assert np.array_equal(ao[st == 0], ao1[st == 0])


@pytest.mark.parametrize("nd", [16, 32])
def test_oracle_pass1_direction_counts(oracle, nd):
    """NUM_DIRECTIONS 16 / 32: the stencil widens to R16Uint / R32Uint and directions above 8 refine;
    with secondaryDepthMode SingleDepth the AO is the per-direction mean (the same scene at 8, 16
    and 32 directions gives close AO: the three radius tables sample the same disc)."""
    from rsd.frame import FrameConfig, make_camera, make_vao, svao_params
    from rsd.scenes import make_scene
    from helpers import to_oracle
    scene = make_scene("arcade_tiny")
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    out = {}
    for n in (8, nd):
        cfg = FrameConfig(visible_w=160, visible_h=96, guard_band=16, divisor=2, sd_samples=4, sd_guard_px=64,
                          radius=1.0, num_directions=n)
        cam = to_oracle(make_camera(scene, cfg), oracle.Camera)
        vao, sdw, sdh = make_vao(cfg)
        z, nrm = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, 1, threads=4)
        ao, st, rmin, rmax = oracle.svao_pass1(cam, to_oracle(vao, oracle.VAOData),
                                               to_oracle(svao_params(cfg), oracle.SVAOParams), z, nrm, sdw, sdh)
        out[n] = (ao, st)
    ao, st = out[nd]
    assert st.dtype == {16: np.uint16, 32: np.uint32}[nd]
    assert (st >> 8).any()  # directions above the eighth requested SD rays
    a8 = out[8][0].astype(np.int32)
    assert np.abs(ao.astype(np.int32) - a8)[out[8][1] == 0].mean() < 12  # same disc, finer sampling


def test_oracle_dual_ao(oracle):
    """dualAO (SVAORaster.ps.slang:13,101-104; SVAORaster2.ps.slang:60-64): the bright channel is the
    single-channel AO bit for bit; the dark channel equals it where no direction needed a ray, and
    after pass 2 dark <= bright everywhere."""
    from rsd.frame import FrameConfig, make_camera, make_vao, sd_params, svao_params
    from rsd.scenes import make_scene
    from helpers import to_oracle
    scene = make_scene("arcade_tiny")
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    res = {}
    for dual in (False, True):
        cfg = FrameConfig(visible_w=160, visible_h=96, guard_band=16, divisor=2, sd_samples=4, sd_guard_px=64,
                          radius=1.0, dual_ao=dual)
        cam = to_oracle(make_camera(scene, cfg), oracle.Camera)
        vao, sdw, sdh = make_vao(cfg)
        ov, svp = to_oracle(vao, oracle.VAOData), to_oracle(svao_params(cfg), oracle.SVAOParams)
        z, nrm = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, 1, threads=4)
        ao1, st, rmin, rmax = oracle.svao_pass1(cam, ov, svp, z, nrm, sdw, sdh)
        sd, _ = oracle.sd_trace(osc, cam, to_oracle(sd_params(cfg, vao.sdGuard), oracle.SDParams), z, rmin, rmax,
                                sdw, sdh, threads=4)
        res[dual] = (ao1, st, oracle.svao_pass2(cam, ov, svp, z, nrm, st, sd, ao1, threads=4))
    ao1, st, ao2 = res[True]
    assert ao1.shape[-1] == 2 and ao2.shape[-1] == 2
    assert np.array_equal(ao1[..., 0], res[False][0]) and np.array_equal(ao2[..., 0], res[False][2])
    assert np.array_equal(ao1[..., 0][st == 0], ao1[..., 1][st == 0])
    assert (st != 0).any() and (ao2[..., 1] <= ao2[..., 0]).all()


def _flat_floor_scene():
    """One 200 x 200 quad at y = 0 under a camera looking down at 45 degrees."""
    from rsd.scenes import Scene
    pos = np.array([[-100, 0, -100], [100, 0, -100], [100, 0, 100], [-100, 0, 100]], np.float32)
    ind = np.array([[0, 2, 1], [0, 3, 2]], np.uint32)
    cam = {"pos": [0.0, 3.0, 6.0], "target": [0.0, 0.0, 0.0], "up": [0.0, 1.0, 0.0]}
    return Scene("flat", pos, ind, np.zeros(2, np.uint32), cam)


def test_oracle_hbao_flat_floor_is_unoccluded(oracle):
    """HBAO (Common.slang:421-430): every sample of a flat floor lies in the pixel's tangent plane, so
    the angle term saturate(dot(n, V) - 0.1) is 0 and the AO saturate(1 - 2 * 0)^2 = 1 everywhere."""
    from rsd.frame import FrameConfig, make_camera, make_vao, svao_params
    from helpers import to_oracle
    scene = _flat_floor_scene()
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    cfg = FrameConfig(visible_w=128, visible_h=96, guard_band=16, divisor=2, sd_guard_px=64, radius=1.0,
                      secondary=0, ao_kernel="hbao", cull_mode=0)
    cam = to_oracle(make_camera(scene, cfg), oracle.Camera)
    vao, sdw, sdh = make_vao(cfg)
    z, nrm = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, 0, threads=4)
    assert (z < 1000.0).mean() > 0.3  # the floor covers the lower part of the frame
    ao, st, _, _ = oracle.svao_pass1(cam, to_oracle(vao, oracle.VAOData), to_oracle(svao_params(cfg), oracle.SVAOParams),
                                     z, nrm, sdw, sdh)
    g = cfg.guard_band
    assert (ao[g:-g, g:-g] == 255).all()


def test_oracle_dual_depth_equal_layers_is_single_depth(oracle):
    """DualDepth (SVAORaster.ps.slang:69-70): a second layer equal to the first adds the same sample
    again (min / max of equal values), so pass 1 equals the SingleDepth pass 1 bit for bit; a layer
    behind the first changes the AO of some refined directions."""
    import dataclasses
    from rsd.frame import FrameConfig, make_camera, make_vao, svao_params
    from rsd.scenes import make_scene
    from helpers import to_oracle
    scene = make_scene("arcade_tiny")
    osc = oracle.Scene(scene.positions, scene.indices, scene.flags)
    for kernel in ("vao", "hbao"):
        cfg = FrameConfig(visible_w=160, visible_h=96, guard_band=16, divisor=2, sd_guard_px=64, radius=1.0,
                          secondary=0, ao_kernel=kernel)
        cam = to_oracle(make_camera(scene, cfg), oracle.Camera)
        vao, sdw, sdh = make_vao(cfg)
        vao = to_oracle(vao, oracle.VAOData)
        z, nrm = oracle.gbuffer(osc, cam, cfg.fb_w, cfg.fb_h, 1, threads=4)
        single = oracle.svao_pass1(cam, vao, to_oracle(svao_params(cfg), oracle.SVAOParams), z, nrm, sdw, sdh)
        dcfg = dataclasses.replace(cfg, primary=1)
        svp = to_oracle(svao_params(dcfg), oracle.SVAOParams)
        same = oracle.svao_pass1(cam, vao, svp, z, nrm, sdw, sdh, depth2=z.copy())
        assert np.array_equal(single[0], same[0]) and np.array_equal(single[1], same[1]), kernel
        behind = oracle.svao_pass1(cam, vao, svp, z, nrm, sdw, sdh, depth2=z * np.float32(1.1) + np.float32(0.25))
        assert not np.array_equal(single[0], behind[0]), kernel
        with pytest.raises(ValueError):
            oracle.svao_pass1(cam, vao, svp, z, nrm, sdw, sdh)  # DualDepth without the second layer
