"""ctypes front end of the CPU oracle (oracle/rsd_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.  Inputs are
numpy arrays and plain Python values; outputs are numpy arrays.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
# RSD_ORACLE_VARIANT=asan: the ASan + UBSan build (make -C oracle asan; tools/asan_cpu_suite.sh)
_VARIANT = os.environ.get("RSD_ORACLE_VARIANT", "")
_LIB_PATH = _HERE / "_build" / (f"librsd_oracle_{_VARIANT}.so" if _VARIANT else "librsd_oracle.so")


def build(quiet: bool = True) -> Path:
    subprocess.run(["make", "-C", str(_HERE)] + ([_VARIANT] if _VARIANT else []), check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return _LIB_PATH


class Camera(C.Structure):
    _fields_ = [("posW", C.c_float * 3), ("nearZ", C.c_float),
                ("U", C.c_float * 3), ("farZ", C.c_float),
                ("V", C.c_float * 3), ("focalLength", C.c_float),
                ("W", C.c_float * 3), ("frameHeight", C.c_float),
                ("frameWidth", C.c_float), ("jitterX", C.c_float), ("jitterY", C.c_float),
                ("aspectRatio", C.c_float), ("viewMat", C.c_float * 16)]


class SDParams(C.Structure):
    _fields_ = [("sample_count", C.c_uint32), ("implementation", C.c_uint32), ("max_count", C.c_uint32),
                ("guard_band", C.c_int32), ("jitter", C.c_uint32), ("normalize", C.c_uint32),
                ("ray_interval", C.c_uint32), ("cull_mode", C.c_uint32), ("alpha_test", C.c_uint32),
                ("alpha", C.c_float), ("hit_order", C.c_uint32), ("use_16bit", C.c_uint32)]


class VAOData(C.Structure):
    _fields_ = [("noiseScale", C.c_float * 2), ("resolution", C.c_float * 2),
                ("lowResolution", C.c_float * 2), ("invResolution", C.c_float * 2),
                ("radius", C.c_float), ("exponent", C.c_float), ("thickness", C.c_float),
                ("sdGuard", C.c_int32), ("ssRadiusCutoff", C.c_float), ("ssMaxRadius", C.c_float)]


class SVAOParams(C.Structure):
    _fields_ = [("num_directions", C.c_uint32), ("sd_samples", C.c_uint32),
                ("secondary_depth_mode", C.c_uint32), ("ray_interval", C.c_uint32),
                ("sd_jitter", C.c_uint32), ("guard_band", C.c_uint32), ("dual_ao", C.c_uint32),
                ("tile_flags_unused", C.c_void_p), ("numerics_unused", C.c_uint32), ("ao_kernel", C.c_uint32),
                ("primary_depth_mode", C.c_uint32), ("depth2", C.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            build()
        L = C.CDLL(str(_LIB_PATH))
        vp, u32, i32, f32 = C.c_void_p, C.c_uint32, C.c_int, C.c_float
        L.ocpu_scene_create.restype = vp
        L.ocpu_scene_create.argtypes = [vp, u32, vp, u32, vp]
        L.ocpu_scene_destroy.argtypes = [vp]
        L.ocpu_scene_node_count.restype = u32
        L.ocpu_scene_node_count.argtypes = [vp]
        L.ocpu_camera_look_at.argtypes = [vp, vp, vp, f32, f32, f32, f32, f32, f32, vp]
        L.ocpu_gbuffer.argtypes = [vp, vp, u32, u32, u32, vp, vp, i32]
        L.ocpu_gbuffer_raster.argtypes = [vp, vp, u32, u32, u32, vp, vp, i32]
        L.ocpu_linearize_depth.argtypes = [vp, vp, C.c_size_t, f32, f32]
        L.ocpu_compress_normals.argtypes = [vp, vp, C.c_size_t, vp]
        L.ocpu_sd_trace.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp, vp, u32, u32, u32, u32, i32, vp]
        L.ocpu_sd_ray.argtypes = [vp, vp, vp, u32, u32, vp, vp, u32, u32, u32, u32, vp, vp, vp, vp]
        L.ocpu_svao_clear.argtypes = [vp, vp, u32]
        L.ocpu_sd_trace_band.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp, vp, u32, u32, u32, u32, u32, u32, i32, vp]
        L.ocpu_sd_trace_ordered.argtypes = [vp, vp, u32, vp, vp, vp, u32, u32, vp, vp, vp, u32, u32, u32, u32, u32, u32,
                                            i32, vp]
        L.ocpu_sd_trace_wavefront.argtypes = [vp, vp, u32, u32, vp, vp, vp, u32, u32, vp, vp, vp, u32, u32, u32, u32, u32,
                                              u32, i32, vp]
        L.ocpu_svao_pass1_band.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp, vp, vp, vp, u32, u32, u32, u32]
        L.ocpu_svao_pass1_rows.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp, vp, vp, vp, u32, u32, u32, u32]
        L.ocpu_svao_pass2_rows.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp, vp, u32, u32, vp, u32, u32, i32]
        L.ocpu_svao_pass2_band.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp, vp, u32, u32, vp, u32, u32, i32]
        L.ocpu_svao_pass1.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp, vp, vp, vp, u32, u32]
        L.ocpu_svao_pass2.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp, vp, u32, u32, vp, i32]
        L.ocpu_svao_pass2_rt_band.argtypes = [vp, vp, vp, vp, vp, vp, u32, u32, vp, vp, u32, u32, u32, u32, u32, i32]
        L.ocpu_scene_set_alpha.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, u32, vp, vp, vp]
        L.ocpu_alpha_fails.restype = i32
        L.ocpu_alpha_fails.argtypes = [vp, u32, f32, f32, i32, f32, vp, f32]
        L.ocpu_alpha_value.restype = f32
        L.ocpu_alpha_value.argtypes = [vp, u32, f32, f32, i32, f32, vp, f32]
        L.ocpu_alpha_threshold.restype = f32
        L.ocpu_alpha_threshold.argtypes = [vp, u32]
        L.ocpu_cross_bilateral_blur.argtypes = [vp, vp, u32, u32, vp, vp, u32, u32, u32, u32, u32]
        L.ocpu_temporal_ao.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, vp, vp, vp, vp]
        L.ocpu_motion_vectors.argtypes = [vp, vp, vp, u32, u32, vp]
        L.ocpu_motion_vectors_raster.argtypes = [vp, vp, vp, u32, u32, vp]
        L.ocpu_taa.argtypes = [vp, vp, vp, u32, u32, f32, f32, u32, vp]
        L.ocpu_ao_flicker_mask.argtypes = [vp, vp, u32, u32, vp, vp]
        L.ocpu_binary_dilation.argtypes = [vp, u32, u32, u32, vp]
        L.ocpu_ray_cone_spread.restype = f32
        L.ocpu_ray_cone_spread.argtypes = [f32, u32]
        L.ocpu_hash.restype = f32
        L.ocpu_hash.argtypes = [f32, f32]
        L.ocpu_jitter.argtypes = [u32, u32, vp, vp]
        L.ocpu_stratified_lut.argtypes = [i32, vp, vp]
        L.ocpu_noise_texture.argtypes = [vp]
        L.ocpu_sample_radius.restype = f32
        L.ocpu_sample_radius.argtypes = [u32, u32]
        L.ocpu_sample_radius_kernel.restype = f32
        L.ocpu_sample_radius_kernel.argtypes = [u32, u32, u32]
        L.ocpu_encode_normal_2x8.restype = u32
        L.ocpu_encode_normal_2x8.argtypes = [vp]
        L.ocpu_decode_normal_2x8.argtypes = [u32, vp]
        L.ocpu_intersect.restype = i32
        L.ocpu_intersect.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def effective_cpus():
    """CPUs this process may use at once: the affinity mask capped by the cgroup CPU quota (a GPU box
    shows 256 CPUs under a 16-CPU quota)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def _threads(n):
    return int(n) if n else effective_cpus()


class Scene:
    """alpha: an object with texcoords [nv,2], tri_material [nt], thresholds / alphas /
    material_textures [m] and textures (list of uint8 [h,w]) -- rsd.scenes.AlphaMaterials."""

    def __init__(self, positions, indices, flags=None, alpha=None):
        self.positions = np.ascontiguousarray(positions, np.float32)
        self.indices = np.ascontiguousarray(indices, np.uint32)
        self.flags = np.ascontiguousarray(flags if flags is not None else np.zeros(len(self.indices)), np.uint32)
        self.h = lib().ocpu_scene_create(_p(self.positions), len(self.positions), _p(self.indices),
                                         len(self.indices), _p(self.flags))
        if alpha is not None:
            uv = np.ascontiguousarray(alpha.texcoords, np.float32)
            tm = np.ascontiguousarray(alpha.tri_material, np.uint32)
            thr = np.ascontiguousarray(alpha.thresholds, np.float32)
            al = np.ascontiguousarray(alpha.alphas, np.float32)
            mt = np.ascontiguousarray(alpha.material_textures, np.uint32)
            tw = np.array([t.shape[1] for t in alpha.textures], np.uint32)
            th = np.array([t.shape[0] for t in alpha.textures], np.uint32)
            mip0 = np.ascontiguousarray(np.concatenate([np.asarray(t, np.uint8).ravel() for t in alpha.textures])
                                        if len(alpha.textures) else np.zeros(1, np.uint8))
            lib().ocpu_scene_set_alpha(self.h, _p(self.indices), _p(uv), _p(tm), len(thr), _p(thr), _p(al), _p(mt),
                                       len(tw), _p(tw), _p(th), _p(mip0))

    def alpha_value(self, prim, bu, bv, lod_ray_cone=False, t=0.0, d=(0.0, 0.0, 1.0), spread=0.0):
        dd = np.ascontiguousarray(d, np.float32)
        return lib().ocpu_alpha_value(self.h, prim, bu, bv, int(lod_ray_cone), t, _p(dd), spread)

    def alpha_threshold(self, material):
        return lib().ocpu_alpha_threshold(self.h, material)

    def alpha_fails(self, prim, bu, bv, lod_ray_cone=False, t=0.0, d=(0.0, 0.0, 1.0), spread=0.0):
        dd = np.ascontiguousarray(d, np.float32)
        return bool(lib().ocpu_alpha_fails(self.h, prim, bu, bv, int(lod_ray_cone), t, _p(dd), spread))

    @property
    def node_count(self):
        return lib().ocpu_scene_node_count(self.h)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ocpu_scene_destroy(self.h)
            self.h = None


def camera_look_at(pos, target, up, focal_length=21.0, frame_height=24.0, aspect=16 / 9, near=0.1, far=1000.0,
                   focal_distance=10000.0) -> Camera:
    cam = Camera()
    f3 = lambda v: np.ascontiguousarray(v, np.float32)
    p, t, u = f3(pos), f3(target), f3(up)
    lib().ocpu_camera_look_at(_p(p), _p(t), _p(u), focal_length, frame_height, aspect, near, far, focal_distance,
                              C.byref(cam))
    return cam


def gbuffer(scene: Scene, cam: Camera, W, H, cull_mode=1, threads=None):
    z = np.zeros((H, W), np.float32)
    n = np.zeros((H, W), np.uint16)
    lib().ocpu_gbuffer(scene.h, C.byref(cam), W, H, cull_mode, _p(z), _p(n), _threads(threads))
    return z, n


def gbuffer_raster(scene: Scene, cam: Camera, W, H, cull_mode=1, threads=None):
    """GBufferRaster.depth (non-linear) and .faceNormalW (H, W, 4) -- the raster G-buffer."""
    d = np.zeros((H, W), np.float32)
    nw = np.zeros((H, W, 4), np.float32)
    lib().ocpu_gbuffer_raster(scene.h, C.byref(cam), W, H, cull_mode, _p(d), _p(nw), _threads(threads))
    return d, nw


def linearize_depth(depth, near, far):
    d = np.ascontiguousarray(depth, np.float32)
    z = np.zeros_like(d)
    lib().ocpu_linearize_depth(_p(d), _p(z), d.size, near, far)
    return z


def compress_normals(normal_w, cam: Camera):
    nw = np.ascontiguousarray(normal_w, np.float32)
    out = np.zeros(nw.shape[:-1], np.uint16)
    lib().ocpu_compress_normals(_p(nw), _p(out), out.size, C.byref(cam))
    return out


def sd_trace(scene: Scene, cam: Camera, params: SDParams, linearZ, rayMin, rayMax, sdW, sdH,
             rows=None, threads=None):
    """The SD trace over the canonical any-hit stream (ascending (t, prim)); independent of any BVH."""
    if params.hit_order != 0:
        raise ValueError("hit_order = traversal needs librsd's BVH: use sd_trace_ordered()")
    N = params.sample_count
    ch, layers = min(N, 4), (N + 3) // 4
    sd = np.zeros((layers, sdH, sdW, ch), np.float32)
    r0, r1 = rows if rows else (0, sdH)
    stats = np.zeros(2, np.uint64)
    lz = np.ascontiguousarray(linearZ, np.float32)
    lib().ocpu_sd_trace(scene.h, C.byref(cam), C.byref(params), _p(lz), lz.shape[1], lz.shape[0],
                        _p(rayMin), _p(rayMax), _p(sd), sdW, sdH, r0, r1, _threads(threads), _p(stats))
    return sd, stats


def sd_trace_ordered(scene: Scene, bvh, tri_offset, cam: Camera, params: SDParams, linearZ, rayMin, rayMax, sdW, sdH,
                     rows=None, band=(0, 1), threads=None):
    """The SD trace over librsd's traversal-order any-hit stream (rsd.h RSD_HIT_ORDER_TRAVERSAL), walking
    librsd's own BVH: `bvh` = the float32 array of rsd_scene_export_bvh, tri_offset in float4 units.
    `scene` supplies the alpha-masked materials."""
    N = params.sample_count
    ch, layers = min(N, 4), (N + 3) // 4
    sd = np.zeros((layers, sdH, sdW, ch), np.float32)
    r0, r1 = rows if rows else (0, sdH)
    stats = np.zeros(2, np.uint64)
    lz = np.ascontiguousarray(linearZ, np.float32)
    b = np.ascontiguousarray(bvh, np.float32)
    lib().ocpu_sd_trace_ordered(scene.h, _p(b), int(tri_offset), C.byref(cam), C.byref(params), _p(lz), lz.shape[1],
                                lz.shape[0], _p(rayMin), _p(rayMax), _p(sd), sdW, sdH, r0, r1, band[0], band[1],
                                _threads(threads), _p(stats))
    return sd, stats


def sd_trace_wavefront(scene: Scene, bvh, tri_offset, pool_soft, cam: Camera, params: SDParams, linearZ, rayMin, rayMax,
                       sdW, sdH, rows=None, band=(0, 1), threads=None):
    """The SD trace over librsd's wavefront any-hit stream (rsd.h RSD_HIT_ORDER_WAVEFRONT) of librsd's own BVH;
    pool_soft = min(208 - 3 wide_depth, 160) (rsd_scene_info.wide_depth), the pool bound its order depends on."""
    N = params.sample_count
    ch, layers = min(N, 4), (N + 3) // 4
    sd = np.zeros((layers, sdH, sdW, ch), np.float32)
    r0, r1 = rows if rows else (0, sdH)
    stats = np.zeros(2, np.uint64)
    lz = np.ascontiguousarray(linearZ, np.float32)
    b = np.ascontiguousarray(bvh, np.float32)
    lib().ocpu_sd_trace_wavefront(scene.h, _p(b), int(tri_offset), int(pool_soft), C.byref(cam), C.byref(params), _p(lz),
                                  lz.shape[1], lz.shape[0], _p(rayMin), _p(rayMax), _p(sd), sdW, sdH, r0, r1, band[0],
                                  band[1], _threads(threads), _p(stats))
    return sd, stats


def sd_ray(cam: Camera, params: SDParams, linearZ, rayMin, rayMax, sdW, sdH, x, y):
    out = np.zeros(6, np.float32)
    tmin, tmax, cosT = C.c_float(), C.c_float(), C.c_float()
    lz = np.ascontiguousarray(linearZ, np.float32)
    lib().ocpu_sd_ray(C.byref(cam), C.byref(params), _p(lz), lz.shape[1], lz.shape[0], _p(rayMin), _p(rayMax),
                      sdW, sdH, x, y, _p(out), C.byref(tmin), C.byref(tmax), C.byref(cosT))
    return out[:3], out[3:], tmin.value, tmax.value, cosT.value


def stencil_dtype(num_directions):
    """The SVAO stencil texel (SVAO.cpp:132-134): R8Uint / R16Uint / R32Uint for 8 / 16 / 32 directions."""
    return {8: np.uint8, 16: np.uint16, 32: np.uint32}[int(num_directions)]


def _host_params(p, depth2=None):
    """A copy of the SVAO params whose DualDepth layer points at host memory (a struct copied from
    librsd carries a device pointer there): `depth2` (float32 H x W) or none; the array must outlive
    the call (the caller holds it)."""
    q = SVAOParams.from_buffer_copy(p)
    q.tile_flags_unused = None
    if q.primary_depth_mode == 1:
        if depth2 is None:
            raise ValueError("DualDepth (primary_depth_mode 1) needs the host depth2 layer")
        q.depth2 = depth2.ctypes.data
    else:
        q.depth2 = None
    return q


def svao_pass1(cam, vao: VAOData, p: SVAOParams, depth, normals, sdW, sdH, depth2=None):
    H, W = depth.shape
    d2 = None if depth2 is None else np.ascontiguousarray(depth2, np.float32)
    p = _host_params(p, d2)
    ao = np.zeros((H, W, 2) if p.dual_ao else (H, W), np.uint8)  # dualAO: RG8Unorm (bright, dark)
    st = np.zeros((H, W), stencil_dtype(p.num_directions))
    rmin = np.zeros((sdH, sdW), np.uint32)
    rmax = np.zeros((sdH, sdW), np.uint32)
    lib().ocpu_svao_clear(_p(rmin), _p(rmax), sdW * sdH)
    lib().ocpu_svao_pass1(C.byref(cam), C.byref(vao), C.byref(p), _p(depth), _p(normals), W, H,
                          _p(ao), _p(st), _p(rmin), _p(rmax), sdW, sdH)
    return ao, st, rmin, rmax


def svao_pass2(cam, vao: VAOData, p: SVAOParams, depth, normals, stencil, sd, ao, threads=None, depth2=None):
    H, W = depth.shape
    d2 = None if depth2 is None else np.ascontiguousarray(depth2, np.float32)
    p = _host_params(p, d2)
    ao = np.array(ao, np.uint8, copy=True)
    sdH, sdW = sd.shape[1], sd.shape[2]
    sdc = np.ascontiguousarray(sd, np.float32)
    stencil = np.ascontiguousarray(stencil, stencil_dtype(p.num_directions))
    lib().ocpu_svao_pass2(C.byref(cam), C.byref(vao), C.byref(p), _p(depth), _p(normals), W, H,
                          _p(stencil), _p(sdc), sdW, sdH, _p(ao), _threads(threads))
    return ao


def ray_cone_spread(focal_length, height):
    return lib().ocpu_ray_cone_spread(focal_length, height)


def svao_pass2_raytraced(scene: Scene, cam, vao: VAOData, p: SVAOParams, depth, normals, stencil, ao, cull=1,
                         ray_pipeline=0, band=(0, 1), threads=None, alpha_test=1, depth2=None):
    """SVAO "AO 2" in the Raytraced secondary mode; returns the updated AO image (VAO or HBAO kernel;
    SingleDepth, or DualDepth primary visibility with the host `depth2` layer)."""
    d2 = None if depth2 is None else np.ascontiguousarray(depth2, np.float32)
    p = _host_params(p, d2)
    H, W = depth.shape
    ao = np.array(ao, np.uint8, copy=True)
    lib().ocpu_svao_pass2_rt_band(scene.h, C.byref(cam), C.byref(vao), C.byref(p), _p(depth), _p(normals), W, H,
                                  _p(np.ascontiguousarray(stencil, stencil_dtype(p.num_directions))), _p(ao), cull,
                                  ray_pipeline, alpha_test,
                                  band[0], band[1], _threads(threads))
    return ao


def hash2(x, y):
    return lib().ocpu_hash(float(x), float(y))


def jitter(x, y):
    a, b = C.c_float(), C.c_float()
    lib().ocpu_jitter(x, y, C.byref(a), C.byref(b))
    return a.value, b.value


def stratified_lut(n):
    idx = np.zeros(n + 1, np.int32)
    lut = np.zeros(1 << n, np.uint32)
    lib().ocpu_stratified_lut(n, _p(idx), _p(lut))
    return idx, lut


def noise_texture():
    out = np.zeros(16, np.uint8)
    lib().ocpu_noise_texture(_p(out))
    return out


def sample_radius(nd, i, kernel=0):
    """Common.slang:51-66: the sample radius of direction i (kernel 0 VAO, 1 HBAO)."""
    return lib().ocpu_sample_radius_kernel(nd, i, kernel)


def encode_normal(n):
    a = np.ascontiguousarray(n, np.float32)
    return lib().ocpu_encode_normal_2x8(_p(a))


def decode_normal(packed):
    out = np.zeros(3, np.float32)
    lib().ocpu_decode_normal_2x8(int(packed), _p(out))
    return out


def intersect(o, d, v0, v1, v2):
    f = lambda v: np.ascontiguousarray(v, np.float32)
    t, u, v, det = C.c_float(), C.c_float(), C.c_float(), C.c_float()
    hit = lib().ocpu_intersect(_p(f(o)), _p(f(d)), _p(f(v0)), _p(f(v1)), _p(f(v2)),
                               C.byref(t), C.byref(u), C.byref(v), C.byref(det))
    return bool(hit), t.value, u.value, v.value, det.value


# ---- in-place, screen-band variants (used by the multi-process sharding tests)
def svao_clear(rmin, rmax):
    lib().ocpu_svao_clear(_p(rmin), _p(rmax), rmin.size)


def svao_pass1_into(cam, vao, p, depth, normals, ao, st, rmin, rmax, band=(0, 1)):
    p = _host_params(p)
    H, W = depth.shape
    sdH, sdW = rmin.shape
    lib().ocpu_svao_pass1_band(C.byref(cam), C.byref(vao), C.byref(p), _p(depth), _p(normals), W, H, _p(ao), _p(st),
                               _p(rmin), _p(rmax), sdW, sdH, band[0], band[1])


def svao_pass1_rows_into(cam, vao, p, depth, normals, ao, st, rmin, rmax, rows):
    """Pass 1 of the visible rows [rows[0], rows[1]) (a contiguous screen band)."""
    p = _host_params(p)
    H, W = depth.shape
    sdH, sdW = rmin.shape
    lib().ocpu_svao_pass1_rows(C.byref(cam), C.byref(vao), C.byref(p), _p(depth), _p(normals), W, H, _p(ao), _p(st),
                               _p(rmin), _p(rmax), sdW, sdH, rows[0], rows[1])


def svao_pass2_rows_into(cam, vao, p, depth, normals, stencil, sd, ao, rows, threads=None):
    p = _host_params(p)
    H, W = depth.shape
    sdc = np.ascontiguousarray(sd, np.float32)
    sdH, sdW = sdc.shape[1], sdc.shape[2]
    lib().ocpu_svao_pass2_rows(C.byref(cam), C.byref(vao), C.byref(p), _p(depth), _p(normals), W, H, _p(stencil),
                               _p(sdc), sdW, sdH, _p(ao), rows[0], rows[1], _threads(threads))


def sd_trace_rows_into(scene, cam, params, linearZ, rmin, rmax, sd, rows, threads=None):
    """The SD trace of SD rows [rows[0], rows[1]) into `sd` (the other rows untouched)."""
    sdH, sdW = sd.shape[1], sd.shape[2]
    stats = np.zeros(2, np.uint64)
    lib().ocpu_sd_trace_band(scene.h, C.byref(cam), C.byref(params), _p(linearZ), linearZ.shape[1], linearZ.shape[0],
                             _p(rmin), _p(rmax), _p(sd), sdW, sdH, rows[0], rows[1], 0, 1, _threads(threads),
                             _p(stats))
    return stats


def sd_trace_into(scene, cam, params, linearZ, rmin, rmax, sd, band=(0, 1), threads=None):
    sdH, sdW = sd.shape[1], sd.shape[2]
    stats = np.zeros(2, np.uint64)
    lib().ocpu_sd_trace_band(scene.h, C.byref(cam), C.byref(params), _p(linearZ), linearZ.shape[1], linearZ.shape[0],
                             _p(rmin), _p(rmax), _p(sd), sdW, sdH, 0, sdH, band[0], band[1], _threads(threads),
                             _p(stats))
    return stats


def svao_pass2_into(cam, vao, p, depth, normals, stencil, sd, ao, band=(0, 1), threads=None):
    p = _host_params(p)
    H, W = depth.shape
    sdH, sdW = sd.shape[1], sd.shape[2]
    lib().ocpu_svao_pass2_band(C.byref(cam), C.byref(vao), C.byref(p), _p(depth), _p(normals), W, H, _p(stencil),
                               _p(sd), sdW, sdH, _p(ao), band[0], band[1], _threads(threads))


def temporal_ao(ao_in, linear_z, mvec, prev_z, prev_ao, prev_history, cam, prev_view_to_cur_view, guard,
                stable_mask=None, ao_dst=None, history_dst=None):
    """TemporalAO (enabled) of one frame (rsd_oracle.c ocpu_temporal_ao, TemporalAO.ps.slang:55-101).
    Pixels outside the guard band keep the destinations' values (zeros by default)."""
    ao_in = np.ascontiguousarray(ao_in, np.uint8)
    H, W = ao_in.shape
    z = np.ascontiguousarray(linear_z, np.float32)
    mv = np.ascontiguousarray(mvec, np.float32)
    pz = np.ascontiguousarray(prev_z, np.float32)
    pa = np.ascontiguousarray(prev_ao, np.uint8)
    pn = np.ascontiguousarray(prev_history, np.uint8)
    assert z.shape == (H, W) and mv.shape == (H, W, 2) and pz.shape == (H, W) and pa.shape == (H, W)
    st = None if stable_mask is None else np.ascontiguousarray(stable_mask, np.uint8)
    m = np.ascontiguousarray(prev_view_to_cur_view, np.float32).reshape(16)
    ao = np.zeros_like(ao_in) if ao_dst is None else np.array(ao_dst, np.uint8, copy=True)
    n = np.zeros_like(ao_in) if history_dst is None else np.array(history_dst, np.uint8, copy=True)
    lib().ocpu_temporal_ao(_p(ao_in), _p(z), _p(mv), _p(pz), _p(pa), _p(pn), None if st is None else _p(st), W, H,
                           guard, C.byref(cam), _p(m), _p(ao), _p(n))
    return ao, n


def motion_vectors(cam, prev_cam, linear_z):
    """GBufferRaster.mvec (RG32F, H x W x 2) for a static scene seen from cam after prev_cam."""
    z = np.ascontiguousarray(linear_z, np.float32)
    out = np.zeros(z.shape + (2,), np.float32)
    lib().ocpu_motion_vectors(C.byref(cam), C.byref(prev_cam), _p(z), z.shape[1], z.shape[0], _p(out))
    return out


def motion_vectors_raster(cam, prev_cam, depth):
    """GBufferRaster.mvec from the non-linear raster depth (background: d >= 1)."""
    d = np.ascontiguousarray(depth, np.float32)
    out = np.zeros(d.shape + (2,), np.float32)
    lib().ocpu_motion_vectors_raster(C.byref(cam), C.byref(prev_cam), _p(d), d.shape[1], d.shape[0], _p(out))
    return out


def ao_flicker_mask(linear_z, normal_w, cam):
    """AOFlickerMask (rsd_oracle.c ocpu_ao_flicker_mask): R8Uint stable mask (H, W)."""
    z = np.ascontiguousarray(linear_z, np.float32)
    n = np.ascontiguousarray(normal_w, np.float32)
    H, W = z.shape
    assert n.shape == (H, W, 4)
    out = np.zeros((H, W), np.uint8)
    lib().ocpu_ao_flicker_mask(_p(z), _p(n), W, H, C.byref(cam), _p(out))
    return out


def binary_dilation(mask, op="min"):
    """BinaryDilation (rsd_oracle.c ocpu_binary_dilation), op 'min' or 'max'."""
    m = np.ascontiguousarray(mask, np.uint8)
    out = np.zeros_like(m)
    lib().ocpu_binary_dilation(_p(m), m.shape[1], m.shape[0], {"min": 0, "max": 1}[op], _p(out))
    return out


def taa(color, mvec, prev_color, alpha=0.1, color_box_sigma=1.0, anti_flicker=True):
    """TAA of one frame (rsd_oracle.c ocpu_taa, TAA.ps.slang:78-150): RGBA32F (H, W, 4) colours,
    RG32F (H, W, 2) motion vectors; returns the RGBA32F output (the next frame's prev_color)."""
    c = np.ascontiguousarray(color, np.float32)
    H, W = c.shape[:2]
    mv = np.ascontiguousarray(mvec, np.float32)
    pv = np.ascontiguousarray(prev_color, np.float32)
    assert c.shape == (H, W, 4) and mv.shape == (H, W, 2) and pv.shape == (H, W, 4)
    out = np.zeros_like(c)
    lib().ocpu_taa(_p(c), _p(mv), _p(pv), W, H, alpha, color_box_sigma, int(bool(anti_flicker)), _p(out))
    return out


def cross_bilateral_blur(src, linear_z, guard, radius=4, better_slope=True, dst=None):
    """CrossBilateralBlur of an R8Unorm image; pixels outside the guard band keep `dst`'s
    values (zeros by default), as the scissored pass leaves them."""
    src = np.ascontiguousarray(src, np.uint8)
    z = np.ascontiguousarray(linear_z, np.float32)
    H, W = src.shape
    out = np.zeros_like(src) if dst is None else np.array(dst, np.uint8, copy=True)
    pp = np.zeros_like(src)
    lib().ocpu_cross_bilateral_blur(_p(src), _p(z), z.shape[1], z.shape[0], _p(pp), _p(out), W, H, guard, radius,
                                    int(better_slope))
    return out, pp
