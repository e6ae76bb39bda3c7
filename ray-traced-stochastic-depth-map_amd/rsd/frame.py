"""Frame-level driver of the Ray-SD + SVAO hot path on one GPU.

`Renderer` owns one rsd_device, one uploaded scene and the device buffers of one
frame, and issues exactly the dispatch sequence of SVAO::execute (SVAO.cpp:192-456):

    clear ray intervals  ->  "AO 1" (pass 1)  ->  StochasticDepthMapRT (SD trace)
    ->  "AO 2" (pass 2)

The G-buffer (linear depth + packed view-space normals) is produced once by the
primary-visibility kernel; it is an input of the hot path, not part of it
(AO frame time excludes the G-buffer and the BVH build).

Device memory comes from torch (plumbing only); every compute step is a librsd
C-ABI call on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os
import weakref

import numpy as np

from . import abi
from .scenes import Scene


@dataclasses.dataclass
class FrameConfig:
    """One BASELINE config: visible size + GuardBand, SD divisor, SD samples, SVAO knobs.

    Defaults follow scripts/SVAO.py:10-12 (guardBand 64, radius 0.2, stochMapDivisor 4)
    and SVAO.h:90-126 (N = 4, MAX_COUNT = 8, jitter, ray interval, back-face culling,
    512-px SD guard band, 8 AO directions)."""
    visible_w: int = 1920
    visible_h: int = 1080
    guard_band: int = 64
    divisor: int = 4
    sd_samples: int = 4
    max_count: int = 8
    implementation: int = abi.SD_DEFAULT
    hit_order: int = abi.HIT_ORDER_CANONICAL  # any-hit order (rsd.h rsd_hit_order; librsd extension)
    use_16bit: bool = False                   # SD pass Use16Bit (standalone SD pass only; N <= 4)
    jitter: bool = True
    ray_interval: bool = True
    cull_mode: int = abi.CULL_BACK
    radius: float = 0.2
    exponent: float = 2.0
    secondary: int = abi.DEPTH_STOCHASTIC  # SVAO secondaryDepthMode: 0 Single, 1 Dual, 2 StochasticDepth, 3 Raytraced
    primary: int = abi.DEPTH_SINGLE        # SVAO primaryDepthMode: 0 Single, 1 Dual (needs Renderer.depth2)
    ao_kernel: str = "vao"                 # SVAO AO kernel (rsd_ao_kernel): "vao" or "hbao" (SVAO.cpp:233)
    ray_pipeline: bool = True              # SVAO rayPipeline (SVAO.h:101): pass-2 extent in Raytraced mode
    alpha_test: bool = True                # SVAO alphaTest (SVAO.h:104) -> SD AlphaTest; no-op on opaque scenes
    thickness: float = 0.0
    sd_guard_px: int = 512
    num_directions: int = 8
    dual_ao: bool = False                  # SVAO dualAO (SVAO.cpp:130): ao is RG8Unorm (bright, dark)
    # arithmetic of the SVAO passes (rsd.h rsd_numerics): "fast" (the product default, AO graded by
    # BASELINE.md section 4's tolerance) or "exact" (bit-identical to the oracle); the environment's
    # RSD_NUMERICS sets the default
    numerics: str = dataclasses.field(default_factory=lambda: os.environ.get("RSD_NUMERICS", "fast"))
    focal_length: float = 21.0
    frame_height: float = 24.0
    near: float = 0.1
    far: float = 1000.0

    @property
    def fb_w(self):
        return self.visible_w + 2 * self.guard_band

    @property
    def fb_h(self):
        return self.visible_h + 2 * self.guard_band


CONFIGS = {
    # BASELINE.json configs[1..4] (configs[0] is the CPU-only plumbing case, see tests)
    "suntemple_1080p_q": (dict(visible_w=1920, visible_h=1080, divisor=4, sd_samples=4), "suntemple"),
    "bistro_1080p_full": (dict(visible_w=1920, visible_h=1080, divisor=1, sd_samples=8), "bistro_exterior"),
    "emerald_4k_q": (dict(visible_w=3840, visible_h=2160, divisor=4, sd_samples=4), "emerald_square"),
    "bistro_4k_full_n16": (dict(visible_w=3840, visible_h=2160, divisor=1, sd_samples=16, max_count=16),
                           "bistro_exterior"),
}

# BASELINE.json configs[0]: the Arcade plumbing case -- 256 x 256, SD N = 1, divisor 1, the SD
# pass driven directly with GuardBand 0 (no SVAO guard band, no SD guard band)
ARCADE_CONFIG = (dict(visible_w=256, visible_h=256, guard_band=0, divisor=1, sd_samples=1, sd_guard_px=0),
                 "arcade_tiny")

# camera path of each config when the bench animates it (BASELINE configs[4]: 120-frame animated camera)
DEFAULT_CAMERA_PATH = {"bistro_4k_full_n16": "orbit120"}


def look_at(pos, target, up, cfg: FrameConfig) -> abi.Camera:
    """Camera::calculateCameraParameters through librsd (rsd_camera_look_at, Camera.cpp:99-185)."""
    cam = abi.Camera()
    f3 = lambda v: (C.c_float * 3)(*[float(x) for x in v])
    aspect = np.float32(cfg.fb_w) / np.float32(cfg.fb_h)
    abi.check(abi.lib().rsd_camera_look_at(f3(pos), f3(target), f3(up), cfg.focal_length, cfg.frame_height,
                                           float(aspect), cfg.near, cfg.far, 10000.0, C.byref(cam)),
              "rsd_camera_look_at")
    return cam


def make_camera(scene: Scene, cfg: FrameConfig) -> abi.Camera:
    return look_at(scene.camera["pos"], scene.camera["target"], scene.camera["up"], cfg)


def camera_path(name: str, seed: int = 5):
    """Look-at poses (pos, target, up) of a named camera path -- the animated camera of
    BASELINE configs[4] (the reference benchmarks along camera paths with PathBenchmark,
    PathBenchmark.cpp:59-90, scripts/SVAO.py:23,54).

    "orbitN": N poses on a closed orbit of the synthetic hall (room 40 x 12 x 40, rsd/scenes.py):
    radius 17 m at 5.5 m height (above every prop, clear of the colonnades at x = +-12.8, which
    are the only full-height objects), bobbing +-0.5 m, looking at a target that wanders around
    the hall centre.  The start angle and the wander phases come from `seed`.  "static": the
    scene's own camera (one pose)."""
    if name == "static":
        return None
    if not name.startswith("orbit"):
        raise ValueError(f"unknown camera path '{name}' (static, orbitN)")
    n = int(name[5:] or 120)
    rng = np.random.default_rng(seed)
    a0, p1, p2 = rng.uniform(0.0, 2.0 * np.pi, 3)
    poses = []
    for i in range(n):
        a = a0 + 2.0 * np.pi * i / n
        pos = [17.0 * np.cos(a), 5.5 + 0.5 * np.sin(2.0 * a + p1), 17.0 * np.sin(a)]
        tgt = [2.0 * np.cos(3.0 * a + p2), 1.0, 2.0 * np.sin(2.0 * a + p1)]
        poses.append(([float(np.float32(v)) for v in pos], [float(np.float32(v)) for v in tgt], [0.0, 1.0, 0.0]))
    return poses


def make_vao(cfg: FrameConfig):
    vao = abi.VAOData()
    w, h = C.c_uint32(), C.c_uint32()
    # getExtraGuardBand (SVAO.cpp:718-723): the SD guard band exists in StochasticDepth mode only
    guard = cfg.sd_guard_px if cfg.secondary == abi.DEPTH_STOCHASTIC else 0
    abi.check(abi.lib().rsd_svao_make_vao_data(cfg.fb_w, cfg.fb_h, cfg.divisor, guard, cfg.radius,
                                               cfg.exponent, cfg.thickness, C.byref(vao), C.byref(w), C.byref(h)),
              "rsd_svao_make_vao_data")
    return vao, w.value, h.value


def sd_params(cfg: FrameConfig, sd_guard: int) -> abi.SDParams:
    # SVAO::compile builds the nested SD pass with these Properties (SVAO.cpp:158-183)
    return abi.SDParams(cfg.sd_samples, cfg.implementation, cfg.max_count, sd_guard, int(cfg.jitter), 1,
                        int(cfg.ray_interval), cfg.cull_mode, int(cfg.alpha_test), float(np.float32(1.5 / cfg.sd_samples)),
                        int(cfg.hit_order), int(cfg.use_16bit))


def svao_params(cfg: FrameConfig) -> abi.SVAOParams:
    if cfg.numerics not in abi.NUMERICS:
        raise ValueError(f"numerics must be one of {sorted(abi.NUMERICS)}, not {cfg.numerics!r}")
    if cfg.ao_kernel not in abi.AO_KERNELS:
        raise ValueError(f"ao_kernel must be one of {sorted(abi.AO_KERNELS)}, not {cfg.ao_kernel!r}")
    return abi.SVAOParams(cfg.num_directions, cfg.sd_samples, cfg.secondary, int(cfg.ray_interval), int(cfg.jitter),
                          cfg.guard_band, int(cfg.dual_ao), None, abi.NUMERICS[cfg.numerics],
                          abi.AO_KERNELS[cfg.ao_kernel], cfg.primary, None)


class Device:
    def __init__(self, index: int = 0):
        h = C.c_void_p()
        abi.check(abi.lib().rsd_device_open(index, C.byref(h)), "rsd_device_open")
        self.h = h
        self.index = index

    def close(self):
        if self.h:
            abi.lib().rsd_device_close(self.h)
            self.h = None


def alpha_desc(a):
    """rsd_alpha_desc of a scenes.AlphaMaterials (and the objects it points into)."""
    mats = (abi.Material * len(a.thresholds))(*[abi.Material(float(t), float(al), int(x)) for t, al, x in
                                                 zip(a.thresholds, a.alphas, a.material_textures)])
    texs = [np.ascontiguousarray(t, np.uint8) for t in a.textures]
    tx = (abi.AlphaTexture * max(1, len(texs)))(*[abi.AlphaTexture(t.shape[1], t.shape[0], t.ctypes.data)
                                                  for t in texs])
    uv = np.ascontiguousarray(a.texcoords, np.float32)
    tm = np.ascontiguousarray(a.tri_material, np.uint32)
    d = abi.AlphaDesc(uv.ctypes.data, tm.ctypes.data, mats, len(mats), tx, len(texs))
    return d, (mats, texs, tx, uv, tm)


def host_bvh(scene: Scene):
    """librsd's BVH of `scene` built on the host without a GPU (rsd_bvh_build): the bytes
    rsd_scene_upload puts in HBM, as (float32 array, triangle-record offset in float4 units)."""
    desc = abi.SceneDesc(scene.positions.ctypes.data, scene.positions.shape[0], scene.indices.ctypes.data,
                         scene.indices.shape[0], scene.flags.ctypes.data)
    n, off = C.c_uint64(), C.c_uint32()
    abi.check(abi.lib().rsd_bvh_build(C.byref(desc), None, 0, C.byref(n), C.byref(off)), "rsd_bvh_build")
    buf = np.zeros(n.value // 4, np.float32)
    abi.check(abi.lib().rsd_bvh_build(C.byref(desc), buf.ctypes.data, n.value, C.byref(n), C.byref(off)),
              "rsd_bvh_build")
    return buf, off.value


class GpuScene:
    def __init__(self, dev: Device, scene: Scene):
        desc = abi.SceneDesc(scene.positions.ctypes.data, scene.positions.shape[0], scene.indices.ctypes.data,
                             scene.indices.shape[0], scene.flags.ctypes.data)
        h = C.c_void_p()
        if scene.alpha is None:
            abi.check(abi.lib().rsd_scene_upload(dev.h, C.byref(desc), C.byref(h)), "rsd_scene_upload")
        else:
            ad, keep = alpha_desc(scene.alpha)
            abi.check(abi.lib().rsd_scene_upload_alpha(dev.h, C.byref(desc), C.byref(ad), C.byref(h)),
                      "rsd_scene_upload_alpha")
            del keep
        self.h = h
        self.info = abi.SceneInfo()
        abi.check(abi.lib().rsd_scene_info_get(h, C.byref(self.info)), "rsd_scene_info_get")

    def export_bvh(self):
        """The device BVH (rsd_scene_export_bvh): (float32 array of the whole allocation,
        triangle-record offset in float4 units) -- what the oracle's traversal-order walk reads."""
        n, off = C.c_uint64(), C.c_uint32()
        abi.check(abi.lib().rsd_scene_export_bvh(self.h, None, 0, C.byref(n), C.byref(off)), "rsd_scene_export_bvh")
        buf = np.zeros(n.value // 4, np.float32)
        abi.check(abi.lib().rsd_scene_export_bvh(self.h, buf.ctypes.data, n.value, C.byref(n), C.byref(off)),
                  "rsd_scene_export_bvh")
        return buf, off.value

    def release(self):
        if self.h:
            abi.lib().rsd_scene_release(self.h)
            self.h = None


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


_raw_stream = None  # torch._C._cuda_getCurrentRawStream (set by the first Renderer)


class Renderer:
    """Owns the frame buffers of one config on one GPU and runs the hot path."""

    def __init__(self, scene: Scene, cfg: FrameConfig, device: int = 0, gpu_scene: GpuScene | None = None,
                 dev: Device | None = None):
        import torch
        global _raw_stream
        self.torch = torch
        if _raw_stream is None:
            _raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        self.cfg = cfg
        self.scene = scene
        self.dev = dev or Device(device)
        torch.cuda.set_device(self.dev.index)
        self.gscene = gpu_scene or GpuScene(self.dev, scene)
        self.cam = make_camera(scene, cfg)
        self.vao, self.sd_w, self.sd_h = make_vao(cfg)
        self.sdp = sd_params(cfg, self.vao.sdGuard)
        self.svp = svao_params(cfg)
        W, H, N = cfg.fb_w, cfg.fb_h, cfg.sd_samples
        dv = torch.device("cuda", self.dev.index)
        self.depth = torch.empty((H, W), dtype=torch.float32, device=dv)
        self.normals = torch.empty((H, W), dtype=torch.int16, device=dv)
        # DualDepth primary mode: the second depth layer (gDepthTex2; DepthPeeling / TemporalDepthPeel in
        # the reference's graphs -- the caller fills it)
        self.depth2 = torch.zeros((H, W), dtype=torch.float32, device=dv) if cfg.primary == abi.DEPTH_DUAL else None
        # SVAO.cpp:307 clears on first use; dualAO: RG8Unorm (bright, dark)
        self.ao = torch.zeros((H, W, 2) if cfg.dual_ao else (H, W), dtype=torch.uint8, device=dv)
        # SVAO.cpp:132-134: R8Uint / R16Uint / R32Uint for 8 / 16 / 32 directions
        st_dtype = {8: torch.uint8, 16: torch.int16, 32: torch.int32}[cfg.num_directions]
        self.stencil = torch.zeros((H, W), dtype=st_dtype, device=dv)
        # rayMin / rayMax in one allocation: a sharded frame all-reduces both in one collective
        self.ray_minmax = torch.empty((2, self.sd_h, self.sd_w), dtype=torch.int32, device=dv)
        self.ray_min, self.ray_max = self.ray_minmax[0], self.ray_minmax[1]
        # Use16Bit (standalone SD pass): R16F / RG16F / RGBA16F
        # the tiled-layout A/B build (RSD_LIB_VARIANT=sdtiled) stores whole 8x8 tiles: pad the rows
        tiled = os.environ.get("RSD_LIB_VARIANT") == "sdtiled"
        sh, sw = ((self.sd_h + 7) // 8 * 8, (self.sd_w + 7) // 8 * 8) if tiled else (self.sd_h, self.sd_w)
        self.sd = torch.empty(((N + 3) // 4, sh, sw, min(N, 4)),
                              dtype=torch.float16 if cfg.use_16bit else torch.float32, device=dv)
        self._bind_tile_flags()

    def _bind_tile_flags(self):
        """Busy 16x16 tiles of this frame's stencil (rsd_svao_params.tile_flags, ABI v4): pass 1 sets
        them, pass 2 visits only flagged tiles and clears them.  One set per stencil buffer (frame slot)."""
        cfg = self.cfg
        n = abi.lib().rsd_svao_tile_count(cfg.fb_w, cfg.fb_h, cfg.guard_band)
        self.tile_flags = self.torch.zeros(max(1, n), dtype=self.torch.uint8, device=self.depth.device)
        # librsd's generation counter of this buffer is forgotten when the tensor is freed: the caching
        # allocator may hand the same address to the next (zeroed) flag buffer
        weakref.finalize(self.tile_flags, abi.lib().rsd_svao_tile_flags_release, self.tile_flags.data_ptr())
        svp = abi.SVAOParams.from_buffer_copy(self.svp)
        # RSD_TILE_FLAGS=off: no flags (pass 2 visits every tile) -- A/B runs only
        svp.tile_flags = None if os.environ.get("RSD_TILE_FLAGS") == "off" else self.tile_flags.data_ptr()
        svp.d_depth2 = self.depth2.data_ptr() if self.depth2 is not None else None
        self.svp = svp

    def keep_clean_tiles(self, on: bool = True):
        """Clean tiles (rsd_sd_params.d_tile_state): librsd's traces of this renderer's SD map skip rewriting the
        8x8 tiles they left at DEFAULT_DEPTH and that have no live ray -- the same bits, a fraction of the
        full-resolution maps' stores.  The map is then librsd's between traces: whoever writes it (or swaps it)
        calls invalidate_sd_tiles().  A frame slot of this renderer gets a stamp buffer of its own."""
        t = self.torch
        sdp = abi.SDParams.from_buffer_copy(self.sdp)
        if on:
            n = abi.lib().rsd_sd_tile_state_count(self.sd_w, self.sd_h)
            self.sd_tile_state = t.zeros(max(1, n), dtype=t.int32, device=self.depth.device)
            sdp.d_tile_state = self.sd_tile_state.data_ptr()
        else:
            self.sd_tile_state = None
            sdp.d_tile_state = None
        self.sdp = sdp

    def invalidate_sd_tiles(self):
        """The SD map was written outside librsd's traces: forget which tiles hold DEFAULT_DEPTH."""
        if getattr(self, "sd_tile_state", None) is not None:
            self.sd_tile_state.zero_()

    def frame_slot(self, own_gbuffer: bool = False) -> "Renderer":
        """Another set of per-frame buffers (ao, stencil, intervals, SD map) over the same scene,
        camera and G-buffer: the state of one more frame in flight.  Frames of different slots
        may run concurrently on different streams -- librsd keeps the SD-trace workspace per
        (scene, stream) -- while frames of one slot stay ordered on its stream.
        own_gbuffer=True: the slot also gets its own camera and G-buffer (an animated camera:
        every frame in flight renders its own pose)."""
        import copy
        t = self.torch
        r = copy.copy(self)
        r._slot = True
        r._desc_key = None  # the slot's own buffers
        r.ao = t.zeros_like(self.ao)
        r.stencil = t.zeros_like(self.stencil)
        r.ray_minmax = t.empty_like(self.ray_minmax)
        r.ray_min, r.ray_max = r.ray_minmax[0], r.ray_minmax[1]
        r.sd = t.empty_like(self.sd)
        r._bind_tile_flags()
        if getattr(self, "sd_tile_state", None) is not None:
            r.keep_clean_tiles()
        if own_gbuffer:
            r.cam = abi.Camera.from_buffer_copy(self.cam)
            r.depth = t.empty_like(self.depth)
            r.normals = t.empty_like(self.normals)
            if self.depth2 is not None:
                r.depth2 = t.empty_like(self.depth2)
                r._bind_tile_flags()
        return r

    def set_pose(self, pos, target, up):
        """Move the camera (an animated camera path): the next gbuffer() / frame() render this
        pose.  librsd copies the camera into every launch's arguments, so frames already
        enqueued keep the pose they were issued with."""
        self.cam = look_at(pos, target, up, self.cfg)

    @property
    def stream(self):
        """torch's current HIP stream of this renderer's device, as the raw handle librsd takes.  (Through
        torch.cuda.current_stream() this cost 3.2 us per call on the GPU box -- a Python Stream object per
        call, ~30 calls per N > 1 frame; the raw accessor is torch's own, the one its code generators use.)"""
        if _raw_stream is not None:
            return _raw_stream(self.dev.index)
        return self.torch.cuda.current_stream().cuda_stream

    @property
    def sd_rays(self) -> int:
        return self.sd_w * self.sd_h

    def gbuffer(self):
        abi.check(abi.lib().rsd_gbuffer(self.gscene.h, C.byref(self.cam), self.cfg.fb_w, self.cfg.fb_h,
                                        self.cfg.cull_mode, _ptr(self.depth), _ptr(self.normals), self.stream),
                  "rsd_gbuffer")

    def clear_intervals(self):
        abi.check(abi.lib().rsd_svao_clear_intervals(_ptr(self.ray_min), _ptr(self.ray_max), self.sd_w * self.sd_h,
                                                     self.stream), "rsd_svao_clear_intervals")

    def pass1(self, band=(0, 1)):
        abi.check(abi.lib().rsd_svao_pass1_band(C.byref(self.cam), C.byref(self.vao), C.byref(self.svp),
                                                _ptr(self.depth), _ptr(self.normals), self.cfg.fb_w, self.cfg.fb_h,
                                                _ptr(self.ao), _ptr(self.stencil), _ptr(self.ray_min),
                                                _ptr(self.ray_max), self.sd_w, self.sd_h, band[0], band[1],
                                                self.stream), "rsd_svao_pass1_band")

    # the trace can reset the interval maps for the next frame (rsd_sd_trace_band_ex)
    can_consume_intervals = True

    def sd_trace(self, counters: bool = False, band=(0, 1), consume: bool = False, throughput: bool = False):
        """consume=True: the trace also resets every interval texel (the next pass 1 needs no
        clear_intervals); needs RayInterval.  throughput=True: the trace overlaps other frames
        (RSD_SD_THROUGHPUT: the work-efficient traversal; same bits)."""
        cnt = abi.Counters() if counters else None
        flags = (abi.SD_CONSUME_INTERVALS if consume else 0) | (abi.SD_THROUGHPUT if throughput else 0)
        abi.check(abi.lib().rsd_sd_trace_band_ex(self.gscene.h, C.byref(self.cam), C.byref(self.sdp),
                                                 _ptr(self.depth), self.cfg.fb_w, self.cfg.fb_h, _ptr(self.ray_min),
                                                 _ptr(self.ray_max), _ptr(self.sd), self.sd_w, self.sd_h, band[0],
                                                 band[1], flags, C.byref(cnt) if cnt is not None else None,
                                                 self.stream), "rsd_sd_trace_band_ex")
        return cnt

    def pass2(self, band=(0, 1)):
        if self.cfg.use_16bit:  # SVAO never sets Use16Bit on its SD pass (SVAO.cpp:158-183)
            raise ValueError("SVAO pass 2 reads 32-bit SD maps; Use16Bit is a standalone SD-pass property")
        abi.check(abi.lib().rsd_svao_pass2_band(C.byref(self.cam), C.byref(self.vao), C.byref(self.svp),
                                                _ptr(self.depth), _ptr(self.normals), self.cfg.fb_w, self.cfg.fb_h,
                                                _ptr(self.stencil), _ptr(self.sd), self.sd_w, self.sd_h,
                                                _ptr(self.ao), band[0], band[1], self.stream), "rsd_svao_pass2_band")

    # ---- contiguous screen bands (rsd/shard.py HaloFrame): visible rows / SD rows [row0, row1)
    def pass1_rows(self, rows):
        abi.check(abi.lib().rsd_svao_pass1_rows(C.byref(self.cam), C.byref(self.vao), C.byref(self.svp),
                                                _ptr(self.depth), _ptr(self.normals), self.cfg.fb_w, self.cfg.fb_h,
                                                _ptr(self.ao), _ptr(self.stencil), _ptr(self.ray_min),
                                                _ptr(self.ray_max), self.sd_w, self.sd_h, rows[0], rows[1],
                                                self.stream), "rsd_svao_pass1_rows")

    def sd_trace_rows(self, rows, consume: bool = False, throughput: bool = False, counters: bool = False):
        cnt = abi.Counters() if counters else None
        flags = (abi.SD_CONSUME_INTERVALS if consume else 0) | (abi.SD_THROUGHPUT if throughput else 0)
        abi.check(abi.lib().rsd_sd_trace_rows(self.gscene.h, C.byref(self.cam), C.byref(self.sdp), _ptr(self.depth),
                                              self.cfg.fb_w, self.cfg.fb_h, _ptr(self.ray_min), _ptr(self.ray_max),
                                              _ptr(self.sd), self.sd_w, self.sd_h, rows[0], rows[1], flags,
                                              C.byref(cnt) if cnt is not None else None, self.stream),
                  "rsd_sd_trace_rows")
        return cnt

    def pass2_rows(self, rows):
        if self.cfg.use_16bit:
            raise ValueError("SVAO pass 2 reads 32-bit SD maps; Use16Bit is a standalone SD-pass property")
        abi.check(abi.lib().rsd_svao_pass2_rows(C.byref(self.cam), C.byref(self.vao), C.byref(self.svp),
                                                _ptr(self.depth), _ptr(self.normals), self.cfg.fb_w, self.cfg.fb_h,
                                                _ptr(self.stencil), _ptr(self.sd), self.sd_w, self.sd_h,
                                                _ptr(self.ao), rows[0], rows[1], self.stream), "rsd_svao_pass2_rows")

    def pass2_raytraced(self, band=(0, 1)):
        abi.check(abi.lib().rsd_svao_pass2_raytraced_band(self.gscene.h, C.byref(self.cam), C.byref(self.vao),
                                                          C.byref(self.svp), _ptr(self.depth), _ptr(self.normals),
                                                          self.cfg.fb_w, self.cfg.fb_h, _ptr(self.stencil),
                                                          _ptr(self.ao), self.cfg.cull_mode, int(self.cfg.ray_pipeline),
                                                          int(self.cfg.alpha_test), band[0], band[1], self.stream),
                  "rsd_svao_pass2_raytraced_band")

    def _frame_desc(self):
        """The rsd_svao_frame_desc of this renderer's buffers (cached; rebuilt when the camera or the
        parameter structs are replaced, e.g. by set_pose)."""
        # the key holds the structs themselves (compared with `is`: a held object's id cannot be reused by a
        # new one, as a freed Camera's could) and the buffers' device addresses (a reassigned tensor)
        objs = (self.cam, self.svp, self.sdp, self.vao, self.gscene)
        ptrs = tuple(t.data_ptr() for t in (self.depth, self.normals, self.ao, self.stencil, self.ray_minmax, self.sd))
        key = getattr(self, "_desc_key", None)
        if key is None or key[1] != ptrs or any(a is not b for a, b in zip(key[0], objs)):
            key = (objs, ptrs)
            cfg = self.cfg
            p = lambda t: t.data_ptr()  # noqa: E731
            self._desc = abi.FrameDesc(self.gscene.h, C.addressof(self.cam), C.addressof(self.vao),
                                       C.addressof(self.svp), C.addressof(self.sdp), p(self.depth), p(self.normals),
                                       cfg.fb_w, cfg.fb_h, p(self.ao), p(self.stencil), p(self.ray_min),
                                       p(self.ray_max), p(self.sd), self.sd_w, self.sd_h, int(cfg.ray_pipeline))
            self._desc_key = key
            self._events = (C.c_void_p * 4)()
        return self._desc

    def svao_frame(self, intervals_clear: bool = False, keep_intervals: bool = False, throughput: bool = False,
                   events=None):
        """One AO frame in ONE librsd call (rsd_svao_frame: clear -> "AO 1" -> SD trace -> "AO 2" issued
        from C++ on the current stream).  intervals_clear: the interval maps are known to be cleared
        (the previous trace consumed them), so no clear launch; keep_intervals: the trace does not
        consume them; events: None or 4 TimingEvents / None recorded before pass 1, before and after
        the SD trace and after pass 2."""
        d = self._frame_desc()
        flags = ((abi.FRAME_INTERVALS_CLEAR if intervals_clear else 0) |
                 (abi.FRAME_KEEP_INTERVALS if keep_intervals else 0) | (abi.SD_THROUGHPUT if throughput else 0))
        ev = None
        if events is not None:
            ev = self._events
            for i, e in enumerate(events):
                ev[i] = e.h.value if e is not None else None
        abi.check(abi.lib().rsd_svao_frame(C.byref(d), flags, ev, self.stream), "rsd_svao_frame")

    def frame(self):
        """One AO frame: the span of the reference's "AO 1" + "AORefine" profile scopes
        (SVAO.cpp:327-455) for the configured secondary depth mode, in one librsd call; the interval
        maps keep what pass 1 wrote (tests read them)."""
        self.svao_frame(keep_intervals=True)

    def numpy(self):
        t = self.torch
        t.cuda.synchronize()
        return dict(depth=self.depth.cpu().numpy(), normals=self.normals.cpu().numpy().view(np.uint16),
                    ao=self.ao.cpu().numpy(), stencil=self.stencil.cpu().numpy().view({1: np.uint8, 2: np.uint16, 4: np.uint32}[self.stencil.element_size()]),
                    ray_min=self.ray_min.cpu().numpy().view(np.uint32),
                    ray_max=self.ray_max.cpu().numpy().view(np.uint32), sd=self.sd.cpu().numpy())

    def close(self):
        if not getattr(self, "_slot", False):  # a frame slot shares the scene of its renderer
            self.gscene.release()
