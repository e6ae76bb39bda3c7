"""TemporalAO (enabled), TAA and the G-buffer's motion vectors on the GPU (librsd rsd_temporal_ao /
rsd_taa / rsd_motion_vectors, include/rsd_graph.h) -- the temporal passes of the reference's AO
chain (scripts/SVAO.py: SVAO -> CrossBilateralBlur -> TemporalAO -> Switch -> ImageEquation -> TAA).

TemporalAO mirrors Source/RenderPasses/TemporalAO/TemporalAO.cpp: properties `enabled` and
`useStableMask` (:42-43), previous-frame depth / AO / history textures (re)allocated on the first
enabled frame and reset when disabled (:128-140), prevViewToCurView = viewMat * inverse(prevViewMat)
(:156), and the end-of-frame copies into the history textures (:165-168)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi

MAX_HISTORY = 30  # TemporalAO.ps.slang:94


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def view_matrix(cam: abi.Camera) -> np.ndarray:
    return np.array(cam.viewMat, np.float64).reshape(4, 4)


def prev_view_to_cur_view(cam: abi.Camera, prev_cam: abi.Camera) -> np.ndarray:
    """viewMat * inverse(prevViewMat) (TemporalAO.cpp:156), row-major float32.  The view matrix is
    rigid (Falcor matrixFromLookAt), so the inverse is its transposed rotation; evaluated in
    float64 and rounded once."""
    p = view_matrix(prev_cam)
    inv = np.eye(4)
    inv[:3, :3] = p[:3, :3].T
    inv[:3, 3] = -p[:3, :3].T @ p[:3, 3]
    return (view_matrix(cam) @ inv).astype(np.float32)


def motion_vectors(cam: abi.Camera, prev_cam: abi.Camera, linear_z, out=None, stream=None):
    """GBufferRaster.mvec (RG32F, H x W x 2) of a static scene seen from `cam` after `prev_cam`."""
    import torch
    H, W = linear_z.shape
    if out is None:
        out = torch.empty((H, W, 2), dtype=torch.float32, device=linear_z.device)
    assert out.shape == (H, W, 2) and out.dtype == torch.float32 and linear_z.dtype == torch.float32
    s = stream if stream is not None else C.c_void_p(torch.cuda.current_stream().cuda_stream)
    abi.check(abi.lib().rsd_motion_vectors(C.byref(cam), C.byref(prev_cam), _ptr(linear_z), W, H, _ptr(out), s),
              "rsd_motion_vectors")
    return out


class TemporalAO:
    """One TemporalAO pass instance: keeps the previous frame's depth, AO and history count."""

    def __init__(self, enabled: bool = True, use_stable_mask: bool = False):
        self.enabled = enabled
        self.use_stable_mask = use_stable_mask
        self.prev_depth = self.prev_ao = self.prev_history = None
        self.history = None  # the pass's internal R8Uint history-count target

    def reset(self):
        """TemporalAO::compile (:105-111): a fresh image after settings changed."""
        self.prev_depth = self.prev_ao = self.prev_history = None

    def _alloc(self, like, dtype):
        import torch
        return torch.zeros(like.shape[:2], dtype=dtype, device=like.device)

    def execute(self, ao_in, linear_z, mvec, cam: abi.Camera, prev_cam: abi.Camera, guard_band: int = 0,
                ao_out=None, stable_mask=None):
        """ao_in: R8Unorm (H, W) uint8; linear_z: (H, W) float32; mvec: (H, W, 2) float32.
        Returns ao_out (allocated when None; pixels outside the guard band keep its values)."""
        import torch
        H, W = ao_in.shape
        if ao_out is None:
            ao_out = torch.zeros_like(ao_in)
        if not self.enabled:  # :128-135 blit, drop the history
            ao_out.copy_(ao_in)
            self.reset()
            return ao_out
        for t, dt, shp in ((ao_in, torch.uint8, (H, W)), (linear_z, torch.float32, (H, W)),
                           (mvec, torch.float32, (H, W, 2)), (ao_out, torch.uint8, (H, W))):
            if t.dtype != dt or tuple(t.shape) != shp or not t.is_contiguous() or t.device != ao_in.device:
                raise ValueError(f"TemporalAO: expected a contiguous {dt} {shp} tensor, got {t.dtype} {tuple(t.shape)}")
        if self.prev_depth is None or tuple(self.prev_depth.shape) != (H, W):  # allocatePrevFrameTexture
            self.prev_depth = self._alloc(ao_in, torch.float32)
            self.prev_ao = self._alloc(ao_in, torch.uint8)
            self.prev_history = self._alloc(ao_in, torch.uint8)
            self.history = self._alloc(ao_in, torch.uint8)
        mask = stable_mask if (stable_mask is not None and self.use_stable_mask) else None
        m = np.ascontiguousarray(prev_view_to_cur_view(cam, prev_cam), np.float32)
        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        abi.check(abi.lib().rsd_temporal_ao(_ptr(ao_in), _ptr(linear_z), _ptr(mvec), _ptr(self.prev_depth),
                                            _ptr(self.prev_ao), _ptr(self.prev_history), _ptr(mask), W, H, guard_band,
                                            C.byref(cam), m.ctypes.data_as(C.c_void_p), _ptr(ao_out),
                                            _ptr(self.history), s), "rsd_temporal_ao")
        # :165-168 save depth, AO and history for the next frame
        self.prev_depth.copy_(linear_z)
        self.prev_ao.copy_(ao_out)
        self.prev_history.copy_(self.history)
        return ao_out


class TAA:
    """One TAA pass instance (TAA.cpp): keeps the previous output; properties `alpha`,
    `colorBoxSigma`, `antiFlicker` with TAA.h's defaults."""

    def __init__(self, alpha: float = 0.1, color_box_sigma: float = 1.0, anti_flicker: bool = True):
        self.alpha, self.color_box_sigma, self.anti_flicker = alpha, color_box_sigma, anti_flicker
        self.prev = None

    def execute(self, color_in, motion_vecs, color_out=None):
        """color_in: (H, W, 4) float32; motion_vecs: (H, W, 2) float32.  Returns color_out."""
        import torch
        H, W = color_in.shape[:2]
        for t, shp in ((color_in, (H, W, 4)), (motion_vecs, (H, W, 2))):
            if t.dtype != torch.float32 or tuple(t.shape) != shp or not t.is_contiguous():
                raise ValueError(f"TAA: expected a contiguous float32 {shp} tensor, got {t.dtype} {tuple(t.shape)}")
        if color_out is None:
            color_out = torch.empty_like(color_in)
        if self.prev is None or tuple(self.prev.shape) != (H, W, 4):  # allocatePrevColor
            self.prev = torch.zeros_like(color_in)
        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        abi.check(abi.lib().rsd_taa(_ptr(color_in), _ptr(motion_vecs), _ptr(self.prev), W, H, self.alpha,
                                    self.color_box_sigma, int(bool(self.anti_flicker)), _ptr(color_out), s), "rsd_taa")
        self.prev.copy_(color_out)  # TAA.cpp:123
        return color_out
