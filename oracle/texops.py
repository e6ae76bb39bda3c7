"""Texture shuffles of the reference's AO graphs, restated in numpy (test infrastructure only).

DeinterleaveTexture (Source/RenderPasses/DeinterleaveTexture/Deinterleave.slang:26-45,
DeinterleaveTexture.cpp:143-158): layer s = dy * 4 + dx of the ceil(H/4) x ceil(W/4) x 16 output
holds src[4y + dy][4x + dx]; `Load` outside the source reads 0.  InterleaveTexture
(Source/RenderPasses/InterleaveTexture/Interleave.slang:7-15): out[y][x] = src[(y % 4) * 4 + x % 4]
[y / 4][x / 4].  Texels are opaque byte strings (the shader's `type` define follows the format).

RayMinMaxLength (Source/RenderPasses/RayMinMaxLength/RayMinMaxLength.ps.slang:4-16): 0 where the
raw rayMax word is 0, else max(0, asfloat(rayMax) - asfloat(rayMin)) / 32 with HLSL max returning
the non-NaN operand."""
import numpy as np


def deinterleave(src):
    """src: (H, W) or (H, W, C) array -> (16, ceil(H/4), ceil(W/4)[, C])."""
    H, W = src.shape[:2]
    h4, w4 = (H + 3) // 4, (W + 3) // 4
    pad = np.zeros((4 * h4, 4 * w4) + src.shape[2:], src.dtype)
    pad[:H, :W] = src
    out = np.empty((16, h4, w4) + src.shape[2:], src.dtype)
    for s in range(16):
        out[s] = pad[s // 4::4, s % 4::4]
    return out


def interleave(layers, H, W):
    """layers: (16, ceil(H/4), ceil(W/4)[, C]) -> (H, W[, C])."""
    y, x = np.mgrid[0:H, 0:W]
    return layers[(y % 4) * 4 + x % 4, y // 4, x // 4]


def ray_min_max_length(ray_min, ray_max):
    """ray_min, ray_max: uint32 interval maps (float bit patterns) -> float32 lengths."""
    mn = np.asarray(ray_min, np.uint32).view(np.float32)
    mx = np.asarray(ray_max, np.uint32)
    with np.errstate(invalid="ignore", over="ignore"):
        d = mx.view(np.float32) - mn
    d = np.where(np.isnan(d) | (d < 0), np.float32(0), d).astype(np.float32)  # max(0, d), NaN -> 0
    return np.where(mx == 0, np.float32(0), d / np.float32(32)).astype(np.float32)
