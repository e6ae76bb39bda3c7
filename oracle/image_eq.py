"""CPU oracle of ImageEquation (TEST INFRASTRUCTURE ONLY: tests/ import it as the checker).

Reference: ImageEquation.ps.slang:8-13 evaluates `float4 result = (FORMULA)` per pixel over
Texture2D<float4> I0..I3 read at int2 xy (ImageEquation.cpp:134-160).  This is an independent
restatement of librsd's definition (csrc/image_eq.h): a recursive-descent evaluator over whole
images as numpy float32 arrays [H, W, 4] (numpy float32 arithmetic rounds each operation like
the device with -ffp-contract=off); exp/log/sin/cos/pow/rsqrt in float64, rounded once; a
scalar is broadcast in all four lanes; two vectors of different widths truncate to the smaller.
"""
import re

import numpy as np

F = np.float32
FMT_R32F, FMT_RG32F, FMT_RGBA32F, FMT_R16U, FMT_R8U, FMT_R8UNORM, FMT_R32U = range(7)


def texel_view(img, fmt, W, H):
    """Texture2D<float4> reads of a whole image, [H, W, 4], zero outside the image / unbound."""
    out = np.zeros((H, W, 4), F)
    if img is None:
        return out
    h, w = img.shape[:2]
    hh, ww = min(h, H), min(w, W)
    v = np.zeros((hh, ww, 4), F)
    v[..., 3] = 1.0
    a = img[:hh, :ww]
    if fmt == FMT_R32F:
        v[..., 0] = a
    elif fmt == FMT_RG32F:
        v[..., :2] = a
    elif fmt == FMT_RGBA32F:
        v[...] = a
    elif fmt == FMT_R8UNORM:
        v[..., 0] = a.astype(F) / F(255.0)
    else:  # integer formats
        v[..., 0] = a.astype(F)
    out[:hh, :ww] = v
    return out


class _Val:
    def __init__(self, a, w):
        self.a, self.w = a, w  # a: [H, W, 4] float32, w: width


def _bw(a, b):
    return b if a == 1 else a if b == 1 else min(a, b)


def _d(f, x):
    return f(x.astype(np.float64)).astype(F)


_F1 = {
    "abs": np.abs, "saturate": lambda x: np.where(x > 0, np.minimum(x, F(1)), F(0)).astype(F),
    "sqrt": np.sqrt, "floor": np.floor, "ceil": np.ceil, "frac": lambda x: x - np.floor(x),
    "exp2": lambda x: _d(np.exp2, x), "log2": lambda x: _d(np.log2, x), "exp": lambda x: _d(np.exp, x),
    "log": lambda x: _d(np.log, x), "sin": lambda x: _d(np.sin, x), "cos": lambda x: _d(np.cos, x),
    "rsqrt": lambda x: (1.0 / np.sqrt(x.astype(np.float64))).astype(F),
    "sign": lambda x: np.where(x > 0, F(1), np.where(x < 0, F(-1), F(0))).astype(F),
}


def _pow(a, b):
    return np.where(b == F(2), a * a, np.power(a.astype(np.float64), b.astype(np.float64)).astype(F)).astype(F)


_F2 = {"min": np.fmin, "max": np.fmax, "pow": _pow,
       "step": lambda a, b: np.where(b >= a, F(1), F(0)).astype(F)}


def evaluate(formula, inputs, W, H):
    """inputs: list of 4 (image or None, fmt).  Returns the float4 result [H, W, 4].

    Arithmetic is IEEE binary32 with the special values HLSL / D3D11 define for it: x / +-0 =
    +-inf (sign of x times sign of 0), 0 / 0 = inf / inf = inf - inf = 0 * inf = NaN -- numpy's
    float32 results, with its floating-point warnings silenced (they are not errors here)."""
    with np.errstate(divide="ignore", invalid="ignore", over="ignore", under="ignore"):
        return _evaluate(formula, inputs, W, H)


def _evaluate(formula, inputs, W, H):
    toks = re.findall(r"\d+\.\d*(?:[eE][-+]?\d+)?[fFhH]?|\.\d+(?:[eE][-+]?\d+)?[fFhH]?|\d+(?:[eE][-+]?\d+)?[fFhH]?"
                      r"|[A-Za-z_]\w*|[-+*/().,\[\]]", formula)
    pos = [0]

    def peek():
        return toks[pos[0]] if pos[0] < len(toks) else None

    def take(t=None):
        tok = peek()
        if t is not None and tok != t:
            raise ValueError(f"expected {t!r}, got {tok!r}")
        pos[0] += 1
        return tok

    def bc(x):  # broadcast lane 0
        return np.repeat(x[..., :1], 4, axis=-1)

    def expr():
        v = term()
        while peek() in ("+", "-"):
            op = take()
            r = term()
            v = _Val(v.a + r.a if op == "+" else v.a - r.a, _bw(v.w, r.w))
        return v

    def term():
        v = unary()
        while peek() in ("*", "/"):
            op = take()
            r = unary()
            v = _Val(v.a * r.a if op == "*" else v.a / r.a, _bw(v.w, r.w))
        return v

    def unary():
        if peek() == "-":
            take()
            v = unary()
            return _Val(-v.a, v.w)
        if peek() == "+":
            take()
            return unary()
        return postfix()

    def postfix():
        v = primary()
        while peek() == ".":
            take()
            sw = take()
            idx = ["xyzw".index(c) if c in "xyzw" else "rgba".index(c) for c in sw]
            if max(idx) >= v.w:
                raise ValueError("swizzle past width")
            lanes = idx + [idx[0]] * (4 - len(idx))
            v = _Val(v.a[..., lanes], len(sw))
        return v

    def primary():
        t = take()
        if re.match(r"[\d.]", t):
            c = F(float(t.rstrip("fFhH")))
            return _Val(np.full((H, W, 4), c, F), 1)
        if t == "(":
            v = expr()
            take(")")
            return v
        m = re.fullmatch(r"I([0-3])", t)
        if m:
            take("[")
            take("xy")
            take("]")
            img, fmt = inputs[int(m.group(1))]
            return _Val(texel_view(img, fmt, W, H), 4)
        take("(")
        args = [expr()]
        while peek() == ",":
            take()
            args.append(expr())
        take(")")
        if t in ("float", "float2", "float3", "float4"):
            n = {"float": 1, "float2": 2, "float3": 3, "float4": 4}[t]
            if len(args) == 1 and args[0].w == 1:
                return _Val(bc(args[0].a), n)
            lanes = np.concatenate([a.a[..., :a.w] for a in args], -1)
            out = np.zeros((H, W, 4), F)
            out[..., :lanes.shape[-1]] = lanes[..., :4]
            return _Val(out, n)
        if t in _F1:
            return _Val(_F1[t](args[0].a).astype(F), args[0].w)
        if t in _F2:
            return _Val(_F2[t](args[0].a, args[1].a).astype(F), _bw(args[0].w, args[1].w))
        if t == "dot":
            w = _bw(args[0].w, args[1].w)
            p = args[0].a * args[1].a
            d = p[..., 0]
            for k in range(1, w):
                d = d + p[..., k]
            return _Val(np.repeat(d[..., None], 4, -1), 1)
        if t == "lerp":
            a, b, s = (x.a for x in args)
            return _Val(a + s * (b - a), _bw(_bw(args[0].w, args[1].w), args[2].w))
        if t == "clamp":
            a, lo, hi = (x.a for x in args)
            return _Val(np.fmin(np.fmax(a, lo), hi), _bw(_bw(args[0].w, args[1].w), args[2].w))
        raise ValueError(f"unknown identifier {t!r}")

    v = expr()
    if pos[0] != len(toks):
        raise ValueError("trailing tokens")
    if v.w not in (1, 4):
        raise ValueError("result must be a scalar or float4")
    return v.a


def store(result, fmt):
    """The render-target write of the result in `fmt`."""
    if fmt == FMT_RGBA32F:
        return result
    if fmt == FMT_RG32F:
        return np.ascontiguousarray(result[..., :2])
    if fmt == FMT_R32F:
        return np.ascontiguousarray(result[..., 0])
    x = result[..., 0]
    x = np.where(np.isnan(x), F(0), x)
    x = np.where(x > 0, np.minimum(x, F(1)), F(0)).astype(F)
    return np.floor(x * F(255.0) + F(0.5)).astype(np.uint8)
