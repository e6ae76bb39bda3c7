// post.hip -- the image passes after SVAO in the reference's graph scripts:
// CrossBilateralBlur and ImageEquation.  Both are HBM-bound streaming kernels over the
// frame; one lane per pixel, 64 x 4 workgroups so every wave reads whole cache lines.
//
// CrossBilateralBlur (RenderPasses/CrossBilateralBlur/CrossBilateralBlur.ps.slang:1-88,
// CrossBilateralBlur.cpp:113-149): separable depth-aware blur, x then y through a ping-pong
// R8Unorm image, KERNEL_RADIUS taps each side with the HBAO+ weights
//   w(d) = exp2(-d^2 falloff - dz^2),  dz = 12 * 16 |z_d - d * slope - z_0| / z_0,
// point sampling at texC + d * dir / size clamped to the guard band's [uvMin, uvMax]
// (GuardBand.cpp:62-63), writes limited to the guard-band scissor (GuardBand.h:4-15).
// Numerics: rsd_device.h contract; exp2 evaluated in double and rounded once.
//
// ImageEquation (ImageEquation.ps.slang:8-13): the formula program of csrc/image_eq.h run
// per pixel; I<k>[xy] reads Texture2D<float4> semantics (missing channels 0, alpha 1;
// unbound or out of range: 0).
#include <cmath>

#include "../../include/rsd_graph.h"
#include "image_eq.h"
#include "rsd_device.h"
#include "rsd_internal.h"

struct rsd_image_program;

namespace rsd {
const IeProgram& image_program(const rsd_image_program* p);

namespace {

constexpr int kPostW = 64, kPostH = 4;

// ---------------------------------------------------------------------- CrossBilateralBlur
struct BlurArgs {
    const uint8_t* src;
    const float* z;
    uint8_t* dst;
    int W, H, g;
    float dirX, dirY;
    float uvMinX, uvMinY, uvMaxX, uvMaxY;
    int zW, zH;
    uint32_t betterSlope;
};

__device__ __forceinline__ int point_texel(float uv, int n) {
    int t = (int)floorf(uv * (float)n);
    return t < 0 ? 0 : (t > n - 1 ? n - 1 : t);
}

template <int R>
__global__ void __launch_bounds__(kPostW * kPostH) blur_kernel(BlurArgs a) {
    const int x = a.g + (int)(blockIdx.x * kPostW + threadIdx.x);
    const int y = a.g + (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= a.W - a.g || y >= a.H - a.g) return;  // guard-band scissor
    const float tcx = ((float)x + 0.5f) / (float)a.W, tcy = ((float)y + 0.5f) / (float)a.H;
    const float dux = (1.0f / (float)a.W) * a.dirX, duy = (1.0f / (float)a.H) * a.dirY;
    float dc[2 * R + 1], ac[2 * R + 1];
#pragma unroll
    for (int d = -R; d <= R; ++d) {
        const float u = fminf(fmaxf(tcx + (float)d * dux, a.uvMinX), a.uvMaxX);
        const float v = fminf(fmaxf(tcy + (float)d * duy, a.uvMinY), a.uvMaxY);
        dc[R + d] = a.z[(size_t)point_texel(v, a.zH) * a.zW + point_texel(u, a.zW)];
        ac[R + d] = unorm8_to_float(a.src[(size_t)point_texel(v, a.H) * a.W + point_texel(u, a.W)]);
    }
    const float sigma = ((float)R + 1.0f) * 0.5f;
    const float falloff = 1.0f / (2.0f * sigma * sigma);
    float ao = ac[R], wsum = 1.0f;
    const float sl = dc[R] - dc[R - 1], sr = dc[R + 1] - dc[R];
    const float minSlope = fabsf(sl) < fabsf(sr) ? sl : sr;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        const int sign = side == 0 ? 1 : -1;
        float slope = side == 0 ? minSlope : -minSlope;
#pragma unroll
        for (int d = 1; d <= R; ++d) {
            const float sAo = ac[R + sign * d];
            float sZ = dc[R + sign * d];
            if (d == 1 && !a.betterSlope) slope = sZ - dc[R];
            sZ -= slope * (float)d;
            float dz = fabsf(sZ - dc[R]) * 16.0f;
            dz = dz * 12.0f / dc[R];
            const float w = (float)exp2((double)(-(float)(d * d) * falloff - dz * dz));
            ao += w * sAo;
            wsum += w;
        }
    }
    a.dst[(size_t)y * a.W + x] = unorm8(ao / wsum);
}

template <int R>
hipError_t launch_blur(const BlurArgs& a, hipStream_t s) {
    const dim3 grid((a.W - 2 * a.g + kPostW - 1) / kPostW, (a.H - 2 * a.g + kPostH - 1) / kPostH);
    hipLaunchKernelGGL(blur_kernel<R>, grid, dim3(kPostW, kPostH), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------- TAA
// TAA.ps.slang:78-150 (TAA.cpp:99-124): YCgCo colour box of the 3x3 neighbourhood (Load: texels
// outside the image read 0), the longest motion vector of the 3x3, the history through the
// 9-tap Catmull-Rom filter (bilinear taps of gSampler: linear, wrap -- Falcor's default address
// mode; librsd's 8-bit sub-texel weights), anti-flicker blend factor, clamp, lerp.  HLSL
// lerp(x, y, s) = x + s * (y - x); clamp / min / max return the non-NaN operand.
struct TaaArgs {
    const float4* color;
    const float2* mvec;
    const float4* prev;
    float4* out;
    int W, H;
    float alpha, sigma;
    uint32_t antiFlicker;
    float invW, invH;  // 1.0 / texDim
};

__device__ __forceinline__ f3 rgb_to_ycgco(float4 c) {
    const float Y = c.x * 0.25f + c.y * 0.50f + c.z * 0.25f;
    const float Cg = c.x * -0.25f + c.y * 0.50f + c.z * -0.25f;
    const float Co = c.x * 0.50f + c.y * 0.00f + c.z * -0.50f;
    return mk(Y, Cg, Co);
}

__device__ __forceinline__ float4 taa_load(const float4* __restrict__ t, int W, int H, int x, int y) {
    if (x < 0 || y < 0 || x >= W || y >= H) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    return t[(size_t)y * W + x];
}

__device__ __forceinline__ int wrap_addr(int i, int n) {
    i %= n;
    return i < 0 ? i + n : i;
}

// bilinear RGB of an RGBA32F texture, wrap addressing, 8-bit sub-texel weights (all 4 taps)
__device__ __forceinline__ f3 taa_bilinear(const float4* __restrict__ t, int W, int H, float u, float v) {
    const float x = u * (float)W - 0.5f, y = v * (float)H - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    float qx = floorf((x - fx0) * 256.0f + 0.5f), qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) { ix += 1; qx = 0.0f; }
    if (qy >= 256.0f) { iy += 1; qy = 0.0f; }
    const float wx = qx * (1.0f / 256.0f), wy = qy * (1.0f / 256.0f);
    const int x0 = wrap_addr(ix, W), x1 = wrap_addr(ix + 1, W), y0 = wrap_addr(iy, H), y1 = wrap_addr(iy + 1, H);
    const float4 a = t[(size_t)y0 * W + x0], b = t[(size_t)y0 * W + x1];
    const float4 c = t[(size_t)y1 * W + x0], d = t[(size_t)y1 * W + x1];
    auto lerp2 = [&](float p, float q, float r, float s) {
        const float r0 = p * (1.0f - wx) + q * wx, r1 = r * (1.0f - wx) + s * wx;
        return r0 * (1.0f - wy) + r1 * wy;
    };
    return mk(lerp2(a.x, b.x, c.x, d.x), lerp2(a.y, b.y, c.y, d.y), lerp2(a.z, b.z, c.z, d.z));
}

__global__ void __launch_bounds__(kPostW * kPostH) taa_kernel(TaaArgs a) {
    const int x = (int)(blockIdx.x * kPostW + threadIdx.x), y = (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= a.W || y >= a.H) return;
    constexpr int ox[8] = {-1, -1, 1, 1, 1, 0, 0, -1}, oy[8] = {-1, 1, -1, 1, 0, -1, 1, 0};
    const float tu = ((float)x + 0.5f) / (float)a.W, tv = ((float)y + 0.5f) / (float)a.H;  // texC
    const f3 color = rgb_to_ycgco(a.color[(size_t)y * a.W + x]);
    f3 avg = color, var = mk(color.x * color.x, color.y * color.y, color.z * color.z);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const f3 c = rgb_to_ycgco(taa_load(a.color, a.W, a.H, x + ox[k], y + oy[k]));
        avg = mk(avg.x + c.x, avg.y + c.y, avg.z + c.z);
        var = mk(var.x + c.x * c.x, var.y + c.y * c.y, var.z + c.z * c.z);
    }
    const float nine = 1.0f / 9.0f;
    avg = mk(avg.x * nine, avg.y * nine, avg.z * nine);
    var = mk(var.x * nine, var.y * nine, var.z * nine);
    const f3 sg = mk(sqrtf(hmax(0.0f, var.x - avg.x * avg.x)), sqrtf(hmax(0.0f, var.y - avg.y * avg.y)),
                     sqrtf(hmax(0.0f, var.z - avg.z * avg.z)));
    const f3 cmin = mk(avg.x - a.sigma * sg.x, avg.y - a.sigma * sg.y, avg.z - a.sigma * sg.z);
    const f3 cmax = mk(avg.x + a.sigma * sg.x, avg.y + a.sigma * sg.y, avg.z + a.sigma * sg.z);
    float2 motion = a.mvec[(size_t)y * a.W + x];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int xx = x + ox[k], yy = y + oy[k];
        const float2 m = (xx < 0 || yy < 0 || xx >= a.W || yy >= a.H) ? make_float2(0.0f, 0.0f)
                                                                        : a.mvec[(size_t)yy * a.W + xx];
        if (m.x * m.x + m.y * m.y > motion.x * motion.x + motion.y * motion.y) motion = m;
    }
    // bicubicSampleCatmullRom((texC + motion) * texDim, texDim)
    const float spx = (tu + motion.x) * (float)a.W, spy = (tv + motion.y) * (float)a.H;
    const float tcx = floorf(spx - 0.5f) + 0.5f, tcy = floorf(spy - 0.5f) + 0.5f;
    float w0[2], w12[2], w3[2], c0[2], c12[2], c3[2];
    const float fv[2] = {spx - tcx, spy - tcy}, tcv[2] = {tcx, tcy}, inv[2] = {a.invW, a.invH};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float f = fv[k], f2 = f * f, f3v = f2 * f;
        const float q0 = f2 - 0.5f * (f3v + f);
        const float q1 = 1.5f * f3v - 2.5f * f2 + 1.0f;
        const float q3 = 0.5f * (f3v - f2);
        const float q2 = 1.0f - q0 - q1 - q3;
        w0[k] = q0;
        w12[k] = q1 + q2;
        w3[k] = q3;
        c0[k] = (tcv[k] - 1.0f) * inv[k];
        c12[k] = (tcv[k] + q2 / w12[k]) * inv[k];
        c3[k] = (tcv[k] + 2.0f) * inv[k];
    }
    const float xs[3] = {c0[0], c12[0], c3[0]}, ys[3] = {c0[1], c12[1], c3[1]};
    const float wxs[3] = {w0[0], w12[0], w3[0]}, wys[3] = {w0[1], w12[1], w3[1]};
    f3 h = mk(0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const f3 t = taa_bilinear(a.prev, a.W, a.H, xs[i], ys[j]);
            const float w = wxs[i] * wys[j];
            if (i == 0 && j == 0) h = mk(t.x * w, t.y * w, t.z * w);
            else h = mk(h.x + t.x * w, h.y + t.y * w, h.z + t.z * w);
        }
    f3 hist = rgb_to_ycgco(make_float4(h.x, h.y, h.z, 0.0f));
    float alpha = a.alpha;
    if (a.antiFlicker) {
        const float dist = hmin(fabsf(cmin.x - hist.x), fabsf(cmax.x - hist.x));
        alpha = hmin(hmax((a.alpha * dist) / (dist + cmax.x - cmin.x), 0.0f), 1.0f);
    }
    hist = mk(hmin(hmax(hist.x, cmin.x), cmax.x), hmin(hmax(hist.y, cmin.y), cmax.y), hmin(hmax(hist.z, cmin.z), cmax.z));
    const f3 l = mk(hist.x + alpha * (color.x - hist.x), hist.y + alpha * (color.y - hist.y),
                    hist.z + alpha * (color.z - hist.z));
    const float tmp = l.x - l.y;
    a.out[(size_t)y * a.W + x] = make_float4(tmp + l.z, l.x + l.y, tmp - l.z, 1.0f);
}

// ---------------------------------------------------------------------- Deinterleave / Interleave
// DeinterleaveTexture (Deinterleave.slang, DeinterleaveTexture.cpp:143-158): a W x H texture ->
// 16 layers of ceil(W/4) x ceil(H/4), layer s = off.y * 4 + off.x holding src[4 y + off.y][4 x +
// off.x] (Loads outside the source read 0).  InterleaveTexture (Interleave.slang): the inverse,
// out[y][x] = src[layer (y % 4) * 4 + x % 4][y / 4][x / 4].  Byte shuffles of ELEM-byte texels.
template <int ELEM>
struct TexelT { uint8_t b[ELEM]; };
template <>
struct TexelT<4> { uint32_t v; };
template <>
struct TexelT<8> { uint2 v; };
template <>
struct TexelT<16> { uint4 v; };

template <int ELEM>
__global__ void __launch_bounds__(kPostW * kPostH) deinterleave_kernel(const TexelT<ELEM>* __restrict__ src, int W,
                                                                        int H, TexelT<ELEM>* __restrict__ dst, int w4,
                                                                        int h4) {
    const int x = (int)(blockIdx.x * kPostW + threadIdx.x), y = (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= w4 || y >= h4) return;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int sx = 4 * x + (s & 3), sy = 4 * y + (s >> 2);
        TexelT<ELEM> t{};
        if (sx < W && sy < H) t = src[(size_t)sy * W + sx];
        dst[((size_t)s * h4 + y) * w4 + x] = t;
    }
}

template <int ELEM>
__global__ void __launch_bounds__(kPostW * kPostH) interleave_kernel(const TexelT<ELEM>* __restrict__ src, int w4,
                                                                      int h4, TexelT<ELEM>* __restrict__ dst, int W,
                                                                      int H) {
    const int x = (int)(blockIdx.x * kPostW + threadIdx.x), y = (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= W || y >= H) return;
    const int xq = x >> 2, yq = y >> 2, s = (y & 3) * 4 + (x & 3);
    TexelT<ELEM> t{};
    if (xq < w4 && yq < h4) t = src[((size_t)s * h4 + yq) * w4 + xq];
    dst[(size_t)y * W + x] = t;
}

// ---------------------------------------------------------------------- RayMinMaxLength
// RayMinMaxLength.ps.slang:4-16: the SD ray interval length of every texel, 0 where rayMax was never
// raised, max(0, rayMax - rayMin) / 32 otherwise (the interval maps hold float bit patterns)
__global__ void __launch_bounds__(256) ray_length_kernel(const uint32_t* __restrict__ rmin,
                                                         const uint32_t* __restrict__ rmax, uint32_t n,
                                                         float* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint32_t mx = rmax[i];
    out[i] = mx == 0u ? 0.0f : hmax(0.0f, __uint_as_float(mx) - __uint_as_float(rmin[i])) / 32.0f;
}

// ---------------------------------------------------------------------- AOFlickerMask
// AOFlickerMask.ps.slang:43-63 (AOFlickerMask.cpp:73-86): a pixel is stable (1) when, in x and
// in y, one of its two neighbours lies in the plane of its view-space normal to within 0.1 (|dot|
// of the unit offset with the normal).  Loads outside the image read 0; HLSL min returns the
// non-NaN operand (a zero offset normalizes to NaN).
__global__ void __launch_bounds__(kPostW * kPostH) flicker_mask_kernel(const float* __restrict__ z,
                                                                        const float4* __restrict__ nw, int W, int H,
                                                                        rsd_camera cam, float isx, float isy,
                                                                        uint8_t* __restrict__ mask) {
    const int x = (int)(blockIdx.x * kPostW + threadIdx.x), y = (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= W || y >= H) return;
    auto ld = [&](int i, int j) { return (i < 0 || j < 0 || i >= W || j >= H) ? 0.0f : z[(size_t)j * W + i]; };
    auto view = [&](int i, int j, float d) {  // UVToViewSpace(PixelToUV(px), d)
        const float u = saturate(((float)i + 0.5f) / (float)W), v = saturate(((float)j + 0.5f) / (float)H);
        const float ndcx = u * 2.0f - 1.0f, ndcy = (1.0f - v) * 2.0f - 1.0f;
        return mk(ndcx * d * isx, ndcy * d * isy, -d);
    };
    const float4 n = nw[(size_t)y * W + x];
    const float* m = cam.viewMat;  // mul(float3x3(viewMat), n)
    const f3 nv = mk(m[0] * n.x + m[1] * n.y + m[2] * n.z, m[4] * n.x + m[5] * n.y + m[6] * n.z,
                     m[8] * n.x + m[9] * n.y + m[10] * n.z);
    const f3 P = view(x, y, ld(x, y));
    auto plane = [&](int i, int j) {
        const f3 q = view(i, j, ld(i, j));
        return fabsf(dot(normalize(P - q), nv));
    };
    const float dx = hmin(plane(x + 1, y), plane(x - 1, y));
    const float dy = hmin(plane(x, y + 1), plane(x, y - 1));
    mask[(size_t)y * W + x] = (dx <= 0.1f && dy <= 0.1f) ? 1u : 0u;
}

// ---------------------------------------------------------------------- BinaryDilation
// BinaryDilation.ps.slang:13-43: OP (min / max) over five Gather footprints (2x2 texels each):
// the centre and four at (+-0.5, +-1.5) px offsets (a radius-2 ring).  Gather's footprint is the
// bilinear footprint of the sample position (librsd's 8-bit sub-texel quantization), wrap
// addressing (the unbound sampler S: Falcor's default).
__device__ __forceinline__ uint32_t gather_op(const uint8_t* __restrict__ t, int W, int H, float u, float v, bool mx) {
    const float x = u * (float)W - 0.5f, y = v * (float)H - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const float qx = floorf((x - fx0) * 256.0f + 0.5f), qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) ix += 1;
    if (qy >= 256.0f) iy += 1;
    const int x0 = wrap_addr(ix, W), x1 = wrap_addr(ix + 1, W), y0 = wrap_addr(iy, H), y1 = wrap_addr(iy + 1, H);
    const uint32_t a = t[(size_t)y1 * W + x0], b = t[(size_t)y1 * W + x1], c = t[(size_t)y0 * W + x1],
                   d = t[(size_t)y0 * W + x0];  // Gather order w, z, ... (irrelevant to min / max)
    return mx ? max(max(a, b), max(c, d)) : min(min(a, b), min(c, d));
}

__global__ void __launch_bounds__(kPostW * kPostH) binary_dilation_kernel(const uint8_t* __restrict__ in, int W, int H,
                                                                           uint32_t opMax, uint8_t* __restrict__ out) {
    const int x = (int)(blockIdx.x * kPostW + threadIdx.x), y = (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= W || y >= H) return;
    const bool mx = opMax != 0u;
    const float u = ((float)x + 0.5f) / (float)W, v = ((float)y + 0.5f) / (float)H;
    const float dx = 0.5f / (float)W, dy = 0.5f / (float)H;
    auto op = [&](uint32_t p, uint32_t q) { return mx ? max(p, q) : min(p, q); };
    uint32_t r0 = gather_op(in, W, H, u + dx, v + 3.0f * dy, mx);
    const uint32_t r1 = gather_op(in, W, H, u + 3.0f * dx, v + -dy, mx);
    const uint32_t r2 = gather_op(in, W, H, u + -dx, v + -3.0f * dy, mx);
    const uint32_t r3 = gather_op(in, W, H, u + -3.0f * dx, v + dy, mx);
    r0 = op(r0, gather_op(in, W, H, u, v, mx));
    out[(size_t)y * W + x] = (uint8_t)op(op(r0, r1), op(r2, r3));
}

// ---------------------------------------------------------------------- TemporalAO
// TemporalAO.ps.slang:55-101 (TemporalAO.cpp:113-163, enabled): reproject the previous frame's
// AO along the motion vector, reject on a > 10 % relative depth change (or a stable-mask pixel),
// accumulate up to 30 frames.  Samplers: gAOSampler linear / clamp (R8Unorm, librsd's 8-bit
// sub-texel bilinear), gDepthSampler at pixel centres (exactly the texel); writes only inside
// the guard-band scissor.
struct TaoArgs {
    const uint8_t* aoIn;
    const float* z;
    const float2* mvec;
    const float* prevZ;
    const uint8_t* prevAo;
    const uint8_t* prevN;
    const uint8_t* stable;  // may be null (unbound: every pixel unstable)
    uint8_t* aoOut;
    uint8_t* nOut;
    int W, H, g;
    float m[16];  // prevViewToCurView, row-major
    float uvMinX, uvMinY, uvMaxX, uvMaxY;
    float isx, isy;  // 0.5 * frameWidth / focalLength, 0.5 * frameHeight / focalLength
};

// bilinear of an R8Unorm texture (clamp), librsd's sampler definition (tex_bilinear on unorm8/255)
__device__ __forceinline__ float unorm8_bilinear(const uint8_t* __restrict__ t, int W, int H, float u, float v) {
    float x = u * (float)W - 0.5f, y = v * (float)H - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    float qx = floorf((x - fx0) * 256.0f + 0.5f), qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) { ix += 1; qx = 0.0f; }
    if (qy >= 256.0f) { iy += 1; qy = 0.0f; }
    const float wx = qx * (1.0f / 256.0f), wy = qy * (1.0f / 256.0f);
    const int x0 = min(max(ix, 0), W - 1), x1 = min(max(ix + 1, 0), W - 1);
    const int y0 = min(max(iy, 0), H - 1), y1 = min(max(iy + 1, 0), H - 1);
    const float t00 = unorm8_to_float(t[(size_t)y0 * W + x0]), t10 = unorm8_to_float(t[(size_t)y0 * W + x1]);
    const float t01 = unorm8_to_float(t[(size_t)y1 * W + x0]), t11 = unorm8_to_float(t[(size_t)y1 * W + x1]);
    const float r0 = t00 * (1.0f - wx) + t10 * wx, r1 = t01 * (1.0f - wx) + t11 * wx;
    return r0 * (1.0f - wy) + r1 * wy;
}

__global__ void __launch_bounds__(kPostW * kPostH) temporal_ao_kernel(TaoArgs a) {
    const int x = a.g + (int)(blockIdx.x * kPostW + threadIdx.x);
    const int y = a.g + (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= a.W - a.g || y >= a.H - a.g) return;  // guard-band scissor
    const size_t o = (size_t)y * a.W + x;
    const float tu = ((float)x + 0.5f) / (float)a.W, tv = ((float)y + 0.5f) / (float)a.H;  // texC
    const float depth = a.z[o];
    float ao = unorm8_to_float(a.aoIn[o]);
    uint32_t n = 1u;
    const float2 mv = a.mvec[o];
    const float pu = tu + mv.x, pv = tv + mv.y;
    if (pu >= a.uvMinX && pu <= a.uvMaxX && pv >= a.uvMinY && pv <= a.uvMaxY) {  // isInValidArea
        const int qx = (int)floorf(pu * (float)a.W), qy = (int)floorf(pv * (float)a.H);  // UVToPixel
        const size_t po = (size_t)min(max(qy, 0), a.H - 1) * a.W + min(max(qx, 0), a.W - 1);
        const float prevRaw = a.prevZ[po];
        // UVToViewSpace(texC + mvec, prevRawDepth), then prevViewToCurView
        const float ndcx = pu * 2.0f - 1.0f, ndcy = (1.0f - pv) * 2.0f - 1.0f;
        const float vx = ndcx * prevRaw * a.isx, vy = ndcy * prevRaw * a.isy, vz = -prevRaw;
        const float pz = a.m[8] * vx + a.m[9] * vy + a.m[10] * vz + a.m[11];
        const float prevDepth = -pz;
        const bool stable = a.stable && a.stable[o] != 0u;
        if (fabsf(1.0f - prevDepth / depth) < 0.1f && !stable) {  // RelativeDepth(depth, prevDepth)
            const float prevAo = unorm8_bilinear(a.prevAo, a.W, a.H, pu, pv);
            const uint32_t prevN = a.prevN[po];
            ao = ((float)prevN * prevAo + ao) / (float)(prevN + 1u);
            n = min(prevN + 1u, 30u);
        }
    }
    a.aoOut[o] = unorm8(ao);
    a.nOut[o] = (uint8_t)n;
}

// GBufferRaster's motion vectors for a static scene and a moving camera (librsd definition):
// the pixel-centre primary hit P = posW + (z / cos) d (z: linear depth, d: the normalized pixel
// ray, cos = dot(normalize(W), d)) projected with the previous camera: mvec = prevUV(P) - uv.
// P behind the previous camera -> mvec = (2, 2) (off screen: TemporalAO resets the pixel).
// Background (no geometry: linear depth >= farZ, i.e. rsd_gbuffer's miss value farZ or the
// linearized cleared raster depth 1.0) -> mvec = (0, 0): GBufferRaster clears mvec
// (GBufferRaster.cpp:176) and writes it only for rasterized geometry (GBufferRaster.3d.slang:117).
struct MvecArgs {
    rsd_camera cam, prev;
    const float* z;
    const float* rawD;  // rsd_motion_vectors_raster: the non-linear raster depth (z unused)
    float2* mvec;
    int W, H;
    float pU[3], pV[3], pW[3];  // prev U / |U|^2, V / |V|^2, W / |W|^2
};

__global__ void __launch_bounds__(kPostW * kPostH) motion_vector_kernel(MvecArgs a) {
    const int x = (int)(blockIdx.x * kPostW + threadIdx.x), y = (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= a.W || y >= a.H) return;
    const rsd_camera& c = a.cam;
    const float u = ((float)x + 0.5f) / (float)a.W, v = ((float)y + 0.5f) / (float)a.H;
    float z;
    if (a.rawD) {
        // GBufferRaster's own depth: background is the cleared depth 1.0 (GBufferRaster.cpp:176), decided
        // on the raw value -- its linearisation can round either side of farZ (near 0.1 / far 10: 9.99996)
        const float dr = a.rawD[(size_t)y * a.W + x];
        if (!(dr < 1.0f)) {
            a.mvec[(size_t)y * a.W + x] = make_float2(0.0f, 0.0f);
            return;
        }
        z = c.nearZ * c.farZ / (c.farZ + dr * (c.nearZ - c.farZ));  // LinearizeDepth (rsd_linearize_depth)
    } else {
        z = a.z[(size_t)y * a.W + x];
        if (!(z < c.farZ)) {
            a.mvec[(size_t)y * a.W + x] = make_float2(0.0f, 0.0f);
            return;
        }
    }
    const f3 wn = normalize(mk(c.W[0], c.W[1], c.W[2]));
    const f3 d = normalize(mk((2.0f * u + -1.0f) * c.U[0] + (-2.0f * v + 1.0f) * c.V[0] + c.W[0],
                              (2.0f * u + -1.0f) * c.U[1] + (-2.0f * v + 1.0f) * c.V[1] + c.W[1],
                              (2.0f * u + -1.0f) * c.U[2] + (-2.0f * v + 1.0f) * c.V[2] + c.W[2]));
    const float t = z / dot(wn, d);
    const f3 rel = mk(c.posW[0] + t * d.x - a.prev.posW[0], c.posW[1] + t * d.y - a.prev.posW[1],
                      c.posW[2] + t * d.z - a.prev.posW[2]);
    const float pa = rel.x * a.pU[0] + rel.y * a.pU[1] + rel.z * a.pU[2];
    const float pb = rel.x * a.pV[0] + rel.y * a.pV[1] + rel.z * a.pV[2];
    const float pw = rel.x * a.pW[0] + rel.y * a.pW[1] + rel.z * a.pW[2];
    float2 mv = make_float2(2.0f, 2.0f);
    if (pw > 0.0f) mv = make_float2((pa / pw + 1.0f) * 0.5f - u, (1.0f - pb / pw) * 0.5f - v);
    a.mvec[(size_t)y * a.W + x] = mv;
}

// ---------------------------------------------------------------------- ImageEquation
struct TexDesc {
    const void* ptr;
    int w, h;
    uint32_t fmt;
};
struct EqArgs {
    IeProgram prog;
    TexDesc in[4];
    void* out;
    int W, H;
    uint32_t outFmt;
};

__device__ __forceinline__ float4 load_texel(const TexDesc& t, int x, int y) {
    if (!t.ptr || x >= t.w || y >= t.h) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const size_t o = (size_t)y * t.w + x;
    switch (t.fmt) {
        case RSD_FMT_R32F: return make_float4(static_cast<const float*>(t.ptr)[o], 0.0f, 0.0f, 1.0f);
        case RSD_FMT_RG32F: {
            const float2 v = static_cast<const float2*>(t.ptr)[o];
            return make_float4(v.x, v.y, 0.0f, 1.0f);
        }
        case RSD_FMT_RGBA32F: return static_cast<const float4*>(t.ptr)[o];
        case RSD_FMT_R8UNORM: return make_float4(unorm8_to_float(static_cast<const uint8_t*>(t.ptr)[o]), 0.0f, 0.0f, 1.0f);
        case RSD_FMT_R8U: return make_float4((float)static_cast<const uint8_t*>(t.ptr)[o], 0.0f, 0.0f, 1.0f);
        case RSD_FMT_R16U: return make_float4((float)static_cast<const uint16_t*>(t.ptr)[o], 0.0f, 0.0f, 1.0f);
        case RSD_FMT_R32U: return make_float4((float)static_cast<const uint32_t*>(t.ptr)[o], 0.0f, 0.0f, 1.0f);
        default: return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
}

__device__ __forceinline__ float lane(float4 v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
__device__ __forceinline__ float dbl1(int f, float x) {
    const double d = (double)x;
    switch (f) {
        case F1_EXP2: return (float)exp2(d);
        case F1_LOG2: return (float)log2(d);
        case F1_EXP: return (float)exp(d);
        case F1_LOG: return (float)log(d);
        case F1_SIN: return (float)sin(d);
        case F1_COS: return (float)cos(d);
        default: return (float)(1.0 / sqrt(d));  // F1_RSQRT
    }
}
__device__ __forceinline__ float f1(int f, float x) {
    switch (f) {
        case F1_ABS: return fabsf(x);
        case F1_SAT: return saturate(x);
        case F1_SQRT: return sqrtf(x);
        case F1_FLOOR: return floorf(x);
        case F1_CEIL: return ceilf(x);
        case F1_FRAC: return x - floorf(x);
        case F1_SIGN: return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f);
        default: return dbl1(f, x);
    }
}
__device__ __forceinline__ float f2(int f, float a, float b) {
    switch (f) {
        case F2_MIN: return fminf(a, b);
        case F2_MAX: return fmaxf(a, b);
        case F2_POW: return acc_pow(a, b);
        default: return b >= a ? 1.0f : 0.0f;  // F2_STEP: step(y, x) = x >= y
    }
}
#define RSD_MAP4(e) make_float4(e(x), e(y), e(z), e(w))

__global__ void __launch_bounds__(kPostW * kPostH) image_equation_kernel(EqArgs a) {
    const int x = (int)(blockIdx.x * kPostW + threadIdx.x), y = (int)(blockIdx.y * kPostH + threadIdx.y);
    if (x >= a.W || y >= a.H) return;
    float4 st[kIeMaxStack];
    int sp = 0;
    for (int pc = 0; pc < a.prog.n; ++pc) {
        const IeInstr in = a.prog.code[pc];
        switch (in.op) {
            case IE_TEX: st[sp++] = load_texel(a.in[in.a], x, y); break;
            case IE_CONST: st[sp++] = make_float4(in.k, in.k, in.k, in.k); break;
            case IE_SWZ: {
                const float4 v = st[sp - 1];
                st[sp - 1] = make_float4(lane(v, in.a & 3), lane(v, (in.a >> 2) & 3), lane(v, (in.a >> 4) & 3),
                                         lane(v, (in.a >> 6) & 3));
                break;
            }
            case IE_NEG: {
                const float4 v = st[sp - 1];
                st[sp - 1] = make_float4(-v.x, -v.y, -v.z, -v.w);
                break;
            }
            case IE_ADD: case IE_SUB: case IE_MUL: case IE_DIV: {
                const float4 p = st[sp - 2], q = st[sp - 1];
                --sp;
                float4 r;
                if (in.op == IE_ADD) r = make_float4(p.x + q.x, p.y + q.y, p.z + q.z, p.w + q.w);
                else if (in.op == IE_SUB) r = make_float4(p.x - q.x, p.y - q.y, p.z - q.z, p.w - q.w);
                else if (in.op == IE_MUL) r = make_float4(p.x * q.x, p.y * q.y, p.z * q.z, p.w * q.w);
                else r = make_float4(p.x / q.x, p.y / q.y, p.z / q.z, p.w / q.w);
                st[sp - 1] = r;
                break;
            }
            case IE_F1: {
                const float4 v = st[sp - 1];
                st[sp - 1] = make_float4(f1(in.a, v.x), f1(in.a, v.y), f1(in.a, v.z), f1(in.a, v.w));
                break;
            }
            case IE_F2: {
                const float4 p = st[sp - 2], q = st[sp - 1];
                --sp;
                st[sp - 1] = make_float4(f2(in.a, p.x, q.x), f2(in.a, p.y, q.y), f2(in.a, p.z, q.z), f2(in.a, p.w, q.w));
                break;
            }
            case IE_F3: {
                const float4 p = st[sp - 3], q = st[sp - 2], t = st[sp - 1];
                sp -= 2;
                float4 r;
                if (in.a == F3_LERP)  // x + s (y - x)
                    r = make_float4(p.x + t.x * (q.x - p.x), p.y + t.y * (q.y - p.y), p.z + t.z * (q.z - p.z),
                                    p.w + t.w * (q.w - p.w));
                else
                    r = make_float4(fminf(fmaxf(p.x, q.x), t.x), fminf(fmaxf(p.y, q.y), t.y),
                                    fminf(fmaxf(p.z, q.z), t.z), fminf(fmaxf(p.w, q.w), t.w));
                st[sp - 1] = r;
                break;
            }
            case IE_DOT: {
                const float4 p = st[sp - 2], q = st[sp - 1];
                --sp;
                float d = p.x * q.x;
                if (in.a > 1) d = d + p.y * q.y;
                if (in.a > 2) d = d + p.z * q.z;
                if (in.a > 3) d = d + p.w * q.w;
                st[sp - 1] = make_float4(d, d, d, d);
                break;
            }
            case IE_CTOR: {
                const int n = in.a;
                float o[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                int k = 0;
                for (int j = 0; j < n; ++j) {
                    const float4 v = st[sp - n + j];
                    const int w = ((in.b >> (2 * j)) & 3) + 1;
                    for (int l = 0; l < w && k < 4; ++l) o[k++] = lane(v, l);
                }
                if (n == 1 && (in.b & 3) == 0) o[1] = o[2] = o[3] = o[0];  // floatN(scalar)
                sp -= n - 1;
                st[sp - 1] = make_float4(o[0], o[1], o[2], o[3]);
                break;
            }
        }
    }
    const float4 r = st[0];
    const size_t o = (size_t)y * a.W + x;
    switch (a.outFmt) {
        case RSD_FMT_RGBA32F: static_cast<float4*>(a.out)[o] = r; break;
        case RSD_FMT_RG32F: static_cast<float2*>(a.out)[o] = make_float2(r.x, r.y); break;
        case RSD_FMT_R32F: static_cast<float*>(a.out)[o] = r.x; break;
        default: static_cast<uint8_t*>(a.out)[o] = unorm8(r.x); break;  // RSD_FMT_R8UNORM
    }
}

}  // namespace
}  // namespace rsd

using namespace rsd;

extern "C" rsd_status rsd_cross_bilateral_blur(const uint8_t* d_src, const float* d_linear_z, uint32_t z_w,
                                               uint32_t z_h, uint8_t* d_pingpong, uint8_t* d_dst, uint32_t width,
                                               uint32_t height, uint32_t guard_band, uint32_t kernel_radius,
                                               uint32_t better_slope, rsd_stream stream) {
    if (!d_src || !d_linear_z || !d_pingpong || !d_dst || width == 0 || height == 0 || z_w == 0 || z_h == 0 ||
        kernel_radius < 1 || kernel_radius > 20 || 2 * guard_band >= width || 2 * guard_band >= height) {
        set_error("rsd_cross_bilateral_blur: invalid argument (radius 1..20, guard band inside the frame)");
        return RSD_ERR_INVALID_ARG;
    }
    BlurArgs a{};
    a.z = d_linear_z;
    a.zW = (int)z_w;
    a.zH = (int)z_h;
    a.W = (int)width;
    a.H = (int)height;
    a.g = (int)guard_band;
    a.betterSlope = better_slope ? 1u : 0u;
    // GuardBand.cpp:62-63
    a.uvMinX = ((float)guard_band + 0.5f) / (float)width;
    a.uvMinY = ((float)guard_band + 0.5f) / (float)height;
    a.uvMaxX = ((float)width - ((float)guard_band + 0.5f)) / (float)width;
    a.uvMaxY = ((float)height - ((float)guard_band + 0.5f)) / (float)height;
    hipStream_t s = (hipStream_t)stream;
    for (int pass = 0; pass < 2; ++pass) {  // blur in x into the ping-pong image, then in y
        a.src = pass == 0 ? d_src : d_pingpong;
        a.dst = pass == 0 ? d_pingpong : d_dst;
        a.dirX = pass == 0 ? 1.0f : 0.0f;
        a.dirY = pass == 0 ? 0.0f : 1.0f;
        hipError_t e = hipSuccess;
        switch (kernel_radius) {
#define RSD_R(r) case r: e = launch_blur<r>(a, s); break;
            RSD_R(1) RSD_R(2) RSD_R(3) RSD_R(4) RSD_R(5) RSD_R(6) RSD_R(7) RSD_R(8) RSD_R(9) RSD_R(10)
            RSD_R(11) RSD_R(12) RSD_R(13) RSD_R(14) RSD_R(15) RSD_R(16) RSD_R(17) RSD_R(18) RSD_R(19) RSD_R(20)
#undef RSD_R
        }
        if (e != hipSuccess) return hip_fail(e, "blur_kernel launch");
    }
    return RSD_OK;
}

namespace {
template <template <int> class KERNEL>
rsd_status launch_by_elem(uint32_t elem, dim3 grid, hipStream_t s, const void* src, int a0, int a1, void* dst, int b0,
                          int b1, const char* what) {
    switch (elem) {
        case 1: hipLaunchKernelGGL(KERNEL<1>::fn, grid, dim3(kPostW, kPostH), 0, s, (const TexelT<1>*)src, a0, a1, (TexelT<1>*)dst, b0, b1); break;
        case 2: hipLaunchKernelGGL(KERNEL<2>::fn, grid, dim3(kPostW, kPostH), 0, s, (const TexelT<2>*)src, a0, a1, (TexelT<2>*)dst, b0, b1); break;
        case 4: hipLaunchKernelGGL(KERNEL<4>::fn, grid, dim3(kPostW, kPostH), 0, s, (const TexelT<4>*)src, a0, a1, (TexelT<4>*)dst, b0, b1); break;
        case 8: hipLaunchKernelGGL(KERNEL<8>::fn, grid, dim3(kPostW, kPostH), 0, s, (const TexelT<8>*)src, a0, a1, (TexelT<8>*)dst, b0, b1); break;
        case 16: hipLaunchKernelGGL(KERNEL<16>::fn, grid, dim3(kPostW, kPostH), 0, s, (const TexelT<16>*)src, a0, a1, (TexelT<16>*)dst, b0, b1); break;
        default:
            set_error(std::string(what) + ": texel size must be 1, 2, 4, 8 or 16 bytes");
            return RSD_ERR_UNSUPPORTED;
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, what);
}
template <int E>
struct DeinterleaveK { static constexpr auto fn = deinterleave_kernel<E>; };
template <int E>
struct InterleaveK { static constexpr auto fn = interleave_kernel<E>; };
}  // namespace

extern "C" rsd_status rsd_deinterleave(const void* d_src, uint32_t width, uint32_t height, uint32_t texel_bytes,
                                       void* d_dst, rsd_stream stream) {
    if (!d_src || !d_dst || width == 0 || height == 0 || d_src == d_dst) {
        set_error("rsd_deinterleave: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t w4 = (width + 3) / 4, h4 = (height + 3) / 4;
    const dim3 grid((w4 + kPostW - 1) / kPostW, (h4 + kPostH - 1) / kPostH);
    return launch_by_elem<DeinterleaveK>(texel_bytes, grid, (hipStream_t)stream, d_src, (int)width, (int)height, d_dst,
                                         (int)w4, (int)h4, "rsd_deinterleave");
}

extern "C" rsd_status rsd_interleave(const void* d_src, uint32_t width, uint32_t height, uint32_t texel_bytes,
                                     void* d_dst, rsd_stream stream) {
    if (!d_src || !d_dst || width == 0 || height == 0 || d_src == d_dst) {
        set_error("rsd_interleave: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t w4 = (width + 3) / 4, h4 = (height + 3) / 4;
    const dim3 grid((width + kPostW - 1) / kPostW, (height + kPostH - 1) / kPostH);
    return launch_by_elem<InterleaveK>(texel_bytes, grid, (hipStream_t)stream, d_src, (int)w4, (int)h4, d_dst,
                                       (int)width, (int)height, "rsd_interleave");
}

extern "C" rsd_status rsd_ray_min_max_length(const uint32_t* d_ray_min, const uint32_t* d_ray_max, uint32_t width,
                                             uint32_t height, float* d_out, rsd_stream stream) {
    if (!d_ray_min || !d_ray_max || !d_out || width == 0 || height == 0) {
        set_error("rsd_ray_min_max_length: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t n = width * height;
    hipLaunchKernelGGL(ray_length_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_ray_min,
                       d_ray_max, n, d_out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "ray_length_kernel launch");
}

extern "C" rsd_status rsd_ao_flicker_mask(const float* d_linear_z, const float* d_normal_w, uint32_t width,
                                          uint32_t height, const rsd_camera* cam, uint8_t* d_mask, rsd_stream stream) {
    if (!d_linear_z || !d_normal_w || !cam || !d_mask || width == 0 || height == 0) {
        set_error("rsd_ao_flicker_mask: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    const float isx = 0.5f * (cam->frameWidth / cam->focalLength), isy = 0.5f * (cam->frameHeight / cam->focalLength);
    const dim3 grid((width + kPostW - 1) / kPostW, (height + kPostH - 1) / kPostH);
    hipLaunchKernelGGL(flicker_mask_kernel, grid, dim3(kPostW, kPostH), 0, (hipStream_t)stream, d_linear_z,
                       reinterpret_cast<const float4*>(d_normal_w), (int)width, (int)height, *cam, isx, isy, d_mask);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "flicker_mask_kernel launch");
}

extern "C" rsd_status rsd_binary_dilation(const uint8_t* d_in, uint32_t width, uint32_t height, uint32_t op_max,
                                          uint8_t* d_out, rsd_stream stream) {
    if (!d_in || !d_out || width == 0 || height == 0 || op_max > 1u || d_in == d_out) {
        set_error("rsd_binary_dilation: invalid argument (op_max 0 = min, 1 = max; no in-place)");
        return RSD_ERR_INVALID_ARG;
    }
    const dim3 grid((width + kPostW - 1) / kPostW, (height + kPostH - 1) / kPostH);
    hipLaunchKernelGGL(binary_dilation_kernel, grid, dim3(kPostW, kPostH), 0, (hipStream_t)stream, d_in, (int)width,
                       (int)height, op_max, d_out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "binary_dilation_kernel launch");
}

extern "C" rsd_status rsd_taa(const float* d_color_in, const float* d_mvec, const float* d_prev_color, uint32_t width,
                              uint32_t height, float alpha, float color_box_sigma, uint32_t anti_flicker,
                              float* d_color_out, rsd_stream stream) {
    if (!d_color_in || !d_mvec || !d_prev_color || !d_color_out || width == 0 || height == 0) {
        set_error("rsd_taa: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    TaaArgs a{};
    a.color = reinterpret_cast<const float4*>(d_color_in);
    a.mvec = reinterpret_cast<const float2*>(d_mvec);
    a.prev = reinterpret_cast<const float4*>(d_prev_color);
    a.out = reinterpret_cast<float4*>(d_color_out);
    a.W = (int)width;
    a.H = (int)height;
    a.alpha = alpha;
    a.sigma = color_box_sigma;
    a.antiFlicker = anti_flicker;
    a.invW = 1.0f / (float)width;  // TAA.ps.slang:47 invTextureSize
    a.invH = 1.0f / (float)height;
    const dim3 grid((width + kPostW - 1) / kPostW, (height + kPostH - 1) / kPostH);
    hipLaunchKernelGGL(taa_kernel, grid, dim3(kPostW, kPostH), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "taa_kernel launch");
}

extern "C" rsd_status rsd_temporal_ao(const uint8_t* d_ao_in, const float* d_linear_z, const float* d_mvec,
                                      const float* d_prev_linear_z, const uint8_t* d_prev_ao,
                                      const uint8_t* d_prev_history, const uint8_t* d_stable_mask, uint32_t width,
                                      uint32_t height, uint32_t guard_band, const rsd_camera* cam,
                                      const float prev_view_to_cur_view[16], uint8_t* d_ao_out,
                                      uint8_t* d_history_out, rsd_stream stream) {
    if (!d_ao_in || !d_linear_z || !d_mvec || !d_prev_linear_z || !d_prev_ao || !d_prev_history || !cam ||
        !prev_view_to_cur_view || !d_ao_out || !d_history_out || width == 0 || height == 0 ||
        2 * guard_band >= width || 2 * guard_band >= height) {
        set_error("rsd_temporal_ao: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    TaoArgs a{};
    a.aoIn = d_ao_in;
    a.z = d_linear_z;
    a.mvec = reinterpret_cast<const float2*>(d_mvec);
    a.prevZ = d_prev_linear_z;
    a.prevAo = d_prev_ao;
    a.prevN = d_prev_history;
    a.stable = d_stable_mask;
    a.aoOut = d_ao_out;
    a.nOut = d_history_out;
    a.W = (int)width;
    a.H = (int)height;
    a.g = (int)guard_band;
    for (int i = 0; i < 16; ++i) a.m[i] = prev_view_to_cur_view[i];
    // GuardBand.cpp:62-63
    a.uvMinX = ((float)guard_band + 0.5f) / (float)width;
    a.uvMinY = ((float)guard_band + 0.5f) / (float)height;
    a.uvMaxX = ((float)width - ((float)guard_band + 0.5f)) / (float)width;
    a.uvMaxY = ((float)height - ((float)guard_band + 0.5f)) / (float)height;
    a.isx = 0.5f * (cam->frameWidth / cam->focalLength);  // TemporalAO.ps.slang:42 imageScale
    a.isy = 0.5f * (cam->frameHeight / cam->focalLength);
    const dim3 grid((width - 2 * guard_band + kPostW - 1) / kPostW, (height - 2 * guard_band + kPostH - 1) / kPostH);
    hipLaunchKernelGGL(temporal_ao_kernel, grid, dim3(kPostW, kPostH), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "temporal_ao_kernel launch");
}

namespace {
rsd_status motion_vectors_impl(const rsd_camera* cam, const rsd_camera* prev_cam, const float* d_linear_z,
                               const float* d_raw, uint32_t width, uint32_t height, float* d_mvec, rsd_stream stream) {
    if (!cam || !prev_cam || !(d_linear_z || d_raw) || !d_mvec || width == 0 || height == 0) {
        set_error("rsd_motion_vectors: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    MvecArgs a{};
    a.cam = *cam;
    a.prev = *prev_cam;
    a.z = d_linear_z;
    a.rawD = d_raw;
    a.mvec = reinterpret_cast<float2*>(d_mvec);
    a.W = (int)width;
    a.H = (int)height;
    auto dot3 = [](const float* p, const float* q) { return (double)p[0] * q[0] + (double)p[1] * q[1] + (double)p[2] * q[2]; };
    const double uu = dot3(prev_cam->U, prev_cam->U), vv = dot3(prev_cam->V, prev_cam->V),
                 ww = dot3(prev_cam->W, prev_cam->W);
    for (int k = 0; k < 3; ++k) {
        a.pU[k] = (float)(prev_cam->U[k] / uu);
        a.pV[k] = (float)(prev_cam->V[k] / vv);
        a.pW[k] = (float)(prev_cam->W[k] / ww);
    }
    const dim3 grid((width + kPostW - 1) / kPostW, (height + kPostH - 1) / kPostH);
    hipLaunchKernelGGL(motion_vector_kernel, grid, dim3(kPostW, kPostH), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "motion_vector_kernel launch");
}
}  // namespace

extern "C" rsd_status rsd_motion_vectors(const rsd_camera* cam, const rsd_camera* prev_cam, const float* d_linear_z,
                                         uint32_t width, uint32_t height, float* d_mvec, rsd_stream stream) {
    if (!d_linear_z) {
        set_error("rsd_motion_vectors: null linear depth");
        return RSD_ERR_INVALID_ARG;
    }
    return motion_vectors_impl(cam, prev_cam, d_linear_z, nullptr, width, height, d_mvec, stream);
}

extern "C" rsd_status rsd_motion_vectors_raster(const rsd_camera* cam, const rsd_camera* prev_cam, const float* d_depth,
                                                uint32_t width, uint32_t height, float* d_mvec, rsd_stream stream) {
    if (!d_depth) {
        set_error("rsd_motion_vectors_raster: null depth");
        return RSD_ERR_INVALID_ARG;
    }
    return motion_vectors_impl(cam, prev_cam, nullptr, d_depth, width, height, d_mvec, stream);
}

extern "C" rsd_status rsd_image_equation_run(const rsd_image_program* prog, const rsd_texture* inputs,
                                             const rsd_texture* out, rsd_stream stream) {
    if (!prog || !out || !out->ptr || out->width == 0 || out->height == 0) {
        set_error("rsd_image_equation_run: null program or output");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t f = out->format;
    if (f != RSD_FMT_RGBA32F && f != RSD_FMT_RG32F && f != RSD_FMT_R32F && f != RSD_FMT_R8UNORM) {
        set_error("rsd_image_equation_run: output format must be RGBA32F, RG32F, R32F or R8Unorm");
        return RSD_ERR_UNSUPPORTED;
    }
    EqArgs a{};
    a.prog = image_program(prog);
    for (int k = 0; k < 4; ++k) {
        if (inputs && inputs[k].ptr) {
            if (inputs[k].format >= RSD_FMT_UNKNOWN) {
                set_error("rsd_image_equation_run: input of unknown format");
                return RSD_ERR_INVALID_ARG;
            }
            a.in[k] = TexDesc{inputs[k].ptr, (int)inputs[k].width, (int)inputs[k].height, inputs[k].format};
        }
    }
    a.out = out->ptr;
    a.W = (int)out->width;
    a.H = (int)out->height;
    a.outFmt = f;
    const dim3 grid((a.W + kPostW - 1) / kPostW, (a.H + kPostH - 1) / kPostH);
    hipLaunchKernelGGL(image_equation_kernel, grid, dim3(kPostW, kPostH), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "image_equation_kernel launch");
}
