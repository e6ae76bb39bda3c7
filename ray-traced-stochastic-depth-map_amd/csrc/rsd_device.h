// rsd_device.h -- device-side math shared by the librsd HIP kernels (gfx950).
//
// Numerics contract (DESIGN.md "Numerics"), identical to the CPU oracle's:
//  * binary32, round-to-nearest, NO contraction: librsd is compiled with
//    -ffp-contract=off, so every expression rounds operation by operation in the
//    order written (only the BVH box test uses explicit fmaf: it decides which
//    nodes are visited, never which hits are reported);
//  * sqrtf / '/' are correctly rounded (hipcc default
//    -fhip-fp32-correctly-rounded-divide-sqrt);
//  * normalize(v) = v * (1 / sqrt(dot(v, v)))     (Falcor VectorMath.h:1731);
//  * sin/cos/pow of a float = (float)f64-libm(double): the reference's HLSL sin/pow
//    precision is implementation-defined; evaluating in double and rounding once makes
//    GPU and host agree bit-for-bit (up to a ~1e-8 chance of a double-rounding tie);
//  * HLSL min/max/saturate: a NaN operand yields the other one (fminf/fmaxf).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsd {

struct f3 { float x, y, z; };

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ f3 normalize(f3 v) {
#ifdef RSD_FAST_NUMERICS  // svao_fast.hip (svao_math.h): the hardware reciprocal square root, 1 ulp
    float inv = __builtin_amdgcn_rsqf(dot(v, v));
#else
    float inv = 1.0f / sqrtf(dot(v, v));
#endif
    return v * inv;
}
__device__ __forceinline__ float length(f3 v) { return sqrtf(dot(v, v)); }
__device__ __forceinline__ float saturate(float x) { return !(x > 0.0f) ? 0.0f : (x > 1.0f ? 1.0f : x); }
__device__ __forceinline__ float hmax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ float hmin(float a, float b) { return fminf(a, b); }
__device__ __forceinline__ float acc_sin(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float acc_pow(float x, float y) {
    // y == 2 (the SVAO default exponent, VAOData.slang:40): x * x is exact in double (48-bit
    // product), so the correctly rounded pow rounds to the binary32 product x * x.
    if (y == 2.0f) return x * x;
    return (float)pow((double)x, (double)y);
}

// R8Unorm store: saturate, round to nearest; NaN -> 0
__device__ __forceinline__ uint8_t unorm8(float x) {
    if (x != x) return 0;
    x = saturate(x);
    return (uint8_t)floorf(x * 255.0f + 0.5f);
}
__device__ __forceinline__ float unorm8_to_float(uint8_t c) { return (float)c / 255.0f; }

// Common.slangh:36-39
__device__ __forceinline__ float sd_hash(float x, float y) {
    float a = 17.0f * x + 0.1f * y;
    float b = 13.0f * y + x;
    float r = 1.0e4f * acc_sin(a) * (0.1f + fabsf(acc_sin(b)));
    return r - floorf(r);
}

// Jitter.slangh:20 jitterPos, indexed (y % 4) * 4 + x % 4 (Jitter.slangh:34-46)
__constant__ static const float kJitter[32] = {
    0.6483604982495308f, 0.914070401340723f,   0.7279119342565536f, 0.1037941575050354f,
    0.48886989802122116f, 0.699178121984005f,  0.3848271369934082f, 0.25951504334807396f,
    0.1555836834013462f, 0.8020274639129639f,  0.2205628715455532f, 0.2412630058825016f,
    0.9962188489735126f, 0.5846633277833462f,  0.8776040785014629f, 0.3954884633421898f,
    0.9271227307617664f, 0.831196017563343f,   0.9490576796233654f, 0.14202157780528069f,
    0.20916065946221352f, 0.5476771481335163f, 0.16468944773077965f, 0.4869129806756973f,
    0.43544455617666245f, 0.9515445046126842f, 0.44085410237312317f, 0.011881716549396515f,
    0.7173641100525856f, 0.6695209294557571f,  0.6563677340745926f, 0.35924511030316353f,
};

__device__ __forceinline__ void sd_jitter(uint32_t x, uint32_t y, bool on, float& jx, float& jy) {
    if (!on) { jx = 0.5f; jy = 0.5f; return; }
    uint32_t i = ((y & 3u) * 4u + (x & 3u)) * 2u;
    jx = kJitter[i];
    jy = kJitter[i + 1];
}

// Linear filtering of an R32F texture (D3D conventions, 8 sub-texel bits).
// wrap: AddressMode::Wrap (Falcor sampler default) else Clamp.
__device__ __forceinline__ int tex_addr(int i, int n, bool wrap) {
    if (wrap) { i %= n; return i < 0 ? i + n : i; }
    return i < 0 ? 0 : (i >= n ? n - 1 : i);
}
__device__ __forceinline__ float tex_bilinear(const float* __restrict__ tex, int W, int H, float u, float v, bool wrap) {
    float x = u * (float)W - 0.5f;
    float y = v * (float)H - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float qx = floorf((x - fx0) * 256.0f + 0.5f);
    float qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) { ix += 1; qx = 0.0f; }
    if (qy >= 256.0f) { iy += 1; qy = 0.0f; }
    float wx = qx * (1.0f / 256.0f), wy = qy * (1.0f / 256.0f);
    int x0 = tex_addr(ix, W, wrap), y0 = tex_addr(iy, H, wrap);
    const float t00 = tex[(size_t)y0 * W + x0];
    // Zero weights: t*(1-0) + t'*0 == t exactly for finite t' (depth texels are finite,
    // DESIGN.md "Numerics"), so the taps with zero weight are not fetched.  Pixel-centre
    // samples (SVAO Init / primary visibility) need 1 fetch instead of 4.
    if (qx == 0.0f && qy == 0.0f) return t00;
    int x1 = tex_addr(ix + 1, W, wrap), y1 = tex_addr(iy + 1, H, wrap);
    if (qy == 0.0f) {
        const float t10 = tex[(size_t)y0 * W + x1];
        return t00 * (1.0f - wx) + t10 * wx;
    }
    const float t01 = tex[(size_t)y1 * W + x0];
    if (qx == 0.0f) return t00 * (1.0f - wy) + t01 * wy;
    const float t10 = tex[(size_t)y0 * W + x1], t11 = tex[(size_t)y1 * W + x1];
    float r0 = t00 * (1.0f - wx) + t10 * wx;
    float r1 = t01 * (1.0f - wx) + t11 * wx;
    return r0 * (1.0f - wy) + r1 * wy;
}

// ---- octahedral 2x8 normals: PackedFormats.slang:35-48, MathHelpers.slang:156-194,
//      FormatConversion.slang:49-95
__device__ __forceinline__ int float_to_snorm8(float v) {
    v = (v != v) ? 0.0f : hmin(hmax(v, -1.0f), 1.0f);
    return (int)truncf(v * 127.0f + (v >= 0.0f ? 0.5f : -0.5f));
}
__device__ __forceinline__ uint32_t encode_normal_2x8(f3 n) {
    float s = 1.0f / (fabsf(n.x) + fabsf(n.y) + fabsf(n.z));
    float px = n.x * s, py = n.y * s;
    if (n.z < 0.0f) {
        float wx = (1.0f - fabsf(py)) * (px >= 0.0f ? 1.0f : -1.0f);
        float wy = (1.0f - fabsf(px)) * (py >= 0.0f ? 1.0f : -1.0f);
        px = wx; py = wy;
    }
    return ((uint32_t)float_to_snorm8(px) & 0xffu) | (((uint32_t)float_to_snorm8(py) << 8) & 0xff00u);
}
__device__ __forceinline__ f3 decode_normal_2x8(uint32_t packed) {
    int bx = (int)(int8_t)(uint8_t)(packed & 0xffu);
    int by = (int)(int8_t)(uint8_t)((packed >> 8) & 0xffu);
    float px = hmax((float)bx / 127.0f, -1.0f), py = hmax((float)by / 127.0f, -1.0f);
    f3 n = mk(px, py, 1.0f - fabsf(px) - fabsf(py));
    if (n.z < 0.0f) {
        float wx = (1.0f - fabsf(n.y)) * (n.x >= 0.0f ? 1.0f : -1.0f);
        float wy = (1.0f - fabsf(n.x)) * (n.y >= 0.0f ? 1.0f : -1.0f);
        n.x = wx; n.y = wy;
    }
    return normalize(n);
}

// SD-map texel addressing.  The product layout is Texture2DArray order [layer][y][x][ch]
// (StochasticDepthMapRT.cpp:177-216).  RSD_SD_TILED (an A/B build only, SURVEY 7.3's "8x8-texel
// tiles"): each layer is stored as 8x8-texel tiles, row-major inside a tile and tiles row-major,
// over a map padded to whole tiles (sd_plane_texels) -- measured no faster, DESIGN.md section 4.
__device__ __forceinline__ size_t sd_texel(int x, int y, int W) {
#ifdef RSD_SD_TILED
    const int tw = (W + 7) >> 3;
    return ((size_t)((y >> 3) * tw + (x >> 3)) << 6) + (size_t)((y & 7) * 8 + (x & 7));
#else
    return (size_t)y * W + x;
#endif
}
__device__ __forceinline__ size_t sd_plane_texels(int W, int H) {
#ifdef RSD_SD_TILED
    return (size_t)((W + 7) >> 3) * ((H + 7) >> 3) * 64u;
#else
    return (size_t)W * H;
#endif
}

__device__ __forceinline__ uint32_t asuint(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float asfloat(uint32_t u) { return __uint_as_float(u); }

}  // namespace rsd
