// svao_math.h -- SVAO per-pixel math shared by the "AO 1" / "AO 2" kernels (svao.hip) and the
// Raytraced secondary mode (svao_rt.hip).
//
// Reference: SVAO/Common.slang:98-496 (BasicAOData, SampleAOData, visibility terms, UV/view
// conversions), SVAO.cpp:663-688 (noise texture).  Numerics contract: rsd_device.h.
#pragma once
#include <cmath>
#include <string>

#include "rsd_device.h"
#include "rsd_internal.h"

namespace rsd {

constexpr int kMaxDirections = 32;  // NUM_DIRECTIONS: 8, 16 or 32 (Common.slang:51-58)

struct SvaoConsts {
    float sinNoise[16], cosNoise[16];
    float sinDir[kMaxDirections], cosDir[kMaxDirections];
    float sampleRadius[kMaxDirections];
    // SampleAOData::Init terms that only depend on the AO radius (Common.slang:358-363),
    // evaluated on the host with the device's float operations for radius == VAOData.radius
    // (every pixel whose screen radius is not clamped to ssMaxRadius)
    float dirRadius[kMaxDirections], dirDx[kMaxDirections], dirDy[kMaxDirections], dirHeight[kMaxDirections];
    float ssrMin2;  // smallest float x with sqrtf(x) > ssRadiusCutoff: sqrtf(x) > c <=> x >= ssrMin2
    // RN(1 / pdf_i) and RN(1 / sphereHeight_i) of those terms (div_rcp); bit i of fastDiv set when
    // both divisors of direction i lie in [2^-30, 2^30]
    float rcpPdf[kMaxDirections], rcpHeight[kMaxDirections];
    // ratioMin[i]: the least float >= M * 2 dirHeight[i] (ratio_le_tenth's exact bound): at the
    // unclamped radius a direction is valid iff sphereStart - sphereEnd >= ratioMin[i]
    float ratioMin[kMaxDirections];
    uint32_t fastDiv;
    uint32_t samePixelInt;  // isSamePixel decided on pixel indices (fill_consts)
    uint32_t nd;            // NUM_DIRECTIONS
    float invNd;            // 1.0 / float(NUM_DIRECTIONS) (SVAORaster.ps.slang:108, Common.slang:660)
    uint32_t hbao;          // AO_KERNEL == AO_KERNEL_HBAO (rsd_ao_kernel)
    float pdfHbao[kMaxDirections];  // HBAO pdf of direction i: 0.9 pow(1 - sampleRadius[i], 1.5) (Common.slang:364)
    float rcpRadius;                // 1 / VAOData.radius (fast numerics: the clamped pixels' scale, sample_init)
};

struct SvaoArgs {
    rsd_camera cam;
    rsd_vao_data d;
    SvaoConsts k;
    const float* depth;
    const uint16_t* normals;
    int W, H;
    uint8_t* ao;
    uint8_t* stencil;  // NUM_DIRECTIONS / 8 bytes per pixel: R8Uint / R16Uint / R32Uint (SVAO.cpp:132-134)
    uint32_t* rayMin;
    uint32_t* rayMax;
    const float* sd;
    int sdW, sdH;
    uint32_t guard, secondary, rayInterval, sdJitter, N;
    uint32_t dual;  // DUAL_AO: ao holds (bright, dark) byte pairs (RG8Unorm)
    uint32_t bandIndex, bandCount;  // 32-row groups g (offset space) with g % count == index
    float isx, isy;  // imageScale (Common.slang:142), hoisted: 0.5 * (frameW / focal), same bits
    float risx, risy;  // 1 / isx, 1 / isy (fast numerics: view-to-uv through one reciprocal of p.z)
    float pzLo, pzHi;  // |p.z| in [pzLo, pzHi] keeps isx p.z and isy p.z in [2^-20, 2^20] (fill_scale)
    const float* snapU;  // getSnappedUV: snapU[k] = (k + 0.5f) / resolution.x for k in [0, resolution.x]
    const float* snapV;  //               snapV[k] = (k + 0.5f) / resolution.y
    const float4* nlut;  // decode_normal_2x8 of every 16-bit code (normal_lut), same bits
    uint32_t* tileFlags;  // rsd_svao_params.tile_flags: one word per busy 16x16 tile (tile_layout), or nullptr
    uint32_t* tileCount;  // the two list counts (after the flags): frame generations alternate between them
    uint32_t tileGen;     // 0 / 1: the count this pass appends to (pass 1) or walks (pass 2), svao.hip tile_gen
    uint32_t tileStamp;   // pass 1: the value it stores in a busy tile's flag (the generation + 1, never 0): a flag
                          // left set by an earlier generation no pass 2 consumed does not keep its tile out of
                          // this generation's list
    uint32_t* tileList;   // busy tiles in the order pass 1 found them (after the count)
    uint32_t tilesX;      // tiles per row of tileFlags
    uint32_t xcdChunk;   // pass 1 (A/B, RSD_PASS1_XCD): > 0 deals chunks of this many workgroups to the XCDs
                         // (workgroups b and b + 8 share an XCD, MI355X_MICROARCH.md "Workgroup dispatch"), so an
                         // XCD's L2 serves neighbouring tiles; 0: the dispatch order as launched
    uint32_t dualDepth;  // PRIMARY_DEPTH_MODE == DualDepth: depth2 refines the raster samples
    const float* depth2; // gDepthTex2 (DualDepth), W x H linear depth
};

constexpr uint32_t kTileEdge = 16;  // busy-tile flag granularity = the pass-2 workgroup tile
inline uint32_t tiles_x(uint32_t W, uint32_t guard) { return (W - 2 * guard + kTileEdge - 1) / kTileEdge; }
inline uint32_t tiles_y(uint32_t H, uint32_t guard) { return (H - 2 * guard + 31u) / 32u * 32u / kTileEdge; }
// the rsd_svao_params.tile_flags buffer (ABI v5) for T tiles: T flag words, {count[2], -, -}, T list
// entries -- rsd_svao_tile_count bytes, zeroed once by its owner
inline uint32_t tile_buffer_bytes(uint32_t T) { return T ? 8u * T + 16u : 0u; }
inline void tile_layout(uint8_t* base, uint32_t T, uint32_t*& flags, uint32_t*& count, uint32_t*& list) {
    flags = reinterpret_cast<uint32_t*>(base);
    count = base ? flags + T : nullptr;
    list = base ? flags + T + 4 : nullptr;
    if (!base) flags = nullptr;
}

struct Basic {
    f3 posV;
    float posVLength;
    f3 normal, tangent, bitangent, normalO, normalV;
    float radiusInPixels, radius;
    float nzRcp;  // rcp_refined(make_nonzero(normalO.z, 1e-4)): set by the all-fast pass-1 loop only
    float rScale, rScaleInv;  // fast numerics, SCALED all-fast loop: radius / VAOData.radius and its inverse
};

struct Sample {
    float sphereStart, sphereEnd, pdf;
    bool isInScreen;
    float su, sv;  // samplePosUV
    float ru, rv;  // rasterSamplePosUV
    int kx, ky;    // the pixel ru, rv is the centre of
    float visibility, objectSpaceZ;
    f3 ip;  // initialSamplePosV (the Raytraced mode needs its length)
    bool fast;             // the host reciprocals below apply (div_rcp)
    float yPdf, yHeight;   // RN(1 / pdf), RN(1 / sphereStart)
};

// RSD_FAST_NUMERICS (svao_fast.hip, svao_kernels.h): the division helpers below become one multiply by
// the hardware reciprocal (v_rcp_f32, 1 ulp) and their range tests constant true; the compiler contracts
// a * b + c into FMAs, '/' and sqrtf lower to v_rcp_f32 / v_sqrt_f32 and float32 denormals flush -- the
// arithmetic D3D permits the reference's HLSL.  Without it (svao.hip, svao_rt.hip): the exact contract.
#ifdef RSD_FAST_NUMERICS
constexpr bool kFastNumerics = true;
#else
constexpr bool kFastNumerics = false;
#endif

#ifdef RSD_FAST_NUMERICS
__device__ __forceinline__ float div_rcp(float a, float b, float y) { return a * y; }
__device__ __forceinline__ float rcp_refined(float b) { return __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ float div_unscaled(float a, float b, float y1) { return a * y1; }
__device__ __forceinline__ float div_unscaled_tail(float a, float b, float y1) { return a * y1; }
__device__ __forceinline__ bool div_unscaled_num_ok(float) { return true; }
__device__ __forceinline__ bool div_unscaled_den_ok(float) { return true; }
#else
// RN(a / b) for b > 0 given y = RN(1 / b), in five operations instead of the IEEE division's
// eleven (v_div_scale x2, v_rcp, 6 fma/mul, v_div_fmas, v_div_fixup).  q0 = RN(a y) is within
// 1.5 ulp of a / b; one residual step (r0 = a - b q0 exact by FMA) brings q1 within 1 ulp; then
// with r1 = a - b q1 (exact) Markstein's theorem (y within 1/2 ulp of 1/b, q1 within 1 ulp of
// a / b) makes RN(q1 + r1 y) = RN(a / b).  Preconditions, which every caller's operands meet:
// no underflow / overflow -- b in [2^-30, 2^30] (host-checked, SvaoConsts::fastDiv) and a = 0
// or |a| in [2^-60, 2^31] (the SVAO visibility numerators, see the callers).  a = +0 gives +0.
__device__ __forceinline__ float div_rcp(float a, float b, float y) {
    const float q0 = a * y;
    const float r0 = __builtin_fmaf(-q0, b, a);
    const float q1 = __builtin_fmaf(r0, y, q0);
    const float r1 = __builtin_fmaf(-q1, b, a);
    return __builtin_fmaf(r1, y, q1);
}

// The gfx950 IEEE binary32 division a / b is: v_div_scale of a and of b, v_rcp of the scaled b, two FMAs
// refining it (y1), q0 = a y1, two residual steps and v_div_fmas, then v_div_fixup.  Where neither the
// scaling nor the fixup acts -- b normal, |b| in [2^-20, 2^20], and a = 0 or |a| in [2^-100, 2^70]
// (exponent difference < 96, a / b and 1 / b normal, |a| >= 2^-103; finite normal operands) -- the
// quotient is that sequence's own value without them: div_unscaled(a, b, rcp_refined(b)), with the
// sign of q0 (the fixup's sign(a) ^ sign(b), which the residual steps lose for a = -0).  Same
// operations, same bits as a / b; a per-pixel divisor pays v_rcp and its refinement once.
__device__ __forceinline__ float rcp_refined(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
}
__device__ __forceinline__ float div_unscaled(float a, float b, float y1) {
    const float q0 = a * y1;
    const float r0 = __builtin_fmaf(-q0, b, a);
    const float q1 = __builtin_fmaf(r0, y1, q0);
    const float r1 = __builtin_fmaf(-q1, b, a);
    return __builtin_copysignf(__builtin_fmaf(r1, y1, q1), q0);
}
// div_unscaled without the sign fix of a zero quotient (callers for which +-0 give the same result)
__device__ __forceinline__ float div_unscaled_tail(float a, float b, float y1) {
    const float q0 = a * y1;
    const float r0 = __builtin_fmaf(-q0, b, a);
    const float q1 = __builtin_fmaf(r0, y1, q0);
    const float r1 = __builtin_fmaf(-q1, b, a);
    return __builtin_fmaf(r1, y1, q1);
}
// the numerator range of div_unscaled (false for NaN / inf)
__device__ __forceinline__ bool div_unscaled_num_ok(float a) {
    const float m = fabsf(a);
    return (m >= 0x1p-100f && m < 0x1p70f) || a == 0.0f;
}
__device__ __forceinline__ bool div_unscaled_den_ok(float b) {
    const float m = fabsf(b);
    return m >= 0x1p-20f && m <= 0x1p20f;
}
#endif  // RSD_FAST_NUMERICS

// n / pdf for n = 0 or n in (0, 2 * sphereHeight]: max(ss - max(se, oz), 0) (>= ulp(ss) / 2 when
// non-zero), ss - se (> 0.2 h after the validity test), saturate(x / ss) * (ss - se)
__device__ __forceinline__ float div_pdf(float n, const Sample& s) {
    return s.fast ? div_rcp(n, s.pdf, s.yPdf) : n / s.pdf;
}

// saturate(x / sphereStart) for x > 0 (calcHaloVisibility): x >= ss gives 1 exactly (x / ss >= 1
// rounds to >= 1); 0 < x < ss is oz - (1 + thickness) r > 0, at least ulp(r) / 2
__device__ __forceinline__ float halo_ratio(float x, const Sample& s) {
    if (s.fast) return x >= s.sphereStart ? 1.0f : saturate(div_rcp(x, s.sphereStart, s.yHeight));
    return saturate(x / s.sphereStart);
}

__device__ __forceinline__ f3 uv_to_view(const SvaoArgs& a, float u, float v, float z) {
    const float ndcx = u * 2.0f - 1.0f, ndcy = (1.0f - v) * 2.0f - 1.0f;
    return mk(ndcx * z * a.isx, ndcy * z * a.isy, -z);
}

__device__ __forceinline__ void view_to_uv(const SvaoArgs& a, f3 p, float& u, float& v) {
    const float ndcx = p.x / (a.isx * p.z), ndcy = p.y / (a.isy * p.z);
    u = ndcx * -0.5f + 0.5f;
    v = ndcy * 0.5f + 0.5f;
}

__device__ __forceinline__ float depth_sample(const SvaoArgs& a, float u, float v) {
    return tex_bilinear(a.depth, a.W, a.H, u, v, false);  // gTextureSampler: linear, clamp
}

// The depth at the centre uv of pixel (kx, ky) (Init's uv, getSnappedUV's rasterSamplePosUV).
// The bilinear filter there resolves to the single texel (kx, ky): uv * size lands within
// (kx + 0.5) +- size * 2^-22, and an offset below 1/512 rounds the 8-bit weights to 0 (or to
// 256 of the next texel, tex_bilinear's carry), so for frames up to 4096 px the fetch is
// direct -- no dependency on the uv arithmetic or the snap-table loads.
// SMALL: the caller guarantees W, H <= 4096 (a specialised kernel: no run-time size test)
template <bool SMALL = false>
__device__ __forceinline__ float depth_center(const SvaoArgs& a, float u, float v, int kx, int ky) {
    if (SMALL || (a.W <= 4096 && a.H <= 4096))
        return a.depth[(size_t)min(max(ky, 0), a.H - 1) * a.W + min(max(kx, 0), a.W - 1)];
    return depth_sample(a, u, v);
}

// Buffer resources of the specialised pass-1 direction loop (gfx9 raw buffers, CK's word-3 flags): the
// snap-table and depth gathers take a 32-bit byte offset from one VALU op instead of 64-bit address
// arithmetic.  The offsets are always inside the buffers (kx in [0, resolution.x], clamped depth texel).
struct P1Bufs {
    __amdgpu_buffer_rsrc_t depth, snapU, snapV;
};
// (the record count only bounds offsets, which are in range here: the maximum keeps the descriptor a
// function of the kernel-argument pointer alone, i.e. in SGPRs -- a count computed in VALU made the
// compiler wrap every load in a readfirstlane loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_buffer(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float buf_load(__amdgpu_buffer_rsrc_t r, uint32_t byteOff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)byteOff, 0, 0));
}
__device__ __forceinline__ P1Bufs p1_bufs(const SvaoArgs& a) {
    P1Bufs b;
    b.depth = raw_buffer(a.depth);
    b.snapU = raw_buffer(a.snapU);
    b.snapV = raw_buffer(a.snapV);
    return b;
}
// depth_center of the specialised kernels (W, H <= 4096): kx, ky >= 0 (floor of a saturated uv)
__device__ __forceinline__ float depth_center_buf(const SvaoArgs& a, const P1Bufs& bf, int kx, int ky) {
    const uint32_t x = min((uint32_t)kx, (uint32_t)a.W - 1u), y = min((uint32_t)ky, (uint32_t)a.H - 1u);
    return buf_load(bf.depth, (y * (uint32_t)a.W + x) * 4u);
}

// the AO of pixel o: one R8Unorm byte, or the (bright, dark) RG8Unorm pair with DUAL_AO
__device__ __forceinline__ void ao_store(const SvaoArgs& a, size_t o, float bright, float dark) {
    if (a.dual) reinterpret_cast<uchar2*>(a.ao)[o] = make_uchar2(unorm8(bright), unorm8(dark));
    else a.ao[o] = unorm8(bright);
}
// Common.slang:326-330 finalize: HBAO maps the average to saturate(1 - 2 avg), then pow(exponent)
__device__ __forceinline__ float ao_finalize(const SvaoArgs& a, float avg) {
    if (a.k.hbao) avg = saturate(1.0f - 2.0f * avg);
    return acc_pow(avg, a.d.exponent);
}

// pass 2's (and the Raytraced pass 2's) end of a refined pixel, SVAORaster2.ps.slang:60-64: the
// direction sums (bright: sum of refined - raster visibility; dark: sum of refined) scaled by
// 2 / NUM_DIRECTIONS (Common.slang:660-661), plus the pass-1 AO (prev: the pixel's (bright, dark)
// bytes as pass 1 stored them), dark = min(bright, dark), finalize
__device__ __forceinline__ void ao_finish(const SvaoArgs& a, size_t o, float accB, float accD, uchar2 prev) {
    float vb = accB;
    vb *= a.k.invNd;
    if (!a.k.hbao) vb *= 2.0f;  // Common.slang:661: VAO only
    if (!a.dual) {
        vb += unorm8_to_float(prev.x);
        a.ao[o] = unorm8(ao_finalize(a, vb));
        return;
    }
    float vd = accD;
    vd *= a.k.invNd;
    if (!a.k.hbao) vd *= 2.0f;
    vb += unorm8_to_float(prev.x);
    vd += unorm8_to_float(prev.y);
    vd = hmin(vb, vd);
    reinterpret_cast<uchar2*>(a.ao)[o] = make_uchar2(unorm8(ao_finalize(a, vb)), unorm8(ao_finalize(a, vd)));
}

// the stencil bitmask of pixel o (one bit per direction)
__device__ __forceinline__ uint32_t stencil_load(const SvaoArgs& a, size_t o) {
    if (a.k.nd == 32u) return reinterpret_cast<const uint32_t*>(a.stencil)[o];
    if (a.k.nd == 16u) return reinterpret_cast<const uint16_t*>(a.stencil)[o];
    return a.stencil[o];
}
__device__ __forceinline__ void stencil_store(const SvaoArgs& a, size_t o, uint32_t m) {
    if (a.k.nd == 32u) reinterpret_cast<uint32_t*>(a.stencil)[o] = m;
    else if (a.k.nd == 16u) reinterpret_cast<uint16_t*>(a.stencil)[o] = (uint16_t)m;
    else a.stencil[o] = (uint8_t)m;
}

// the reads of basic_init: the pixel's depth and its packed normal (0 outside the frame)
template <bool SMALL = false>
__device__ __forceinline__ void basic_reads(const SvaoArgs& a, float u, float v, float& z, uint32_t& packed) {
    const rsd_vao_data& d = a.d;
    z = depth_center<SMALL>(a, u, v, (int)(u * d.resolution[0]), (int)(v * d.resolution[1]));
    const uint32_t ix = (uint32_t)(u * d.resolution[0]), iy = (uint32_t)(v * d.resolution[1]);
    packed = (ix < (uint32_t)a.W && iy < (uint32_t)a.H) ? a.normals[(size_t)iy * a.W + ix] : 0u;
}

// Common.slang:285-324 from the reads above (z, nl = decode_normal_2x8(packed) from the device table)
// noise: null, or an LDS copy of the 16 noise sines then the 16 cosines (pass 2's specialised tiles)
__device__ __forceinline__ bool basic_from(const SvaoArgs& a, float u, float v, float z, float4 nl, Basic& b,
                                           const float* noise = nullptr);

// Common.slang:285-324
template <bool SMALL = false>
__device__ __forceinline__ bool basic_init(const SvaoArgs& a, float u, float v, Basic& b, const float* noise = nullptr) {
    float z;
    uint32_t packed;
    basic_reads<SMALL>(a, u, v, z, packed);
    return basic_from(a, u, v, z, a.nlut[packed], b, noise);  // nlut = decode_normal_2x8, tabulated on the device
}

__device__ __forceinline__ bool basic_from(const SvaoArgs& a, float u, float v, float z, float4 nl, Basic& b,
                                           const float* noise) {
    const rsd_vao_data& d = a.d;
    float rux, ruy;
    if constexpr (kFastNumerics) {  // one hardware reciprocal of the pixel's depth for both radii
        const float rz = __builtin_amdgcn_rcpf(z);
        rux = (d.radius * a.cam.focalLength) * __builtin_amdgcn_rcpf(a.cam.frameWidth) * rz;
        ruy = (d.radius * a.cam.focalLength) * __builtin_amdgcn_rcpf(a.cam.frameHeight) * rz;
    } else {
        rux = (d.radius * a.cam.focalLength) / (a.cam.frameWidth * z);
        ruy = (d.radius * a.cam.focalLength) / (a.cam.frameHeight * z);
    }
    const float pa = rux * d.resolution[0], pb = ruy * d.resolution[1];
    b.radiusInPixels = pa + 0.5f * (pb - pa);
    b.radius = d.radius;
    const float maxRadius = d.ssMaxRadius;
    if (b.radiusInPixels > maxRadius) {
        b.radius = b.radius / b.radiusInPixels * maxRadius;
        b.radiusInPixels = maxRadius;
    }
    if (b.radiusInPixels < 0.5f) return false;
    b.posV = uv_to_view(a, u, v, z);
    b.posVLength = length(b.posV);
    b.normalV = mk(nl.x, nl.y, nl.z);
    if (dot(b.posV, b.normalV) > 0.0f) b.normalV = -b.normalV;
    const float nu = u * d.noiseScale[0], nv = v * d.noiseScale[1];
    const int ni = ((int)floorf(nu * 4.0f)) & 3, nj = ((int)floorf(nv * 4.0f)) & 3;
    const f3 rd = noise ? mk(noise[nj * 4 + ni], noise[16 + nj * 4 + ni], 0.0f)
                        : mk(a.k.sinNoise[nj * 4 + ni], a.k.cosNoise[nj * 4 + ni], 0.0f);
    if constexpr (kFastNumerics) {
        const float il = __builtin_amdgcn_rcpf(b.posVLength);
        b.normal = mk(-b.posV.x * il, -b.posV.y * il, -b.posV.z * il);
    } else {
        b.normal = mk(-b.posV.x / b.posVLength, -b.posV.y / b.posVLength, -b.posV.z / b.posVLength);
    }
    b.bitangent = normalize(cross(b.normal, rd));
    b.tangent = cross(b.bitangent, b.normal);
    b.normalO = mk(dot(b.normalV, b.tangent), dot(b.normalV, b.bitangent), dot(b.normalV, b.normal));
    return true;
}

// the SCALED all-fast loop's per-pixel factors (fast numerics): exactly 1 for an unclamped pixel
__device__ __forceinline__ void set_radius_scale(const SvaoArgs& a, Basic& b) {
    const bool unclamped = b.radius == a.d.radius;
    b.rScale = unclamped ? 1.0f : b.radius * a.k.rcpRadius;
    b.rScaleInv = unclamped ? 1.0f : a.d.radius * __builtin_amdgcn_rcpf(b.radius);
}

__device__ __forceinline__ float make_nonzero(float v, float eps) {
    const float av = hmax(fabsf(v), eps);
    return v >= 0.0f ? av : -av;
}

// Common.slang:354-399 (VAO kernel)
// RN(n / D) <= 0.1f for n >= 0, D >= 0 (Common.slang:378), without the division: 0.1f has an odd
// significand, so RN(q) <= 0.1f <=> q < M = 0.1f + ulp(0.1f) / 2 (a tie rounds up, to even), and
// for D > 0 q < M <=> n < M * D, a product of 25- and 24-bit significands: exact in double.
// D = 0 gives +inf / NaN in the reference (never <= 0.1): n < 0 is false here as well.
__device__ __forceinline__ bool ratio_le_tenth(float n, float D) {
#ifdef RSD_FAST_NUMERICS
    return n * __builtin_amdgcn_rcpf(D) <= 0.1f;  // the reference's (n / D) <= 0.1 with a 1-ulp '/'
#else
    constexpr double M = (double)0.1f + 0x1p-28;
    return (double)n < M * (double)D;
#endif
}

// ssrAbove = (screenSpaceRadius > ssRadiusCutoff), decided on the squared radius (no sqrt).
// ALLFAST: the caller guarantees b.radius == VAOData.radius and every fastDiv bit (the host terms
// and div_rcp apply; a wave-uniform case of the specialised pass 1)
// VAO: the caller is a VAO-only (specialised) kernel -- the HBAO branches compile away
// SCALED (fast numerics only, with ALLFAST): the pixel's radius may be clamped to ssMaxRadius; every
// radius-dependent term of the direction is linear in it (Common.slang:358-365: radius_i = r_i R,
// sphereHeight = R sqrt(1 - r_i^2), pdf = 2 sphereHeight), so the host terms at VAOData.radius are
// scaled by b.rScale = R / VAOData.radius (1 exactly when unclamped) -- the rounding differs from the
// reference's order of operations by a few ulp, inside the fast-numerics tolerance
// KL > 0 (with ALLFAST): the direction terms come from an LDS copy kl[6][KL] (dirDx, dirDy, dirHeight, rcpPdf,
// rcpHeight, ratioMin) -- pass 2, whose lanes hold different directions: the kernel-argument tables would be
// per-lane vector loads, one more dependent memory round trip per pair
template <bool ALLFAST = false, bool VAO = false, bool SCALED = false, int KL = 0>
__device__ __forceinline__ bool sample_init(const SvaoArgs& a, float u, float v, const Basic& b, int i, Sample& s,
                                            bool& ssrAbove, const P1Bufs* bf = nullptr, const float* kl = nullptr) {
    const rsd_vao_data& d = a.d;
    float radius, dx, dy, sphereHeight;
    s.fast = false;
    float ratioMin = 0.0f;
    if (ALLFAST) {
        radius = a.k.dirRadius[i];
        s.fast = true;
        if constexpr (KL > 0) {
            dx = kl[i];
            dy = kl[KL + i];
            sphereHeight = kl[2 * KL + i];
            s.yPdf = kl[3 * KL + i];
            s.yHeight = kl[4 * KL + i];
            ratioMin = kl[5 * KL + i];
        } else {
            dx = a.k.dirDx[i];
            dy = a.k.dirDy[i];
            sphereHeight = a.k.dirHeight[i];
            s.yPdf = a.k.rcpPdf[i];
            s.yHeight = a.k.rcpHeight[i];
            ratioMin = a.k.ratioMin[i];
        }
        if constexpr (SCALED) {
            dx *= b.rScale;
            dy *= b.rScale;
            sphereHeight *= b.rScale;
            s.yPdf *= b.rScaleInv;
            s.yHeight *= b.rScaleInv;
            ratioMin *= b.rScale;
        }
    } else if (b.radius == d.radius) {  // the host-evaluated terms (same operations, same bits)
        radius = a.k.dirRadius[i];
        dx = a.k.dirDx[i];
        dy = a.k.dirDy[i];
        sphereHeight = a.k.dirHeight[i];
        s.fast = (a.k.fastDiv >> i) & 1u;
        s.yPdf = a.k.rcpPdf[i];
        s.yHeight = a.k.rcpHeight[i];
    } else {
        radius = a.k.sampleRadius[i] * b.radius;
        dx = radius * a.k.sinDir[i];
        dy = radius * a.k.cosDir[i];
        sphereHeight = sqrtf(b.radius * b.radius - radius * radius);
    }
    s.pdf = (!VAO && a.k.hbao) ? a.k.pdfHbao[i] : 2.0f * sphereHeight;  // Common.slang:362-365
    s.sphereStart = sphereHeight;
    float zi;  // ALLFAST: the validity test below is one compare against the host bound ratioMin
    if (ALLFAST) {  // the pixel's divisor is in div_unscaled's range (checked with ALLFAST)
        const float num = -(dx * b.normalO.x + dy * b.normalO.y), den = make_nonzero(b.normalO.z, 0.0001f);
        zi = (kFastNumerics || __ballot(!div_unscaled_num_ok(num)) == 0u) ? div_unscaled(num, den, b.nzRcp) : num / den;
    } else {
        zi = -(dx * b.normalO.x + dy * b.normalO.y) / make_nonzero(b.normalO.z, 0.0001f);
    }
    s.sphereEnd = hmin(hmax(zi, -sphereHeight), sphereHeight);
    // (sphereStart - sphereEnd is never NaN: hmax maps a NaN zi to -sphereHeight)
    if (ALLFAST ? !(s.sphereStart - s.sphereEnd >= ratioMin)
                : ratio_le_tenth(s.sphereStart - s.sphereEnd, 2.0f * sphereHeight))
        return false;
    const f3 ip = b.posV + b.tangent * dx + b.bitangent * dy;
    s.ip = ip;
    // ALLFAST: the two view-to-uv divisions through div_unscaled when every lane's p.z keeps both
    // divisors in [2^-20, 2^20].  Exact for |p.x|, |p.y| in [2^-100, 2^70] (|posV| < 2^60 per pixel, the
    // sample offset < radius); a smaller numerator gives |x / den| < 2^-80, and then u = x / den * -0.5 +
    // 0.5 rounds to 0.5 whichever tiny quotient the sequence returns, and su is all that is used of it.
    if (ALLFAST && kFastNumerics) {  // x / (isx z) = x (1 / isx) (1 / z): one hardware reciprocal for both
        const float rz = __builtin_amdgcn_rcpf(ip.z);
        s.su = (ip.x * a.risx * rz) * -0.5f + 0.5f;
        s.sv = (ip.y * a.risy * rz) * 0.5f + 0.5f;
    } else if (ALLFAST && __ballot(!(fabsf(ip.z) >= a.pzLo && fabsf(ip.z) <= a.pzHi)) == 0u) {
        const float dx2 = a.isx * ip.z, dy2 = a.isy * ip.z;
        const float ndcx = div_unscaled_tail(ip.x, dx2, rcp_refined(dx2));
        const float ndcy = div_unscaled_tail(ip.y, dy2, rcp_refined(dy2));
        s.su = ndcx * -0.5f + 0.5f;
        s.sv = ndcy * 0.5f + 0.5f;
    } else {
        view_to_uv(a, ip, s.su, s.sv);
    }
    s.visibility = 0.0f;
    s.objectSpaceZ = 0.0f;
    const float ex = (u - s.su) * d.resolution[0], ey = (v - s.sv) * d.resolution[1];
    ssrAbove = ex * ex + ey * ey >= a.k.ssrMin2;
    // ALLFAST: saturate as fmin(fmax(x, 0), 1) (NaN -> 0 as well); it may differ from saturate only in
    // the sign of a zero, which neither use of cu below can see (-0 == +0; floor(+-0 * res) = 0)
    const float cu = ALLFAST ? fminf(fmaxf(s.su, 0.0f), 1.0f) : saturate(s.su);
    const float cv = ALLFAST ? fminf(fmaxf(s.sv, 0.0f), 1.0f) : saturate(s.sv);
    s.isInScreen = (s.su == cu) && (s.sv == cv);
    // getSnappedUV (Common.slang:116-120): (floor(uv * res) + 0.5) / res from the host table
    s.kx = (int)floorf(cu * d.resolution[0]);
    s.ky = (int)floorf(cv * d.resolution[1]);
    if (kFastNumerics) {  // (k + 0.5) / res with the hardware reciprocal: no table loads
        s.ru = ((float)s.kx + 0.5f) * d.invResolution[0];
        s.rv = ((float)s.ky + 0.5f) * d.invResolution[1];
    } else if (bf) {
        s.ru = buf_load(bf->snapU, (uint32_t)s.kx * 4u);
        s.rv = buf_load(bf->snapV, (uint32_t)s.ky * 4u);
    } else {
        s.ru = a.snapU[s.kx];
        s.rv = a.snapV[s.ky];
    }
    return true;
}

// Common.slang:180-184 calcHaloVisibility (HALO_RADIUS = sphereStart, Common.slang:38)
__device__ __forceinline__ float calc_halo_visibility(const rsd_vao_data& d, float oz, float ss, float se, float pdf,
                                                      float radius) {
    return saturate((oz - (1.0f + d.thickness) * radius) / ss) * (ss - se) / pdf;
}

// Common.slang:180-196
__device__ __forceinline__ float calc_visibility(const rsd_vao_data& d, float oz, float ss, float se, float pdf,
                                                 float radius) {
    const float sphere = hmax(ss - hmax(se, oz), 0.0f) / pdf;
    // saturate(x / ss) with ss > 0 is +0 for x <= 0 (and for NaN), so the halo term is then
    // exactly +0 * (ss - se) / pdf = +0: its two divisions are skipped
    const float x = oz - (1.0f + d.thickness) * radius;
    const float halo = x > 0.0f ? saturate(x / ss) * (ss - se) / pdf : 0.0f;
    return sphere + halo;
}

// calc_visibility of a Sample (same bits; divisions by its pdf / sphereStart via div_rcp)
__device__ __forceinline__ float sample_visibility(const rsd_vao_data& d, float oz, const Sample& s, float radius) {
    const float sphere = div_pdf(hmax(s.sphereStart - hmax(s.sphereEnd, oz), 0.0f), s);
    const float x = oz - (1.0f + d.thickness) * radius;
    const float halo = x > 0.0f ? div_pdf(halo_ratio(x, s) * (s.sphereStart - s.sphereEnd), s) : 0.0f;
    return sphere + halo;
}

// Common.slang:421-430 HBAOKernel (gData.radius: the VAOData radius, not the pixel's clamped one)
__device__ __forceinline__ float hbao_kernel(const SvaoArgs& a, const Basic& b, f3 S) {
    const f3 V = S - b.posV;
    const float angleTerm = saturate(dot(b.normalV, normalize(V)) - 0.1f);  // NdotVBias
    const float distanceTerm = saturate(1.0f - dot(V, V) / (a.d.radius * a.d.radius));
    return angleTerm * distanceTerm;
}

// Common.slang:463-483: VAO -- min of calcVisibility; HBAO -- max of saturate(HBAOKernel / pdf)
template <bool VAO = false>
__device__ __forceinline__ void add_sample(const SvaoArgs& a, const Basic& b, Sample& s, f3 spV, bool init) {
    const float oz = dot(spV - b.posV, b.normal);
    s.objectSpaceZ = init ? oz : hmin(s.objectSpaceZ, oz);
    if (!VAO && a.k.hbao) {
        const float v = saturate(hbao_kernel(a, b, spV) / s.pdf);
        s.visibility = init ? v : hmax(s.visibility, v);
        return;
    }
    const float vis = sample_visibility(a.d, oz, s, b.radius);
    s.visibility = init ? vis : hmin(s.visibility, vis);
}

// Common.slang:455-461 requireRay: VAO (CONST_RADIUS, Common.slang:37) or HBAO
__device__ __forceinline__ bool require_ray(const SvaoArgs& a, const Basic& b, const Sample& s, bool ssrAbove) {
    if (a.k.hbao) return s.objectSpaceZ > hmax(s.sphereStart, b.radius * 0.1f) && ssrAbove;
    const float constRadius = (1.0f + a.d.thickness) * b.radius - s.sphereStart;
    return s.objectSpaceZ > s.sphereStart + constRadius && ssrAbove;
}

// Common.slang:498-505 evalDualVisibility: the second depth layer at the raster sample's texel, only
// where the sample still requires a ray
__device__ __forceinline__ void eval_dual(const SvaoArgs& a, const Basic& b, Sample& s, bool ssrAbove, bool init) {
    if (!require_ray(a, b, s, ssrAbove)) return;
    const float z = (a.W <= 4096 && a.H <= 4096)
                        ? a.depth2[(size_t)min(max(s.ky, 0), a.H - 1) * a.W + min(max(s.kx, 0), a.W - 1)]
                        : tex_bilinear(a.depth2, a.W, a.H, s.ru, s.rv, false);
    add_sample(a, b, s, uv_to_view(a, s.ru, s.rv, z), init);
}


// Common.slang:492-496
template <bool SMALL = false, bool VAO = false>
__device__ __forceinline__ void eval_primary(const SvaoArgs& a, const Basic& b, Sample& s, const P1Bufs* bf = nullptr) {
    const float z = bf ? depth_center_buf(a, *bf, s.kx, s.ky) : depth_center<SMALL>(a, s.ru, s.rv, s.kx, s.ky);
    add_sample<VAO>(a, b, s, uv_to_view(a, s.ru, s.rv, z), true);
}

// Common.slang:164-168
__device__ __forceinline__ int uv_to_sd(float uv, float low, int guard) {
    const int p = (int)floorf(uv * low) + guard;
    const int hi = (int)low + guard * 2 - 1;
    return p < 0 ? 0 : (p > hi ? hi : p);
}

inline void fill_scale(SvaoArgs& a) {
    // Common.slang:142/150 imageScale, evaluated once on the host (IEEE float, same bits)
    a.isx = 0.5f * (a.cam.frameWidth / a.cam.focalLength);
    a.isy = 0.5f * (a.cam.frameHeight / a.cam.focalLength);
    a.risx = a.isx != 0.0f ? 1.0f / a.isx : 0.0f;
    a.risy = a.isy != 0.0f ? 1.0f / a.isy : 0.0f;
    // with a factor-2 margin for the rounding of isx * p.z (0 when the scales are not finite and positive)
    const double lo = std::min(a.isx, a.isy), hi = std::max(a.isx, a.isy);
    const bool ok = lo > 0.0 && hi < 1e30;
    a.pzLo = ok ? (float)(0x1p-19 / lo) : INFINITY;
    a.pzHi = ok ? (float)(0x1p19 / hi) : 0.0f;
}

inline void fill_consts(SvaoConsts& k, const rsd_vao_data& d, uint32_t nd, uint32_t kernel = RSD_AO_KERNEL_VAO) {
    // SVAO.cpp:670-684 -> R8Unorm noise; Common.slang:311-312 randRotation, :357 alpha
    static const float dither[16] = {0.0f, 8.0f, 2.0f, 10.0f, 12.0f, 4.0f, 14.0f, 6.0f,
                                     3.0f, 11.0f, 1.0f, 9.0f, 15.0f, 7.0f, 13.0f, 5.0f};
    for (int i = 0; i < 16; ++i) {
        const uint8_t byte = (uint8_t)(dither[i] / 16.0f * 255.0f);
        const float rr = (float)byte / 255.0f * 2.0f * 3.141f;
        k.sinNoise[i] = (float)std::sin((double)rr);
        k.cosNoise[i] = (float)std::cos((double)rr);
    }
    // Common.slang:52-58 (VAO kernel): the 16 / 32 tables are double literals there, rounded to float
    static const float radius8[8] = {0.917883f, 0.564429f, 0.734504f, 0.359545f,
                                     0.820004f, 0.470149f, 0.650919f, 0.205215f};
    static const float radius16[16] = {
        0.949098221604059, 0.5865639019441775, 0.7554681720909893, 0.3895439574863043,
        0.8425560503012255, 0.4948003867747738, 0.6719196866381647, 0.25203100417434543,
        0.8908588816103737, 0.5418210823278604, 0.7136427497994143, 0.32724136087586453,
        0.7980920320691521, 0.4445340224611676, 0.6297373536812639, 0.1447182620692375,
    };
    static const float radius32[32] = {
        0.9682458365518543, 0.5974803093982587, 0.7660169295429302, 0.4038472576817624,
        0.8541535023444914, 0.5068159098187986, 0.6823727109604635, 0.2726076670970059,
        0.904018191941786, 0.5531894754180758, 0.7240656647095169, 0.34372202910162664,
        0.8089818132350507, 0.45747336127867605, 0.640354849019649, 0.17748061996818404,
        0.9327350969376332, 0.5755500192397054, 0.7449678114312224, 0.37479566486456295,
        0.8311856199411515, 0.4825843210309559, 0.6614378277661477, 0.22975243551455923,
        0.878233108646881, 0.5303115209931901, 0.7032256306171377, 0.3099952198410562,
        0.7873133907642258, 0.43130429537268, 0.6190581352335289, 0.10219580968897692,
    };
    // Common.slang:60-66 (HBAO kernel), double literals rounded to float
    static const float hbao8[8] = {0.019897607325877215, 0.3239192018939078, 0.15013283288204182, 0.5608856339193332,
                                   0.07874804859295396, 0.4306374970658152, 0.23159241868180838, 0.74770696488701};
    static const float hbao16[16] = {
        0.008364792005390745, 0.29968419137477154, 0.13131974798930376, 0.5251597224509892,
        0.06264063727314514, 0.40226410430222115, 0.21027995621089465, 0.6906178807859765,
        0.03303993608633204, 0.34903099295095424, 0.16956281924775551, 0.5996160679614535,
        0.09559795810145842, 0.46040865279052423, 0.25357218870257175, 0.8218290863578166,
    };
    static const float hbao32[32] = {
        0.0035168784979124203, 0.28787249889929795, 0.12214740408236834, 0.5082189968610005,
        0.05489041689357717, 0.38854375322009427, 0.19986558164830323, 0.6656225173745592,
        0.02630214826181389, 0.33636038195532914, 0.15977097044845298, 0.579825376399601,
        0.08708424832212604, 0.44533522627083877, 0.24249692822679572, 0.7816464549941924,
        0.013886447731081395, 0.3116969449839127, 0.14064876764650994, 0.5426920213922799,
        0.07059703986067731, 0.41628837439340993, 0.22085459126773643, 0.7177502077720759,
        0.04006955250785802, 0.36194276200351894, 0.17950859741413544, 0.6203897476558216,
        0.10428292232859922, 0.47588885313824597, 0.2648228762567681, 0.8740952987729764,
    };
    k.nd = nd == 16u || nd == 32u ? nd : 8u;
    k.invNd = 1.0f / (float)k.nd;
    k.hbao = kernel == RSD_AO_KERNEL_HBAO ? 1u : 0u;
    const float* radius = k.hbao ? (k.nd == 32u ? hbao32 : k.nd == 16u ? hbao16 : hbao8)
                                 : (k.nd == 32u ? radius32 : k.nd == 16u ? radius16 : radius8);
    for (int i = 0; i < (int)k.nd; ++i) {
        const float al = ((float)i / (float)k.nd) * 2.0f * 3.141f;  // Common.slang:357
        k.sinDir[i] = (float)std::sin((double)al);
        k.cosDir[i] = (float)std::cos((double)al);
        k.sampleRadius[i] = radius[i];
        // Common.slang:358-361 at radius = VAOData.radius (float ops as on the device)
        k.dirRadius[i] = k.sampleRadius[i] * d.radius;
        k.dirDx[i] = k.dirRadius[i] * k.sinDir[i];
        k.dirDy[i] = k.dirRadius[i] * k.cosDir[i];
        k.dirHeight[i] = std::sqrt(d.radius * d.radius - k.dirRadius[i] * k.dirRadius[i]);
        // pow of a float in double, rounded once (rsd_device.h numerics contract)
        k.pdfHbao[i] = 0.9f * (float)std::pow((double)(1.0f - k.sampleRadius[i]), 1.5);
    }
    // sqrtf is correctly rounded and monotone: the least x with sqrtf(x) > c
    const float c = d.ssRadiusCutoff;
    float x = (float)((double)c * (double)c);
    while (x > 0.0f && std::sqrt(std::nextafter(x, 0.0f)) > c) x = std::nextafter(x, 0.0f);
    while (!(std::sqrt(x) > c)) x = std::nextafter(x, INFINITY);
    k.ssrMin2 = x;
    // div_rcp reciprocals: RN(RN64(1 / b)) = RN(1 / b) (double rounding is innocuous for a
    // quotient when 53 >= 2 * 24 + 2)
    // isSamePixel (Common.slang:129-133): |texC - rasterSamplePosUV| < 0.9 / res per axis.  Both
    // uvs are pixel centres within a few ulp (<= 2^-22 for uv < 2) of (k + 0.5) / res, so the test
    // holds exactly when the pixel indices agree (difference < 2^-21 << 0.9 / res) and fails when
    // they differ (difference >= 1 / res - 2^-21 > 0.9 / res) for res <= 2^18
    k.samePixelInt = d.resolution[0] <= 262144.0f && d.resolution[1] <= 262144.0f;
    k.rcpRadius = d.radius > 0.0f ? (float)(1.0 / (double)d.radius) : 0.0f;
    k.fastDiv = 0u;
    for (int i = 0; i < (int)k.nd; ++i) {
        const float pdf = 2.0f * k.dirHeight[i], h = k.dirHeight[i];
        k.rcpPdf[i] = (float)(1.0 / (double)pdf);
        k.rcpHeight[i] = (float)(1.0 / (double)h);
        // (HBAO divides by its own pdf and takes no div_rcp path: no fast bits)
        const bool ok = !k.hbao && h >= 0x1p-30f && pdf <= 0x1p30f;
        if (ok) k.fastDiv |= 1u << i;
        // ratio_le_tenth(n, D) is n < M D in exact arithmetic (M D exact in double): valid iff
        // n >= M D iff n >= the least float >= M D
        const double bound = ((double)0.1f + 0x1p-28) * (double)pdf;
        float t = (float)bound;
        if ((double)t < bound) t = std::nextafter(t, INFINITY);
        k.ratioMin[i] = t;
    }
}

// getSnappedUV tables for a frame size (device copies cached per thread, grow-only)
rsd_status snap_tables(const rsd_vao_data& d, const float** u, const float** v);
// decode_normal_2x8 for all 65536 codes, computed by a device kernel (bit-identical), cached
rsd_status normal_lut(const float4** out);

inline rsd_status check_common(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                               const float* depth, const uint16_t* normals, uint32_t W, uint32_t H, const char* who) {
    if (!cam || !vao || !p || !depth || !normals || W == 0 || H == 0) {
        set_error(std::string(who) + ": null argument or empty extent");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->num_directions != 8 && p->num_directions != 16 && p->num_directions != 32) {
        // Common.slang:51-58 holds sample radii for 8, 16 and 32 directions only
        set_error(std::string(who) + ": NUM_DIRECTIONS must be 8, 16 or 32");
        return RSD_ERR_UNSUPPORTED;
    }
    if (p->ao_kernel != RSD_AO_KERNEL_VAO && p->ao_kernel != RSD_AO_KERNEL_HBAO) {
        set_error(std::string(who) + ": ao_kernel must be RSD_AO_KERNEL_VAO or RSD_AO_KERNEL_HBAO");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->primary_depth_mode > 1 || (p->primary_depth_mode == 1 && !p->d_depth2)) {
        set_error(std::string(who) + ": primary_depth_mode must be 0 (SingleDepth) or 1 (DualDepth with d_depth2)");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->numerics != RSD_NUMERICS_FAST && p->numerics != RSD_NUMERICS_EXACT) {
        set_error(std::string(who) + ": numerics must be RSD_NUMERICS_FAST or RSD_NUMERICS_EXACT");
        return RSD_ERR_INVALID_ARG;
    }
    if (2 * p->guard_band >= W || 2 * p->guard_band >= H) {
        set_error(std::string(who) + ": guard band leaves no visible region");
        return RSD_ERR_INVALID_ARG;
    }
    return RSD_OK;
}

}  // namespace rsd
