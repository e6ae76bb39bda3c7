// svao.hip -- SVAO "AO 1" and "AO 2" compute passes on gfx950.
//
// Reference: SVAORaster.ps.slang:29-122 (pass 1), SVAORaster2.ps.slang:48-65 (pass 2),
//            SVAO/Common.slang:98-663 (BasicAOData / SampleAOData / calcAO2),
//            SVAO.cpp:327-354 (clears + pass-1 dispatch), :450-454 (pass-2 dispatch),
//            SVAO.cpp:663-688 (noise texture).
// Both passes are screen-space, HBM/L2-bound: pass 1 does ~10 depth fetches per pixel and
// two device-scope integer atomics per refined direction; pass 2 gathers popc(mask) x N
// SD depths at texels up to ssMaxRadius away.  Per-pixel transcendentals are tables
// (16 noise angles, 8 direction angles) computed on the host in double and rounded once;
// the only per-pixel libm call left is pow() in finalize (SVAO Common.slang:326-330).
#include <cfloat>
#include <cmath>

#include "rsd_device.h"
#include "rsd_internal.h"

namespace rsd {

struct SvaoConsts {
    float sinNoise[16], cosNoise[16];
    float sinDir[8], cosDir[8];
    float sampleRadius[8];
};

struct SvaoArgs {
    rsd_camera cam;
    rsd_vao_data d;
    SvaoConsts k;
    const float* depth;
    const uint16_t* normals;
    int W, H;
    uint8_t* ao;
    uint8_t* stencil;
    uint32_t* rayMin;
    uint32_t* rayMax;
    const float* sd;
    int sdW, sdH;
    uint32_t guard, secondary, rayInterval, sdJitter, N;
    uint32_t bandIndex, bandCount;  // 32-row groups g (offset space) with g % count == index
    float isx, isy;  // imageScale (Common.slang:142), hoisted: 0.5 * (frameW / focal), same bits
};

struct Basic {
    f3 posV;
    float posVLength;
    f3 normal, tangent, bitangent, normalO, normalV;
    float radiusInPixels, radius;
};

struct Sample {
    float sphereStart, sphereEnd, pdf;
    bool isInScreen;
    float su, sv;  // samplePosUV
    float ru, rv;  // rasterSamplePosUV
    float visibility, objectSpaceZ;
};

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

// Common.slang:285-324
__device__ __forceinline__ bool basic_init(const SvaoArgs& a, float u, float v, Basic& b) {
    const rsd_vao_data& d = a.d;
    const float z = depth_sample(a, u, v);
    const float rux = (d.radius * a.cam.focalLength) / (a.cam.frameWidth * z);
    const float ruy = (d.radius * a.cam.focalLength) / (a.cam.frameHeight * z);
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
    const uint32_t ix = (uint32_t)(u * d.resolution[0]), iy = (uint32_t)(v * d.resolution[1]);
    const uint32_t packed = (ix < (uint32_t)a.W && iy < (uint32_t)a.H) ? a.normals[(size_t)iy * a.W + ix] : 0u;
    b.normalV = decode_normal_2x8(packed);
    if (dot(b.posV, b.normalV) > 0.0f) b.normalV = -b.normalV;
    const float nu = u * d.noiseScale[0], nv = v * d.noiseScale[1];
    const int ni = ((int)floorf(nu * 4.0f)) & 3, nj = ((int)floorf(nv * 4.0f)) & 3;
    const f3 rd = mk(a.k.sinNoise[nj * 4 + ni], a.k.cosNoise[nj * 4 + ni], 0.0f);
    b.normal = mk(-b.posV.x / b.posVLength, -b.posV.y / b.posVLength, -b.posV.z / b.posVLength);
    b.bitangent = normalize(cross(b.normal, rd));
    b.tangent = cross(b.bitangent, b.normal);
    b.normalO = mk(dot(b.normalV, b.tangent), dot(b.normalV, b.bitangent), dot(b.normalV, b.normal));
    return true;
}

__device__ __forceinline__ float make_nonzero(float v, float eps) {
    const float av = hmax(fabsf(v), eps);
    return v >= 0.0f ? av : -av;
}

// Common.slang:354-399 (VAO kernel)
__device__ __forceinline__ bool sample_init(const SvaoArgs& a, float u, float v, const Basic& b, int i, Sample& s,
                                            float& screenSpaceRadius) {
    const rsd_vao_data& d = a.d;
    const float radius = a.k.sampleRadius[i] * b.radius;
    const float dx = radius * a.k.sinDir[i], dy = radius * a.k.cosDir[i];
    const float sphereHeight = sqrtf(b.radius * b.radius - radius * radius);
    s.pdf = 2.0f * sphereHeight;
    s.sphereStart = sphereHeight;
    const float zi = -(dx * b.normalO.x + dy * b.normalO.y) / make_nonzero(b.normalO.z, 0.0001f);
    s.sphereEnd = hmin(hmax(zi, -sphereHeight), sphereHeight);
    if ((s.sphereStart - s.sphereEnd) / (2.0f * sphereHeight) <= 0.1f) return false;
    const f3 ip = b.posV + b.tangent * dx + b.bitangent * dy;
    view_to_uv(a, ip, s.su, s.sv);
    s.visibility = 0.0f;
    s.objectSpaceZ = 0.0f;
    const float ex = (u - s.su) * d.resolution[0], ey = (v - s.sv) * d.resolution[1];
    screenSpaceRadius = sqrtf(ex * ex + ey * ey);
    const float cu = saturate(s.su), cv = saturate(s.sv);
    s.isInScreen = (s.su == cu) && (s.sv == cv);
    s.ru = (floorf(cu * d.resolution[0]) + 0.5f) / d.resolution[0];
    s.rv = (floorf(cv * d.resolution[1]) + 0.5f) / d.resolution[1];
    return true;
}

// Common.slang:180-196
__device__ __forceinline__ float calc_visibility(const rsd_vao_data& d, float oz, float ss, float se, float pdf,
                                                 float radius) {
    const float sphere = hmax(ss - hmax(se, oz), 0.0f) / pdf;
    const float halo = saturate((oz - (1.0f + d.thickness) * radius) / ss) * (ss - se) / pdf;
    return sphere + halo;
}

// Common.slang:463-483
__device__ __forceinline__ void add_sample(const SvaoArgs& a, const Basic& b, Sample& s, f3 spV, bool init) {
    const float oz = dot(spV - b.posV, b.normal);
    s.objectSpaceZ = init ? oz : hmin(s.objectSpaceZ, oz);
    const float vis = calc_visibility(a.d, oz, s.sphereStart, s.sphereEnd, s.pdf, b.radius);
    s.visibility = init ? vis : hmin(s.visibility, vis);
}

// Common.slang:492-496
__device__ __forceinline__ void eval_primary(const SvaoArgs& a, const Basic& b, Sample& s) {
    const float z = depth_sample(a, s.ru, s.rv);
    add_sample(a, b, s, uv_to_view(a, s.ru, s.rv, z), true);
}

// Common.slang:164-168
__device__ __forceinline__ int uv_to_sd(float uv, float low, int guard) {
    const int p = (int)floorf(uv * low) + guard;
    const int hi = (int)low + guard * 2 - 1;
    return p < 0 ? 0 : (p > hi ? hi : p);
}

// SVAO.cpp:334-340
__global__ void clear_intervals_kernel(uint32_t* rmin, uint32_t* rmax, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        rmax[i] = 0u;
        rmin[i] = 0x7f7fffffu;  // asuint(FLT_MAX)
    }
}

// SVAORaster.ps.slang:29-122, [numthreads(16,16,1)] with the 2x2 group interleave
__global__ void __launch_bounds__(256) svao_pass1_kernel(SvaoArgs a) {
    const uint32_t bx = blockIdx.x, by = blockIdx.y;
    const uint32_t ox = (bx / 2u) * 32u + 2u * threadIdx.x + (bx % 2u);
    const uint32_t oy = ((by / 2u) * a.bandCount + a.bandIndex) * 32u + 2u * threadIdx.y + (by % 2u);
    const uint32_t px = ox + a.guard, py = oy + a.guard;
    const rsd_vao_data& d = a.d;
    const float u = ((float)px + 0.5f) * d.invResolution[0];
    const float v = ((float)py + 0.5f) * d.invResolution[1];
    float ao = 0.0f;
    uint32_t st = 0;
    Basic b;
    if (!basic_init(a, u, v, b)) {
        ao = 1.0f;
    } else {
#pragma unroll 1
        for (int i = 0; i < 8; ++i) {
            Sample s;
            float ssr;
            if (!sample_init(a, u, v, b, i, s, ssr)) continue;
            if (fabsf(u - s.ru) < d.invResolution[0] * 0.9f && fabsf(v - s.rv) < d.invResolution[1] * 0.9f) {
                ao += (s.sphereStart - s.sphereEnd) / s.pdf;  // isSamePixel
                continue;
            }
            eval_primary(a, b, s);
            ao += s.visibility;
            bool forceRay = false;
            if (!s.isInScreen && d.sdGuard > 0) {
                forceRay = true;
                s.objectSpaceZ = 3.402823466e+38f;
            }
            const float constRadius = (1.0f + d.thickness) * b.radius - s.sphereStart;
            const bool req = s.objectSpaceZ > s.sphereStart + constRadius && ssr > d.ssRadiusCutoff;
            if (req || forceRay) {
                st |= 1u << i;
                if (a.secondary == 2u) {
                    const int sx = uv_to_sd(s.su, d.lowResolution[0], d.sdGuard);
                    const int sy = uv_to_sd(s.sv, d.lowResolution[1], d.sdGuard);
                    const size_t o = (size_t)sy * a.sdW + sx;
                    if (a.rayInterval) {
                        const float osMin = hmin(s.objectSpaceZ, b.radius + d.thickness * b.radius + s.sphereStart);
                        atomicMin(&a.rayMin[o], asuint(hmax(b.posVLength - osMin, 0.0f)));
                        atomicMax(&a.rayMax[o], asuint(hmax(b.posVLength - s.sphereEnd, 0.0f)));
                    } else {
                        a.rayMax[o] = 1u;
                    }
                }
            }
        }
        ao *= 1.0f / 8.0f;
        ao *= 2.0f;
        if (a.secondary == 0u || st == 0u) ao = acc_pow(ao, d.exponent);
    }
    if (px < (uint32_t)a.W && py < (uint32_t)a.H) {
        a.ao[(size_t)py * a.W + px] = unorm8(ao);
        a.stencil[(size_t)py * a.W + px] = (uint8_t)st;
    }
}

// SVAORaster2.ps.slang:48-65 -> calcAO2 (Common.slang:523-597), stochastic-depth branch
template <int N>
__global__ void __launch_bounds__(256) svao_pass2_kernel(SvaoArgs a) {
    const uint32_t bx = blockIdx.x, by = blockIdx.y;
    const uint32_t px = bx * 16u + threadIdx.x + a.guard;
    const uint32_t py = ((by / 2u) * a.bandCount + a.bandIndex) * 32u + (by % 2u) * 16u + threadIdx.y + a.guard;
    if (px >= (uint32_t)a.W - a.guard || py >= (uint32_t)a.H - a.guard) return;
    const size_t o = (size_t)py * a.W + px;
    uint32_t mask = a.stencil[o];
    if (mask == 0u) return;
    const rsd_vao_data& d = a.d;
    const float u = ((float)px + 0.5f) * d.invResolution[0];
    const float v = ((float)py + 0.5f) * d.invResolution[1];
    Basic b;
    basic_init(a, u, v, b);
    const float depthRange = a.cam.farZ - a.cam.nearZ, depthOffset = a.cam.nearZ;
    const size_t plane = (size_t)a.sdW * a.sdH;
    float vis = 0.0f;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        if (!(mask & (1u << i))) continue;
        Sample s;
        float ssr;
        sample_init(a, u, v, b, i, s, ssr);
        eval_primary(a, b, s);
        vis -= s.visibility;
        const int cx = uv_to_sd(s.su, d.lowResolution[0], d.sdGuard);
        const int cy = uv_to_sd(s.sv, d.lowResolution[1], d.sdGuard);
        float jx, jy;
        sd_jitter((uint32_t)cx, (uint32_t)cy, a.sdJitter != 0u, jx, jy);
        const float su = ((float)(cx - d.sdGuard) + jx) / d.lowResolution[0];
        const float sv = ((float)(cy - d.sdGuard) + jy) / d.lowResolution[1];
        const size_t so = (size_t)cy * a.sdW + cx;
        float dep[N];
        if constexpr (N == 1) {
            dep[0] = a.sd[so];
        } else if constexpr (N == 2) {
            const float2 t = reinterpret_cast<const float2*>(a.sd)[so];
            dep[0] = t.x; dep[1] = t.y;
        } else {
#pragma unroll
            for (int l = 0; l < N / 4; ++l) {
                const float4 t = reinterpret_cast<const float4*>(a.sd)[l * plane + so];
                dep[4 * l] = t.x; dep[4 * l + 1] = t.y; dep[4 * l + 2] = t.z; dep[4 * l + 3] = t.w;
            }
        }
        if (!s.isInScreen) { s.visibility = 1.0f; s.objectSpaceZ = 3.402823466e+38f; }  // resetSample
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const float lz = dep[k] * depthRange + depthOffset;
            add_sample(a, b, s, uv_to_view(a, su, sv, lz), false);
        }
        vis += s.visibility;
    }
    vis *= 1.0f / 8.0f;
    vis *= 2.0f;
    vis += unorm8_to_float(a.ao[o]);
    vis = acc_pow(vis, d.exponent);
    a.ao[o] = unorm8(vis);
}

static void fill_scale(SvaoArgs& a) {
    // Common.slang:142/150 imageScale, evaluated once on the host (IEEE float, same bits)
    a.isx = 0.5f * (a.cam.frameWidth / a.cam.focalLength);
    a.isy = 0.5f * (a.cam.frameHeight / a.cam.focalLength);
}

static void fill_consts(SvaoConsts& k) {
    // SVAO.cpp:670-684 -> R8Unorm noise; Common.slang:311-312 randRotation, :357 alpha
    static const float dither[16] = {0.0f, 8.0f, 2.0f, 10.0f, 12.0f, 4.0f, 14.0f, 6.0f,
                                     3.0f, 11.0f, 1.0f, 9.0f, 15.0f, 7.0f, 13.0f, 5.0f};
    for (int i = 0; i < 16; ++i) {
        const uint8_t byte = (uint8_t)(dither[i] / 16.0f * 255.0f);
        const float rr = (float)byte / 255.0f * 2.0f * 3.141f;
        k.sinNoise[i] = (float)std::sin((double)rr);
        k.cosNoise[i] = (float)std::cos((double)rr);
    }
    static const float radius8[8] = {0.917883f, 0.564429f, 0.734504f, 0.359545f,
                                     0.820004f, 0.470149f, 0.650919f, 0.205215f};  // Common.slang:53
    for (int i = 0; i < 8; ++i) {
        const float al = ((float)i / 8.0f) * 2.0f * 3.141f;
        k.sinDir[i] = (float)std::sin((double)al);
        k.cosDir[i] = (float)std::cos((double)al);
        k.sampleRadius[i] = radius8[i];
    }
}

static rsd_status check_common(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                               const float* depth, const uint16_t* normals, uint32_t W, uint32_t H, const char* who) {
    if (!cam || !vao || !p || !depth || !normals || W == 0 || H == 0) {
        set_error(std::string(who) + ": null argument or empty extent");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->num_directions != 8) {
        set_error(std::string(who) + ": only NUM_DIRECTIONS = 8 (the SVAO default) is implemented");
        return RSD_ERR_UNSUPPORTED;
    }
    if (2 * p->guard_band >= W || 2 * p->guard_band >= H) {
        set_error(std::string(who) + ": guard band leaves no visible region");
        return RSD_ERR_INVALID_ARG;
    }
    return RSD_OK;
}

}  // namespace rsd

using namespace rsd;

extern "C" rsd_status rsd_svao_clear_intervals(uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t count,
                                               rsd_stream stream) {
    if (!d_ray_min || !d_ray_max) {
        set_error("rsd_svao_clear_intervals: null buffer");
        return RSD_ERR_INVALID_ARG;
    }
    if (count == 0) return RSD_OK;
    hipLaunchKernelGGL(clear_intervals_kernel, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_ray_min,
                       d_ray_max, count);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "clear_intervals_kernel launch");
}

static rsd_status check_band(uint32_t index, uint32_t count, const char* who) {
    if (count == 0 || index >= count) {
        set_error(std::string(who) + ": band_index must be < band_count");
        return RSD_ERR_INVALID_ARG;
    }
    return RSD_OK;
}

extern "C" rsd_status rsd_svao_pass1_band(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                                          uint32_t sd_w, uint32_t sd_h, uint32_t band_index, uint32_t band_count,
                                          rsd_stream stream) {
    rsd_status st = check_band(band_index, band_count, "rsd_svao_pass1_band");
    if (st != RSD_OK) return st;
    st = check_common(cam, vao, p, d_depth, d_normals, W, H, "rsd_svao_pass1");
    if (st != RSD_OK) return st;
    if (!d_ao || !d_stencil || (p->secondary_depth_mode == 2 && (!d_ray_min || !d_ray_max || !sd_w || !sd_h))) {
        set_error("rsd_svao_pass1: null output buffer");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->secondary_depth_mode == 2 &&
        (sd_w != (uint32_t)vao->lowResolution[0] + 2u * (uint32_t)vao->sdGuard ||
         sd_h != (uint32_t)vao->lowResolution[1] + 2u * (uint32_t)vao->sdGuard)) {
        set_error("rsd_svao_pass1: SD map size does not match lowResolution + 2 sdGuard");
        return RSD_ERR_INVALID_ARG;
    }
    SvaoArgs a{};
    a.cam = *cam;
    a.d = *vao;
    fill_consts(a.k);
    fill_scale(a);
    a.depth = d_depth;
    a.normals = d_normals;
    a.W = (int)W;
    a.H = (int)H;
    a.ao = d_ao;
    a.stencil = d_stencil;
    a.rayMin = d_ray_min;
    a.rayMax = d_ray_max;
    a.sdW = (int)sd_w;
    a.sdH = (int)sd_h;
    a.guard = p->guard_band;
    a.secondary = p->secondary_depth_mode;
    a.rayInterval = p->ray_interval;
    a.sdJitter = p->sd_jitter;
    a.N = p->sd_samples;
    // SVAO.cpp:347-350: nThreads = roundup32(dims - 2 guardBand), 16x16 groups
    const uint32_t nx = (W - 2 * p->guard_band + 31u) / 32u * 32u, ny = (H - 2 * p->guard_band + 31u) / 32u * 32u;
    const uint32_t groups = ny / 32u;
    const uint32_t bandGroups = groups > band_index ? (groups - band_index + band_count - 1) / band_count : 0u;
    a.bandIndex = band_index;
    a.bandCount = band_count;
    if (bandGroups == 0) return RSD_OK;
    hipLaunchKernelGGL(svao_pass1_kernel, dim3(nx / 16, 2 * bandGroups), dim3(16, 16), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "svao_pass1_kernel launch");
}

extern "C" rsd_status rsd_svao_pass2_band(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                                          uint8_t* d_ao, uint32_t band_index, uint32_t band_count, rsd_stream stream) {
    rsd_status st = check_band(band_index, band_count, "rsd_svao_pass2_band");
    if (st != RSD_OK) return st;
    st = check_common(cam, vao, p, d_depth, d_normals, W, H, "rsd_svao_pass2");
    if (st != RSD_OK) return st;
    if (!d_stencil || !d_sd || !d_ao || !sd_w || !sd_h) {
        set_error("rsd_svao_pass2: null buffer");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t N = p->sd_samples;
    if (N != 1 && N != 2 && N != 4 && N != 8 && N != 16) {
        set_error("rsd_svao_pass2: MSAA_SAMPLES must be 1, 2, 4, 8 or 16");
        return RSD_ERR_UNSUPPORTED;
    }
    SvaoArgs a{};
    a.cam = *cam;
    a.d = *vao;
    fill_consts(a.k);
    fill_scale(a);
    a.depth = d_depth;
    a.normals = d_normals;
    a.W = (int)W;
    a.H = (int)H;
    a.ao = d_ao;
    a.stencil = const_cast<uint8_t*>(d_stencil);
    a.sd = d_sd;
    a.sdW = (int)sd_w;
    a.sdH = (int)sd_h;
    a.guard = p->guard_band;
    a.secondary = p->secondary_depth_mode;
    a.rayInterval = p->ray_interval;
    a.sdJitter = p->sd_jitter;
    a.N = N;
    const uint32_t vw = W - 2 * p->guard_band, vh = H - 2 * p->guard_band;
    const uint32_t groups = (vh + 31u) / 32u;
    const uint32_t bandGroups = groups > band_index ? (groups - band_index + band_count - 1) / band_count : 0u;
    a.bandIndex = band_index;
    a.bandCount = band_count;
    if (bandGroups == 0) return RSD_OK;
    dim3 grid((vw + 15) / 16, 2 * bandGroups), block(16, 16);
    hipStream_t s = (hipStream_t)stream;
    switch (N) {
        case 1: hipLaunchKernelGGL(svao_pass2_kernel<1>, grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL(svao_pass2_kernel<2>, grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL(svao_pass2_kernel<4>, grid, block, 0, s, a); break;
        case 8: hipLaunchKernelGGL(svao_pass2_kernel<8>, grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL(svao_pass2_kernel<16>, grid, block, 0, s, a); break;
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "svao_pass2_kernel launch");
}

extern "C" rsd_status rsd_svao_pass1(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                     const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                     uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                                     uint32_t sd_w, uint32_t sd_h, rsd_stream stream) {
    return rsd_svao_pass1_band(cam, vao, p, d_depth, d_normals, W, H, d_ao, d_stencil, d_ray_min, d_ray_max, sd_w,
                               sd_h, 0, 1, stream);
}

extern "C" rsd_status rsd_svao_pass2(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                     const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                     const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                                     uint8_t* d_ao, rsd_stream stream) {
    return rsd_svao_pass2_band(cam, vao, p, d_depth, d_normals, W, H, d_stencil, d_sd, sd_w, sd_h, d_ao, 0, 1, stream);
}
