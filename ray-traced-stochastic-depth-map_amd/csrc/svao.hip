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
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "rsd_device.h"
#include "rsd_internal.h"
#include "svao_math.h"

#ifndef RSD_P1_UNROLL
#define RSD_P1_UNROLL 1
#endif

namespace rsd {

// SVAO.cpp:334-340
__global__ void clear_intervals_kernel(uint32_t* rmin, uint32_t* rmax, uint32_t n) {
    // 4 texels per lane with 16-B stores where both buffers are 16-B aligned
    const uint32_t i = 4u * (blockIdx.x * blockDim.x + threadIdx.x);
    const bool vec = ((reinterpret_cast<uintptr_t>(rmin) | reinterpret_cast<uintptr_t>(rmax)) & 15u) == 0u;
    if (vec && i + 4u <= n) {
        reinterpret_cast<uint4*>(rmax)[i / 4u] = make_uint4(0u, 0u, 0u, 0u);
        reinterpret_cast<uint4*>(rmin)[i / 4u] = make_uint4(0x7f7fffffu, 0x7f7fffffu, 0x7f7fffffu, 0x7f7fffffu);
        return;
    }
    for (uint32_t k = i; k < n && k < i + 4u; ++k) {
        rmax[k] = 0u;
        rmin[k] = 0x7f7fffffu;  // asuint(FLT_MAX)
    }
}

// One direction of SVAORaster.ps.slang:49-105 for one pixel: the reference loop body.  (Issuing the
// reads of 2 or 4 directions before their bodies measured 77 / 91 vs 70 us: 77 / 105 VGPRs, 6 / 4 waves
// per SIMD -- DESIGN.md section 4.)  SPEC: the specialised kernel of the StochasticDepth frame with ray
// intervals, an SD guard band, pixel-index isSamePixel and a frame of at most 4096 x 4096 (every
// BASELINE config) -- the run-time tests of those settings are compile-time constants there.
template <bool SPEC, bool ALLFAST = false>
__device__ __forceinline__ void pass1_dir_generic(const SvaoArgs& a, float u, float v, uint32_t px, uint32_t py,
                                                  const Basic& b, int i, float& ao, float& aoD, uint32_t& st,
                                                  const P1Bufs* bf = nullptr) {
    const rsd_vao_data& d = a.d;
    Sample s;
    bool ssrAbove;
    if (!sample_init<ALLFAST>(a, u, v, b, i, s, ssrAbove, bf)) return;
    const bool same = (SPEC || a.k.samePixelInt) ? (s.kx == (int)px && s.ky == (int)py)
                                                 : (fabsf(u - s.ru) < d.invResolution[0] * 0.9f &&
                                                    fabsf(v - s.rv) < d.invResolution[1] * 0.9f);
    if (same) {
        const float w = div_pdf(s.sphereStart - s.sphereEnd, s);  // isSamePixel
        ao += w;
        aoD += w;
        return;
    }
    // SVAORaster.ps.slang:62-66: Raytraced mode with TRACE_OUT_OF_SCREEN (SVAO.h:104)
    bool forceRay = !SPEC && a.secondary == 3u && !s.isInScreen;
    eval_primary<SPEC>(a, b, s, bf);
    ao += s.visibility;
    if (!s.isInScreen && (SPEC || d.sdGuard > 0)) {
        forceRay = true;
        s.objectSpaceZ = 3.402823466e+38f;
    }
    const float constRadius = (1.0f + d.thickness) * b.radius - s.sphereStart;
    const bool req = s.objectSpaceZ > s.sphereStart + constRadius && ssrAbove;
    if (req || forceRay) {
        st |= 1u << i;
        if (SPEC || a.secondary == 2u) {
            const int sx = uv_to_sd(s.su, d.lowResolution[0], d.sdGuard);
            const int sy = uv_to_sd(s.sv, d.lowResolution[1], d.sdGuard);
            const size_t o = (size_t)sy * a.sdW + sx;
            if (SPEC || a.rayInterval) {
                const float osMin = hmin(s.objectSpaceZ, b.radius + d.thickness * b.radius + s.sphereStart);
                atomicMin(&a.rayMin[o], asuint(hmax(b.posVLength - osMin, 0.0f)));
                atomicMax(&a.rayMax[o], asuint(hmax(b.posVLength - s.sphereEnd, 0.0f)));
            } else {
                a.rayMax[o] = 1u;
            }
        }
    } else {
        aoD += s.visibility;  // darkmap: the dark channel keeps directions that need no ray
    }
}

// SVAORaster.ps.slang:29-122, [numthreads(16,16,1)] with the 2x2 group interleave.  (A branch-free
// "lean" direction body -- host constants in SGPRs, predicated updates, one float ratio compare --
// measured 74 vs 70 us at configs[1]: more VALU per direction and 64-73 VGPRs)
// ND > 0: NUM_DIRECTIONS known at compile time (the specialised kernel); 0: a.k.nd
template <bool SPEC, int ND>
__global__ void __launch_bounds__(256) svao_pass1_kernel(SvaoArgs a) {
    const uint32_t bx = blockIdx.x, by = blockIdx.y;
    const uint32_t ox = (bx / 2u) * 32u + 2u * threadIdx.x + (bx % 2u);
    const uint32_t oy = ((by / 2u) * a.bandCount + a.bandIndex) * 32u + 2u * threadIdx.y + (by % 2u);
    const uint32_t px = ox + a.guard, py = oy + a.guard;
    const rsd_vao_data& d = a.d;
    const float u = ((float)px + 0.5f) * d.invResolution[0];
    const float v = ((float)py + 0.5f) * d.invResolution[1];
    float ao = 0.0f, aoD = 0.0f;  // bright, dark (DUAL_AO: SVAORaster.ps.slang:13 ao_t = float2)
    uint32_t st = 0;
    Basic b;
    const P1Bufs bf = p1_bufs(a);  // uniform: built before any divergent branch
    if (!basic_init<SPEC>(a, u, v, b)) {
        ao = aoD = 1.0f;
    } else {
        const int nd = ND > 0 ? ND : (int)a.k.nd;
        // every lane of the wave at the unclamped AO radius (all but the pixels nearest the camera):
        // the host terms and div_rcp for all, no per-lane choice of path (the specialised kernel runs
        // only when every direction's fastDiv bit is set), and the per-direction zi division by the
        // pixel's make_nonzero(normalO.z) through its refined reciprocal (div_unscaled)
        const float nzd = make_nonzero(b.normalO.z, 0.0001f);
        const bool posOk = fabsf(b.posV.x) < 0x1p60f && fabsf(b.posV.y) < 0x1p60f;  // (div_unscaled bounds)
        if (SPEC && __ballot(b.radius != d.radius || !div_unscaled_den_ok(nzd) || !posOk) == 0u) {
            b.nzRcp = rcp_refined(nzd);
#pragma unroll RSD_P1_UNROLL
            for (int i = 0; i < nd; ++i) pass1_dir_generic<SPEC, true>(a, u, v, px, py, b, i, ao, aoD, st, &bf);
        } else {
#pragma unroll RSD_P1_UNROLL
            for (int i = 0; i < nd; ++i) pass1_dir_generic<SPEC>(a, u, v, px, py, b, i, ao, aoD, st);
        }
        ao *= a.k.invNd;  // SVAORaster.ps.slang:108-109
        ao *= 2.0f;
        aoD *= a.k.invNd;
        aoD *= 2.0f;
        if ((!SPEC && a.secondary == 0u) || st == 0u) {
            ao = acc_pow(ao, d.exponent);
            aoD = acc_pow(aoD, d.exponent);
        }
    }
    if (px < (uint32_t)a.W && py < (uint32_t)a.H) {
        ao_store(a, (size_t)py * a.W + px, ao, aoD);
        stencil_store(a, (size_t)py * a.W + px, st);
    }
    if (a.tileFlags) {
        // busy 16x16 tiles for pass 2: a wave is 4 thread rows of this 16x16 group = one tile row
        // and two tiles (threadIdx.x < 8: the left one, the 2x2 interleave spreads 16 threads over
        // 32 pixels); one byte store per busy tile and wave
        const uint64_t mL = __ballot(st != 0u && threadIdx.x < 8u), mR = __ballot(st != 0u && threadIdx.x >= 8u);
        const uint32_t lane = __lane_id();
        if ((lane == 0u && mL) || (lane == 8u && mR)) a.tileFlags[(oy / kTileEdge) * a.tilesX + ox / kTileEdge] = 1u;
    }
}

// SVAORaster2.ps.slang:48-65 -> calcAO2 (Common.slang:523-597), stochastic-depth branch: one
// refined direction i of a pixel -> its primary visibility p (subtracted) and refined r (added)
// SPEC / ALLFAST as in pass 1 (the specialised kernel: frame <= 4096 x 4096, every fastDiv bit, SD map
// width / height in [1, 2^20]; ALLFAST: every lane's pixel at the unclamped radius with b.nzRcp set).
// (ylx, yly) = rcp_refined of the SD resolution: the texel-centre uv divisions (cx - guard + jx) / low
// go through div_unscaled -- the numerator is never 0 and >= 0.0037 in magnitude (the jitter table
// lies in (0.0037, 0.9963), or 0.5 without jitter), so its preconditions hold.
template <int N, bool SPEC = false, bool ALLFAST = false>
__device__ __forceinline__ void svao_pass2_dir(const SvaoArgs& a, const Basic& b, float u, float v, int i, float& p,
                                               float& r, float ylx = 0.0f, float yly = 0.0f) {
    const rsd_vao_data& d = a.d;
    const float depthRange = a.cam.farZ - a.cam.nearZ, depthOffset = a.cam.nearZ;
    const size_t plane = sd_plane_texels(a.sdW, a.sdH);
    Sample s;
    bool ssrAbove;
    sample_init<ALLFAST>(a, u, v, b, i, s, ssrAbove);
    eval_primary<SPEC>(a, b, s);
    p = s.visibility;
    const int cx = uv_to_sd(s.su, d.lowResolution[0], d.sdGuard);
    const int cy = uv_to_sd(s.sv, d.lowResolution[1], d.sdGuard);
    float jx, jy;
    sd_jitter((uint32_t)cx, (uint32_t)cy, a.sdJitter != 0u, jx, jy);
    const float nu = (float)(cx - d.sdGuard) + jx, nv = (float)(cy - d.sdGuard) + jy;
    const float su = SPEC ? div_unscaled(nu, d.lowResolution[0], ylx) : nu / d.lowResolution[0];
    const float sv = SPEC ? div_unscaled(nv, d.lowResolution[1], yly) : nv / d.lowResolution[1];
    const size_t so = sd_texel(cx, cy, a.sdW);
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
    // addSample x N (Common.slang:583-596): visibility = min over k of sphere_k + halo_k.
    // Where halo_k is exactly +0 the term is RN(y_k / pdf), monotone in y_k, so those k
    // share ONE division of their least numerator (the result is the same float).
    float ymin = INFINITY;
    bool plain = false;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const float lz = dep[k] * depthRange + depthOffset;
        const float oz = dot(uv_to_view(a, su, sv, lz) - b.posV, b.normal);
        s.objectSpaceZ = hmin(s.objectSpaceZ, oz);
        const float y = hmax(s.sphereStart - hmax(s.sphereEnd, oz), 0.0f);
        const float x = oz - (1.0f + d.thickness) * b.radius;
        if (x > 0.0f) {
            const float halo = div_pdf(halo_ratio(x, s) * (s.sphereStart - s.sphereEnd), s);
            s.visibility = hmin(s.visibility, div_pdf(y, s) + halo);
        } else {
            ymin = hmin(ymin, y);
            plain = true;
        }
    }
    if (plain) s.visibility = hmin(s.visibility, div_pdf(ymin, s));
    r = s.visibility;
}

// Only stencilled pixels (~7 % at 1080p, ~1.7 refined directions each) have work, and each
// direction is a chain of dependent gathers (depth, then the SD map).  A workgroup owns a
// kP2Tile^2 tile of a 32-row band group and lists the
// tile's (pixel, direction) pairs in LDS, grouped per pixel in direction order; its
// lanes evaluate one pair each, then the pixel's running sum is applied in direction order,
// vis = (vis - p_i) + r_i as in calcAO2, and finally the AO store.  A sparse tile is one
// short pass instead of 256 lanes idling around a few busy ones; a dense tile takes as
// many passes as its mean direction count (<= the old per-lane maximum).
constexpr int kP2Tile = 16;                   // pass-2 tile edge (pixels): 16 measured 33 us, 8 35 us, 32 65 us
constexpr int kP2Lanes = kP2Tile * kP2Tile;   // lanes per workgroup = pixels per tile
static_assert(kP2Tile == (int)kTileEdge, "busy-tile flags are per pass-2 tile");
// the LDS of one pass-2 tile (26 KB: 6 workgroups per CU)
template <int ND>
struct P2Shared {
    uint32_t pix[kP2Lanes];        // active pixel slot: local index
    uint16_t pair[ND * kP2Lanes];  // pair: slot << 5 | direction
    uint16_t first[kP2Lanes];      // first pair of each slot
    float acc[kP2Lanes];           // running vis of each slot (bright)
    float accD[kP2Lanes];          // ... dark channel (DUAL_AO)
    float p[kP2Lanes], r[kP2Lanes];
    uchar2 aoPrev[kP2Lanes];       // the pixel's pass-1 AO (bright, dark), read with the stencil
    // the pixel's BasicAOData, evaluated once per pixel, not per pair: the 16 floats pass 2 reads
    // (posVLength, normalV, radiusInPixels stay out)
    alignas(16) float basic[kP2Lanes][16];
    uint32_t nPix, nPair;
};

// One kP2Tile^2 tile whose top-left pixel is (x0, y0); flag: its busy-tile flag (cleared) or null
template <int N, int ND, bool SPEC>
__device__ __forceinline__ void pass2_tile(const SvaoArgs& a, uint32_t x0, uint32_t y0, uint8_t* flag,
                                           P2Shared<ND>& sh) {
    constexpr uint32_t T = kP2Tile, L = kP2Lanes;
    const uint32_t tid = threadIdx.x;
    const rsd_vao_data& d = a.d;
    if (tid == 0) { sh.nPix = 0u; sh.nPair = 0u; }
    __syncthreads();
    {
        // every read of the tile's pixels is issued at once, independent of the stencil: the stencil, the
        // pixel's depth and packed normal (basic_init's reads) and the pass-1 AO the finish adds to; then
        // the normal-table read.  (Round 2 read the stencil first and the rest behind it: two more
        // dependent memory round trips per tile.)
        const uint32_t px = x0 + (tid % T), py = y0 + (tid / T);
        const bool inb = px < (uint32_t)a.W - a.guard && py < (uint32_t)a.H - a.guard;
        const size_t po = (size_t)py * a.W + px;
        const float u = ((float)px + 0.5f) * d.invResolution[0];
        const float v = ((float)py + 0.5f) * d.invResolution[1];
        uint32_t m = 0u, packed = 0u;
        float z = 0.0f;
        uchar2 prev = make_uchar2(0, 0);
        if (inb) {
            m = stencil_load(a, po);
            basic_reads<SPEC>(a, u, v, z, packed);
            if (a.dual) prev = reinterpret_cast<const uchar2*>(a.ao)[po];
            else prev.x = a.ao[po];
        }
        const float4 nl = a.nlut[packed];
        if (m) {
            const uint32_t slot = atomicAdd(&sh.nPix, 1u), base = atomicAdd(&sh.nPair, (uint32_t)__popc(m));
            sh.pix[slot] = tid;
            sh.first[slot] = (uint16_t)base;
            sh.acc[slot] = 0.0f;
            sh.accD[slot] = 0.0f;
            uint32_t j = base;
            for (int i = 0; i < ND; ++i)
                if (m & (1u << i)) sh.pair[j++] = (uint16_t)(slot << 5 | i);
            // a non-zero stencil means pass 1's basic_init of this pixel succeeded (same bits)
            Basic b;
            basic_from(a, u, v, z, nl, b);
            sh.aoPrev[slot] = prev;
            float* q = sh.basic[slot];
            q[0] = b.posV.x; q[1] = b.posV.y; q[2] = b.posV.z;
            q[3] = b.normal.x; q[4] = b.normal.y; q[5] = b.normal.z;
            q[6] = b.tangent.x; q[7] = b.tangent.y; q[8] = b.tangent.z;
            q[9] = b.bitangent.x; q[10] = b.bitangent.y; q[11] = b.bitangent.z;
            q[12] = b.normalO.x; q[13] = b.normalO.y; q[14] = b.normalO.z;
            q[15] = b.radius;
        }
    }
    __syncthreads();
    if (flag && tid == 0) *flag = 0u;  // consumed: the next pass 1 on this stream starts from zero
    const uint32_t nPix = sh.nPix, nPair = sh.nPair;
    for (uint32_t c = 0; c < nPair; c += L) {
        const uint32_t k = c + tid;
        uint32_t slot = 0;
        if (k < nPair) {
            const uint32_t e = sh.pair[k];
            slot = e >> 5;
            const uint32_t lp = sh.pix[slot] & 255u;
            const float u = ((float)(x0 + lp % T) + 0.5f) * d.invResolution[0];
            const float v = ((float)(y0 + lp / T) + 0.5f) * d.invResolution[1];
            const float* q = sh.basic[slot];
            Basic b;
            b.posV = mk(q[0], q[1], q[2]);
            b.normal = mk(q[3], q[4], q[5]);
            b.tangent = mk(q[6], q[7], q[8]);
            b.bitangent = mk(q[9], q[10], q[11]);
            b.normalO = mk(q[12], q[13], q[14]);
            b.radius = q[15];
            b.posVLength = 0.0f;  // not read by pass 2
            b.normalV = b.normal;
            b.radiusInPixels = 0.0f;
            float p, r;
            if constexpr (SPEC) {
                const float nzd = make_nonzero(b.normalO.z, 0.0001f);
                const float ylx = rcp_refined(d.lowResolution[0]), yly = rcp_refined(d.lowResolution[1]);
                const bool posOk = fabsf(b.posV.x) < 0x1p60f && fabsf(b.posV.y) < 0x1p60f;
                if (__ballot(b.radius != d.radius || !div_unscaled_den_ok(nzd) || !posOk) == 0u) {
                    b.nzRcp = rcp_refined(nzd);
                    svao_pass2_dir<N, true, true>(a, b, u, v, (int)(e & 31u), p, r, ylx, yly);
                } else {
                    svao_pass2_dir<N, true, false>(a, b, u, v, (int)(e & 31u), p, r, ylx, yly);
                }
            } else {
                svao_pass2_dir<N>(a, b, u, v, (int)(e & 31u), p, r);
            }
            sh.p[tid] = p;
            sh.r[tid] = r;
        }
        __syncthreads();
        // the lane of a pixel's first pair in this chunk applies its pairs in direction order
        if (k < nPair && k == max((uint32_t)sh.first[slot], c)) {
            float acc = sh.acc[slot], accD = sh.accD[slot];
            for (uint32_t j = k; j < nPair && j < c + L && (uint32_t)(sh.pair[j] >> 5) == slot; ++j) {
                acc = (acc - sh.p[j - c]) + sh.r[j - c];  // calcAO2: visibility.x -= raster; visibility += refined
                accD = accD + sh.r[j - c];
            }
            sh.acc[slot] = acc;
            sh.accD[slot] = accD;
        }
        __syncthreads();
    }
    for (uint32_t sl = tid; sl < nPix; sl += L) {
        const uint32_t lp = sh.pix[sl] & 255u;
        const size_t o = (size_t)(y0 + lp / T) * a.W + (x0 + lp % T);
        ao_finish(a, o, sh.acc[sl], sh.accD[sl], sh.aoPrev[sl]);
    }
}

// One workgroup per tile of the band's 32-row groups; an unflagged tile (busy-tile flags of pass 1)
// returns before any barrier.  (A persistent grid of 6 workgroups per CU striding over the flagged
// tiles measured 48-51 vs 36-38 us at configs[1]: the busy tiles cluster, so some workgroups
// serialise several dependent tile chains -- tools/pass2_probe.py)
template <int N, int ND, bool SPEC = false>
__global__ void __launch_bounds__(kP2Lanes) svao_pass2_kernel(SvaoArgs a) {
    constexpr uint32_t kPerGroup = 32u / kP2Tile;  // tile rows per 32-row band group
    __shared__ P2Shared<ND> sh;
    const uint32_t y0 = ((blockIdx.y / kPerGroup) * a.bandCount + a.bandIndex) * 32u + (blockIdx.y % kPerGroup) * kP2Tile +
                        a.guard;
    uint8_t* flag = a.tileFlags ? a.tileFlags + ((y0 - a.guard) / kP2Tile) * a.tilesX + blockIdx.x : nullptr;
    if (flag && *flag == 0u) return;  // uniform over the workgroup
    pass2_tile<N, ND, SPEC>(a, blockIdx.x * kP2Tile + a.guard, y0, flag, sh);
}

}  // namespace rsd

namespace rsd {
namespace {
// Device-resident constant tables, cached per device for the life of the process (a few KB to
// 1 MB each, never freed: a table may still be read by kernels in flight on any stream).
// Process-wide with a lock: one rsd_device per GPU per host thread (rsd.h), any thread, any GPU.
constexpr int kMaxDevices = 64;
std::mutex g_tab_mutex;

__global__ void normal_lut_kernel(float4* lut) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 65536u) {
        const f3 n = decode_normal_2x8(i);
        lut[i] = make_float4(n.x, n.y, n.z, 0.0f);
    }
}
float4* g_nlut[kMaxDevices] = {};

struct SnapTable {
    int w, h;
    float* d;
};
std::vector<SnapTable> g_snap[kMaxDevices];  // per device: one table per frame-buffer size

int current_device(int* dev) {
    if (hipGetDevice(dev) != hipSuccess || *dev < 0 || *dev >= kMaxDevices) return -1;
    return 0;
}
}  // namespace

rsd_status normal_lut(const float4** out) {
    int dev = 0;
    if (current_device(&dev)) {
        set_error("normal_lut: no current HIP device (or device index >= 64)");
        return RSD_ERR_NO_DEVICE;
    }
    std::lock_guard<std::mutex> lock(g_tab_mutex);
    if (!g_nlut[dev]) {
        float4* d = nullptr;
        RSD_HIP(hipMalloc(&d, 65536 * sizeof(float4)));
        hipLaunchKernelGGL(normal_lut_kernel, dim3(256), dim3(256), 0, (hipStream_t)0, d);
        RSD_HIP(hipGetLastError());
        RSD_HIP(hipDeviceSynchronize());  // once per device
        g_nlut[dev] = d;
    }
    *out = g_nlut[dev];
    return RSD_OK;
}

// pixel-centre UVs (k + 0.5) / resolution of every column and row of the frame buffer
rsd_status snap_tables(const rsd_vao_data& vd, const float** u, const float** v) {
    const int w = (int)vd.resolution[0], h = (int)vd.resolution[1];
    int dev = 0;
    if (current_device(&dev)) {
        set_error("snap_tables: no current HIP device (or device index >= 64)");
        return RSD_ERR_NO_DEVICE;
    }
    std::lock_guard<std::mutex> lock(g_tab_mutex);
    for (const SnapTable& t : g_snap[dev])
        if (t.w == w && t.h == h) {
            *u = t.d;
            *v = t.d + w + 1;
            return RSD_OK;
        }
    std::vector<float> t((size_t)w + 1 + (size_t)h + 1);
    for (int k = 0; k <= w; ++k) t[k] = ((float)k + 0.5f) / vd.resolution[0];
    for (int k = 0; k <= h; ++k) t[(size_t)w + 1 + k] = ((float)k + 0.5f) / vd.resolution[1];
    float* d = nullptr;
    RSD_HIP(hipMalloc(&d, t.size() * sizeof(float)));
    RSD_HIP(hipMemcpy(d, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
    g_snap[dev].push_back({w, h, d});
    *u = d;
    *v = d + w + 1;
    return RSD_OK;
}
}  // namespace rsd

using namespace rsd;

extern "C" uint32_t rsd_svao_tile_count(uint32_t width, uint32_t height, uint32_t guard_band) {
    if (2 * guard_band >= width || 2 * guard_band >= height) return 0u;
    return tiles_x(width, guard_band) * tiles_y(height, guard_band);
}

extern "C" rsd_status rsd_svao_clear_intervals(uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t count,
                                               rsd_stream stream) {
    if (!d_ray_min || !d_ray_max) {
        set_error("rsd_svao_clear_intervals: null buffer");
        return RSD_ERR_INVALID_ARG;
    }
    if (count == 0) return RSD_OK;
    hipLaunchKernelGGL(clear_intervals_kernel, dim3((count + 1023) / 1024), dim3(256), 0, (hipStream_t)stream, d_ray_min,
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

// 32-row groups g = start + k * step, k < n -- or, with n = ~0u, every group of an interleaved band
// (start = index, step = count) -- counted from the first visible row
namespace {
rsd_status pass1_impl(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p, const float* d_depth,
                      const uint16_t* d_normals, uint32_t W, uint32_t H, uint8_t* d_ao, uint8_t* d_stencil,
                      uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h, uint32_t start,
                      uint32_t step, uint32_t n, rsd_stream stream) {
    rsd_status st = check_common(cam, vao, p, d_depth, d_normals, W, H, "rsd_svao_pass1");
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
    fill_consts(a.k, a.d, p->num_directions);
    {
        rsd_status ts = snap_tables(a.d, &a.snapU, &a.snapV);
        if (ts == RSD_OK) ts = normal_lut(&a.nlut);
        if (ts != RSD_OK) return ts;
    }
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
    a.dual = p->dual_ao ? 1u : 0u;
    a.rayInterval = p->ray_interval;
    a.sdJitter = p->sd_jitter;
    a.N = p->sd_samples;
    a.tileFlags = p->tile_flags;
    a.tilesX = tiles_x(W, p->guard_band);
    // SVAO.cpp:347-350: nThreads = roundup32(dims - 2 guardBand), 16x16 groups
    const uint32_t nx = (W - 2 * p->guard_band + 31u) / 32u * 32u, ny = (H - 2 * p->guard_band + 31u) / 32u * 32u;
    const uint32_t groups = ny / 32u;
    const uint32_t bandGroups = std::min(n, groups > start ? (groups - start + step - 1) / step : 0u);
    a.bandIndex = start;
    a.bandCount = step;
    if (bandGroups == 0) return RSD_OK;
    // the specialised kernel for the StochasticDepth frame (every BASELINE config); RSD_PASS1=generic
    // forces the generic one (A/B runs)
    const char* p1Env = std::getenv("RSD_PASS1");
    const uint32_t allDirs = a.k.nd == 32u ? 0xffffffffu : (1u << a.k.nd) - 1u;
    const bool spec = !(p1Env && std::strcmp(p1Env, "generic") == 0) && a.secondary == 2u && a.rayInterval &&
                      a.k.samePixelInt && a.d.sdGuard > 0 && W <= 4096u && H <= 4096u &&
                      (a.k.fastDiv & allDirs) == allDirs && a.d.radius < 0x1p58f;
    const dim3 grid(nx / 16, 2 * bandGroups), block(16, 16);
    hipStream_t s = (hipStream_t)stream;
    if (spec && a.k.nd == 8u) hipLaunchKernelGGL((svao_pass1_kernel<true, 8>), grid, block, 0, s, a);
    else if (spec) hipLaunchKernelGGL((svao_pass1_kernel<true, 0>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((svao_pass1_kernel<false, 0>), grid, block, 0, s, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "svao_pass1_kernel launch");
}
}  // namespace

extern "C" rsd_status rsd_svao_pass1_band(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                                          uint32_t sd_w, uint32_t sd_h, uint32_t band_index, uint32_t band_count,
                                          rsd_stream stream) {
    rsd_status st = check_band(band_index, band_count, "rsd_svao_pass1_band");
    if (st != RSD_OK) return st;
    return pass1_impl(cam, vao, p, d_depth, d_normals, W, H, d_ao, d_stencil, d_ray_min, d_ray_max, sd_w, sd_h,
                      band_index, band_count, ~0u, stream);
}

extern "C" rsd_status rsd_svao_pass1_rows(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                                          uint32_t sd_w, uint32_t sd_h, uint32_t row0, uint32_t row1,
                                          rsd_stream stream) {
    if (!p) {
        set_error("rsd_svao_pass1_rows: null params");
        return RSD_ERR_INVALID_ARG;
    }
    if (row0 > row1 || row0 % 32u != 0u || (row1 % 32u != 0u && row1 + 2u * (uint32_t)p->guard_band < H)) {
        set_error("rsd_svao_pass1_rows: rows must be multiples of 32 from the first visible row (row1 may end the frame)");
        return RSD_ERR_INVALID_ARG;
    }
    return pass1_impl(cam, vao, p, d_depth, d_normals, W, H, d_ao, d_stencil, d_ray_min, d_ray_max, sd_w, sd_h,
                      row0 / 32u, 1u, (row1 - row0 + 31u) / 32u, stream);
}

namespace {
rsd_status pass2_impl(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p, const float* d_depth,
                      const uint16_t* d_normals, uint32_t W, uint32_t H, const uint8_t* d_stencil, const float* d_sd,
                      uint32_t sd_w, uint32_t sd_h, uint8_t* d_ao, uint32_t start, uint32_t step, uint32_t n,
                      rsd_stream stream) {
    rsd_status st = check_common(cam, vao, p, d_depth, d_normals, W, H, "rsd_svao_pass2");
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
    fill_consts(a.k, a.d, p->num_directions);
    {
        rsd_status ts = snap_tables(a.d, &a.snapU, &a.snapV);
        if (ts == RSD_OK) ts = normal_lut(&a.nlut);
        if (ts != RSD_OK) return ts;
    }
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
    a.dual = p->dual_ao ? 1u : 0u;
    a.rayInterval = p->ray_interval;
    a.sdJitter = p->sd_jitter;
    a.N = N;
    a.tileFlags = p->tile_flags;
    a.tilesX = tiles_x(W, p->guard_band);
    const uint32_t vw = W - 2 * p->guard_band, vh = H - 2 * p->guard_band;
    const uint32_t groups = (vh + 31u) / 32u;
    const uint32_t bandGroups = std::min(n, groups > start ? (groups - start + step - 1) / step : 0u);
    a.bandIndex = start;
    a.bandCount = step;
    if (bandGroups == 0) return RSD_OK;
    dim3 grid((vw + kP2Tile - 1) / kP2Tile, (32 / kP2Tile) * bandGroups), block(kP2Lanes);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t nd = a.k.nd;
    // the specialised kernel (8 directions; RSD_PASS2=generic forces the generic one for A/B runs)
    const char* p2Env = std::getenv("RSD_PASS2");
    const bool spec = !(p2Env && std::strcmp(p2Env, "generic") == 0) && nd == 8u && W <= 4096u && H <= 4096u &&
                      (a.k.fastDiv & 0xffu) == 0xffu && a.d.lowResolution[0] >= 1.0f &&
                      a.d.lowResolution[0] <= 0x1p20f && a.d.lowResolution[1] >= 1.0f && a.d.lowResolution[1] <= 0x1p20f &&
                      a.d.radius < 0x1p58f;
#define RSD_P2(NN)                                                                                           \
    if (nd == 32u) hipLaunchKernelGGL((svao_pass2_kernel<NN, 32>), grid, block, 0, s, a);                  \
    else if (nd == 16u) hipLaunchKernelGGL((svao_pass2_kernel<NN, 16>), grid, block, 0, s, a);             \
    else if (spec) hipLaunchKernelGGL((svao_pass2_kernel<NN, 8, true>), grid, block, 0, s, a);             \
    else hipLaunchKernelGGL((svao_pass2_kernel<NN, 8>), grid, block, 0, s, a);
    switch (N) {
        case 1: RSD_P2(1) break;
        case 2: RSD_P2(2) break;
        case 4: RSD_P2(4) break;
        case 8: RSD_P2(8) break;
        default: RSD_P2(16) break;
    }
#undef RSD_P2
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "svao_pass2_kernel launch");
}
}  // namespace

extern "C" rsd_status rsd_svao_pass2_band(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                                          uint8_t* d_ao, uint32_t band_index, uint32_t band_count, rsd_stream stream) {
    rsd_status st = check_band(band_index, band_count, "rsd_svao_pass2_band");
    if (st != RSD_OK) return st;
    return pass2_impl(cam, vao, p, d_depth, d_normals, W, H, d_stencil, d_sd, sd_w, sd_h, d_ao, band_index, band_count,
                      ~0u, stream);
}

extern "C" rsd_status rsd_svao_pass2_rows(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                                          uint8_t* d_ao, uint32_t row0, uint32_t row1, rsd_stream stream) {
    if (!p) {
        set_error("rsd_svao_pass2_rows: null params");
        return RSD_ERR_INVALID_ARG;
    }
    if (row0 > row1 || row0 % 32u != 0u || (row1 % 32u != 0u && row1 + 2u * (uint32_t)p->guard_band < H)) {
        set_error("rsd_svao_pass2_rows: rows must be multiples of 32 from the first visible row (row1 may end the frame)");
        return RSD_ERR_INVALID_ARG;
    }
    return pass2_impl(cam, vao, p, d_depth, d_normals, W, H, d_stencil, d_sd, sd_w, sd_h, d_ao, row0 / 32u, 1u,
                      (row1 - row0 + 31u) / 32u, stream);
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
