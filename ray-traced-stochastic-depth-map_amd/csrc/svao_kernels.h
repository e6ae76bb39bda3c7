// svao_kernels.h -- the SVAO "AO 1" / "AO 2" kernels, compiled twice (DESIGN.md section 2 "Numerics"):
//
//   svao.hip       namespace rsd::exact  -ffp-contract=off, correctly rounded '/' and sqrt: the numerics
//                                        contract of rsd_device.h, bit-identical to the CPU oracle
//                                        (RSD_NUMERICS_EXACT);
//   svao_fast.hip  namespace rsd::fast   RSD_FAST_NUMERICS: FMA contraction, v_rcp_f32 / v_sqrt_f32 /
//                                        v_rsq_f32, float32 denormals flushed -- the arithmetic D3D allows
//                                        the reference's HLSL (mad may fuse, '/' is 2.5 ulp, denormals
//                                        flush), graded against the oracle by BASELINE.md section 4's AO
//                                        tolerance (RSD_NUMERICS_FAST, the product default).
//
// Reference: SVAORaster.ps.slang:29-122 (pass 1), SVAORaster2.ps.slang:48-65 (pass 2),
//            SVAO/Common.slang:98-663.  The including file defines RSD_SVAO_NS (exact / fast) and
//            includes svao_math.h first.
#pragma once
#ifndef RSD_SVAO_NS
#error "define RSD_SVAO_NS (exact or fast) before including svao_kernels.h"
#endif

#ifndef RSD_P1_UNROLL
#define RSD_P1_UNROLL 1
#endif
// fast numerics: clamped-radius pixels take the SCALED all-fast loops (sample_init); 0 = the per-lane
// generic loops as in the exact build (A/B builds: make variant V=noscaled DEFS=-DRSD_SCALED_ALLFAST=0)
// diagnostic builds only (make variant V=noatom DEFS=-DRSD_DIAG_P1_NOATOM=1; results wrong by design): pass 1
// without its interval atomics, to price them
#ifndef RSD_DIAG_P1_NOATOM
#define RSD_DIAG_P1_NOATOM 0
#endif
#ifndef RSD_SCALED_ALLFAST
#define RSD_SCALED_ALLFAST 1
#endif

namespace rsd {
namespace RSD_SVAO_NS {

// One direction of SVAORaster.ps.slang:49-105 for one pixel: the reference loop body.  (Issuing the
// reads of 2 or 4 directions before their bodies measured 77 / 91 vs 70 us: 77 / 105 VGPRs, 6 / 4 waves
// per SIMD -- DESIGN.md section 4; in the fast build 2 directions at 62 VGPRs, 8 waves, measured 48.7-49.0
// vs 47.5 us, and 2-3 us per frame slower with frames in flight, profiles/round4/ab_pass/.)  SPEC: the specialised kernel of the StochasticDepth frame with ray
// intervals, an SD guard band, pixel-index isSamePixel and a frame of at most 4096 x 4096 (every
// BASELINE config) -- the run-time tests of those settings are compile-time constants there.
template <bool SPEC, bool ALLFAST = false, bool SCALED = false>
__device__ __forceinline__ void pass1_dir_generic(const SvaoArgs& a, float u, float v, uint32_t px, uint32_t py,
                                                  const Basic& b, int i, float& ao, float& aoD, uint32_t& st,
                                                  const P1Bufs* bf = nullptr) {
    const rsd_vao_data& d = a.d;
    Sample s;
    bool ssrAbove;
    if (!sample_init<ALLFAST, SPEC, SCALED>(a, u, v, b, i, s, ssrAbove, bf)) return;
    const bool same = (SPEC || a.k.samePixelInt) ? (s.kx == (int)px && s.ky == (int)py)
                                                 : (fabsf(u - s.ru) < d.invResolution[0] * 0.9f &&
                                                    fabsf(v - s.rv) < d.invResolution[1] * 0.9f);
    if (same) {
        if (SPEC || !a.k.hbao) {  // isSamePixel (SVAORaster.ps.slang:55-60: HBAO adds 0)
            const float w = div_pdf(s.sphereStart - s.sphereEnd, s);
            ao += w;
            aoD += w;
        }
        return;
    }
    // SVAORaster.ps.slang:62-66: Raytraced mode with TRACE_OUT_OF_SCREEN (SVAO.h:104)
    bool forceRay = !SPEC && a.secondary == 3u && !s.isInScreen;
    eval_primary<SPEC, SPEC>(a, b, s, bf);
    if (!SPEC && a.dualDepth) eval_dual(a, b, s, ssrAbove, false);  // SVAORaster.ps.slang:69-70
    ao += s.visibility;
    if (!s.isInScreen && (SPEC || d.sdGuard > 0)) {
        forceRay = true;
        s.objectSpaceZ = 3.402823466e+38f;
    }
    bool req;
    if (SPEC) {
        const float constRadius = (1.0f + d.thickness) * b.radius - s.sphereStart;
        req = s.objectSpaceZ > s.sphereStart + constRadius && ssrAbove;
    } else {
        req = require_ray(a, b, s, ssrAbove);
    }
    if (req || forceRay) {
        st |= 1u << i;
        if (SPEC || a.secondary == 2u) {
            const int sx = uv_to_sd(s.su, d.lowResolution[0], d.sdGuard);
            const int sy = uv_to_sd(s.sv, d.lowResolution[1], d.sdGuard);
            const size_t o = (size_t)sy * a.sdW + sx;
            if (SPEC || a.rayInterval) {
                // SVAORaster.ps.slang:90-91
                const float osMin = (!SPEC && a.k.hbao) ? hmin(s.objectSpaceZ, s.sphereStart)
                                                        : hmin(s.objectSpaceZ, b.radius + d.thickness * b.radius + s.sphereStart);
                if (!RSD_DIAG_P1_NOATOM) {
                    atomicMin(&a.rayMin[o], asuint(hmax(b.posVLength - osMin, 0.0f)));
                    atomicMax(&a.rayMax[o], asuint(hmax(b.posVLength - s.sphereEnd, 0.0f)));
                }
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
// (A workgroup-wide LDS copy of the depth texels around the 32 x 32 pixels plus a 16-texel apron, 16 KB, serving the
// gathers inside it was measured slower at configs[1]-[3]: 46 -> 52 us, the copy costs more than the gathers it
// serves; round 6, profiles/round6/pass1_window/.)
template <bool SPEC, int ND>
__global__ void __launch_bounds__(256) svao_pass1_kernel(SvaoArgs a) {
    uint32_t bx = blockIdx.x, by = blockIdx.y;
    if (a.xcdChunk) {  // chunks of C workgroups dealt round-robin to the 8 XCD groups (bijective on the full chunks)
        const uint32_t C = a.xcdChunk, gx = gridDim.x, n = gx * gridDim.y, L = by * gx + bx;
        const uint32_t full = n / (8u * C) * (8u * C);
        if (L < full) {
            const uint32_t xcd = L % 8u, j = L / 8u;
            const uint32_t T = ((j / C) * 8u + xcd) * C + j % C;
            bx = T % gx;
            by = T / gx;
        }
    }
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
    // the specialised kernels: the 16 noise sines and cosines in LDS (a lane's noise index is its own, so the
    // kernel-argument table would be a per-lane vector load, one more dependent round trip per pixel)
    __shared__ float sNoise[SPEC ? 32 : 1];
    if constexpr (SPEC) {
        const uint32_t t = threadIdx.y * 16u + threadIdx.x;
        if (t < 32u) sNoise[t] = t < 16u ? a.k.sinNoise[t] : a.k.cosNoise[t - 16u];
        __syncthreads();
    }
    if (!basic_init<SPEC>(a, u, v, b, SPEC ? sNoise : nullptr)) {
        ao = aoD = 1.0f;
    } else {
        const int nd = ND > 0 ? ND : (int)a.k.nd;
        // every lane of the wave at the unclamped AO radius (all but the pixels nearest the camera):
        // the host terms and div_rcp for all, no per-lane choice of path (the specialised kernel runs
        // only when every direction's fastDiv bit is set), and the per-direction zi division by the
        // pixel's make_nonzero(normalO.z) through its refined reciprocal (div_unscaled)
        const float nzd = make_nonzero(b.normalO.z, 0.0001f);
        const bool posOk = kFastNumerics || (fabsf(b.posV.x) < 0x1p60f && fabsf(b.posV.y) < 0x1p60f);  // (div_unscaled bounds)
        if (SPEC && __ballot(b.radius != d.radius || !div_unscaled_den_ok(nzd) || !posOk) == 0u) {
            b.nzRcp = rcp_refined(nzd);
#pragma unroll RSD_P1_UNROLL
            for (int i = 0; i < nd; ++i) pass1_dir_generic<SPEC, true>(a, u, v, px, py, b, i, ao, aoD, st, &bf);
        } else if (SPEC && kFastNumerics && RSD_SCALED_ALLFAST) {
            // fast numerics: a wave with clamped-radius pixels (nearest the camera) takes the same lean
            // loop with the direction terms scaled per pixel instead of the per-lane IEEE paths
            b.nzRcp = rcp_refined(nzd);
            set_radius_scale(a, b);
#pragma unroll RSD_P1_UNROLL
            for (int i = 0; i < nd; ++i) pass1_dir_generic<SPEC, true, true>(a, u, v, px, py, b, i, ao, aoD, st, &bf);
        } else {
#pragma unroll RSD_P1_UNROLL
            for (int i = 0; i < nd; ++i) pass1_dir_generic<SPEC>(a, u, v, px, py, b, i, ao, aoD, st);
        }
        ao *= a.k.invNd;  // SVAORaster.ps.slang:108-109 (x 2: VAO only)
        aoD *= a.k.invNd;
        if (SPEC || !a.k.hbao) {
            ao *= 2.0f;
            aoD *= 2.0f;
        }
        if ((!SPEC && a.secondary == 0u) || st == 0u) {
            ao = SPEC ? acc_pow(ao, d.exponent) : ao_finalize(a, ao);
            aoD = SPEC ? acc_pow(aoD, d.exponent) : ao_finalize(a, aoD);
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
        // only visible pixels vote: the padded dispatch (roundup32 of the visible size) also runs up to 31
        // columns / rows beyond it, whose tile index would alias the next row's first tile (or lie past
        // the last flag byte) when the visible width is not a multiple of 16
        const bool vote = st != 0u && ox < (uint32_t)a.W - 2u * a.guard && oy < (uint32_t)a.H - 2u * a.guard;
        const uint64_t mL = __ballot(vote && threadIdx.x < 8u), mR = __ballot(vote && threadIdx.x >= 8u);
        const uint32_t lane = __lane_id();
        if ((lane == 0u && mL) || (lane == 8u && mR)) {
            // the first wave to flag a tile appends it to the busy-tile list pass 2 walks
            const uint32_t t = (oy / kTileEdge) * a.tilesX + ox / kTileEdge;
            if (atomicExch(&a.tileFlags[t], a.tileStamp) != a.tileStamp)
                a.tileList[atomicAdd(a.tileCount + a.tileGen, 1u)] = t;
        }
        // the other list count (read by the previous frame's pass 2, earlier on this stream) starts the
        // next frame's list at zero: no workgroup of pass 2 has to reset anything (svao.hip tile_gen)
        if (blockIdx.x == 0u && blockIdx.y == 0u && threadIdx.x == 0u && threadIdx.y == 0u)
            a.tileCount[a.tileGen ^ 1u] = 0u;
    }
}

// SVAORaster2.ps.slang:48-65 -> calcAO2 (Common.slang:523-597), stochastic-depth branch: one
// refined direction i of a pixel -> its primary visibility p (subtracted) and refined r (added)
// SPEC / ALLFAST as in pass 1 (the specialised kernel: frame <= 4096 x 4096, every fastDiv bit, SD map
// width / height in [1, 2^20]; ALLFAST: every lane's pixel at the unclamped radius with b.nzRcp set).
// (ylx, yly) = rcp_refined of the SD resolution: the texel-centre uv divisions (cx - guard + jx) / low
// go through div_unscaled -- the numerator is never 0 and >= 0.0037 in magnitude (the jitter table
// lies in (0.0037, 0.9963), or 0.5 without jitter), so its preconditions hold.
// KL > 0 (the specialised all-fast kernels): kl = the tile's LDS copy of the direction terms (sample_init)
// followed by the 16 SD jitter pairs (rsd_device.h kJitter); the pair's reads -- the primary depth and the
// N SD depths, no table -- are issued back to back, the depth first (vmcnt returns in order, so waiting for
// the depth leaves the SD reads in flight)
template <int N, bool SPEC = false, bool ALLFAST = false, bool SCALED = false, int KL = 0>
__device__ __forceinline__ void svao_pass2_dir(const SvaoArgs& a, const Basic& b, float u, float v, int i, float& p,
                                               float& r, float ylx = 0.0f, float yly = 0.0f,
                                               const float* kl = nullptr) {
    const rsd_vao_data& d = a.d;
    const float depthRange = a.cam.farZ - a.cam.nearZ, depthOffset = a.cam.nearZ;
    const size_t plane = sd_plane_texels(a.sdW, a.sdH);
    Sample s;
    bool ssrAbove;
    sample_init<ALLFAST, SPEC, SCALED, KL>(a, u, v, b, i, s, ssrAbove, nullptr, kl);
    float zp = 0.0f;
    if constexpr (SPEC) {
        zp = depth_center<true>(a, s.ru, s.rv, s.kx, s.ky);  // evalPrimaryVisibility's read, issued first
    } else {
        if (a.dualDepth) eval_dual(a, b, s, ssrAbove, true);  // Common.slang:555-558 (force init)
        else eval_primary<SPEC, SPEC>(a, b, s);
        p = s.visibility;
        if (a.secondary == 1u) {
            // secondary DualDepth: calcAO2 has no branch for it (Common.slang:562-651), so the raster
            // visibility is subtracted and added back unchanged
            r = p;
            return;
        }
    }
    const int cx = uv_to_sd(s.su, d.lowResolution[0], d.sdGuard);
    const int cy = uv_to_sd(s.sv, d.lowResolution[1], d.sdGuard);
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
    float jx, jy;
    if constexpr (KL > 0) {
        const uint32_t ji = ((uint32_t)(cy & 3) * 4u + (uint32_t)(cx & 3)) * 2u;
        jx = a.sdJitter ? kl[6 * KL + ji] : 0.5f;
        jy = a.sdJitter ? kl[6 * KL + ji + 1] : 0.5f;
    } else {
        sd_jitter((uint32_t)cx, (uint32_t)cy, a.sdJitter != 0u, jx, jy);
    }
    if constexpr (SPEC) {
        add_sample<true>(a, b, s, uv_to_view(a, s.ru, s.rv, zp), true);  // evalPrimaryVisibility
        p = s.visibility;
    }
    const float nu = (float)(cx - d.sdGuard) + jx, nv = (float)(cy - d.sdGuard) + jy;
    const float su = SPEC ? div_unscaled(nu, d.lowResolution[0], ylx) : nu / d.lowResolution[0];
    const float sv = SPEC ? div_unscaled(nv, d.lowResolution[1], yly) : nv / d.lowResolution[1];
    if (!s.isInScreen) {  // resetSample (Common.slang:485-490)
        s.visibility = (!SPEC && a.k.hbao) ? 0.0f : 1.0f;
        s.objectSpaceZ = 3.402823466e+38f;
    }
    if (!SPEC && a.k.hbao) {  // addSample x N, HBAO: the max of saturate(HBAOKernel / pdf)
#pragma unroll
        for (int k = 0; k < N; ++k) add_sample(a, b, s, uv_to_view(a, su, sv, dep[k] * depthRange + depthOffset), false);
        r = s.visibility;
        return;
    }
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
template <int ND, int NB = 16, int KC = 0>
struct P2Shared {
    // the specialised kernels (KC = 6 ND + 64): the direction terms and SD jitter pairs sample_init and
    // svao_pass2_dir read per pair (kl, KL = ND) and the noise terms basic_from reads per pixel, copied
    // from the kernel arguments once per tile (per-lane indices: vector loads of kernel-argument memory,
    // one dependent round trip each, otherwise)
    float kc[KC > 0 ? KC : 1];
    uint32_t pix[kP2Lanes];        // active pixel slot: local index
    uint16_t pair[ND * kP2Lanes];  // pair: slot << 5 | direction
    uint16_t first[kP2Lanes];      // first pair of each slot
    float acc[kP2Lanes];           // running vis of each slot (bright)
    float accD[kP2Lanes];          // ... dark channel (DUAL_AO)
    float p[kP2Lanes], r[kP2Lanes];
    uchar2 aoPrev[kP2Lanes];       // the pixel's pass-1 AO (bright, dark), read with the stencil
    // the pixel's BasicAOData, evaluated once per pixel, not per pair: the 16 floats pass 2 reads
    // (posVLength, radiusInPixels stay out; normalV too, except in the generic kernels, NB = 20: HBAO)
    alignas(16) float basic[kP2Lanes][NB];
    uint32_t nPix, nPair;
};

// One kP2Tile^2 tile whose top-left pixel is (x0, y0); flag: its busy-tile flag (cleared) or null
template <int N, int ND, bool SPEC, int NB, int KC>
__device__ __forceinline__ void pass2_tile(const SvaoArgs& a, uint32_t x0, uint32_t y0, uint32_t* flag,
                                           P2Shared<ND, NB, KC>& sh, uint32_t tid = threadIdx.x) {
    constexpr uint32_t T = kP2Tile, L = kP2Lanes;
    const rsd_vao_data& d = a.d;
    if (tid == 0) { sh.nPix = 0u; sh.nPair = 0u; }
    if constexpr (KC > 0) {
        static_assert(KC == 6 * ND + 64, "kc layout: 6 direction tables of ND, 16 jitter pairs, 16 + 16 noise terms");
        if (tid < (uint32_t)KC) {
            const uint32_t t = tid % ND, w = tid / ND, j = tid - 6u * ND;
            const float* src = w == 0 ? a.k.dirDx : w == 1 ? a.k.dirDy : w == 2 ? a.k.dirHeight
                             : w == 3 ? a.k.rcpPdf : w == 4 ? a.k.rcpHeight : a.k.ratioMin;
            sh.kc[tid] = tid < 6u * ND ? src[t] : j < 32u ? kJitter[j] : j < 48u ? a.k.sinNoise[j - 32u]
                                                                                  : a.k.cosNoise[j - 48u];
        }
    }
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
            basic_from(a, u, v, z, nl, b, KC > 0 ? sh.kc + 6 * ND + 32 : nullptr);
            sh.aoPrev[slot] = prev;
            float* q = sh.basic[slot];
            q[0] = b.posV.x; q[1] = b.posV.y; q[2] = b.posV.z;
            q[3] = b.normal.x; q[4] = b.normal.y; q[5] = b.normal.z;
            q[6] = b.tangent.x; q[7] = b.tangent.y; q[8] = b.tangent.z;
            q[9] = b.bitangent.x; q[10] = b.bitangent.y; q[11] = b.bitangent.z;
            q[12] = b.normalO.x; q[13] = b.normalO.y; q[14] = b.normalO.z;
            q[15] = b.radius;
            if constexpr (NB > 16) { q[16] = b.normalV.x; q[17] = b.normalV.y; q[18] = b.normalV.z; }
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
            if constexpr (NB > 16) b.normalV = mk(q[16], q[17], q[18]);  // HBAOKernel
            else b.normalV = b.normal;  // not read by the VAO kernel
            b.radiusInPixels = 0.0f;
            float p, r;
            if constexpr (SPEC) {
                const float nzd = make_nonzero(b.normalO.z, 0.0001f);
                const float ylx = rcp_refined(d.lowResolution[0]), yly = rcp_refined(d.lowResolution[1]);
                const bool posOk = kFastNumerics || (fabsf(b.posV.x) < 0x1p60f && fabsf(b.posV.y) < 0x1p60f);
                if (kFastNumerics && RSD_SCALED_ALLFAST) {
                    // fast numerics: every pair through the scaled lean path (pass 1's SCALED loop; the
                    // scale is exactly 1 for an unclamped pixel) -- one copy of the pair body, no vote
                    b.nzRcp = rcp_refined(nzd);
                    set_radius_scale(a, b);
                    svao_pass2_dir<N, true, true, true, ND>(a, b, u, v, (int)(e & 31u), p, r, ylx, yly, sh.kc);
                } else if (__ballot(b.radius != d.radius || !div_unscaled_den_ok(nzd) || !posOk) == 0u) {
                    b.nzRcp = rcp_refined(nzd);
                    svao_pass2_dir<N, true, true, false, ND>(a, b, u, v, (int)(e & 31u), p, r, ylx, yly, sh.kc);
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
    __shared__ P2Shared<ND, SPEC ? 16 : 20, SPEC ? 6 * ND + 64 : 0> sh;
    const uint32_t y0 = ((blockIdx.y / kPerGroup) * a.bandCount + a.bandIndex) * 32u + (blockIdx.y % kPerGroup) * kP2Tile +
                        a.guard;
    uint32_t* flag = a.tileFlags ? a.tileFlags + ((y0 - a.guard) / kP2Tile) * a.tilesX + blockIdx.x : nullptr;
    if (!flag || *flag != 0u) pass2_tile<N, ND, SPEC, SPEC ? 16 : 20, SPEC ? 6 * ND + 64 : 0>(a, blockIdx.x * kP2Tile + a.guard, y0, flag, sh);
}

// Whole-frame pass 2 over the busy-tile list pass 1 appended (tile_flags, ABI v5): workgroup i takes list
// entry i, so the busy tiles' workgroups are dispatched first and the empty ones (i >= count) form the
// tail, retiring at once while the busy ones run.  The flag-grid kernel above interleaves them (8160
// workgroups at configs[1], 21 % busy), and each holds its LDS until its own flag load returns.  One
// tile per workgroup: a grid-stride loop over the list keeps the loop-invariant tile set-up in registers
// (105-109 VGPRs, occupancy 4, vs 78 and 6).
template <int N, int ND, bool SPEC = false>
__global__ void __launch_bounds__(kP2Lanes) svao_pass2_list_kernel(SvaoArgs a) {
    __shared__ P2Shared<ND, SPEC ? 16 : 20, SPEC ? 6 * ND + 64 : 0> sh;
    // the count of this frame's list (pass 1 of the same generation appended to it; the next pass 1
    // appends to the other one): read-only here, no reset and no completion ticket
    const uint32_t n = __builtin_amdgcn_readfirstlane(a.tileCount[a.tileGen]);
    if (blockIdx.x >= n) return;
    // uniform: the tile origin stays in scalar registers like blockIdx in the flag-grid kernel
    const uint32_t t = __builtin_amdgcn_readfirstlane(a.tileList[blockIdx.x]);
    pass2_tile<N, ND, SPEC, SPEC ? 16 : 20, SPEC ? 6 * ND + 64 : 0>(a, (t % a.tilesX) * kP2Tile + a.guard, (t / a.tilesX) * kP2Tile + a.guard,
                                            a.tileFlags + t, sh);
}

// The specialised kernel's busy-tile list in a grid of the resident workgroups (launch_pass2: occupancy x
// CUs): workgroup i takes list entries i, i + grid, ..., so the empty tail is never dispatched -- with
// frames in flight its ~6 K empty workgroups held dispatch slots the other frames' passes wait for
// (configs[1], 200 frames with 4 in flight: 77.5-78.1 -> 74.5-75.2 us per frame; pass 2 alone 23.0-23.2
// -> 22.7-23.0 us; profiles/round4/pass2_loop/).  Only for frames of at most 8 tiles per resident
// workgroup (1080p): at 4K (~6 busy tiles per workgroup) the static stride serialises clustered busy
// tiles and one workgroup per tile is faster (pass 2 62.8 vs 73.6 us at configs[3]).  90 VGPRs (5 waves
// per SIMD) with the two opaque re-reads below; a 6-wave target spills.
template <int N, int ND, bool SPEC = false>
__global__ void __launch_bounds__(kP2Lanes) svao_pass2_loop_kernel(SvaoArgs a) {
    __shared__ P2Shared<ND, SPEC ? 16 : 20, SPEC ? 6 * ND + 64 : 0> sh;
    const uint32_t n = __builtin_amdgcn_readfirstlane(a.tileCount[a.tileGen]);
#pragma nounroll
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        // the arguments re-read from the kernel-argument segment per tile through an opaque pointer: values
        // derived from them cannot be hoisted out of the loop into registers (111 VGPRs otherwise)
        const __attribute__((address_space(4))) SvaoArgs* ka =
            (const __attribute__((address_space(4))) SvaoArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ka));
        const SvaoArgs& aa = *(const SvaoArgs*)ka;
        uint32_t tid = threadIdx.x;  // likewise the lane's LDS and pixel addresses
        asm volatile("" : "+v"(tid));
        const uint32_t t = __builtin_amdgcn_readfirstlane(aa.tileList[i]);
        pass2_tile<N, ND, SPEC, SPEC ? 16 : 20, SPEC ? 6 * ND + 64 : 0>(aa, (t % aa.tilesX) * kP2Tile + aa.guard,
                                                                        (t / aa.tilesX) * kP2Tile + aa.guard, aa.tileFlags + t, sh,
                                                                        tid);
        __syncthreads();  // the tile's last LDS reads before the next tile's writes
    }
}

// ---- host launchers of this TU's kernels (svao.hip picks the TU by rsd_svao_params.numerics)
// pass 1: variant 0 = generic, 1 = specialised with NUM_DIRECTIONS = 8, 2 = specialised, any count
void launch_pass1(const SvaoArgs& a, int variant, dim3 grid, dim3 block, hipStream_t s) {
    if (variant == 1) hipLaunchKernelGGL((svao_pass1_kernel<true, 8>), grid, block, 0, s, a);
    else if (variant == 2) hipLaunchKernelGGL((svao_pass1_kernel<true, 0>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((svao_pass1_kernel<false, 0>), grid, block, 0, s, a);
}

// the loop kernel's resident workgroups (its occupancy x CUs; 0 if unknown)
template <int N>
static uint32_t loop_resident() {
    static const uint32_t g = [] {
        int dev = 0, cus = 0, nb = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, svao_pass2_loop_kernel<N, 8, true>, kP2Lanes, 0) != hipSuccess)
            return 0u;
        return (uint32_t)(std::max(nb, 0) * std::max(cus, 0));
    }();
    return g;
}

// pass 2: N SD samples, nd directions; spec: the specialised 8-direction kernel; list: the busy-tile
// list kernel (workgroup i: list entry i) instead of the flag grid; loop: the specialised list in the
// resident grid (svao_pass2_loop_kernel)
void launch_pass2(const SvaoArgs& a, uint32_t N, uint32_t nd, bool spec, dim3 grid, dim3 block, hipStream_t s,
                  bool list, bool loop) {
#define RSD_P2K(K, NN, D, SP) hipLaunchKernelGGL((K<NN, D, SP>), grid, block, 0, s, a)
#define RSD_P2(NN)                                                                                           \
    if (list) {                                                                                              \
        if (nd == 32u) RSD_P2K(svao_pass2_list_kernel, NN, 32, false);                                       \
        else if (nd == 16u) RSD_P2K(svao_pass2_list_kernel, NN, 16, false);                                  \
        else if (spec && loop && loop_resident<NN>() && grid.x <= 8u * loop_resident<NN>())                  \
            hipLaunchKernelGGL((svao_pass2_loop_kernel<NN, 8, true>), dim3(std::min(grid.x, loop_resident<NN>())),  \
                               block, 0, s, a);                                                              \
        else if (spec) RSD_P2K(svao_pass2_list_kernel, NN, 8, true);                                          \
        else RSD_P2K(svao_pass2_list_kernel, NN, 8, false);                                                   \
    } else if (nd == 32u) RSD_P2K(svao_pass2_kernel, NN, 32, false);                                         \
    else if (nd == 16u) RSD_P2K(svao_pass2_kernel, NN, 16, false);                                           \
    else if (spec) RSD_P2K(svao_pass2_kernel, NN, 8, true);                                                   \
    else RSD_P2K(svao_pass2_kernel, NN, 8, false);
    switch (N) {
        case 1: RSD_P2(1) break;
        case 2: RSD_P2(2) break;
        case 4: RSD_P2(4) break;
        case 8: RSD_P2(8) break;
        default: RSD_P2(16) break;
    }
#undef RSD_P2
#undef RSD_P2K
}

}  // namespace RSD_SVAO_NS
}  // namespace rsd
