// sd_trace.hip -- the Ray-SD hot path on gfx950: BVH2 k-nearest any-hit traversal
// that fills the stochastic depth map, plus the primary-visibility (G-buffer) kernel
// built on the same traversal.
//
// Reference: StochasticDepthMapRT.rt.slang:39-105 (rayGen / anyHit),
//            Common.slangh:65-92 (initRayDesc), :102-254 (algorithm),
//            IntersectionHelpers.slang:109-180 (watertight triangle test),
//            Camera.slang:46-90 (pinhole rays).
//
// Any-hit order.  DXR calls any-hit in an unspecified order.  Here the
// any-hit stream is CANONICAL: ascending (t, primitive id), each triangle at most once.
// The Default reservoir and the KBuffer commit no later than the MAX_COUNT-th hit and a
// commit ends the stream (TMax = t), so the result only depends on the MAX_COUNT nearest
// hits: each lane keeps a sorted k-list of the k nearest (t, prim) keys in VGPRs, prunes
// the traversal with the k-th key exactly like a DXR commit shrinks TMax, and runs the
// reference algorithm over the sorted list afterwards.  The coverage-mask variant (no
// count bound) continues in chunks of k keys after the last one processed.  The result is
// independent of the BVH and of the traversal order -- the property the CPU oracle checks.
//
// Kernel shape: one lane per SD texel, one 64-lane wave per 8x8 texel tile (coherent
// primary rays), node stack in LDS (16 entries / lane) with a private overflow.  Nodes are
// 4-wide 128-B {child boxes, refs} records fetched as 8 x 16-B loads; triangles are 48-B
// records, a whole leaf (<= 4) fetched before it is tested.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "bvh_traverse.h"
#include "entry_grid.h"
#include "rsd_device.h"
#include "rsd_internal.h"

namespace rsd {

// ------------------------------------------------------------------------------------
// SD map kernel
// ------------------------------------------------------------------------------------
// queue-control words of one trace: {count[32], head[32]} of the live-ray queue partitions, the
// raster walk's live-tile count, spare
constexpr int kQctlWords = 5 * (int)kQueueParts + 32;
constexpr int kQctlTouch = 4 * (int)kQueueParts + 32;  // two-pass setup: touched texels listed per partition
constexpr int kQctlHead2 = 3 * (int)kQueueParts + 32;  // hybrid walk: the row walk's own dequeue heads
constexpr int kQctlLiveTiles = 2 * (int)kQueueParts;
constexpr int kQctlShort = 2 * (int)kQueueParts + 32;  // lpt: short-ray counts (filled from the partition's end)
#ifndef RSD_SETUP_WAVES
#define RSD_SETUP_WAVES 4
#endif
constexpr int kSetupWaves = RSD_SETUP_WAVES;  // sd_setup_kernel: tiles (waves) per workgroup (A/B: RSD_SETUP_WAVES)
struct SDArgs {
    const float4* nodes;  // BVH base (wide nodes, then triangle records)
    const float4* tris;   // = nodes + triOff
    uint32_t triOff;
    rsd_camera cam;
    const float* linearZ;
    int zW, zH;
    const uint32_t* rayMin;
    const uint32_t* rayMax;
    float* sd;
    int sdW, sdH;
    int guard;
    uint32_t impl, maxCount, jitter, normalize, rayInterval, cull;
    float alpha;
    const int32_t* lutIdx;  // coverage mask: stratified indices [N+1]
    const uint32_t* lut;    // coverage mask: look-up table [2^N]
    unsigned long long* counters;
    uint32_t partCap;  // live-ray queue: capacity of one partition
    // screen-band sharding: the 8-row tile rows t = bandStart + k * bandStep, k < bandN (an
    // interleaved band: start = index, step = count; a contiguous row range: step = 1)
    int bandStart, bandStep, bandN;
    int poolSoft;      // row traversal: above this many pooled items a row pops one item per step
    const float* rayTab;  // per-column / per-row ray terms (ray_table_kernel), see sd_ray
    uint32_t deadFast;    // setup may classify rayMin == asuint(FLT_MAX) texels as dead directly
    uint32_t* qctlNext;   // the other queue-control buffer, zeroed by the setup kernel
    uint32_t consume;     // RSD_SD_CONSUME_INTERVALS: setup resets every texel's interval after use
    uint32_t* rayMinW;    // writable aliases of rayMin / rayMax (consume only)
    uint32_t* rayMaxW;
    uint32_t alphaTest;   // USE_ALPHA_TEST and the scene has alpha data
    AlphaData alphaData;  // spread = RAY_CONE_SPREAD
    uint32_t f16;         // Use16Bit: the map is R16F / RG16F / RGBA16F (N <= 4)
    // raster walk (RSD_WALK_RASTER): per-texel queue slot (-1: no live ray), per-8x8-tile view-depth
    // range of its live rays, the K-key lists of the live rays (64-bit (t bits, prim) keys), the
    // prim -> triangle record map, and the camera projection onto the SD texel grid
    uint32_t raster, keysK, nTris;
    int32_t* slotMap;
    float2* tileRec;
    uint32_t* liveTiles;  // the tiles with live rays (count: qctl[kQctlLiveTiles])
    unsigned long long* keys64;
    const uint32_t* primRec;
    int tilesW;
    float projU[3], projV[3], projW[3];  // U / |U|^2, V / |V|^2, W / |W|^2
    float camWn[3];                      // normalize(W): view depth of a point = dot(P - o, Wn)
    float wClip;                         // near clip in projW units below every valid hit
    // longest-first queue (fused row walk): rays with TMax - TMin > lptLen go to the front of their
    // partition, the others to its back, so the expensive rays are dequeued first
    uint32_t lpt;
    float lptLen;
    // spread (row and quad walks): the static first rays of the persistent waves are dealt row-major over
    // the partition's waves (queue index i -> wave i % waves, row i / waves), so the longest-first rays land
    // one per wave instead of eight to a wave; 0: wave-major (index i -> wave i / rows, row i % rows)
    uint32_t spread;
    uint32_t quadStack;  // entries of each ray's LDS stack in the quad walks (quad_stack_entries)
    uint32_t qrange;     // diagnostics (RSD_TRACE_QRANGE): 0 every ray, 1 the longest-first rays only, 2 the others
    uint32_t hybridRowBlocks;  // hybrid walk: its first blocks run the row walk (sd_trace_hybrid_kernel)
    // two-pass setup (the full-resolution maps): sd_classify_kernel lists the texels pass 1 touched, partition p at
    // touchList[p * touchCap ..), and sd_live_kernel evaluates only those
    uint32_t* touchList;
    uint32_t touchCap;
    uint32_t liveBlocks;  // sd_live_kernel's grid (a multiple of kQueueParts)
    uint32_t rowPrio;          // hybrid walk: issue priority of the row blocks' waves (s_setprio; A/B, RSD_TRACE_ROWPRIO)
    uint32_t prio;             // issue priority of every setup and walk wave (s_setprio; A/B, RSD_TRACE_PRIO)
    // clean tiles (rsd_sd_params.d_tile_state): per 8x8 tile, tileSig when the last trace left every texel it
    // wrote at DEFAULT_DEPTH (0: unknown); such a tile without a live ray is not rewritten
    uint32_t* tileState;
    uint32_t tileSig;
    uint32_t tileCount;  // 8x8 tiles of the map: the texel masks follow the stamps in tileState (2 words per tile)
    // segment entry grid (entry_grid.h, canonical walks): the setup kernel looks up the frontier of
    // each live ray's segment and copies its items to entQ[slot * kEntryCap ..]
    uint32_t entOn;
    const uint4* entSlots;
    const float4* entItems;  // 2 x float4 per entry: {code, lo.xyz} {hi.xyz, 0}
    uint32_t entBits, entProbe;
    int entRmax;
    float entOrigin[3], entExtent;
    uint32_t* entQ;
    // diagnostics (instrumented fused walk, RSD_TRACE_RAYLOG): 8 words per queue slot {texel, steps,
    // nodes, leaves, keys found, clocks, TMax - TMin, TMin}
    uint32_t* rayLog;
    // diagnostics (RSD_SETUP_DIAG, results wrong by design): 1 the setup kernel returns at once (the launch floor of a
    // trace with an empty queue), 2 no texel is live (the setup's streaming part without the live rays' chains)
    uint32_t diag;
};

// tile stamp of a tile whose texel mask (the words after the stamps in tileState) names the texels the last trace left
// at DEFAULT_DEPTH (sd_classify_kernel; the one-pass setup treats it as unknown and rewrites the tile)
constexpr uint32_t kTileMaskSig = 0x100u;

// entry_lookup results besides first << 4 | count
constexpr uint32_t kEntryRoot = 0u;           // walk from the root
constexpr uint32_t kEntryDead = 0xffffffffu;  // no BVH box near the segment: no hit

// The frontier of the segment [TMin, TMax] of the ray (o, d) (entry_grid.h).  The segment's AABB
// is padded by 2^-14 of the coordinate magnitude (float rounding of o + d t, of the watertight
// test's hit point, and of the cell index below are all ~2^-23 relative); the loose cell of its
// centre at the finest level with m <= cell edge contains it.
__device__ __forceinline__ uint32_t entry_lookup(const SDArgs& a, f3 o, f3 d, float TMin, float TMax) {
    const float pad = 0x1p-14f * (fabsf(o.x) + fabsf(o.y) + fabsf(o.z) + TMax) + 1e-30f;
    const f3 p0 = o + d * TMin, p1 = o + d * TMax;
    const float lx = fminf(p0.x, p1.x) - pad, hx = fmaxf(p0.x, p1.x) + pad;
    const float ly = fminf(p0.y, p1.y) - pad, hy = fmaxf(p0.y, p1.y) + pad;
    const float lz = fminf(p0.z, p1.z) - pad, hz = fmaxf(p0.z, p1.z) + pad;
    const float m = fmaxf(fmaxf(hx - lx, hy - ly), hz - lz);
    const float E = a.entExtent;
    if (!(m <= E)) return kEntryRoot;  // longer than the scene (or NaN): the root
    int R = min(a.entRmax, ilogbf(E / m));
    while (R > 0 && m > ldexpf(E, -R)) --R;
    const float sc = ldexpf(1.0f, R) / E;
    const int i = (int)floorf((0.5f * (lx + hx) - a.entOrigin[0]) * sc);
    const int j = (int)floorf((0.5f * (ly + hy) - a.entOrigin[1]) * sc);
    const int k = (int)floorf((0.5f * (lz + hz) - a.entOrigin[2]) * sc);
    const int hi = 1 << R;
    if (i < -1 || j < -1 || k < -1 || i > hi || j > hi || k > hi) return kEntryDead;  // outside every box
    const unsigned long long key = ((unsigned long long)(R + 1) << 60) | ((unsigned long long)(i + 1) << 40) |
                                   ((unsigned long long)(j + 1) << 20) | (unsigned long long)(k + 1);
    uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - a.entBits));
    const uint32_t mask = (1u << a.entBits) - 1u;
    const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
    // linear probing, four slots per round trip (the same slots, checked in the same order, as one at a time: a
    // lane's chain of dependent probe loads is a quarter as long; round 6: configs[2] 180 -> 178 us, configs[1] and
    // [3] unchanged -- the setup's live-ray path is not bound by its probe chain)
    for (uint32_t n = 0; n <= a.entProbe; n += 4u, h = (h + 4u) & mask) {
        uint4 sl[4];
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) sl[k] = a.entSlots[(h + k) & mask];
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) {
            if (n + k > a.entProbe) return kEntryDead;
            if (sl[k].x == klo && sl[k].y == khi) return sl[k].z;
            if (sl[k].x == 0u && sl[k].y == 0u) return kEntryDead;
        }
    }
    return kEntryDead;  // the level is complete: an absent cell overlaps no BVH box
}

// queue slot of the qi-th ray of partition part (lpt: the long rays [0, nLong) from the front, the
// short ones from the back)
__device__ __forceinline__ uint32_t queue_slot(const SDArgs& a, uint32_t part, uint32_t qi, uint32_t nLong) {
    const uint32_t base = part * a.partCap;
    return (!a.lpt || qi < nLong) ? base + qi : base + a.partCap - 1u - (qi - nLong);
}

// Per-column and per-row terms of initRayDesc, evaluated once per frame size with exactly the
// operations sd_ray used to evaluate per texel (so the bits are unchanged):
//   [0, W)        cx[x]  = (sx + 0.5) / dimx + -jitterX      (pixel-centre dir, TMax)
//   [W, 2W)       u0[x]  = (sx + 0.5) / dimx                 (linearZ sample)
//   [2W, 6W)      jx[r][x] = (sx + jitterPos[r][x % 4].x) / dimx, r = y % 4
//   [6W, 6W+H)    cy[y]  = (sy + 0.5) / dimy + jitterY
//   [.., +H)      v0[y]  = (sy + 0.5) / dimy
//   [.., +4H)     jy[r][y] = (sy + jitterPos[y % 4][r].y) / dimy, r = x % 4
//   [.., +3)      normalize(camera W)
__global__ void ray_table_kernel(float* __restrict__ tab, int W, int H, int guard, uint32_t jitter, float jitterX,
                                 float jitterY, f3 camW) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int dimx = W - 2 * guard, dimy = H - 2 * guard;
    if (i < W) {
        const int sx = i - guard;
        tab[i] = ((float)sx + 0.5f) / (float)dimx + -jitterX;
        tab[W + i] = ((float)sx + 0.5f) / (float)dimx;
        for (int r = 0; r < 4; ++r) {
            float jx, jy;
            sd_jitter((uint32_t)i, (uint32_t)r, jitter != 0u, jx, jy);
            tab[2 * W + r * W + i] = ((float)sx + jx) / (float)dimx;
        }
    }
    if (i < H) {
        const int sy = i - guard;
        float* t = tab + 6 * W;
        t[i] = ((float)sy + 0.5f) / (float)dimy + jitterY;
        t[H + i] = ((float)sy + 0.5f) / (float)dimy;
        for (int r = 0; r < 4; ++r) {
            float jx, jy;
            sd_jitter((uint32_t)r, (uint32_t)i, jitter != 0u, jx, jy);
            t[2 * H + r * H + i] = ((float)sy + jy) / (float)dimy;
        }
    }
    if (i == 0) {
        const f3 wn = normalize(camW);
        float* t = tab + 6 * W + 6 * H;
        t[0] = wn.x;
        t[1] = wn.y;
        t[2] = wn.z;
    }
}


// initRayDesc, Common.slangh:65-92 (with Camera.slang:46-90).  Returns true if the ray
// interval is non-empty (TMin <= TMax): only those rays reach TraceRay.
__device__ __forceinline__ bool sd_ray(const SDArgs& a, int x, int y, f3& d, float& TMin, float& TMax, float& cosT) {
    const rsd_camera& c = a.cam;
    const int W = a.sdW, H = a.sdH;
    const int dimx = W - 2 * a.guard, dimy = H - 2 * a.guard;
    const int sx = x - a.guard, sy = y - a.guard;
    const float* t = a.rayTab;  // ray_table_kernel
    const float* ty = t + 6 * W;
    const f3 wn = mk(ty[6 * H], ty[6 * H + 1], ty[6 * H + 2]);  // normalize(camera W)
    const f3 dc = normalize(cam_dir(c, t[x], ty[y]));
    const float invCos = 1.0f / dot(wn, dc);
    TMax = c.farZ * invCos;  // computeRayPinhole tMax (pixel centre)
    d = normalize(cam_dir(c, t[2 * W + (y & 3) * W + x], ty[2 * H + (x & 3) * H + y]));  // SD jitter
    const float eps = 0.1f * c.nearZ;
    float depth = 0.0f;
    if (sx >= 0 && sy >= 0 && sx < dimx && sy < dimy) depth = tex_bilinear(a.linearZ, a.zW, a.zH, t[W + x], ty[H + y], true);
    cosT = dot(wn, d);
    TMin = depth / cosT + eps;
    if (a.rayInterval) {
        const size_t o = (size_t)y * a.sdW + x;
        const uint32_t iMin = a.rayMin ? a.rayMin[o] : 0u;
        if (iMin != 0u) TMin = hmax(asfloat(iMin), TMin);
        const uint32_t iMax = a.rayMax ? a.rayMax[o] : 0u;
        if (iMax != 0u) TMax = hmin(asfloat(iMax), TMax);
    }
    return TMin <= TMax;
}

// store, StochasticDepthMapRT.rt.slang:90-104 (Texture2DArray layout [layer][y][x][ch]).
// Use16Bit (StochasticDepthMapRT.cpp:192-198, N <= 4): the typed store converts to binary16,
// round to nearest even (v_cvt_f16_f32; overflow -> inf, e.g. DEFAULT_DEPTH without NORMALIZE).
__device__ __forceinline__ uint32_t f16_bits(float v) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)v);
}
template <int N>
__device__ __forceinline__ void sd_store(const SDArgs& a, int x, int y, const float (&depths)[N]) {
    const size_t plane = sd_plane_texels(a.sdW, a.sdH);
    const size_t o = sd_texel(x, y, a.sdW);
    if constexpr (N <= 4) {
        if (a.f16) {
            if constexpr (N == 1) {
                reinterpret_cast<uint16_t*>(a.sd)[o] = (uint16_t)f16_bits(depths[0]);
            } else if constexpr (N == 2) {
                reinterpret_cast<uint32_t*>(a.sd)[o] = f16_bits(depths[0]) | (f16_bits(depths[1]) << 16);
            } else {
                reinterpret_cast<uint2*>(a.sd)[o] = make_uint2(f16_bits(depths[0]) | (f16_bits(depths[1]) << 16),
                                                               f16_bits(depths[2]) | (f16_bits(depths[3]) << 16));
            }
            return;
        }
    }
    if constexpr (N == 1) {
        a.sd[o] = depths[0];
    } else if constexpr (N == 2) {
        reinterpret_cast<float2*>(a.sd)[o] = make_float2(depths[0], depths[1]);
    } else {
#pragma unroll
        for (int l = 0; l < N / 4; ++l)
            reinterpret_cast<float4*>(a.sd)[l * plane + o] =
                make_float4(depths[4 * l], depths[4 * l + 1], depths[4 * l + 2], depths[4 * l + 3]);
    }
}

// anyHit -> algorithm (Common.slangh:102-254) for ONE delivered hit: hash `rng` of its
// barycentrics, normalized view depth `z`, `af` = the alpha test failed.  Returns the commit
// decision (true: the any-hit shader accepts the hit, DXR TMax = t).
template <int N, int IMPL>
__device__ __forceinline__ bool sd_any_hit_impl(const SDArgs& a, float rng, float z, bool af, float (&depths)[N],
                                                uint32_t& cnt) {
    // IMPL >= 0: the implementation known at compile time (the specialised row walk: 0 = Default)
    if (IMPL < 0 && a.impl == 1u) {  // CoverageMask, Common.slangh:117-131, 189-209
        const int R = (int)floorf(a.alpha * (float)N + rng);
        uint32_t mask = 0u;
        if (R >= N) mask = 0xffffu;
        else if (R != 0) {
            const float rng2 = sd_hash(rng, z);  // hash3D(float3(bary, t))
            const float lo = (float)a.lutIdx[R], hi = (float)a.lutIdx[R + 1];
            mask = a.lut[(int)(lo + rng2 * (hi - lo))];
        }
        if (af) return cnt >= a.maxCount;  // alpha test failed: ignore the hit (count is 0 here)
        float maxT = 0.0f;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if ((mask & (1u << i)) && z < depths[i]) depths[i] = z;
            maxT = hmax(maxT, depths[i]);
        }
        return !(z < maxT);
    } else if (IMPL < 0 && a.impl == 3u) {  // KBuffer, Common.slangh:132-135, 211-232
        if (z >= depths[N - 1]) return true;
        cnt++;
        if (af) return cnt >= a.maxCount;
        const float rayT = z;
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (z < depths[i]) { const float tmp = depths[i]; depths[i] = z; z = tmp; }
        return (depths[N - 1] == rayT) || cnt >= a.maxCount;
    } else {  // Default reservoir, Common.slangh:136-153, 234-247
        uint32_t slot = cnt++;
        if (cnt > (uint32_t)N) slot = (uint32_t)(rng * (float)cnt);
#pragma unroll
        for (int i = 0; i < N; ++i)
            if ((uint32_t)i == slot && !(depths[i] <= z) && !af) depths[i] = z;
        return cnt >= a.maxCount;
    }
}
template <int N>
__device__ __forceinline__ bool sd_any_hit(const SDArgs& a, float rng, float z, bool af, float (&depths)[N],
                                           uint32_t& cnt) {
    return sd_any_hit_impl<N, -1>(a, rng, z, af, depths, cnt);
}

// ------------------------------------------------------------------------------------
// Quad-cooperative traversal (the SD trace).  A live SD ray is latency-bound: few rays,
// long dependent chains (MI355X: one wave alone issues a VALU op every ~4 cycles).  So
// each ray is walked by a QUAD of 4 lanes: in a node step lane q fetches and tests child
// q (the node is SoA, so the quad's 8 loads of 4 B are 16-B coalesced rows); in a leaf
// step lane q tests triangle q.  The 4 child keys are sorted across the quad with
// __shfl_xor compare-exchanges, the nearest is taken and the rest go to the ray's LDS
// stack.  Every lane keeps an identical copy of the ray's k-list; accepted hits are
// broadcast one by one and inserted by all 4 lanes.  A wave walks 16 rays.
// ------------------------------------------------------------------------------------
constexpr int kQuadRays = kBlock / 4;   // rays per wave
// per-ray LDS stack of the quad walks, sized per scene at launch (dynamic LDS, SDArgs.quadStack): a
// depth-first 4-wide walk holds <= 3 pushed siblings per level below its start, plus the entry items it
// has not popped yet, so quad_stack_entries(wide depth) entries never overflow.  Sized to the tree, the
// stack of configs[1]-[4]'s trees (4-wide depth 15-18: 56-64 entries) takes 7-8 KB per wave instead of round 4's fixed 96
// entries (12 KB), and LDS no longer caps the persistent waves below their register limit (13 per CU).
constexpr uint32_t quad_stack_entries(uint32_t wideDepth) { return (3u * wideDepth + 7u + 7u) & ~7u; }

// Quad-local exchange through DPP quad_perm (a VALU modifier: no LDS round trip, unlike
// __shfl / ds_bpermute).  CTRL = quad_perm(p0,p1,p2,p3) = p0 | p1<<2 | p2<<4 | p3<<6.
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppXor3 = 0x1B;
template <int CTRL>
__device__ __forceinline__ uint32_t dppu(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int L>  // value of quad lane L, in every lane of the quad
__device__ __forceinline__ float qbcf(float v) { return dppf<L * 0x55>(v); }
template <int L>
__device__ __forceinline__ uint32_t qbcu(uint32_t v) { return dppu<L * 0x55>(v); }
__device__ __forceinline__ float qself(float v, int j) {
    const float b0 = qbcf<0>(v), b1 = qbcf<1>(v), b2 = qbcf<2>(v), b3 = qbcf<3>(v);
    return j == 0 ? b0 : (j == 1 ? b1 : (j == 2 ? b2 : b3));
}
__device__ __forceinline__ uint32_t qselu(uint32_t v, int j) {
    const uint32_t b0 = qbcu<0>(v), b1 = qbcu<1>(v), b2 = qbcu<2>(v), b3 = qbcu<3>(v);
    return j == 0 ? b0 : (j == 1 ? b1 : (j == 2 ? b2 : b3));
}

template <int CTRL>
__device__ __forceinline__ void quad_cx(float& k, uint32_t& it, bool low) {
    const float ok = dppf<CTRL>(k);
    const uint32_t oi = dppu<CTRL>(it);
    const bool takeOther = low ? (ok < k) : (k < ok);
    k = takeOther ? ok : k;
    it = takeOther ? oi : it;
}

// Step clocks of the instrumented quad walk (rsd_counters.step_*; the latency floor of bench.py): per
// step of a ray -- one iteration of its quad's loop -- the wait for the step's own fetch (the
// instrumented build waits right after issuing it), its own box / triangle tests and merge, the stack
// push / pop from the point where the quad's branches reconverge, and the whole iteration from loop top
// to loop top (the remainder is the other branch of the wave: divergence).  s_memtime is wave-uniform;
// every quad's lane 0 accumulates its own ray's steps.
struct QuadClk {
    unsigned long long fetch = 0, tests = 0, stack = 0, total = 0, steps = 0;
};

// The quad walk's K nearest keys, distributed over the quad (round 5): lane q holds keys j = 4 s + q (slot s
// of S = K / 4), so each lane keeps K / 4 keys instead of a copy of all K (at K = 16: 8 instead of 32 VGPRs,
// and the record index is not kept at all -- the epilogue finds a key's triangle record through the scene's
// primitive -> record map).  Lane q's slots are exactly the keys whose terms lane q prepares in the epilogue.
// Every lane of the quad inserts the same key: its position is the quad-wide count of keys before it, and
// each slot at or after it takes the key before it -- lane q - 1's same slot, or (lane 0) lane 3's previous
// slot -- through one quad rotation per slot.  The K-th key is kept replicated for the pruning tests.
constexpr int kDppQuadRotR = 0x93;  // quad_perm [3, 0, 1, 2]: lane q reads lane q - 1 (lane 0: lane 3)
template <int K>
struct QuadKeys {
    static constexpr int S = K / 4;
    float t[S];
    uint32_t p[S];
    float kthT;  // key K - 1 (every lane)
    uint32_t kthP;
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < S; ++i) { t[i] = INFINITY; p[i] = 0xffffffffu; }
        kthT = INFINITY;
        kthP = 0xffffffffu;
    }
    __device__ __forceinline__ void insert(float nt, uint32_t np, int q) {
        uint32_t c = 0u;
#pragma unroll
        for (int i = 0; i < S; ++i) c += key_less(t[i], p[i], nt, np) ? 1u : 0u;
        c += dppu<kDppXor1>(c);
        c += dppu<kDppXor2>(c);  // every lane: the keys before the new one
        float rt[S];
        uint32_t rp[S];
#pragma unroll
        for (int i = 0; i < S; ++i) {
            rt[i] = dppf<kDppQuadRotR>(t[i]);
            rp[i] = dppu<kDppQuadRotR>(p[i]);
        }
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const uint32_t j = 4u * (uint32_t)i + (uint32_t)q;
            const float prevT = q > 0 ? rt[i] : (i > 0 ? rt[i > 0 ? i - 1 : 0] : INFINITY);
            const uint32_t prevP = q > 0 ? rp[i] : (i > 0 ? rp[i > 0 ? i - 1 : 0] : 0xffffffffu);
            const bool put = j == c, shift = j > c;
            t[i] = put ? nt : (shift ? prevT : t[i]);
            p[i] = put ? np : (shift ? prevP : p[i]);
        }
        kthT = qbcf<3>(t[S - 1]);
        kthP = qbcu<3>(p[S - 1]);
    }
};

template <int K>
__device__ __forceinline__ int trace_knearest_quad(const float4* __restrict__ bvh, uint32_t triOff, const RayCtx& r,
                                                   float tmin, float tmax, uint32_t cull, bool useLB, float lbT,
                                                   uint32_t lbP, QuadKeys<K>& kl, uint32_t* __restrict__ sItem,
                                                   float* __restrict__ sT, int q, int quadBase, TraceStats& st,
                                                   const uint32_t* __restrict__ ent, uint32_t nEnt,
                                                   QuadClk* clk = nullptr) {
    kl.clear();
    int sp = 0, found = 0;
    unsigned long long tTop = clk ? __builtin_amdgcn_s_memtime() : 0ull, tA = 0ull, tF = 0ull;
    uint32_t item = 0;
    if (nEnt) {
        // the segment's entry-grid frontier (entry_grid.h): item 0 first, the rest on the stack
        // (entry distance -inf: always popped; the result does not depend on the order)
        item = ent[0];
        if (q == 0)
            for (uint32_t e = 1; e < nEnt; ++e) {
                sItem[(e - 1) * kQuadRays] = ent[e];
                sT[(e - 1) * kQuadRays] = -INFINITY;
            }
        sp = (int)nEnt - 1;
    }
    const float tlo = useLB ? fmaxf(tmin, lbT) : tmin;
    const float* bf = reinterpret_cast<const float*>(bvh);
    while (true) {
        const uint32_t off = item & kOffMask;
        uint32_t next = kNoItem;
        if (clk) tA = __builtin_amdgcn_s_memtime();
        if (item & kLeafBit) {
            st.leaves++;
            const uint32_t cnt = ((item >> 29) & 3u) + 1u;
            bool acc = false;
            float t = 0.0f;
            uint32_t prim = 0u;
            float4 va = make_float4(0.0f, 0.0f, 0.0f, 0.0f), vb = va, vc = va;
            if ((uint32_t)q < cnt) {
                const float4* tp = bvh + off + 3u * (uint32_t)q;
                va = tp[0];
                vb = tp[1];
                vc = tp[2];
            }
            if (clk) {  // the step's fetch (the instrumented build waits here)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                tF = __builtin_amdgcn_s_memtime();
                if (q == 0) clk->fetch += tF - tA;
            }
            if ((uint32_t)q < cnt) {
                st.tris++;
                float bu, bv, det;
                if (intersect_tri(r, va, vb, vc, t, bu, bv, det) && t >= tmin && t <= tmax) {
                    prim = __float_as_uint(va.w);
                    acc = !culled(det, __float_as_uint(vb.w), cull) && (!useLB || key_less(lbT, lbP, t, prim)) &&
                          key_less(t, prim, kl.kthT, kl.kthP);
                }
            }
            uint32_t m = (uint32_t)(__ballot(acc) >> quadBase) & 0xfu;
            while (m) {
                const int j = __ffs(m) - 1;
                m &= m - 1u;
                const float tj = qself(t, j);
                const uint32_t pj = qselu(prim, j);
                if (key_less(tj, pj, kl.kthT, kl.kthP)) {
                    kl.insert(tj, pj, q);
                    found = found < K ? found + 1 : K;
                }
            }
            if (clk && q == 0) clk->tests += __builtin_amdgcn_s_memtime() - tF;
        } else {
            st.nodes++;
            const float thi = fminf(tmax, kl.kthT);
            const float* nb = bf + 4u * off;
            const float lox = nb[q], hix = nb[4 + q], loy = nb[8 + q], hiy = nb[12 + q], loz = nb[16 + q],
                        hiz = nb[20 + q];
            const uint32_t ref = __float_as_uint(nb[24 + q]), cnt = __float_as_uint(nb[28 + q]);
            if (clk) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                tF = __builtin_amdgcn_s_memtime();
                if (q == 0) clk->fetch += tF - tA;
            }
            float tn;
            const bool hit = ref != kNoItem && box_hit(r, lox, hix, loy, hiy, loz, hiz, tlo, thi, tn);
            float k = hit ? tn : INFINITY;
            uint32_t it = hit ? (cnt ? (kLeafBit | ((cnt - 1u) << 29) | (triOff + 3u * ref)) : 8u * ref) : kNoItem;
            const int m = __popc((uint32_t)(__ballot(hit) >> quadBase) & 0xfu);
            // sorting network (0,1)(2,3) (0,2)(1,3) (1,2) across the quad
            quad_cx<kDppXor1>(k, it, (q & 1) == 0);
            quad_cx<kDppXor2>(k, it, (q & 2) == 0);
            {
                const float ok = dppf<kDppXor3>(k);
                const uint32_t oi = dppu<kDppXor3>(it);
                const bool mid = q == 1 || q == 2;
                const bool takeOther = mid && ((q == 1) ? (ok < k) : (k < ok));
                k = takeOther ? ok : k;
                it = takeOther ? oi : it;
            }
            next = qbcu<0>(it);
            if (clk && q == 0) clk->tests += __builtin_amdgcn_s_memtime() - tF;
            if (q >= 1 && q < m) {
                const int slot = sp + (m - 1 - q);  // farthest deepest
                sItem[slot * kQuadRays] = it;
                sT[slot * kQuadRays] = k;
            }
            sp += m > 0 ? m - 1 : 0;
        }
        if (clk) tA = __builtin_amdgcn_s_memtime();  // the branches reconverged
        if (next == kNoItem) {
            const float thi = fminf(tmax, kl.kthT);
            while (sp > 0) {
                --sp;
                const float tt = sT[sp * kQuadRays];
                if (tt <= thi) { next = sItem[sp * kQuadRays]; break; }
            }
        }
        if (clk) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (q == 0) {
                clk->stack += t - tA;
                clk->total += t - tTop;
                clk->steps++;
            }
            tTop = t;
        }
        if (next == kNoItem) break;
        item = next;
    }
    return found;
}

// TraceRay + anyHit -> algorithm (Common.slangh:102-254) over the canonical hit stream,
// for the ray of this quad.  All 4 lanes end with identical depths.
template <int K, int N, bool SPEC = false>
__device__ __forceinline__ void sd_resolve(const SDArgs& a, f3 d, float TMin, float TMax, float cosT, float (&depths)[N],
                                           uint32_t* sItem, float* sT, int q, int quadBase, TraceStats& st,
                                           uint32_t& hitsDelivered, const uint32_t* ent = nullptr,
                                           uint32_t nEnt = 0u, QuadClk* clk = nullptr) {
    const rsd_camera& c = a.cam;
    RayCtx r;
    ray_setup(r, mk(c.posW[0], c.posW[1], c.posW[2]), d);
    QuadKeys<K> kl;
    uint32_t count = 0;
    bool commit = false, useLB = false;
    float lbT = 0.0f;
    uint32_t lbP = 0u;
    constexpr int J = (K + 3) / 4;  // hits per lane in the epilogue
    while (!commit) {
        // SPEC (as the row walk's): one chunk of K keys decides the texel -- no lower bound, no alpha test
        const int found = trace_knearest_quad<K>(a.nodes, a.triOff, r, TMin, TMax, a.cull, SPEC ? false : useLB, lbT, lbP, kl, sItem,
                                                 sT, q, quadBase, st, ent, nEnt, SPEC ? nullptr : clk);
        // barycentrics + hash of hit j are computed by lane j % 4 (re-running the identical
        // triangle test on the hit's record), then shared with the quad
        float rngL[J], zL[J];
        uint32_t afL = 0u;  // bit i: hit 4 i + q fails the alpha test
#pragma unroll
        for (int i = 0; i < J; ++i) {
            const int j = 4 * i + q;
            rngL[i] = 0.0f;
            zL[i] = 0.0f;
            uint32_t ti = 0u;
            if (j < found) ti = a.primRec[kl.p[i]];  // key j = 4 i + q is this lane's slot i
            if (j < found) {
                float t, bu, bv, det;
                const float4 v0 = a.tris[3 * ti], v1 = a.tris[3 * ti + 1], v2 = a.tris[3 * ti + 2];
                intersect_tri(r, v0, v1, v2, t, bu, bv, det);
                rngL[i] = sd_hash(bu, bv);
                float z = t * cosT;  // RayToViewDepth
                if (a.normalize) z = saturate((z - c.nearZ) / (c.farZ - c.nearZ));
                zL[i] = z;
                if (!SPEC && a.alphaTest && (__float_as_uint(v1.w) & 4u) &&
                    alpha_test_fails(a.alphaData, __float_as_uint(v0.w), v0, v1, v2, bu, bv, true, t, r.d))
                    afL |= 1u << i;
            }
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const float rng = qself(rngL[j / 4], j % 4);
            float z = qself(zL[j / 4], j % 4);
            const bool af = (qselu(afL, j % 4) >> (j / 4)) & 1u;
            if (commit || j >= found) continue;
            hitsDelivered++;
            commit = sd_any_hit_impl<N, SPEC ? 0 : -1>(a, rng, z, af, depths, count);
        }
        if (SPEC || found < K) break;  // stream exhausted (SPEC: a commit by the K-th key)
        useLB = true;
        lbT = kl.kthT;
        lbP = kl.kthP;
    }
}

// A live ray in the queue: 2 x 16 B {dir.xyz, TMin} {TMax, cosT, texel, nEnt}; nEnt > 0: the walk starts
// from the nEnt entry-grid items at entQ[slot * kEntryCap] instead of the root
__device__ __forceinline__ void ray_rec_load(const float4* __restrict__ q, uint32_t slot, f3& d, float& TMin,
                                             float& TMax, float& cosT, uint32_t& texel, uint32_t& nEnt) {
    const float4 r0 = q[2u * slot], r1 = q[2u * slot + 1u];
    d = mk(r0.x, r0.y, r0.z);
    TMin = r0.w;
    TMax = r1.x;
    cosT = r1.y;
    texel = __float_as_uint(r1.z);
    nEnt = __float_as_uint(r1.w);
}
__device__ __forceinline__ void ray_rec_load(const float4* __restrict__ q, uint32_t slot, f3& d, float& TMin,
                                             float& TMax, float& cosT, uint32_t& texel) {
    uint32_t nEnt;
    ray_rec_load(q, slot, d, TMin, TMax, cosT, texel, nEnt);
}

// The frontier of a live ray's segment (entry_grid.h) and the items whose boxes the ray passes (the walk's own child
// test); false: the segment can hit nothing (a culled ray: DEFAULT_DEPTH, no walk).  keep = 0 with true: from the root.
// B: frontier items loaded (and tested) per round trip -- kEntryCap (all at once: the one-pass setup, latency-bound),
// or kEntryCap / 2 (sd_live_kernel: half the box registers, more waves resident; the second batch only for a segment
// with more items)
template <uint32_t B = kEntryCap>
__device__ __forceinline__ bool entry_frontier(const SDArgs& a, f3 d, float TMin, float TMax, uint32_t& keep,
                                               uint32_t (&code)[kEntryCap]) {
    const f3 o = mk(a.cam.posW[0], a.cam.posW[1], a.cam.posW[2]);
    uint32_t ent = entry_lookup(a, o, d, TMin, TMax);
    if (a.counters) {  // roofline bytes of the lookup (rsd_counters.entry_*)
        atomicAdd(&a.counters[19], 1ull);
        if (ent != kEntryRoot && ent != kEntryDead) atomicAdd(&a.counters[20], (unsigned long long)(ent & 15u));
    }
    if (ent != kEntryRoot && ent != kEntryDead) {
        RayCtx r;
        ray_setup(r, o, d);
        const uint32_t first = ent >> 4, n = ent & 15u;
        if constexpr (B == kEntryCap) {
            float4 b0[kEntryCap], b1[kEntryCap];
#pragma unroll
            for (uint32_t e = 0; e < kEntryCap; ++e)  // every load before the first test
                if (e < n) { b0[e] = a.entItems[2u * (first + e)]; b1[e] = a.entItems[2u * (first + e) + 1u]; }
#pragma unroll
            for (uint32_t e = 0; e < kEntryCap; ++e) {
                float tn;
                code[e] = __float_as_uint(b0[e].x);
                if (e < n && box_hit(r, b0[e].y, b1[e].x, b0[e].z, b1[e].y, b0[e].w, b1[e].z, TMin, TMax, tn))
                    keep |= 1u << e;
            }
        } else {
#pragma unroll
        for (uint32_t e0 = 0; e0 < kEntryCap; e0 += B) {
            if (e0 >= n) break;
            float4 b0[B], b1[B];
#pragma unroll
            for (uint32_t k = 0; k < B; ++k)  // every load of the batch before its first test
                if (e0 + k < n) { b0[k] = a.entItems[2u * (first + e0 + k)]; b1[k] = a.entItems[2u * (first + e0 + k) + 1u]; }
#pragma unroll
            for (uint32_t k = 0; k < B; ++k) {
                float tn;
                code[e0 + k] = __float_as_uint(b0[k].x);
                if (e0 + k < n && box_hit(r, b0[k].y, b1[k].x, b0[k].z, b1[k].y, b0[k].w, b1[k].z, TMin, TMax, tn))
                    keep |= 1u << (e0 + k);
            }
        }
        }
        if (keep == 0u) ent = kEntryDead;
    }
    return ent != kEntryDead;
}

// Queue slots of a wave's live rays in partition `part` (every lane calls it; the queue is split in kQueueParts
// partitions, each with its own counters: one counter word serialises ~90 atomics/us) -- with a.lpt the rays
// longer than lptLen from the partition's front, the others from its back -- and their records + entry items.
__device__ __forceinline__ uint32_t queue_live(const SDArgs& a, float4* __restrict__ queue, uint32_t* __restrict__ qctl,
                                               uint32_t part, int lane, bool live, f3 d, float TMin, float TMax,
                                               float cosT, uint32_t texel, uint32_t keep,
                                               const uint32_t (&code)[kEntryCap]) {
    const unsigned long long m = __ballot(live);
    uint32_t slot;
    if (a.lpt) {
        // lptLen > 0: absolute interval length; < 0: relative to TMin
        const bool isLong = live && TMax - TMin > (a.lptLen >= 0.0f ? a.lptLen : -a.lptLen * TMin);
        const unsigned long long ml = __ballot(isLong), ms = m & ~ml;
        const uint32_t nl = (uint32_t)__popcll(ml), ns = (uint32_t)__popcll(ms);
        uint32_t bl = 0, bs = 0;
        if (lane == 0 && nl) bl = atomicAdd(&qctl[part], nl);
        if (lane == 0 && ns) bs = atomicAdd(&qctl[kQctlShort + part], ns);
        bl = __shfl(bl, 0);
        bs = __shfl(bs, 0);
        const unsigned long long below = (1ull << lane) - 1ull;
        slot = isLong ? part * a.partCap + bl + (uint32_t)__popcll(ml & below)
                      : part * a.partCap + a.partCap - 1u - (bs + (uint32_t)__popcll(ms & below));
    } else {
        uint32_t base = 0;
        if (lane == 0 && m) base = atomicAdd(&qctl[part], (uint32_t)__popcll(m));
        base = __shfl(base, 0);
        slot = part * a.partCap + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    }
    if (live) {
        // record word 7: the number of entry items stored to entQ (0: walk from the root)
        queue[2u * slot] = make_float4(d.x, d.y, d.z, TMin);
        queue[2u * slot + 1u] = make_float4(TMax, cosT, __uint_as_float(texel), __uint_as_float(__popc(keep)));
#pragma unroll
        for (uint32_t e = 0; e < kEntryCap; ++e)
            if ((keep >> e) & 1u) a.entQ[(size_t)slot * kEntryCap + __popc(keep & ((1u << e) - 1u))] = code[e];
    }
    return slot;
}

// Phase 1 (rayGen up to TraceRay): one lane per SD texel of the band.  Rays whose interval
// is empty keep DEFAULT_DEPTH and are written here; the others are appended to a compact
// queue of ray records (one atomic per wave) so that phase 2 runs full waves of live rays
// and starts traversing without recomputing the ray.
// The queue control words {count[32], head[32]} are double-buffered across calls: call k
// uses buffer k % 2 (zero on entry) and its setup kernel zeroes buffer (k + 1) % 2, which
// call k - 1 finished with (stream order) -- no memset launch per trace.
template <int N>
__global__ void __launch_bounds__(kSetupWaves * kBlock) sd_setup_kernel(SDArgs a, float4* __restrict__ queue,
                                                                        uint32_t* __restrict__ qctl,
                                                                        uint32_t* __restrict__ qctlNext) {
    if (a.prio) __builtin_amdgcn_s_setprio(2);
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int w = threadIdx.x; w < kQctlWords; w += kSetupWaves * kBlock) qctlNext[w] = 0u;
    if (a.diag == 1u) return;
    // one wave per 8x8 tile, kSetupWaves tiles of a tile row per workgroup
    const int lane = threadIdx.x & (kBlock - 1);
    const int tileX = (int)blockIdx.x * kSetupWaves + (int)(threadIdx.x / kBlock);
    const int tilesX = (a.sdW + kTile - 1) / kTile;
    const int x = tileX * kTile + (lane & (kTile - 1));
    // consume: the grid covers every tile row of the map; other bands' rows only get their
    // intervals reset (SVAO.cpp:334-340's clear for the next frame)
    const int tileRow = a.consume ? (int)blockIdx.y : (int)blockIdx.y * a.bandStep + a.bandStart;
    const int y = tileRow * kTile + (lane / kTile);
    const bool inside = x < a.sdW && y < a.sdH;
    if (a.consume && (tileRow < a.bandStart || (tileRow - a.bandStart) % a.bandStep != 0 ||
                      (tileRow - a.bandStart) / a.bandStep >= a.bandN)) {
        // only texels whose words are not at their reset values (8 B read instead of 8 B written: HBM reads
        // are the cheaper direction, and most texels were never touched)
        if (inside && (a.rayMinW[(size_t)y * a.sdW + x] != 0x7f7fffffu || a.rayMaxW[(size_t)y * a.sdW + x] != 0u)) {
            a.rayMinW[(size_t)y * a.sdW + x] = 0x7f7fffffu;  // asuint(FLT_MAX)
            a.rayMaxW[(size_t)y * a.sdW + x] = 0u;
        }
        return;  // uniform over the workgroup
    }
    // the tile's clean stamp (one word per wave), loaded first so that its latency hides behind the texel's
    const bool tileIn = tileX < tilesX;
    const uint32_t tilePrev = a.tileState && tileIn ? a.tileState[(size_t)tileRow * tilesX + tileX] : 0u;
    bool live = false, culled = false;
    uint32_t keep = 0u;                    // keep: the frontier items the ray passes
    uint32_t code[kEntryCap];              // their item codes
    f3 d = mk(0.0f, 0.0f, 0.0f);
    float TMin = 0.0f, TMax = 0.0f, cosT = 0.0f;
    if (inside) {
        // rayMin never lowered by pass 1 (still asuint(FLT_MAX)): TMin >= FLT_MAX > TMax, the
        // texel is dead without evaluating its ray (a.deadFast: the host proved TMax < FLT_MAX)
        const uint32_t rmin = a.rayMin[(size_t)y * a.sdW + x];
        const bool untouched = a.deadFast && rmin == 0x7f7fffffu;
        // consume: words already at their reset values are not rewritten (both read here, one round trip)
        const bool atReset = a.consume && rmin == 0x7f7fffffu && a.rayMax[(size_t)y * a.sdW + x] == 0u;
        live = !untouched && sd_ray(a, x, y, d, TMin, TMax, cosT) && a.diag != 2u;
        if (a.consume && !atReset) {  // after the last read of this texel's interval
            a.rayMinW[(size_t)y * a.sdW + x] = 0x7f7fffffu;
            a.rayMaxW[(size_t)y * a.sdW + x] = 0u;
        }
        if (live && a.entOn && !entry_frontier(a, d, TMin, TMax, keep, code)) {
            live = false;  // a live interval that can hit nothing: DEFAULT_DEPTH, no walk
            culled = true;
        }
    }
    const unsigned long long m = __ballot(live);
    // a tile without a live ray whose texels the previous trace of this map left at DEFAULT_DEPTH already
    // holds this trace's bits (the full-resolution maps: most of the map, 64 B per texel at N = 16)
    const bool clean = a.tileState && m == 0ull && tilePrev == a.tileSig;
    if (inside && !live && !clean) {
        float depths[N];
        const float DEFAULT = a.normalize ? 1.0f : 3.40282347e+37f;  // Common.slangh:16
#pragma unroll
        for (int i = 0; i < N; ++i) depths[i] = DEFAULT;
        sd_store<N>(a, x, y, depths);
    }
    if (a.tileState && tileIn && lane == 0) {  // a live ray may store anything: the tile is unknown again
        const uint32_t now = m == 0ull ? a.tileSig : 0u;
        if (now != tilePrev) a.tileState[(size_t)tileRow * tilesX + tileX] = now;
    }
    const uint32_t n = (uint32_t)__popcll(m);
    // the queue is split in kQueueParts partitions (block b -> partition b % kQueueParts), each
    // with its own counter: one counter word serialises ~90 atomics/us.
    const uint32_t lin = blockIdx.y * (uint32_t)tilesX + (uint32_t)tileX;
    const uint32_t part = lin % kQueueParts;
    const uint32_t slot = queue_live(a, queue, qctl, part, lane, live, d, TMin, TMax, cosT,
                                     (uint32_t)y * (uint32_t)a.sdW + x, keep, code);
    if (a.counters && culled) atomicAdd(&a.counters[1], 1ull);  // still an active ray (rsd_counters)
    if (a.raster) {
        // the raster walk's inputs: slot map, the tile's view-depth range, empty key lists
        if (inside) a.slotMap[(size_t)y * a.sdW + x] = live ? (int32_t)slot : -1;
        float zlo = live ? TMin * cosT : INFINITY, zhi = live ? TMax * cosT : -INFINITY;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            zlo = fminf(zlo, __shfl_xor(zlo, o));
            zhi = fmaxf(zhi, __shfl_xor(zhi, o));
        }
        if (lane == 0 && tileX < tilesX) {
            a.tileRec[(size_t)tileRow * a.tilesW + tileX] = make_float2(zlo, zhi);
            if (n) a.liveTiles[atomicAdd(&qctl[kQctlLiveTiles], 1u)] = (uint32_t)tileRow * (uint32_t)a.tilesW + tileX;
        }
        if (live)
            for (uint32_t k = 0; k < a.keysK; ++k) a.keys64[(size_t)slot * a.keysK + k] = ~0ull;
        if (a.counters && lane == 0) atomicAdd(&a.counters[1], (unsigned long long)n);
    }
    const unsigned long long in = __ballot(inside);
    if (a.counters && lane == 0) atomicAdd(&a.counters[0], (unsigned long long)__popcll(in));
    if (a.counters && clean && lane == 0) atomicAdd(&a.counters[25], (unsigned long long)__popcll(in));
}

// Phase 2: persistent waves pull 16 live rays (one per quad) at a time from the queue
// until it drains (every wave reaches the exit: the head only grows, the count is fixed).
// The first chunk of each wave is static (blockIdx); later ones come from one atomic head
// that starts after the static range, so a wave with no static chunk exits without an
// atomic (one head word serialises ~90 dequeues/us, MI355X_MICROARCH.md "dequeue").

// Two-pass setup (round 6; the full-resolution maps).  The one-pass setup evaluates each texel's
// ray in the lane of its texel, so every wave that holds a live ray carries its lookup chain (the ray, the entry-grid
// probe, the frontier boxes, the queue atomics: ~5 dependent round trips), and at configs[4] 258 K such waves pass
// through 24 slots per CU -- 42 rounds of that chain.  Here pass A streams over the map with one light lane per
// texel (interval words, the tiles' clean stamps, DEFAULT_DEPTH where no texel of a tile was touched and the tile is
// not clean) and lists the touched texels -- rayMin lowered by pass 1 -- per queue partition (one atomic per
// workgroup); pass B gives every listed texel a lane, densely, for the chain.  Same records, same stores: the
// bits of the map are the one-pass setup's (a tile with touched but dead texels is stamped unknown instead of
// clean: it is rewritten once more on its next trace, conservatively).
constexpr int kClassWaves = 4;   // sd_classify_kernel: waves per workgroup
#ifndef RSD_CLASS_TILES
#define RSD_CLASS_TILES 4
#endif
constexpr int kClassTiles = RSD_CLASS_TILES;  // sd_classify_kernel: 8x8 tiles per wave (their loads in one round trip)
constexpr int kLiveBlock = 256;  // sd_live_kernel: lanes per workgroup (4 waves)

template <int N>
__global__ void __launch_bounds__(kClassWaves * kBlock) sd_classify_kernel(SDArgs a, uint32_t* __restrict__ qctl,
                                                                           uint32_t* __restrict__ qctlNext) {
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int w = threadIdx.x; w < kQctlWords; w += kClassWaves * kBlock) qctlNext[w] = 0u;
    __shared__ uint32_t sCount[kClassWaves + 1];
    const int lane = threadIdx.x & (kBlock - 1), wave = (int)(threadIdx.x / kBlock);
    const int tilesX = (a.sdW + kTile - 1) / kTile;
    const int tileX0 = ((int)blockIdx.x * kClassWaves + wave) * kClassTiles;  // the wave's kClassTiles tiles
    const int tileRow = a.consume ? (int)blockIdx.y : (int)blockIdx.y * a.bandStep + a.bandStart;
    const int y = tileRow * kTile + (lane / kTile);
    const bool otherBand = a.consume && (tileRow < a.bandStart || (tileRow - a.bandStart) % a.bandStep != 0 ||
                                         (tileRow - a.bandStart) / a.bandStep >= a.bandN);
    // every load of the wave's texels and tile stamps first (one round trip for the kClassTiles tiles)
    uint32_t rmin[kClassTiles], rmax[kClassTiles], prev[kClassTiles], mlo[kClassTiles], mhi[kClassTiles];
#pragma unroll
    for (int t = 0; t < kClassTiles; ++t) {
        const int x = (tileX0 + t) * kTile + (lane & (kTile - 1));
        const bool inside = x < a.sdW && y < a.sdH;
        const size_t o = (size_t)y * a.sdW + x;
        rmin[t] = inside ? a.rayMin[o] : 0x7f7fffffu;
        rmax[t] = inside && a.consume ? a.rayMax[o] : 0u;
        prev[t] = a.tileState && !otherBand && tileX0 + t < tilesX ? a.tileState[(size_t)tileRow * tilesX + tileX0 + t] : 0u;
        // the tile's texel mask (stamp kSubSig: the texels the last trace left at DEFAULT_DEPTH), loaded with the stamp
        const size_t mw = a.tileCount + 2u * ((size_t)tileRow * tilesX + tileX0 + t);
        mlo[t] = a.tileState && !otherBand && tileX0 + t < tilesX ? a.tileState[mw] : 0u;
        mhi[t] = a.tileState && !otherBand && tileX0 + t < tilesX ? a.tileState[mw + 1u] : 0u;
    }
    if (otherBand) {
        // other bands' rows: the intervals are reset only (sd_setup_kernel)
#pragma unroll
        for (int t = 0; t < kClassTiles; ++t) {
            const int x = (tileX0 + t) * kTile + (lane & (kTile - 1));
            const size_t o = (size_t)y * a.sdW + x;
            if (x < a.sdW && y < a.sdH && (rmin[t] != 0x7f7fffffu || rmax[t] != 0u)) {
                a.rayMinW[o] = 0x7f7fffffu;
                a.rayMaxW[o] = 0u;
            }
        }
        return;  // uniform over the workgroup
    }
    const float DEFAULT = a.normalize ? 1.0f : 3.40282347e+37f;  // Common.slangh:16
    unsigned long long m[kClassTiles];
    uint32_t waveCount = 0;
#pragma unroll
    for (int t = 0; t < kClassTiles; ++t) {
        const int x = (tileX0 + t) * kTile + (lane & (kTile - 1));
        m[t] = __ballot(x < a.sdW && y < a.sdH && rmin[t] != 0x7f7fffffu);  // touched (a.deadFast: else dead)
        waveCount += (uint32_t)__popcll(m[t]);
    }
    // the touched texels of the workgroup: one atomic on its partition's list counter, issued before the stores
    // below so that its round trip overlaps them
    if (lane == 0) sCount[wave] = waveCount;
    __syncthreads();
    uint32_t wgBase = 0, tot = 0;
    if (threadIdx.x == 0) {
        for (int w = 0; w < kClassWaves; ++w) { const uint32_t c = sCount[w]; sCount[w] = tot; tot += c; }
        if (tot) wgBase = atomicAdd(&qctl[kQctlTouch + (blockIdx.y * gridDim.x + blockIdx.x) % kQueueParts], tot);
    }
#pragma unroll
    for (int t = 0; t < kClassTiles; ++t) {
        const int x = (tileX0 + t) * kTile + (lane & (kTile - 1));
        const bool inside = x < a.sdW && y < a.sdH;
        const size_t o = (size_t)y * a.sdW + x;
        const bool touched = (m[t] >> lane) & 1ull;
        // consume: untouched words not at their reset values are reset here; pass B resets the touched ones after
        // reading them
        if (a.consume && inside && !touched && rmax[t] != 0u) a.rayMaxW[o] = 0u;
        const bool clean = a.tileState && m[t] == 0ull && prev[t] == a.tileSig;
        // per-texel: the last trace left this texel at DEFAULT_DEPTH (a whole-tile stamp, or the tile's mask)
        const uint64_t mask = ((uint64_t)mhi[t] << 32) | mlo[t];
        const bool known = a.tileState && (prev[t] == a.tileSig || (prev[t] == (a.tileSig | kTileMaskSig) && ((mask >> lane) & 1ull)));
#ifdef RSD_DIAG_CLASSIFY_NOSTORE
        if (false) {  // diagnostics (results wrong by design): the classify pass without its DEFAULT_DEPTH stores
#else
        if (inside && !touched && !known) {
#endif
            float depths[N];
#pragma unroll
            for (int i = 0; i < N; ++i) depths[i] = DEFAULT;
            sd_store<N>(a, x, y, depths);
        }
        if (a.tileState && tileX0 + t < tilesX && lane == 0) {
            // no touched texel: the whole tile is DEFAULT_DEPTH now; else its untouched texels are (a touched one may
            // turn live: unknown), recorded in the tile's mask
            const uint32_t now = m[t] == 0ull ? a.tileSig : (a.tileSig | kTileMaskSig);
            if (now != prev[t]) a.tileState[(size_t)tileRow * tilesX + tileX0 + t] = now;
            if (m[t] != 0ull) {
                const uint64_t nm = ~m[t];
                const size_t mw = a.tileCount + 2u * ((size_t)tileRow * tilesX + tileX0 + t);
                if (prev[t] != now || (uint32_t)nm != mlo[t]) a.tileState[mw] = (uint32_t)nm;
                if (prev[t] != now || (uint32_t)(nm >> 32) != mhi[t]) a.tileState[mw + 1u] = (uint32_t)(nm >> 32);
            }
        }
        if (a.counters) {
            const unsigned long long in = __ballot(inside), kept = __ballot(inside && !touched && known);
            if (lane == 0) atomicAdd(&a.counters[0], (unsigned long long)__popcll(in));
            if (lane == 0) atomicAdd(&a.counters[25], (unsigned long long)__popcll(kept));
        }
    }
    if (threadIdx.x == 0)
        sCount[kClassWaves] = tot ? ((blockIdx.y * gridDim.x + blockIdx.x) % kQueueParts) * a.touchCap + wgBase : 0u;
    __syncthreads();
    uint32_t at = sCount[kClassWaves] + sCount[wave];
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (int t = 0; t < kClassTiles; ++t) {
        if ((m[t] >> lane) & 1ull)
            a.touchList[at + (uint32_t)__popcll(m[t] & below)] =
                (uint32_t)y * (uint32_t)a.sdW + (uint32_t)((tileX0 + t) * kTile + (lane & (kTile - 1)));
        at += (uint32_t)__popcll(m[t]);
    }
}

// Pass B: lane i of list partition p's texels (blocks b with b % kQueueParts == p stride over them).  A list partition
// holds whole classify workgroups (128 x 8-texel strips), so the rays of one cluster of long segments would share a
// queue partition -- and the static rows of the walk that read it; the wave of 64 listed texels c therefore appends to
// queue partition (p + c) % kQueueParts (one-pass setup: tile t -> t % kQueueParts), which holds at most
// touchCap + 2 * 64 * kQueueParts rays (partCap covers that).
#ifndef RSD_LIVE_WAVES
#define RSD_LIVE_WAVES 1
#endif
template <int N>
__global__ void __launch_bounds__(kLiveBlock) __attribute__((amdgpu_waves_per_eu(RSD_LIVE_WAVES))) sd_live_kernel(SDArgs a, float4* __restrict__ queue,
                                                             uint32_t* __restrict__ qctl) {
    const uint32_t part = blockIdx.x % kQueueParts, blocksPerPart = gridDim.x / kQueueParts;
    const uint32_t count = min(__hip_atomic_load(&qctl[kQctlTouch + part], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               a.touchCap);
    const int lane = threadIdx.x & (kBlock - 1);
    const float DEFAULT = a.normalize ? 1.0f : 3.40282347e+37f;  // Common.slangh:16
    for (uint32_t base = (blockIdx.x / kQueueParts) * kLiveBlock; base < count; base += blocksPerPart * kLiveBlock) {
        const uint32_t i = base + threadIdx.x;  // (wave-uniform loop: every lane of a wave reaches the ballots)
        bool live = false, culled = false;
        uint32_t keep = 0u, code[kEntryCap];
        f3 d = mk(0.0f, 0.0f, 0.0f);
        float TMin = 0.0f, TMax = 0.0f, cosT = 0.0f;
        uint32_t texel = 0u;
        int x = 0, y = 0;
        if (i < count) {
            texel = a.touchList[part * a.touchCap + i];
            x = (int)(texel % (uint32_t)a.sdW);
            y = (int)(texel / (uint32_t)a.sdW);
            live = sd_ray(a, x, y, d, TMin, TMax, cosT);
            if (a.consume) {  // after the last read of this texel's interval
                a.rayMinW[texel] = 0x7f7fffffu;
                a.rayMaxW[texel] = 0u;
            }
            if (live && a.entOn && !entry_frontier<kEntryCap / 2>(a, d, TMin, TMax, keep, code)) {
                live = false;
                culled = true;
            }
            if (!live) {
                float depths[N];
#pragma unroll
                for (int k = 0; k < N; ++k) depths[k] = DEFAULT;
                sd_store<N>(a, x, y, depths);
            }
        }
        const uint32_t qpart = (part + (base + threadIdx.x - (uint32_t)lane) / (uint32_t)kBlock) % kQueueParts;
        queue_live(a, queue, qctl, qpart, lane, live, d, TMin, TMax, cosT, texel, keep, code);
        if (a.counters && culled) atomicAdd(&a.counters[1], 1ull);  // still an active ray (rsd_counters)
    }
}

template <int K, int N, bool SPEC = false, bool CNT = false>
__device__ __forceinline__ void sd_trace_queue_body(const SDArgs& a, const float4* __restrict__ queue,
                                                    uint32_t* __restrict__ qctl, uint32_t* sQuadStack, uint32_t bid,
                                                    uint32_t nb, uint32_t qr) {
    // sQuadStack: a.quadStack entries per ray, items then their entry distances; (bid, nb): this wave's block
    // among the walk's blocks (the hybrid kernel's quad blocks follow its row blocks); qr: the queue range
    uint32_t* sItem = sQuadStack;
    float* sT = reinterpret_cast<float*>(sQuadStack + a.quadStack * kQuadRays);
    const int lane = threadIdx.x;
    const int q = lane & 3, quad = lane >> 2, quadBase = lane & ~3;
    // wave w serves partition w % kQueueParts (nb is a multiple of kQueueParts)
    const uint32_t part = bid % kQueueParts, wavesPerPart = nb / kQueueParts;
    const uint32_t nLong = __hip_atomic_load(&qctl[part], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (RSD_TRACE_QRANGE, diagnostics: only the longest-first rays, or only the others)
    const uint32_t q0 = qr == 2u ? nLong : 0u;
    const uint32_t count = (qr == 1u ? nLong : nLong + (a.lpt ? __hip_atomic_load(&qctl[kQctlShort + part],
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u)) - q0;
    TraceStats st{0u, 0u, 0u};
    uint32_t active = 0, hitsDelivered = 0, maxNodes = 0, maxSteps = 0;
    unsigned long long sumCycles = 0, maxCycles = 0;
    // instrumented traces (counters): the step clocks of every ray (QuadClk) and the clock calibration of
    // the first wave (s_memtime ticks against the 100 MHz s_memrealtime), as the row walk's
    QuadClk clk;
    unsigned long long cal0 = 0, calR0 = 0;
    if (CNT && bid == 0) {
        cal0 = __builtin_amdgcn_s_memtime();
        calR0 = __builtin_amdgcn_s_memrealtime();
    }
    uint32_t base = (bid / kQueueParts) * (uint32_t)kQuadRays;
    bool firstChunk = true;
    while (base < count || (firstChunk && a.spread)) {
        // the static first chunk (spread: quad q of the partition's wave w takes index q * waves + w)
        const uint32_t qi = firstChunk && a.spread ? (uint32_t)quad * wavesPerPart + bid / kQueueParts
                                                   : base + (uint32_t)quad;
        firstChunk = false;
        if (qi < count) {
            f3 d;
            float TMin, TMax, cosT;
            uint32_t idx, nEnt;
            const uint32_t slot = queue_slot(a, part, qi + q0, nLong);
            ray_rec_load(queue, slot, d, TMin, TMax, cosT, idx, nEnt);
            const int x = (int)(idx % (uint32_t)a.sdW), y = (int)(idx / (uint32_t)a.sdW);
            float depths[N];
            const float DEFAULT = a.normalize ? 1.0f : 3.40282347e+37f;
#pragma unroll
            for (int i = 0; i < N; ++i) depths[i] = DEFAULT;
            const uint32_t n0 = st.nodes, l0 = st.leaves;
            const unsigned long long c0 = a.counters ? __builtin_amdgcn_s_memtime() : 0ull;
            sd_resolve<K, N, SPEC>(a, d, TMin, TMax, cosT, depths, &sItem[quad], &sT[quad], q, quadBase, st,
                             hitsDelivered, a.entOn ? a.entQ + (size_t)slot * kEntryCap : nullptr, nEnt,
                             CNT ? &clk : nullptr);
            if (q == 0) {
                if (a.counters) {
                    const unsigned long long dc = __builtin_amdgcn_s_memtime() - c0;
                    sumCycles += dc;
                    maxCycles = dc > maxCycles ? dc : maxCycles;
                }
                maxNodes = max(maxNodes, st.nodes - n0);
                maxSteps = max(maxSteps, st.nodes - n0 + st.leaves - l0);
                active++;
                sd_store<N>(a, x, y, depths);
            }
        }
        if (lane == 0)
            base = wavesPerPart * (uint32_t)kQuadRays + atomicAdd(&qctl[kQueueParts + part], (uint32_t)kQuadRays);
        base = __shfl(base, 0);
    }
    if (a.counters) {
        if (q != 0) hitsDelivered = 0;
        atomicAdd(&a.counters[1], (unsigned long long)active);
        atomicAdd(&a.counters[2], (unsigned long long)(q == 0 ? st.nodes : 0u));
        atomicAdd(&a.counters[3], (unsigned long long)st.tris);
        atomicAdd(&a.counters[4], (unsigned long long)hitsDelivered);
        atomicMax(&a.counters[5], (unsigned long long)maxNodes);
        atomicMax(&a.counters[6], (unsigned long long)maxSteps);
        atomicAdd(&a.counters[7], sumCycles);
        atomicMax(&a.counters[8], maxCycles);
        atomicAdd(&a.counters[9], (unsigned long long)(q == 0 ? st.leaves : 0u));
        if (CNT && q == 0) {  // step clocks (rsd_counters.step_*): compute = own tests + the other branch
            atomicAdd(&a.counters[14], clk.steps);
            atomicAdd(&a.counters[16], clk.fetch);
            atomicAdd(&a.counters[17], clk.total - clk.fetch - clk.stack);
            atomicAdd(&a.counters[18], clk.stack);
            atomicAdd(&a.counters[24], clk.tests);
        }
        if (CNT && bid == 0 && lane == 0) {
            const unsigned long long cal1 = __builtin_amdgcn_s_memtime(), calR1 = __builtin_amdgcn_s_memrealtime();
            atomicMax(&a.counters[21], cal1 - cal0);
            atomicMax(&a.counters[22], calR1 - calR0);
        }
    }
}

template <int K, int N, bool SPEC = false, bool CNT = false>
__global__ void __launch_bounds__(kBlock) sd_trace_queue_kernel(SDArgs a, const float4* __restrict__ queue,
                                                                uint32_t* __restrict__ qctl) {
    extern __shared__ uint32_t sQuadStack[];
    sd_trace_queue_body<K, N, SPEC, CNT>(a, queue, qctl, sQuadStack, blockIdx.x, gridDim.x, a.qrange);
}

// ------------------------------------------------------------------------------------
// Traversal-order any-hit stream (rsd_sd_params.hit_order = RSD_HIT_ORDER_TRAVERSAL, rsd.h).
// The DXR-like order: a depth-first walk of the 4-wide BVH, children nearest entry distance
// first (the quad sorting network below; ties keep child-slot order), leaf triangles in record
// order, each triangle delivered once to anyHit -> algorithm as it is found.  A committed hit
// (Common.slangh: algorithm() == true, the any-hit shader does not IgnoreHit) shrinks the ray's
// TMax to its t, and later candidates must be nearer (t < TMax), so the reservoir's random slot
// replacement (Common.slangh:137-151) really samples: the texel depends on the BVH (the oracle
// walks the same tree, rsd_scene_export_bvh).  A quad (4 lanes) walks one ray: lane q tests
// child q / triangle q, the leaf's candidates are delivered one by one in record order with the
// TMax test repeated against the current TMax.  All 4 lanes keep identical algorithm state.
// ------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void sd_trace_ordered_ray(const SDArgs& a, f3 d, float TMin, float TMax, float cosT,
                                                     float (&depths)[N], uint32_t* __restrict__ sItem,
                                                     float* __restrict__ sT, int q, int quadBase, TraceStats& st,
                                                     uint32_t& delivered) {
    const rsd_camera& c = a.cam;
    RayCtx r;
    ray_setup(r, mk(c.posW[0], c.posW[1], c.posW[2]), d);
    uint32_t cnt = 0;
    float tCur = TMax;       // RayTCurrent(): TMax, then the t of the last committed hit
    bool committed = false;  // after a commit only nearer hits (t < tCur) are candidates
    int sp = 0;
    uint32_t item = 0;       // the root node
    const float* bf = reinterpret_cast<const float*>(a.nodes);
    while (true) {
        const uint32_t off = item & kOffMask;
        uint32_t next = kNoItem;
        if (item & kLeafBit) {
            st.leaves++;
            const uint32_t n = ((item >> 29) & 3u) + 1u;
            bool cand = false, af = false;
            float t = 0.0f, rng = 0.0f, z = 0.0f;
            if ((uint32_t)q < n) {
                const float4* tp = a.nodes + off + 3u * (uint32_t)q;
                const float4 va = tp[0], vb = tp[1], vc = tp[2];
                st.tris++;
                float bu, bv, det;
                if (intersect_tri(r, va, vb, vc, t, bu, bv, det) && t >= TMin && t <= tCur &&
                    !culled(det, __float_as_uint(vb.w), a.cull)) {
                    cand = true;
                    rng = sd_hash(bu, bv);
                    z = t * cosT;  // RayToViewDepth
                    if (a.normalize) z = saturate((z - c.nearZ) / (c.farZ - c.nearZ));
                    af = a.alphaTest && (__float_as_uint(vb.w) & 4u) &&
                         alpha_test_fails(a.alphaData, __float_as_uint(va.w), va, vb, vc, bu, bv, true, t, r.d);
                }
            }
            const uint32_t afBits = (uint32_t)(__ballot(af) >> quadBase) & 0xfu;
            for (uint32_t m = (uint32_t)(__ballot(cand) >> quadBase) & 0xfu; m; m &= m - 1u) {
                const int j = __ffs(m) - 1;
                const float tj = qself(t, j), rj = qself(rng, j), zj = qself(z, j);
                if (committed ? !(tj < tCur) : !(tj <= tCur)) continue;  // behind the committed hit
                delivered++;
                if (sd_any_hit<N>(a, rj, zj, ((afBits >> j) & 1u) != 0u, depths, cnt)) {
                    tCur = tj;  // AcceptHit: TMax = t
                    committed = true;
                }
            }
        } else {
            st.nodes++;
            const float* nb = bf + 4u * off;
            const float lox = nb[q], hix = nb[4 + q], loy = nb[8 + q], hiy = nb[12 + q], loz = nb[16 + q],
                        hiz = nb[20 + q];
            const uint32_t ref = __float_as_uint(nb[24 + q]), ccnt = __float_as_uint(nb[28 + q]);
            float tn;
            const bool hit = ref != kNoItem && box_hit(r, lox, hix, loy, hiy, loz, hiz, TMin, tCur, tn);
            float k = hit ? tn : INFINITY;
            uint32_t it = hit ? (ccnt ? (kLeafBit | ((ccnt - 1u) << 29) | (a.triOff + 3u * ref)) : 8u * ref) : kNoItem;
            const int m = __popc((uint32_t)(__ballot(hit) >> quadBase) & 0xfu);
            // sorting network (0,1)(2,3) (0,2)(1,3) (1,2): a pair swaps only if strictly out of order
            quad_cx<kDppXor1>(k, it, (q & 1) == 0);
            quad_cx<kDppXor2>(k, it, (q & 2) == 0);
            {
                const float ok = dppf<kDppXor3>(k);
                const uint32_t oi = dppu<kDppXor3>(it);
                const bool mid = q == 1 || q == 2;
                const bool takeOther = mid && ((q == 1) ? (ok < k) : (k < ok));
                k = takeOther ? ok : k;
                it = takeOther ? oi : it;
            }
            next = qbcu<0>(it);
            if (q >= 1 && q < m) {
                const int slot = sp + (m - 1 - q);  // the nearest of the rest on top
                sItem[slot * kQuadRays] = it;
                sT[slot * kQuadRays] = k;
            }
            sp += m > 0 ? m - 1 : 0;
        }
        if (next == kNoItem) {
            while (sp > 0) {
                --sp;
                if (sT[sp * kQuadRays] <= tCur) { next = sItem[sp * kQuadRays]; break; }
            }
            if (next == kNoItem) break;
        }
        item = next;
    }
}

// Persistent waves over the live-ray queue (as sd_trace_queue_kernel), 16 rays per wave.
template <int N>
__global__ void __launch_bounds__(kBlock) sd_trace_ordered_kernel(SDArgs a, const float4* __restrict__ queue,
                                                                  uint32_t* __restrict__ qctl) {
    extern __shared__ uint32_t sQuadStack[];  // a.quadStack entries per ray: items, then their entry distances
    uint32_t* sItem = sQuadStack;
    float* sT = reinterpret_cast<float*>(sQuadStack + a.quadStack * kQuadRays);
    const int lane = threadIdx.x;
    const int q = lane & 3, quad = lane >> 2, quadBase = lane & ~3;
    const uint32_t part = blockIdx.x % kQueueParts, wavesPerPart = gridDim.x / kQueueParts;
    const uint32_t nLong = __hip_atomic_load(&qctl[part], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t count = nLong + (a.lpt ? __hip_atomic_load(&qctl[kQctlShort + part], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT) : 0u);
    const float DEFAULT = a.normalize ? 1.0f : 3.40282347e+37f;  // Common.slangh:16
    TraceStats st{0u, 0u, 0u};
    uint32_t active = 0, delivered = 0, maxNodes = 0, maxSteps = 0;
    uint32_t base = (blockIdx.x / kQueueParts) * (uint32_t)kQuadRays;
    bool firstChunk = true;
    while (base < count || (firstChunk && a.spread)) {
        // the static first chunk (spread: quad q of the partition's wave w takes index q * waves + w)
        const uint32_t qi = firstChunk && a.spread ? (uint32_t)quad * wavesPerPart + blockIdx.x / kQueueParts
                                                   : base + (uint32_t)quad;
        firstChunk = false;
        if (qi < count) {
            f3 d;
            float TMin, TMax, cosT;
            uint32_t idx;
            ray_rec_load(queue, queue_slot(a, part, qi, nLong), d, TMin, TMax, cosT, idx);
            float depths[N];
#pragma unroll
            for (int i = 0; i < N; ++i) depths[i] = DEFAULT;
            const uint32_t n0 = st.nodes, l0 = st.leaves;
            sd_trace_ordered_ray<N>(a, d, TMin, TMax, cosT, depths, &sItem[quad], &sT[quad], q, quadBase, st,
                                    delivered);
            if (q == 0) {
                maxNodes = max(maxNodes, st.nodes - n0);
                maxSteps = max(maxSteps, st.nodes - n0 + st.leaves - l0);
                active++;
                sd_store<N>(a, (int)(idx % (uint32_t)a.sdW), (int)(idx / (uint32_t)a.sdW), depths);
            }
        }
        if (lane == 0)
            base = wavesPerPart * (uint32_t)kQuadRays + atomicAdd(&qctl[kQueueParts + part], (uint32_t)kQuadRays);
        base = __shfl(base, 0);
    }
    if (a.counters) {
        atomicAdd(&a.counters[1], (unsigned long long)active);
        atomicAdd(&a.counters[2], (unsigned long long)(q == 0 ? st.nodes : 0u));
        atomicAdd(&a.counters[3], (unsigned long long)st.tris);
        atomicAdd(&a.counters[4], (unsigned long long)(q == 0 ? delivered : 0u));
        atomicMax(&a.counters[5], (unsigned long long)maxNodes);
        atomicMax(&a.counters[6], (unsigned long long)maxSteps);
        atomicAdd(&a.counters[9], (unsigned long long)(q == 0 ? st.leaves : 0u));
    }
}

// ------------------------------------------------------------------------------------
// Raster walk (RSD_WALK_RASTER).  Every SD ray starts at the camera position, so the canonical
// any-hit set of a texel -- the triangles its ray hits with TMin <= t <= TMax, culling applied --
// can be found from the triangles' side: project each triangle onto the SD texel grid (texel x's
// ray passes through image-plane x coordinate (sx + jitter) / dimx, jitter in (0, 1)), and run the
// exact watertight test (intersect_tri, the traversal's own) for the live texels under its
// footprint.  Hits go into the texel's K-list of 64-bit keys (t bits << 32 | prim: t > 0, so the
// integer order is the (t, prim) order) by the atomicMin insertion chain: the list ends with the K
// smallest keys whatever the insertion order, i.e. exactly the K nearest keys the BVH walks find,
// so sd_resolve_row_kernel<..., RASTER> gives the same bits.  The work is throughput-bound (one
// thread per triangle record, no dependent traversal chain): tiles whose live rays' view-depth
// range misses the triangle's are skipped, footprints over kRasterSmall texels are walked by the
// whole wave.
// ------------------------------------------------------------------------------------
constexpr int kRasterBlock = 256;
constexpr int kRasterSmall = 16;

__device__ __forceinline__ float dot3(const float* a, f3 v) { return a[0] * v.x + a[1] * v.y + a[2] * v.z; }

// footprint of the triangle on the SD texel grid (clipped at the near plane wClip) and its view-
// depth range; false if it covers no texel of the map
__device__ __forceinline__ bool raster_footprint(const SDArgs& a, float4 v0, float4 v1, float4 v2, int& bx0, int& bx1,
                                                 int& by0, int& by1, float& zlo, float& zhi) {
    const rsd_camera& c = a.cam;
    const f3 o = mk(c.posW[0], c.posW[1], c.posW[2]);
    const f3 p[3] = {mk(v0.x - o.x, v0.y - o.y, v0.z - o.z), mk(v1.x - o.x, v1.y - o.y, v1.z - o.z),
                     mk(v2.x - o.x, v2.y - o.y, v2.z - o.z)};
    float pa[3], pb[3], pw[3];
    zlo = INFINITY;
    zhi = -INFINITY;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        pa[i] = dot3(a.projU, p[i]);
        pb[i] = dot3(a.projV, p[i]);
        pw[i] = dot3(a.projW, p[i]);
        const float z = dot3(a.camWn, p[i]);
        zlo = fminf(zlo, z);
        zhi = fmaxf(zhi, z);
    }
    // conservative depth range (float error of the dot products)
    const float zm = 1e-4f * fmaxf(fabsf(zlo), fabsf(zhi)) + 1e-4f;
    zlo -= zm;
    zhi += zm;
    const float wc = a.wClip;
    if (!(pw[0] >= wc || pw[1] >= wc || pw[2] >= wc)) return false;  // wholly behind the near clip
    float xlo = INFINITY, xhi = -INFINITY, ylo = INFINITY, yhi = -INFINITY;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int j = i == 2 ? 0 : i + 1;
        if (pw[i] >= wc) {
            const float u = pa[i] / pw[i], v = pb[i] / pw[i];
            xlo = fminf(xlo, u); xhi = fmaxf(xhi, u); ylo = fminf(ylo, v); yhi = fmaxf(yhi, v);
        }
        if ((pw[i] >= wc) != (pw[j] >= wc)) {  // the edge crosses the clip plane
            const float s = (wc - pw[i]) / (pw[j] - pw[i]);
            const float u = (pa[i] + s * (pa[j] - pa[i])) / wc, v = (pb[i] + s * (pb[j] - pb[i])) / wc;
            xlo = fminf(xlo, u); xhi = fmaxf(xhi, u); ylo = fminf(ylo, v); yhi = fmaxf(yhi, v);
        }
    }
    // NDC -> texel: sx + jitter = (ndcx + 1) / 2 * dimx, sy + jitter = (1 - ndcy) / 2 * dimy; 0.05 texel margin
    const int dimx = a.sdW - 2 * a.guard, dimy = a.sdH - 2 * a.guard;
    const float fx0 = (xlo + 1.0f) * 0.5f * (float)dimx - 0.05f, fx1 = (xhi + 1.0f) * 0.5f * (float)dimx + 0.05f;
    const float fy0 = (1.0f - yhi) * 0.5f * (float)dimy - 0.05f, fy1 = (1.0f - ylo) * 0.5f * (float)dimy + 0.05f;
    const float lim = 1e8f;  // near-clipped vertices project far away: clamp before converting
    bx0 = max((int)floorf(fmaxf(fx0, -lim)) + a.guard, 0);
    bx1 = min((int)floorf(fminf(fx1, lim)) + a.guard, a.sdW - 1);
    by0 = max((int)floorf(fmaxf(fy0, -lim)) + a.guard, 0);
    by1 = min((int)floorf(fminf(fy1, lim)) + a.guard, a.sdH - 1);
    return bx0 <= bx1 && by0 <= by1;
}

// may the live rays of 8x8 tile (tx, ty) hit a triangle of view depth [zlo, zhi]?  (false for tiles
// of other bands: their records may be stale)
__device__ __forceinline__ bool raster_tile(const SDArgs& a, int tx, int ty, float zlo, float zhi) {
    if (ty < a.bandStart || (ty - a.bandStart) % a.bandStep != 0 || (ty - a.bandStart) / a.bandStep >= a.bandN)
        return false;
    const float2 tr = a.tileRec[(size_t)ty * a.tilesW + tx];
    return zhi >= tr.x && zlo <= tr.y;  // a tile without live rays has the empty range [inf, -inf]
}

// one (triangle, texel) pair of a tile that passed raster_tile: slot, exact test, K-list insertion
template <int K>
__device__ __forceinline__ uint32_t raster_texel(const SDArgs& a, int x, int y, float4 v0, float4 v1, float4 v2,
                                                 const float4* __restrict__ queue) {
    const int32_t slot = a.slotMap[(size_t)y * a.sdW + x];
    if (slot < 0) return 0u;
    const float4 r0 = queue[2u * (uint32_t)slot], r1 = queue[2u * (uint32_t)slot + 1u];
    RayCtx r;
    ray_setup(r, mk(a.cam.posW[0], a.cam.posW[1], a.cam.posW[2]), mk(r0.x, r0.y, r0.z));
    float t, bu, bv, det;
    if (!intersect_tri(r, v0, v1, v2, t, bu, bv, det) || !(t >= r0.w && t <= r1.x) ||
        culled(det, __float_as_uint(v1.w), a.cull))
        return 1u;
    unsigned long long key = ((unsigned long long)__float_as_uint(t) << 32) | (unsigned long long)__float_as_uint(v0.w);
    unsigned long long* L = a.keys64 + (size_t)slot * K;
    if (key >= __hip_atomic_load(&L[K - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return 1u;
#pragma unroll
    for (int j = 0; j < K; ++j) {  // sorted insertion: each slot keeps the smaller key, the larger moves on
        const unsigned long long old = atomicMin(&L[j], key);
        if (old == ~0ull) break;
        key = old > key ? old : key;
    }
    return 1u;
}

template <int K>
__global__ void __launch_bounds__(kRasterBlock) sd_raster_kernel(SDArgs a, const float4* __restrict__ queue,
                                                                 const uint32_t* __restrict__ qctl) {
    const uint32_t i = blockIdx.x * kRasterBlock + threadIdx.x;
    const uint32_t liveCount = qctl[kQctlLiveTiles];
    const int lane = (int)(threadIdx.x & 63u);
    float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0, v2 = v0;
    int bx0 = 0, bx1 = -1, by0 = 0, by1 = -1;
    float zlo = 0.0f, zhi = 0.0f;
    bool any = false;
    if (i < a.nTris) {
        v0 = a.tris[3u * i];
        v1 = a.tris[3u * i + 1u];
        v2 = a.tris[3u * i + 2u];
        any = raster_footprint(a, v0, v1, v2, bx0, bx1, by0, by1, zlo, zhi);
    }
    const int area = any ? (bx1 - bx0 + 1) * (by1 - by0 + 1) : 0;
    uint32_t tests = 0u;
    if (any && area <= kRasterSmall)
        for (int y = by0; y <= by1; ++y)
            for (int x = bx0; x <= bx1; ++x)
                if (raster_tile(a, x >> 3, y >> 3, zlo, zhi)) tests += raster_texel<K>(a, x, y, v0, v1, v2, queue);
    // large footprints, one triangle at a time for the whole wave: the lanes test its 8x8 tiles,
    // then walk the texels of each passing tile (one lane per texel)
    for (unsigned long long bm = __ballot(area > kRasterSmall); bm; bm &= bm - 1ull) {
        const int b = __ffsll((long long)bm) - 1;
        const float4 w0 = make_float4(__shfl(v0.x, b), __shfl(v0.y, b), __shfl(v0.z, b), __shfl(v0.w, b));
        const float4 w1 = make_float4(__shfl(v1.x, b), __shfl(v1.y, b), __shfl(v1.z, b), __shfl(v1.w, b));
        const float4 w2 = make_float4(__shfl(v2.x, b), __shfl(v2.y, b), __shfl(v2.z, b), __shfl(v2.w, b));
        const int cx0 = __shfl(bx0, b), cx1 = __shfl(bx1, b), cy0 = __shfl(by0, b), cy1 = __shfl(by1, b);
        const float czlo = __shfl(zlo, b), czhi = __shfl(zhi, b);
        const int tx0 = cx0 >> 3, ty0 = cy0 >> 3, tw = (cx1 >> 3) - tx0 + 1, nt = tw * ((cy1 >> 3) - ty0 + 1);
        // the footprint's tiles, or the list of tiles with live rays when that is shorter
        const bool byList = nt > (int)liveCount;
        const int nIter = byList ? (int)liveCount : nt;
        for (int k0 = 0; k0 < nIter; k0 += 64) {
            const int k = k0 + lane;
            int tx = 0, ty = 0;
            bool pass = false;
            if (k < nIter) {
                if (byList) {
                    const uint32_t t = a.liveTiles[k];
                    tx = (int)(t % (uint32_t)a.tilesW);
                    ty = (int)(t / (uint32_t)a.tilesW);
                    pass = tx >= tx0 && tx < tx0 + tw && ty >= ty0 && ty <= (cy1 >> 3);
                } else {
                    tx = tx0 + k % tw;
                    ty = ty0 + k / tw;
                    pass = true;
                }
                pass = pass && raster_tile(a, tx, ty, czlo, czhi);
            }
            for (unsigned long long tm = __ballot(pass); tm; tm &= tm - 1ull) {
                const int src = __ffsll((long long)tm) - 1;
                const int x = __shfl(tx, src) * 8 + (lane & 7), y = __shfl(ty, src) * 8 + (lane >> 3);
                if (x >= cx0 && x <= cx1 && y >= cy0 && y <= cy1) tests += raster_texel<K>(a, x, y, w0, w1, w2, queue);
            }
        }
    }
    if (a.counters) {
        atomicAdd(&a.counters[3], (unsigned long long)tests);                        // exact tests
        if (i < a.nTris) atomicAdd(&a.counters[9], 1ull);                              // records read
    }
}

// ------------------------------------------------------------------------------------
// Row-parallel traversal (the default SD trace).  The quad walk above is depth-first: its
// critical path is every node and leaf the ray visits, one dependent fetch after the other
// (the slowest live ray of a 1080p/4 frame visits ~130 items, and the launch lasts as long
// as that ray).  Here a ray is walked by a ROW of 16 lanes (a quarter wave): each step, up
// to 16 work items (4-wide nodes or leaves) taken from the top of the ray's LDS pool are
// processed at once, one per lane, and their surviving children are pushed back, nearest on
// top.  The critical path becomes ~ the tree depth plus (visited items / 16).
// The ray's k-list is sorted ACROSS the row (lane j holds key j, up to 16 keys): inserting a
// hit is one ballot and three shuffles.  Pruning is the depth-first walk's: an item is
// dropped once the K-th key is nearer than its box, which only depends on keys found, so the
// K nearest keys -- and the SD texel -- do not depend on the visiting order.
// Pool bound: a row pops 16 items per step while the pool holds <= poolSoft items and one
// item (a depth-first step, +3 items per level at most) above, so the pool never exceeds
// poolSoft + 48 + 3 * (wide tree depth) <= kPoolCap (poolSoft is derived from the depth).
// A wave walks 4 rays; every row refills from the live-ray queue on its own.
// ------------------------------------------------------------------------------------
constexpr int kPoolCap = 256;  // work items per ray (LDS: rays per wave x 256 x 8 B)

template <int ROW>
__device__ __forceinline__ uint32_t row_bits(bool p, int base) {
    return (uint32_t)(__ballot(p) >> base) & ((1u << ROW) - 1u);
}

// Row-local moves without the LDS crossbar (8-lane rows: two per 16-lane DPP row; 16-lane
// rows fall back to __shfl).  DPP row_shr:n -> lane i reads lane i - n, row_shl:n -> i + n.
constexpr int kDppRowShr1 = 0x111, kDppRowShr4 = 0x114, kDppRowShl4 = 0x104;
// value of row lane L (3 or 7 for 8-lane rows) in every lane of the row
template <int ROW, int L>
__device__ __forceinline__ uint32_t row_bcast(uint32_t v, int l, int base) {
    if constexpr (ROW == 8) {
        const uint32_t q = dppu<(L & 3) * 0x55>(v);  // lanes 0-3 <- lane L % 4, lanes 4-7 <- lane 4 + L % 4
        if constexpr (L >= 4) {
            const uint32_t w = dppu<kDppRowShl4>(q);  // lanes 0-3 <- lane L
            return l < 4 ? w : q;
        } else {
            const uint32_t w = dppu<kDppRowShr4>(q);  // lanes 4-7 <- lane L
            return l < 4 ? q : w;
        }
    } else {
        return (uint32_t)__shfl((int)v, base + L);
    }
}
template <int ROW, int L>
__device__ __forceinline__ float row_bcastf(float v, int l, int base) {
    return __uint_as_float(row_bcast<ROW, L>(__float_as_uint(v), l, base));
}
// value of row lane l - 1 (lane 0's result is unspecified)
template <int ROW>
__device__ __forceinline__ uint32_t row_prev(uint32_t v, int l, int base) {
    if constexpr (ROW == 8) return dppu<kDppRowShr1>(v);
    else return (uint32_t)__shfl((int)v, base + (l > 0 ? l - 1 : 0));
}

// insert key (nt, np) into the row-distributed sorted list (lane j holds key j); the largest key
// falls off the last lane.  Keys are (t, prim): the resolve pass finds a key's triangle record by
// its primitive id (rsd_scene.d_prim_rec), so the list carries no record index.
template <int ROW>
__device__ __forceinline__ void row_insert(float& kt, uint32_t& kp, float nt, uint32_t np, int l, int base) {
    const int pos = __popc(row_bits<ROW>(key_less(kt, kp, nt, np), base));
    const float st = __uint_as_float(row_prev<ROW>(__float_as_uint(kt), l, base));
    const uint32_t sp = row_prev<ROW>(kp, l, base);
    if (l == pos) {
        kt = nt; kp = np;
    } else if (l > pos) {
        kt = st; kp = sp;
    }
}
// the same with the key's barycentrics (the fused walk's hit terms)
template <int ROW>
__device__ __forceinline__ void row_insert(float& kt, uint32_t& kp, float& ku, float& kv, float nt, uint32_t np,
                                           float nu, float nv, int l, int base) {
    const int pos = __popc(row_bits<ROW>(key_less(kt, kp, nt, np), base));
    const float st = __uint_as_float(row_prev<ROW>(__float_as_uint(kt), l, base));
    const uint32_t sp = row_prev<ROW>(kp, l, base);
    const float su = __uint_as_float(row_prev<ROW>(__float_as_uint(ku), l, base));
    const float sv = __uint_as_float(row_prev<ROW>(__float_as_uint(kv), l, base));
    if (l == pos) {
        kt = nt; kp = np; ku = nu; kv = nv;
    } else if (l > pos) {
        kt = st; kp = sp; ku = su; kv = sv;
    }
}

// two keys per lane (K = 2 ROW, the specialised walk at K = 16 on 8-lane rows): lane l holds keys 2l (slot 0) and
// 2l + 1 (slot 1) of the sorted list; the insert counts the keys below the new one in both slots and shifts every key
// at or above that position by one (slot 1 <- own slot 0, slot 0 <- the previous lane's slot 1)
template <int ROW>
__device__ __forceinline__ void row_insert2(float& kt0, uint32_t& kp0, float& ku0, float& kv0, float& kt1, uint32_t& kp1,
                                            float& ku1, float& kv1, float nt, uint32_t np, float nu, float nv, int l,
                                            int base) {
    const int pos = __popc(row_bits<ROW>(key_less(kt0, kp0, nt, np), base)) +
                    __popc(row_bits<ROW>(key_less(kt1, kp1, nt, np), base));
    const float st = __uint_as_float(row_prev<ROW>(__float_as_uint(kt1), l, base));
    const uint32_t sp = row_prev<ROW>(kp1, l, base);
    const float su = __uint_as_float(row_prev<ROW>(__float_as_uint(ku1), l, base));
    const float sv = __uint_as_float(row_prev<ROW>(__float_as_uint(kv1), l, base));
    const int i0 = 2 * l, i1 = 2 * l + 1;
    if (i1 == pos) {
        kt1 = nt; kp1 = np; ku1 = nu; kv1 = nv;
    } else if (i1 > pos) {
        kt1 = kt0; kp1 = kp0; ku1 = ku0; kv1 = kv0;
    }
    if (i0 == pos) {
        kt0 = nt; kp0 = np; ku0 = nu; kv0 = nv;
    } else if (i0 > pos) {
        kt0 = st; kp0 = sp; ku0 = su; kv0 = sv;
    }
}

// exclusive prefix sum (and total) of v in [0, 7] over the lanes of a row
template <int ROW>
__device__ __forceinline__ int row_prefix(int v, int l, int base, int& total) {
    const uint32_t below = (1u << l) - 1u;
    int pre = 0;
    total = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const uint32_t m = row_bits<ROW>((v >> b) & 1, base);
        pre += __popc(m & below) << b;
        total += __popc(m) << b;
    }
    return pre;
}

// anyHit -> algorithm (Common.slangh:102-254) over `found` keys in ascending (t, prim) order;
// lane j of the row holds key j's hash `rng` and normalized view depth `z`.  Every lane of
// the row ends with the same depths / cnt / commit.
template <int K, int N, int IMPL = -1>
__device__ __forceinline__ bool sd_algorithm_row(const SDArgs& a, float rng, float z, bool afl, int found,
                                                 int base, float (&depths)[N], uint32_t& cnt, uint32_t& delivered) {
    bool commit = false;
    const uint64_t afm = __ballot(afl);  // bit base + j: key j fails the alpha test
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const float rj = __shfl(rng, base + j);
        float zj = __shfl(z, base + j);
        const bool af = (afm >> (base + j)) & 1u;
        if (commit || j >= found) continue;
        delivered++;
        commit = sd_any_hit_impl<N, IMPL>(a, rj, zj, af, depths, cnt);
    }
    return commit;
}

// the same with two keys per lane (row_insert2's layout: key j in lane j / 2, slot j % 2), no alpha-tested keys
template <int K, int N, int IMPL = -1>
__device__ __forceinline__ bool sd_algorithm_row2(const SDArgs& a, float rng0, float z0, float rng1, float z1, int found,
                                                  int base, float (&depths)[N], uint32_t& cnt, uint32_t& delivered) {
    bool commit = false;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const float rj = __shfl((j & 1) ? rng1 : rng0, base + j / 2);
        const float zj = __shfl((j & 1) ? z1 : z0, base + j / 2);
        if (commit || j >= found) continue;
        delivered++;
        commit = sd_any_hit_impl<N, IMPL>(a, rj, zj, false, depths, cnt);
    }
    return commit;
}

// hash + normalized view depth of the hit (t, triangle record tri) -- the barycentrics come
// from re-running the identical triangle test (Common.slangh:110-115)
// (af: an alpha-masked triangle fails the alpha test at the ray-cone LOD of the hit,
// StochasticDepthMapRT.rt.slang:31-37 + Common.slangh:155-175)
__device__ __forceinline__ void sd_hit_terms(const SDArgs& a, const RayCtx& r, float cosT, uint32_t tri, float& rng,
                                             float& z, bool& af) {
    float t, bu, bv, det;
    const float4 v0 = a.tris[3 * tri], v1 = a.tris[3 * tri + 1], v2 = a.tris[3 * tri + 2];
    intersect_tri(r, v0, v1, v2, t, bu, bv, det);
    rng = sd_hash(bu, bv);
    z = t * cosT;  // RayToViewDepth
    if (a.normalize) z = saturate((z - a.cam.nearZ) / (a.cam.farZ - a.cam.nearZ));
    af = a.alphaTest && (__float_as_uint(v1.w) & 4u) &&
         alpha_test_fails(a.alphaData, __float_as_uint(v0.w), v0, v1, v2, bu, bv, true, t, r.d);
}

// ROW lanes per ray (8 or 16, >= K: lane j of the row holds key j), 64 / ROW rays per wave.
// SPLIT: the walk only collects the K nearest keys and writes them to `keys` (one K-key slot
// per queue slot); sd_resolve_row_kernel runs the algorithm.  Valid when one chunk of K keys
// always decides the texel: Default / KBuffer with MaxCount <= K.  Otherwise the algorithm
// runs here and the walk continues after the K-th key while it has not committed.
// SPEC: the specialised fused walk of the common trace -- the Default reservoir with MaxCount <= K (a
// commit by the K-th key, so no second chunk of keys) and no alpha-tested triangles: the lower-bound
// (useLB) tests, the alpha test, the other implementations and the chunk continuation compile away.
// (Round 6, not kept: deferring a row's leaves to a second pool stack and giving the WAVE separate node steps and
// leaf steps -- every row then tests up to ROW deferred leaves at once -- so that node steps run the box tests alone
// instead of the union of the box and triangle paths of a wave's mixed items.  Same bits, slower at every config:
// configs[1] 67.5 -> 69.1 us, configs[2] 179 -> 223, configs[3] 197 -> 216 (profiles/round6/trace_ab/defer_*).)
template <int K, int N, int ROW, bool SPLIT, bool CNT, int POOL = kPoolCap, bool SPEC = false>
__device__ __forceinline__ void sd_trace_row_body(const SDArgs& a, const float4* __restrict__ queue,
                                                  uint32_t* __restrict__ qctl, uint2* __restrict__ keys,
                                                  uint32_t* sItem, float* sT, uint32_t bid, uint32_t nb, uint32_t qr) {
    // sItem / sT: the rows' LDS pools (kBlock / ROW x POOL entries each); (bid, nb, qr) as sd_trace_queue_body's
    // one key per lane, or (the specialised fused walk, K = 16 on 8-lane rows) two: row_insert2
    static_assert(K <= ROW || (K == 2 * ROW && SPEC && !SPLIT), "one key per lane, or two in the specialised walk");
    constexpr int KPL = K <= ROW ? 1 : 2;
    constexpr int kKthLane = (K - 1) / KPL;  // the lane holding key K - 1 (slot KPL - 1)
    static_assert(kEntryCap <= (uint32_t)ROW, "entry items start one per lane");
    constexpr int kRow = ROW, kRowRays = kBlock / ROW;
    const int lane = threadIdx.x;
    const int l = lane & (kRow - 1), base = lane & ~(kRow - 1), row = lane / kRow;
    uint32_t* pItem = sItem + row * POOL;
    float* pT = sT + row * POOL;
    const uint32_t part = bid % kQueueParts, wavesPerPart = nb / kQueueParts;
    const uint32_t nLong = __hip_atomic_load(&qctl[part], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (RSD_TRACE_QRANGE, diagnostics: only the longest-first rays, or only the others)
    const uint32_t q0 = qr == 2u ? nLong : 0u;
    const uint32_t count = (qr == 1u ? nLong : nLong + (a.lpt ? __hip_atomic_load(&qctl[kQctlShort + part],
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u)) - q0;
    const rsd_camera& c = a.cam;
    const float DEFAULT = a.normalize ? 1.0f : 3.40282347e+37f;  // Common.slangh:16
    const int soft = a.poolSoft;
    uint32_t slot = 0;  // queue slot of the row's ray
    uint32_t nEnt = 0;  // entry-grid items of the row's ray (0: the root)

    // ---- per-row state (the same value in the 16 lanes of a row unless noted)
    constexpr int kFetch = 0, kTrace = 1, kExit = 2;
    int phase = kFetch;
    bool first = true;
    int x = 0, y = 0;
    RayCtx r;
    float TMin = 0.0f, TMax = 0.0f, cosT = 0.0f;
    float depths[N];
    uint32_t cnt = 0;     // algorithm count (Common.slangh:137)
    bool useLB = false;   // coverage mask / MaxCount > K: keys after (lbT, lbP) only
    float lbT = 0.0f;
    uint32_t lbP = 0u;
    int pool = 0;         // items in this ray's LDS pool
    uint32_t item = kNoItem;  // per lane: the work item of this step
    float kt = INFINITY;  // per lane: key l of the row's sorted k-list
    uint32_t kp = kNoItem;
    float ku = 0.0f, kv = 0.0f;  // per lane: key l's barycentrics (fused walk: the hit terms' inputs)
    float kt2 = INFINITY, ku2 = 0.0f, kv2 = 0.0f;  // KPL = 2: lane l holds keys 2l (kt ...) and 2l + 1 (kt2 ...)
    uint32_t kp2 = kNoItem;
    // ---- statistics (counters build)
    TraceStats st{0u, 0u, 0u};
    uint32_t active = 0, hitsDelivered = 0, maxSteps = 0, raySteps = 0, maxNodes = 0, rayNodes = 0, rayLeaves = 0;
    unsigned long long sumCycles = 0, maxCycles = 0, c0 = 0;

    unsigned long long tFetch = 0, tStep = 0, tResolve = 0, nStep = 0, nLoop = 0, tS0 = 0, tS1 = 0;
    unsigned long long tMem = 0, tComp = 0, tPool = 0, tMark = 0;  // step split (instrumented build)
    unsigned long long tBox = 0, tTri = 0, tB = 0, tT = 0;  // compute split: box tests + sort, triangle tests
    // clock calibration (instrumented build): the first wave's span in s_memtime ticks and in the
    // 100 MHz s_memrealtime ticks converts the step clocks to microseconds (rsd_counters.shader_clock_mhz)
    unsigned long long cal0 = 0, calR0 = 0;
    if constexpr (CNT) {
        if (bid == 0) {
            cal0 = __builtin_amdgcn_s_memtime();
            calR0 = __builtin_amdgcn_s_memrealtime();
        }
    }
    while (__ballot(phase != kExit) != 0ull) {
        if constexpr (CNT) { tS0 = __builtin_amdgcn_s_memtime(); nLoop += lane == 0; }
        const bool fetching = phase == kFetch;
        if (phase == kFetch) {
            uint32_t qi;
            if (first) {  // the static first ray
                qi = a.spread ? (uint32_t)row * wavesPerPart + bid / kQueueParts
                              : (bid / kQueueParts) * (uint32_t)kRowRays + (uint32_t)row;
                first = false;
            } else {
                uint32_t h = 0;
                if (l == 0) h = atomicAdd(&qctl[(qr == 1u ? kQctlHead2 : kQueueParts) + part], 1u);
                qi = wavesPerPart * (uint32_t)kRowRays + __shfl(h, base);
            }
            if (qi >= count) {
                phase = kExit;
            } else {
                slot = queue_slot(a, part, qi + q0, nLong);
                f3 d;
                uint32_t idx;
                // the entry items load with the record (the setup kernel wrote both)
                const uint32_t e = a.entOn && l < (int)kEntryCap ? a.entQ[(size_t)slot * kEntryCap + l] : kNoItem;
                ray_rec_load(queue, slot, d, TMin, TMax, cosT, idx, nEnt);
                x = (int)(idx % (uint32_t)a.sdW);
                y = (int)(idx / (uint32_t)a.sdW);
                ray_setup(r, mk(c.posW[0], c.posW[1], c.posW[2]), d);
#pragma unroll
                for (int i = 0; i < N; ++i) depths[i] = DEFAULT;
                cnt = 0u;
                useLB = false;
                pool = 0;
                // the root node, or the segment's entry-grid frontier (one item per lane)
                item = nEnt ? ((uint32_t)l < nEnt ? e : kNoItem) : (l == 0 ? 0u : kNoItem);
                kt = INFINITY; kp = kNoItem; ku = kv = 0.0f;
                kt2 = INFINITY; kp2 = kNoItem; ku2 = kv2 = 0.0f;
                phase = kTrace;
                if constexpr (CNT) {
                    active += l == 0;
                    raySteps = 0;
                    rayNodes = 0;
                    rayLeaves = 0;
                    c0 = __builtin_amdgcn_s_memtime();
                }
            }
        }
        if constexpr (CNT) {
            tS1 = __builtin_amdgcn_s_memtime();
            if (fetching && l == 0) tFetch += tS1 - tS0;
        }
        if (phase != kTrace) continue;

        // ---- one traversal step of this row
        if constexpr (SPEC) useLB = false;
        const float tlo = useLB ? fmaxf(TMin, lbT) : TMin;
        float kthT = row_bcastf<ROW, kKthLane>(KPL == 2 ? kt2 : kt, l, base);
        uint32_t kthP = row_bcast<ROW, kKthLane>(KPL == 2 ? kp2 : kp, l, base);
        float thi = fminf(TMax, kthT);
        float ck[4];
        uint32_t ci[4];
        int nc = 0;
        // one fetch per step, all loads issued before the first use: a 4-wide node (128 B), or the
        // leaf's triangle records (48 B each; a leaf of 3-4 triangles reads 192 B -- the BVH
        // allocation is padded by 192 B, so the tail loads never leave it)
        const float4* p = a.nodes + (item & kOffMask);
        float4 q[12];
        const bool isLeaf = item != kNoItem && (item & kLeafBit);
        if constexpr (CNT) tMark = __builtin_amdgcn_s_memtime();
        if (item != kNoItem) {
#pragma unroll
            for (int j = 0; j < 8; ++j) q[j] = p[j];
            if (isLeaf && (item >> 29 & 3u) >= 2u) {
#pragma unroll
                for (int j = 8; j < 12; ++j) q[j] = p[j];
            }
        }
        if constexpr (CNT) {  // the step's fetch latency (the instrumented build waits here)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (l == 0) tMem += t - tMark;
            tMark = t;
        }
        if (item != kNoItem && !isLeaf) {
            st.nodes++;
            rayNodes++;
            const uint32_t rf[4] = {__float_as_uint(q[6].x), __float_as_uint(q[6].y), __float_as_uint(q[6].z),
                                    __float_as_uint(q[6].w)};
            const uint32_t cn[4] = {__float_as_uint(q[7].x), __float_as_uint(q[7].y), __float_as_uint(q[7].z),
                                    __float_as_uint(q[7].w)};
            const float lox[4] = {q[0].x, q[0].y, q[0].z, q[0].w}, hix[4] = {q[1].x, q[1].y, q[1].z, q[1].w};
            const float loy[4] = {q[2].x, q[2].y, q[2].z, q[2].w}, hiy[4] = {q[3].x, q[3].y, q[3].z, q[3].w};
            const float loz[4] = {q[4].x, q[4].y, q[4].z, q[4].w}, hiz[4] = {q[5].x, q[5].y, q[5].z, q[5].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float tn;
                const bool h = rf[j] != kNoItem && box_hit(r, lox[j], hix[j], loy[j], hiy[j], loz[j], hiz[j], tlo,
                                                          thi, tn);
                ck[j] = h ? tn : INFINITY;
                ci[j] = h ? (cn[j] ? (kLeafBit | ((cn[j] - 1u) << 29) | (a.triOff + 3u * rf[j])) : 8u * rf[j])
                          : kNoItem;
                nc += h;
            }
            // ascending entry distance; misses (INF) sort last
            cswap(ck[0], ci[0], ck[1], ci[1]);
            cswap(ck[2], ci[2], ck[3], ci[3]);
            cswap(ck[0], ci[0], ck[2], ci[2]);
            cswap(ck[1], ci[1], ck[3], ci[3]);
            cswap(ck[1], ci[1], ck[2], ci[2]);
        }
        if constexpr (CNT) { tB = __builtin_amdgcn_s_memtime(); tT = tB; }
        // ---- leaves: every triangle test of the step first (independent dependency chains), then
        //      the row merges the accepted hits into its k-list, one insert each (the merge
        //      re-checks each hit against the current K-th key)
        const uint32_t lc = isLeaf ? ((item >> 29) & 3u) + 1u : 0u;
        if (isLeaf) st.leaves++;
        if (CNT && isLeaf) rayLeaves++;
        if (__ballot(lc != 0u) != 0ull) {
            float tj[4], uj[4], vj[4];
            uint32_t pj[4];
            bool aj[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                aj[j] = false;
                tj[j] = 0.0f; uj[j] = 0.0f; vj[j] = 0.0f;
                pj[j] = 0u;
                if ((uint32_t)j < lc) {
                    st.tris++;
                    const float4 v0 = q[3 * j], v1 = q[3 * j + 1], v2 = q[3 * j + 2];
                    float det, t, bu, bv;
                    if (intersect_tri(r, v0, v1, v2, t, bu, bv, det) && t >= TMin && t <= TMax) {
                        const uint32_t prim = __float_as_uint(v0.w);
                        aj[j] = !culled(det, __float_as_uint(v1.w), a.cull) &&
                                (!useLB || key_less(lbT, lbP, t, prim)) && key_less(t, prim, kthT, kthP);
                        tj[j] = t; pj[j] = prim; uj[j] = bu; vj[j] = bv;
                    }
                }
            }
            if constexpr (CNT) tT = __builtin_amdgcn_s_memtime();
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                for (uint32_t m = row_bits<ROW>(aj[j], base); m; m &= m - 1u) {
                    const int srcLane = base + __ffs(m) - 1;
                    const float bt = __shfl(tj[j], srcLane);
                    const uint32_t bp = __shfl(pj[j], srcLane);
                    float nu = 0.0f, nv = 0.0f;
                    if constexpr (!SPLIT) {
                        nu = __shfl(uj[j], srcLane);
                        nv = __shfl(vj[j], srcLane);
                    }
                    if (key_less(bt, bp, kthT, kthP)) {
                        if constexpr (SPLIT) row_insert<ROW>(kt, kp, bt, bp, l, base);
                        else if constexpr (KPL == 2) row_insert2<ROW>(kt, kp, ku, kv, kt2, kp2, ku2, kv2, bt, bp, nu, nv, l, base);
                        else row_insert<ROW>(kt, kp, ku, kv, bt, bp, nu, nv, l, base);
                        kthT = row_bcastf<ROW, kKthLane>(KPL == 2 ? kt2 : kt, l, base);
                        kthP = row_bcast<ROW, kKthLane>(KPL == 2 ? kp2 : kp, l, base);
                    }
                }
            }
        }
        thi = fminf(TMax, kthT);
        // ---- push the surviving children, nearest on top
        int keep = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) keep += (j < nc && ck[j] <= thi) ? 1 : 0;  // ck ascending: a prefix
        int total;
        const int pre = row_prefix<ROW>(keep, l, base, total);
        if (pool + total > POOL) {  // unreachable by the pool bound; never write out of range
            if (a.counters && l == 0) atomicAdd(&a.counters[10], 1ull);  // always checked
            keep = max(0, min(keep, POOL - pool - pre));
            total = POOL - pool;
        }
        if constexpr (CNT) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (l == 0) {
                tComp += t - tMark;
                tBox += tB - tMark;
                tTri += tT - tB;
            }
            tMark = t;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j < keep) {
                const int slot = pool + pre + (keep - 1 - j);
                pItem[slot] = ci[j];
                pT[slot] = ck[j];
            }
        }
        pool += total;
        __builtin_amdgcn_wave_barrier();  // LDS pushes above before the pops below (one wave)
        // ---- pop the next items
        const int take = min(pool, pool <= soft ? kRow : 1);
        item = kNoItem;
        if (l < take) {
            const uint32_t it = pItem[pool - 1 - l];
            const float tt = pT[pool - 1 - l];
            item = tt <= thi ? it : kNoItem;
        }
        pool -= take;
        __builtin_amdgcn_wave_barrier();
        if constexpr (CNT) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (l == 0) tPool += __builtin_amdgcn_s_memtime() - tMark;
            raySteps++;
            const unsigned long long t2 = __builtin_amdgcn_s_memtime();
            if (l == 0) { tStep += t2 - tS1; nStep++; }
            tS1 = t2;
        }
        if (pool > 0 || row_bits<ROW>(item != kNoItem, base) != 0u) continue;

        // ---- traversal done
        if constexpr (SPLIT) {
            // the K nearest keys of the ray -> sd_resolve_row_kernel
            if (l < K) keys[(size_t)slot * K + l] = make_uint2(__float_as_uint(kt), kp);
            phase = kFetch;
            if constexpr (CNT) {
                uint32_t n = rayNodes;
#pragma unroll
                for (int o = ROW / 2; o >= 1; o >>= 1) n += __shfl_xor(n, o);
                maxNodes = max(maxNodes, n);
                maxSteps = max(maxSteps, raySteps);
                const unsigned long long t3 = __builtin_amdgcn_s_memtime();
                if (l == 0) {
                    tResolve += t3 - tS1;
                    sumCycles += t3 - c0;
                    maxCycles = t3 - c0 > maxCycles ? t3 - c0 : maxCycles;
                }
            }
            continue;
        }
        // TraceRay + anyHit -> algorithm (Common.slangh:102-254) over the found keys, in
        // ascending (t, prim) order; lane j prepares key j
        const int found = min(K, __popc(row_bits<ROW>(kp != kNoItem, base)) +
                                     (KPL == 2 ? __popc(row_bits<ROW>(kp2 != kNoItem, base)) : 0));
        // lane j: key j's terms from the (t, barycentrics) its leaf test found -- sd_hit_terms'
        // values bit for bit; the alpha test (alpha scenes only) re-reads the triangle
        float rng = 0.0f, z = 0.0f;
        bool af = false;
        uint32_t delivered = 0;
        if constexpr (KPL == 2) {  // lane l: keys 2l and 2l + 1 (no alpha test: SPEC)
            float rng2 = 0.0f, z2 = 0.0f;
            if (2 * l < found) {
                rng = sd_hash(ku, kv);
                z = kt * cosT;
                if (a.normalize) z = saturate((z - a.cam.nearZ) / (a.cam.farZ - a.cam.nearZ));
            }
            if (2 * l + 1 < found) {
                rng2 = sd_hash(ku2, kv2);
                z2 = kt2 * cosT;
                if (a.normalize) z2 = saturate((z2 - a.cam.nearZ) / (a.cam.farZ - a.cam.nearZ));
            }
            sd_algorithm_row2<K, N, 0>(a, rng, z, rng2, z2, found, base, depths, cnt, delivered);
            if (l == 0) hitsDelivered += delivered;
            if (l == 0) sd_store<N>(a, x, y, depths);
            phase = kFetch;
            continue;
        }
        if (l < found) {
            if (!SPEC && a.alphaTest) {
                sd_hit_terms(a, r, cosT, a.primRec[kp], rng, z, af);
            } else {
                rng = sd_hash(ku, kv);
                z = kt * cosT;  // RayToViewDepth
                if (a.normalize) z = saturate((z - a.cam.nearZ) / (a.cam.farZ - a.cam.nearZ));
            }
        }
        const bool commit = sd_algorithm_row<K, N, SPEC ? 0 : -1>(a, rng, z, af, found, base, depths, cnt, delivered);
        if (l == 0) hitsDelivered += delivered;
        if (CNT && l == 0) tResolve += __builtin_amdgcn_s_memtime() - tS1;
        if (!SPEC && !commit && found == K) {
            // the stream continues after the K-th key: trace the next chunk of K keys
            useLB = true;
            lbT = __shfl(kt, base + K - 1);
            lbP = __shfl(kp, base + K - 1);
            pool = 0;
            item = nEnt ? ((uint32_t)l < nEnt ? a.entQ[(size_t)slot * kEntryCap + l] : kNoItem) : (l == 0 ? 0u : kNoItem);
            kt = INFINITY; kp = kNoItem; ku = kv = 0.0f;
            continue;
        }
        if (l == 0) sd_store<N>(a, x, y, depths);
        phase = kFetch;
        if constexpr (CNT) {
            // per-ray totals: row sums of the lanes' node counts
            uint32_t n = rayNodes;
#pragma unroll
            for (int o = ROW / 2; o >= 1; o >>= 1) n += __shfl_xor(n, o);
            maxNodes = max(maxNodes, n);
            maxSteps = max(maxSteps, raySteps);
            const unsigned long long dc = __builtin_amdgcn_s_memtime() - c0;
            uint32_t nl = rayLeaves;
#pragma unroll
            for (int o = ROW / 2; o >= 1; o >>= 1) nl += __shfl_xor(nl, o);
            if (l == 0) {
                sumCycles += dc;
                maxCycles = dc > maxCycles ? dc : maxCycles;
                if (a.rayLog) {
                    uint32_t* g = a.rayLog + (size_t)slot * 8u;
                    g[0] = (uint32_t)y * (uint32_t)a.sdW + (uint32_t)x;
                    g[1] = raySteps;
                    g[2] = n;
                    g[3] = nl;
                    g[4] = (uint32_t)found;
                    g[5] = (uint32_t)min(dc, 0xffffffffull);
                    g[6] = __float_as_uint(TMax - TMin);
                    g[7] = __float_as_uint(TMin);
                }
            }
        }
    }
    if constexpr (CNT) {
        atomicAdd(&a.counters[1], (unsigned long long)active);
        atomicAdd(&a.counters[2], (unsigned long long)st.nodes);
        atomicAdd(&a.counters[3], (unsigned long long)st.tris);
        atomicAdd(&a.counters[4], (unsigned long long)hitsDelivered);
        atomicMax(&a.counters[5], (unsigned long long)maxNodes);
        atomicMax(&a.counters[6], (unsigned long long)maxSteps);
        atomicAdd(&a.counters[7], sumCycles);
        atomicMax(&a.counters[8], maxCycles);
        atomicAdd(&a.counters[9], (unsigned long long)st.leaves);
        atomicAdd(&a.counters[11], tFetch);
        atomicAdd(&a.counters[12], tStep);
        atomicAdd(&a.counters[13], tResolve);
        atomicAdd(&a.counters[14], nStep);
        atomicAdd(&a.counters[15], nLoop);
        atomicAdd(&a.counters[16], tMem);
        atomicAdd(&a.counters[17], tComp);
        atomicAdd(&a.counters[18], tPool);
        atomicAdd(&a.counters[23], tBox);
        atomicAdd(&a.counters[24], tTri);
        if (bid == 0 && lane == 0) {
            const unsigned long long cal1 = __builtin_amdgcn_s_memtime(), calR1 = __builtin_amdgcn_s_memrealtime();
            atomicMax(&a.counters[21], cal1 - cal0);
            atomicMax(&a.counters[22], calR1 - calR0);
        }
    }
}

template <int K, int N, int ROW, bool SPLIT, bool CNT, int POOL = kPoolCap, bool SPEC = false>
__global__ void __launch_bounds__(kBlock) sd_trace_row_kernel(SDArgs a, const float4* __restrict__ queue,
                                                              uint32_t* __restrict__ qctl, uint2* __restrict__ keys) {
    constexpr int kRowRays = kBlock / ROW;
    __shared__ uint32_t sItem[kRowRays * POOL];
    __shared__ float sT[kRowRays * POOL];
    sd_trace_row_body<K, N, ROW, SPLIT, CNT, POOL, SPEC>(a, queue, qctl, keys, sItem, sT, blockIdx.x, gridDim.x, a.qrange);
}

// The hybrid walk (walk 6): one launch whose first a.hybridRowBlocks blocks walk the longest-first rays with the
// specialised row walk and whose other blocks walk the remaining rays with the specialised quad walk, so the long
// rays' chains (which set a quad-walk launch) take 8 items per step while the bulk keeps the quad walk's lane use.
// One dynamic LDS allocation serves either role (max of the two).
template <int K, int N, int ROW, int POOL>
__global__ void __launch_bounds__(kBlock) sd_trace_hybrid_kernel(SDArgs a, const float4* __restrict__ queue,
                                                                 uint32_t* __restrict__ qctl, uint2* __restrict__ keys) {
    extern __shared__ uint32_t sDyn[];
    const uint32_t rb = a.hybridRowBlocks;
    if ((blockIdx.x < rb && a.rowPrio) || a.prio) __builtin_amdgcn_s_setprio(2);  // (rowPrio: neutral, trace_ab/prio_*)
    if (blockIdx.x < rb)
        sd_trace_row_body<K, N, ROW, false, false, POOL, true>(
            a, queue, qctl, keys, sDyn, reinterpret_cast<float*>(sDyn + (kBlock / ROW) * POOL), blockIdx.x, rb, 1u);
    else
        sd_trace_queue_body<K, N, true>(a, queue, qctl, sDyn, blockIdx.x - rb, gridDim.x - rb, 2u);
}

// Wavefront traversal-order any-hit stream (rsd_sd_params.hit_order = RSD_HIT_ORDER_WAVEFRONT, rsd.h): the
// canonical row walk's traversal -- a row of 8 lanes per ray, each lane one work item per step, the surviving
// children pushed nearest-on-top onto the ray's LIFO pool in LDS and up to 8 popped per step (1 while the pool
// is above poolSoft) -- but every candidate hit goes to any-hit as the walk finds it: per step the lanes' leaves
// in lane order, a leaf's triangles in record order; a committed hit sets TMax = t (AcceptHit), later
// candidates need t < TMax, and boxes are tested against the TMax of the step's start.  Like the depth-first
// order (sd_trace_ordered_kernel) it is one definition of DXR's implementation-defined order, walked from the
// root (no entry grid: the frontier would reorder the stream); the oracle restates it step for step
// (oracle/rsd_oracle.c o_wavefront_walk) over the exported BVH.  Rows stride over the live-ray queue as the
// canonical row walk does (longest-first partitions).
template <int N>
__global__ void __launch_bounds__(kBlock) sd_trace_wavefront_kernel(SDArgs a, const float4* __restrict__ queue,
                                                                    uint32_t* __restrict__ qctl) {
    constexpr int kRow = 8, kRowRays = kBlock / kRow, POOL = kPoolCap;
    __shared__ uint32_t sItem[kRowRays * POOL];
    __shared__ float sT[kRowRays * POOL];
    const int lane = threadIdx.x;
    const int l = lane & (kRow - 1), base = lane & ~(kRow - 1), row = lane / kRow;
    uint32_t* pItem = sItem + row * POOL;
    float* pT = sT + row * POOL;
    const uint32_t part = blockIdx.x % kQueueParts, wavesPerPart = gridDim.x / kQueueParts;
    const uint32_t nLong = __hip_atomic_load(&qctl[part], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t count = nLong + (a.lpt ? __hip_atomic_load(&qctl[kQctlShort + part], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT) : 0u);
    const rsd_camera& c = a.cam;
    const float DEFAULT = a.normalize ? 1.0f : 3.40282347e+37f;  // Common.slangh:16
    const int soft = a.poolSoft;
    constexpr int kFetch = 0, kTrace = 1, kExit = 2;
    int phase = kFetch;
    bool first = true;
    int x = 0, y = 0, pool = 0;
    RayCtx r;
    float TMin = 0.0f, TMax = 0.0f, cosT = 0.0f, tCur = 0.0f;
    bool committed = false;
    float depths[N];
    uint32_t cnt = 0, item = kNoItem;
    TraceStats st{0u, 0u, 0u};
    uint32_t active = 0, delivered = 0, raySteps = 0, maxSteps = 0;
    while (__ballot(phase != kExit) != 0ull) {
        if (phase == kFetch) {
            uint32_t qi;
            if (first) {
                qi = (blockIdx.x / kQueueParts) * (uint32_t)kRowRays + (uint32_t)row;
                first = false;
            } else {
                uint32_t h = 0;
                if (l == 0) h = atomicAdd(&qctl[kQueueParts + part], 1u);
                qi = wavesPerPart * (uint32_t)kRowRays + __shfl(h, base);
            }
            if (qi >= count) {
                phase = kExit;
            } else {
                f3 d;
                uint32_t idx;
                ray_rec_load(queue, queue_slot(a, part, qi, nLong), d, TMin, TMax, cosT, idx);
                x = (int)(idx % (uint32_t)a.sdW);
                y = (int)(idx / (uint32_t)a.sdW);
                ray_setup(r, mk(c.posW[0], c.posW[1], c.posW[2]), d);
#pragma unroll
                for (int i = 0; i < N; ++i) depths[i] = DEFAULT;
                cnt = 0u;
                tCur = TMax;  // RayTCurrent()
                committed = false;
                pool = 0;
                item = l == 0 ? 0u : kNoItem;  // the root
                phase = kTrace;
                active += l == 0;
                raySteps = 0;
            }
        }
        if (phase != kTrace) continue;

        // ---- one step of this row: every box against the TMax of the step's start
        const float thi0 = tCur;
        float ck[4];
        uint32_t ci[4];
        int nc = 0;
        const float4* p = a.nodes + (item & kOffMask);
        float4 q[12];
        const bool isLeaf = item != kNoItem && (item & kLeafBit);
        if (item != kNoItem) {
#pragma unroll
            for (int j = 0; j < 8; ++j) q[j] = p[j];
            if (isLeaf && (item >> 29 & 3u) >= 2u) {
#pragma unroll
                for (int j = 8; j < 12; ++j) q[j] = p[j];
            }
        }
        if (item != kNoItem && !isLeaf) {
            st.nodes++;
            const uint32_t rf[4] = {__float_as_uint(q[6].x), __float_as_uint(q[6].y), __float_as_uint(q[6].z),
                                    __float_as_uint(q[6].w)};
            const uint32_t cn[4] = {__float_as_uint(q[7].x), __float_as_uint(q[7].y), __float_as_uint(q[7].z),
                                    __float_as_uint(q[7].w)};
            const float lox[4] = {q[0].x, q[0].y, q[0].z, q[0].w}, hix[4] = {q[1].x, q[1].y, q[1].z, q[1].w};
            const float loy[4] = {q[2].x, q[2].y, q[2].z, q[2].w}, hiy[4] = {q[3].x, q[3].y, q[3].z, q[3].w};
            const float loz[4] = {q[4].x, q[4].y, q[4].z, q[4].w}, hiz[4] = {q[5].x, q[5].y, q[5].z, q[5].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float tn;
                const bool h = rf[j] != kNoItem && box_hit(r, lox[j], hix[j], loy[j], hiy[j], loz[j], hiz[j], TMin,
                                                          thi0, tn);
                ck[j] = h ? tn : INFINITY;
                ci[j] = h ? (cn[j] ? (kLeafBit | ((cn[j] - 1u) << 29) | (a.triOff + 3u * rf[j])) : 8u * rf[j])
                          : kNoItem;
                nc += h;
            }
            cswap(ck[0], ci[0], ck[1], ci[1]);
            cswap(ck[2], ci[2], ck[3], ci[3]);
            cswap(ck[0], ci[0], ck[2], ci[2]);
            cswap(ck[1], ci[1], ck[3], ci[3]);
            cswap(ck[1], ci[1], ck[2], ci[2]);
        }
        // ---- leaves: every triangle test of the step first, then the row delivers the candidates in lane
        //      order, a leaf's triangles in record order, each against the current TMax
        const uint32_t lc = isLeaf ? ((item >> 29) & 3u) + 1u : 0u;
        if (isLeaf) st.leaves++;
        if (__ballot(lc != 0u) != 0ull) {
            float tj[4], rj[4], zj[4];
            uint32_t cand = 0u, afm = 0u;  // bit j: triangle j is a candidate / fails the alpha test
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                tj[j] = 0.0f; rj[j] = 0.0f; zj[j] = 0.0f;
                if ((uint32_t)j < lc) {
                    st.tris++;
                    const float4 v0 = q[3 * j], v1 = q[3 * j + 1], v2 = q[3 * j + 2];
                    float det, t, bu, bv;
                    if (intersect_tri(r, v0, v1, v2, t, bu, bv, det) && t >= TMin && t <= thi0 &&
                        !culled(det, __float_as_uint(v1.w), a.cull)) {  // ray flags: before any-hit
                        cand |= 1u << j;
                        tj[j] = t;
                        rj[j] = sd_hash(bu, bv);
                        float z = t * cosT;  // RayToViewDepth
                        if (a.normalize) z = saturate((z - c.nearZ) / (c.farZ - c.nearZ));
                        zj[j] = z;
                        if (a.alphaTest && (__float_as_uint(v1.w) & 4u) &&
                            alpha_test_fails(a.alphaData, __float_as_uint(v0.w), v0, v1, v2, bu, bv, true, t, r.d))
                            afm |= 1u << j;
                    }
                }
            }
            for (uint32_t m = row_bits<kRow>(cand != 0u, base); m; m &= m - 1u) {
                const int src = base + __ffs(m) - 1;
                const uint32_t cs = (uint32_t)__shfl((int)cand, src), as = (uint32_t)__shfl((int)afm, src);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float bt = __shfl(tj[j], src), br = __shfl(rj[j], src), bz = __shfl(zj[j], src);
                    if (!((cs >> j) & 1u) || (committed ? !(bt < tCur) : !(bt <= tCur))) continue;
                    delivered += l == 0;
                    if (sd_any_hit<N>(a, br, bz, ((as >> j) & 1u) != 0u, depths, cnt)) {
                        tCur = bt;  // AcceptHit: TMax = t
                        committed = true;
                    }
                }
            }
        }
        const float thi = tCur;
        // ---- push the surviving children, nearest on top; pop the next items
        int keep = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) keep += (j < nc && ck[j] <= thi) ? 1 : 0;  // ck ascending: a prefix
        int total;
        const int pre = row_prefix<kRow>(keep, l, base, total);
        if (pool + total > POOL) {  // unreachable by the pool bound; never write out of range
            if (a.counters && l == 0) atomicAdd(&a.counters[10], 1ull);
            keep = max(0, min(keep, POOL - pool - pre));
            total = POOL - pool;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j < keep) {
                const int slot = pool + pre + (keep - 1 - j);
                pItem[slot] = ci[j];
                pT[slot] = ck[j];
            }
        }
        pool += total;
        __builtin_amdgcn_wave_barrier();
        const int take = min(pool, pool <= soft ? kRow : 1);
        item = kNoItem;
        if (l < take) {
            const uint32_t it = pItem[pool - 1 - l];
            const float tt = pT[pool - 1 - l];
            item = tt <= thi ? it : kNoItem;
        }
        pool -= take;
        __builtin_amdgcn_wave_barrier();
        raySteps++;
        if (pool > 0 || row_bits<kRow>(item != kNoItem, base) != 0u) continue;
        if (l == 0) sd_store<N>(a, x, y, depths);
        maxSteps = max(maxSteps, raySteps);
        phase = kFetch;
    }
    if (a.counters) {
        atomicAdd(&a.counters[1], (unsigned long long)active);
        atomicAdd(&a.counters[2], (unsigned long long)st.nodes);
        atomicAdd(&a.counters[3], (unsigned long long)st.tris);
        atomicAdd(&a.counters[4], (unsigned long long)delivered);
        atomicMax(&a.counters[6], (unsigned long long)maxSteps);
        atomicAdd(&a.counters[9], (unsigned long long)st.leaves);
    }
}

// Phase 3 of the split trace: anyHit -> algorithm over the K nearest keys of every live ray
// (one row of ROW lanes per ray, lane j prepares key j), then the SD texel store
// (StochasticDepthMapRT.rt.slang:90-104).  Persistent rows stride over the queue partitions.
template <int K, int N, int ROW, bool RASTER = false>
__global__ void __launch_bounds__(kBlock) sd_resolve_row_kernel(SDArgs a, const float4* __restrict__ queue,
                                                                uint32_t* __restrict__ qctl,
                                                                const uint2* __restrict__ keys) {
    constexpr int kRowRays = kBlock / ROW;
    const int lane = threadIdx.x;
    const int l = lane & (ROW - 1), base = lane & ~(ROW - 1), row = lane / ROW;
    const uint32_t rows = gridDim.x * (uint32_t)kRowRays, me = blockIdx.x * (uint32_t)kRowRays + (uint32_t)row;
    const rsd_camera& c = a.cam;
    const float DEFAULT = a.normalize ? 1.0f : 3.40282347e+37f;  // Common.slangh:16
    uint32_t delivered = 0;
    // live ray g of the frame = partition part, entry g - (rays in partitions < part)
    uint32_t part = 0, partStart = 0, partCount = qctl[0];
    for (uint32_t g = me;; g += rows) {
        while (part < kQueueParts && g >= partStart + partCount) {
            partStart += partCount;
            if (++part < kQueueParts) partCount = qctl[part];
        }
        if (part >= kQueueParts) break;
        {
            const uint32_t slot = part * a.partCap + (g - partStart);
            f3 d;
            float TMin, TMax, cosT;
            uint32_t idx;
            ray_rec_load(queue, slot, d, TMin, TMax, cosT, idx);
            RayCtx r;
            ray_setup(r, mk(c.posW[0], c.posW[1], c.posW[2]), d);
            float rng = 0.0f, z = 0.0f;
            bool valid = false, af = false;
            if (l < K) {
                if constexpr (RASTER) {  // 64-bit (t, prim) keys of the raster walk
                    const unsigned long long k = a.keys64[(size_t)slot * K + l];
                    valid = k != ~0ull;
                    if (valid) sd_hit_terms(a, r, cosT, a.primRec[(uint32_t)k], rng, z, af);
                } else {  // (t bits, prim) keys of the row walk
                    const uint2 k = keys[(size_t)slot * K + l];
                    valid = k.y != kNoItem;
                    if (valid) sd_hit_terms(a, r, cosT, a.primRec[k.y], rng, z, af);
                }
            }
            const int found = __popc(row_bits<ROW>(valid, base));  // keys are sorted: a prefix
            float depths[N];
#pragma unroll
            for (int i = 0; i < N; ++i) depths[i] = DEFAULT;
            uint32_t cnt = 0;
            sd_algorithm_row<K, N>(a, rng, z, af, found, base, depths, cnt, delivered);
            if (l == 0) sd_store<N>(a, (int)(idx % (uint32_t)a.sdW), (int)(idx / (uint32_t)a.sdW), depths);
        }
    }
    if (a.counters && l == 0 && delivered) atomicAdd(&a.counters[4], (unsigned long long)delivered);
}

// ------------------------------------------------------------------------------------
// Primary visibility: closest (t, prim) hit in [near/cos, far/cos] (Camera.slang:46-59),
// linear depth = t * cos (LinearizeDepth), view-space face normal packed 2x8
// (CompressNormals.ps.slang, viewSpace + use16Bit).  Miss: depth = farZ, normal = 0.
// ------------------------------------------------------------------------------------
struct GBArgs {
    const float4* nodes;
    const float4* tris;
    uint32_t triOff;
    rsd_camera cam;
    int W, H;
    uint32_t cull;
    float* z;
    uint16_t* n;
    float4* nw;  // raster mode: world face normal (RGBA32F); z then holds non-linear depth
    uint32_t alphaTest;  // the scene has alpha data: alpha test at LOD 0 (GBufferRaster useAlphaTest)
    AlphaData alpha;
};

__global__ void __launch_bounds__(kBlock) gbuffer_kernel(GBArgs a) {
    __shared__ uint32_t sstack[kLdsStack * kBlock];
    __shared__ float sstackT[kLdsStack * kBlock];
    const int lane = threadIdx.x;
    const int x = blockIdx.x * kTile + (lane & (kTile - 1));
    const int y = blockIdx.y * kTile + (lane / kTile);
    if (x >= a.W || y >= a.H) return;
    const rsd_camera& c = a.cam;
    const f3 wn = normalize(mk(c.W[0], c.W[1], c.W[2]));
    const f3 d = normalize(cam_dir(c, ((float)x + 0.5f) / (float)a.W + -c.jitterX,
                                   ((float)y + 0.5f) / (float)a.H + c.jitterY));
    const float cosT = dot(wn, d);
    const float invCos = 1.0f / cosT;
    RayCtx r;
    ray_setup(r, mk(c.posW[0], c.posW[1], c.posW[2]), d);
    KList<1> kl;
    TraceStats st{0u, 0u, 0u};
    const int found = trace_knearest<1>(a.nodes, a.triOff, r, c.nearZ * invCos, c.farZ * invCos, a.cull, false,
                                        0.0f, 0u, kl, &sstack[lane], &sstackT[lane], st, a.alphaTest != 0u, a.alpha);
    const size_t o = (size_t)y * a.W + x;
    if (!found) {
        if (a.nw) {
            a.z[o] = 1.0f;  // cleared depth
            a.nw[o] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        } else {
            a.z[o] = c.farZ;
            a.n[o] = 0;
        }
        return;
    }
    const float zlin = kl.t[0] * cosT;
    const uint32_t ti = kl.l[0];
    const float4 v0 = a.tris[3 * ti], v1 = a.tris[3 * ti + 1], v2 = a.tris[3 * ti + 2];
    const f3 e1 = mk(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z);
    const f3 e2 = mk(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z);
    const f3 nw = normalize(cross(e1, e2));
    if (a.nw) {
        // D3D-style [0,1] depth of a right-handed perspective: far (z - near) / (z (far - near))
        a.z[o] = c.farZ * (zlin - c.nearZ) / (zlin * (c.farZ - c.nearZ));
        a.nw[o] = make_float4(nw.x, nw.y, nw.z, 0.0f);
        return;
    }
    a.z[o] = zlin;
    const float* m = c.viewMat;
    const f3 nv = mk(m[0] * nw.x + m[1] * nw.y + m[2] * nw.z, m[4] * nw.x + m[5] * nw.y + m[6] * nw.z,
                     m[8] * nw.x + m[9] * nw.y + m[10] * nw.z);
    a.n[o] = (uint16_t)encode_normal_2x8(nv);
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
// walk: 0 = quad (depth-first), 1 = row walk + in-kernel algorithm, 2 = split (row walk ->
// keys -> resolve kernel), 3 = traversal-order any-hit stream (rsd_hit_order), 4 = raster (triangles
// -> 64-bit key lists -> resolve kernel)
static size_t quad_stack_bytes(const SDArgs& a) { return (size_t)a.quadStack * kQuadRays * 8u; }

// RSD_TRACE_SPEC=off: the generic walks (A/B runs)
static bool specEnvOff() {
    const char* e = std::getenv("RSD_TRACE_SPEC");
    return e && std::string(e) == "off";
}

template <int K, int N>
static hipError_t launch_sd_kn(const SDArgs& a, dim3 grid, uint32_t persistentBlocks, float4* queue, uint32_t* qctl,
                               uint2* keys, int walk, int pool, hipStream_t s) {
    constexpr int ROW = K <= 8 ? 8 : 16;
    uint32_t* qctlNext = a.qctlNext;
    if (a.touchList) {  // the two-pass setup
        const dim3 cgrid((grid.x + kClassWaves * kClassTiles - 1) / (kClassWaves * kClassTiles), grid.y);
        hipLaunchKernelGGL((sd_classify_kernel<N>), cgrid, dim3(kClassWaves * kBlock), 0, s, a, qctl, qctlNext);
        hipError_t e0 = hipGetLastError();
        if (e0 != hipSuccess) return e0;
        hipLaunchKernelGGL((sd_live_kernel<N>), dim3(a.liveBlocks), dim3(kLiveBlock), 0, s, a, queue, qctl);
    } else {
        const dim3 sgrid((grid.x + kSetupWaves - 1) / kSetupWaves, grid.y);
        hipLaunchKernelGGL((sd_setup_kernel<N>), sgrid, dim3(kSetupWaves * kBlock), 0, s, a, queue, qctl, qctlNext);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const dim3 pg(persistentBlocks), wb(kBlock);
    if (walk == 2) {
        if (a.counters) hipLaunchKernelGGL((sd_trace_row_kernel<K, N, ROW, true, true>), pg, wb, 0, s, a, queue, qctl, keys);
        else if (pool == 128) hipLaunchKernelGGL((sd_trace_row_kernel<K, N, ROW, true, false, 128>), pg, wb, 0, s, a, queue, qctl, keys);
        else hipLaunchKernelGGL((sd_trace_row_kernel<K, N, ROW, true, false>), pg, wb, 0, s, a, queue, qctl, keys);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL((sd_resolve_row_kernel<K, N, ROW>), pg, wb, 0, s, a, queue, qctl, keys);
    } else if (walk == 3) {
        hipLaunchKernelGGL((sd_trace_ordered_kernel<N>), pg, wb, quad_stack_bytes(a), s, a, queue, qctl);
    } else if (walk == 5) {
        hipLaunchKernelGGL((sd_trace_wavefront_kernel<N>), pg, wb, 0, s, a, queue, qctl);
    } else if (walk == 6) {
        // 8-lane rows at every K (K = 16: two keys per lane, row_insert2)
        const size_t rowLds = (size_t)(kBlock / 8) * pool * 8u, lds = std::max(rowLds, quad_stack_bytes(a));
        if (pool == 128) hipLaunchKernelGGL((sd_trace_hybrid_kernel<K, N, 8, 128>), pg, wb, lds, s, a, queue, qctl, keys);
        else hipLaunchKernelGGL((sd_trace_hybrid_kernel<K, N, 8, kPoolCap>), pg, wb, lds, s, a, queue, qctl, keys);
    } else if (walk == 4) {
        hipLaunchKernelGGL((sd_raster_kernel<K>), dim3((a.nTris + kRasterBlock - 1) / kRasterBlock), dim3(kRasterBlock),
                           0, s, a, queue, qctl);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL((sd_resolve_row_kernel<K, N, ROW, true>), pg, wb, 0, s, a, queue, qctl, keys);
    } else if (walk == 1) {
        // the specialised walk (RSD_TRACE_SPEC=off: the generic one, A/B runs)
        const char* specEnv = std::getenv("RSD_TRACE_SPEC");
        const bool spec = !(specEnv && std::string(specEnv) == "off") && !a.alphaTest && a.impl != 1u &&
                          a.impl != 3u && a.maxCount <= (uint32_t)K;
        if (a.counters) hipLaunchKernelGGL((sd_trace_row_kernel<K, N, ROW, false, true>), pg, wb, 0, s, a, queue, qctl, keys);
        else if (spec && pool == 128) hipLaunchKernelGGL((sd_trace_row_kernel<K, N, ROW, false, false, 128, true>), pg, wb, 0, s, a, queue, qctl, keys);
        else if (spec) hipLaunchKernelGGL((sd_trace_row_kernel<K, N, ROW, false, false, kPoolCap, true>), pg, wb, 0, s, a, queue, qctl, keys);
        else hipLaunchKernelGGL((sd_trace_row_kernel<K, N, ROW, false, false>), pg, wb, 0, s, a, queue, qctl, keys);
    } else {
        // the specialised quad walk (the row walk's conditions; RSD_TRACE_SPEC=off: the generic one)
        const char* specEnv = std::getenv("RSD_TRACE_SPEC");
        const bool spec = !(specEnv && std::string(specEnv) == "off") && !a.alphaTest && a.impl != 1u &&
                          a.impl != 3u && a.maxCount <= (uint32_t)K && !a.counters;
        const size_t lds = quad_stack_bytes(a);
        if (a.counters) hipLaunchKernelGGL((sd_trace_queue_kernel<K, N, false, true>), pg, wb, lds, s, a, queue, qctl);
        else if (spec) hipLaunchKernelGGL((sd_trace_queue_kernel<K, N, true>), pg, wb, lds, s, a, queue, qctl);
        else hipLaunchKernelGGL((sd_trace_queue_kernel<K, N>), pg, wb, lds, s, a, queue, qctl);
    }
    return hipGetLastError();
}

template <int K>
static hipError_t launch_sd_k(const SDArgs& a, uint32_t N, dim3 grid, uint32_t pb, float4* q, uint32_t* qc, uint2* keys,
                              int walk, int pool, hipStream_t s) {
    switch (N) {
        case 1: return launch_sd_kn<K, 1>(a, grid, pb, q, qc, keys, walk, pool, s);
        case 2: return launch_sd_kn<K, 2>(a, grid, pb, q, qc, keys, walk, pool, s);
        case 4: return launch_sd_kn<K, 4>(a, grid, pb, q, qc, keys, walk, pool, s);
        case 8: return launch_sd_kn<K, 8>(a, grid, pb, q, qc, keys, walk, pool, s);
        case 16: return launch_sd_kn<K, 16>(a, grid, pb, q, qc, keys, walk, pool, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rsd

using namespace rsd;

namespace {
// coverage-mask tables per (device, N), process-wide, never freed (kernels in flight on any
// stream may read them)
struct LutCache {
    int32_t* d_idx = nullptr;
    uint32_t* d_lut = nullptr;
};
constexpr int kLutDevices = 64;
LutCache g_lut[kLutDevices][17];
std::mutex g_lut_mutex;

// the SD-trace workspace of (scene, stream); created on the stream's first trace.  Host threads may trace
// one scene on their own streams (the band frame's rank threads): the list is locked; a workspace is only
// used by its stream's calls, which the caller orders
constexpr size_t kMaxWorkspaces = 64;
rsd_status sd_workspace(rsd_scene* scene, hipStream_t s, SdWorkspace** out) {
    std::lock_guard<std::mutex> lock(scene->ws_mutex);
    for (SdWorkspace* w : scene->sd_ws)
        if (w->stream == s) { *out = w; return RSD_OK; }
    if (scene->sd_ws.size() >= kMaxWorkspaces) {
        // a caller cycling through many transient streams: drain the device (no trace of this
        // scene can still be using a workspace) and start over instead of growing without bound
        RSD_HIP(hipDeviceSynchronize());
        release_sd_workspaces(scene);
    }
    SdWorkspace* w = new SdWorkspace();
    w->stream = s;
    hipError_t e = hipMalloc(&w->qctl, 2 * kQctlWords * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&w->counters, 32 * sizeof(unsigned long long));
    if (e != hipSuccess) {
        (void)hipFree(w->qctl);
        delete w;
        return hip_fail(e, "sd workspace");
    }
    scene->sd_ws.push_back(w);
    *out = w;
    return RSD_OK;
}

rsd_status ensure_lut(int dev, uint32_t N, const int32_t** idx, const uint32_t** lut) {
    if (dev < 0 || dev >= kLutDevices || N > 16) {
        set_error("rsd_sd_trace: device index >= 64 or N > 16");
        return RSD_ERR_UNSUPPORTED;
    }
    std::lock_guard<std::mutex> lock(g_lut_mutex);
    LutCache& c = g_lut[dev][N];
    if (!c.d_lut) {
        // StochasticDepthMapRT.cpp:79-124 generateStratifiedLookupTable
        std::vector<int32_t> ind(N + 1);
        std::vector<uint32_t> tab(1u << N);
        auto binom = [](int n, int k) {
            std::vector<int> C(k + 1, 0);
            C[0] = 1;
            for (int i = 1; i <= n; i++)
                for (int j = std::min(i, k); j > 0; j--) C[j] = C[j] + C[j - 1];
            return C[k];
        };
        ind[0] = 0;
        for (uint32_t i = 1; i <= N; i++) ind[i] = binom((int)N, (int)i - 1) + ind[i - 1];
        std::vector<int32_t> cur(ind);
        tab[0] = 0;
        for (uint32_t i = 1; i < (1u << N); i++) {
            int pc = __builtin_popcount(i);
            tab[cur[pc]] = i;
            cur[pc]++;
        }
        int32_t* di = nullptr;
        uint32_t* dl = nullptr;
        RSD_HIP(hipMalloc(&di, sizeof(int32_t) * ind.size()));
        RSD_HIP(hipMalloc(&dl, sizeof(uint32_t) * tab.size()));
        RSD_HIP(hipMemcpy(di, ind.data(), sizeof(int32_t) * ind.size(), hipMemcpyHostToDevice));
        RSD_HIP(hipMemcpy(dl, tab.data(), sizeof(uint32_t) * tab.size(), hipMemcpyHostToDevice));
        c.d_idx = di;
        c.d_lut = dl;
    }
    *idx = c.d_idx;
    *lut = c.d_lut;
    return RSD_OK;
}
}  // namespace

namespace {
// The SD trace of the 8-row tile rows t = start + k * step, k < n (rsd_sd_trace_band_ex: an
// interleaved band; rsd_sd_trace_rows: a contiguous range).
rsd_status sd_trace_impl(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* p, const float* d_linear_z,
                         uint32_t z_w, uint32_t z_h, uint32_t* d_ray_min, uint32_t* d_ray_max, float* d_sd_out,
                         uint32_t sd_w, uint32_t sd_h, uint32_t start, uint32_t step, uint32_t n, uint32_t flags,
                         rsd_counters* counters, rsd_stream stream) {
    const bool consume = (flags & RSD_SD_CONSUME_INTERVALS) != 0u;
    const bool throughput = (flags & RSD_SD_THROUGHPUT) != 0u;
    if (flags & ~(RSD_SD_CONSUME_INTERVALS | RSD_SD_THROUGHPUT)) {
        set_error("rsd_sd_trace_band_ex: unknown flag");
        return RSD_ERR_INVALID_ARG;
    }
    if (consume && (!p || !p->ray_interval || !d_ray_min || !d_ray_max)) {
        set_error("rsd_sd_trace_band_ex: RSD_SD_CONSUME_INTERVALS needs RayInterval and both interval maps");
        return RSD_ERR_INVALID_ARG;
    }
    if (!scene || !cam || !p || !d_linear_z || !d_sd_out || sd_w == 0 || sd_h == 0 || z_w == 0 || z_h == 0) {
        set_error("rsd_sd_trace: null argument or empty extent");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t N = p->sample_count;
    if (N != 1 && N != 2 && N != 4 && N != 8 && N != 16) {
        // StochasticDepthMapRT.cpp:190 throws for other N; 16 is the documented extension
        set_error("rsd_sd_trace: SampleCount must be 1, 2, 4, 8 or 16");
        return RSD_ERR_UNSUPPORTED;
    }
    if (p->implementation == RSD_SD_RESERVOIR_SAMPLING || p->implementation > RSD_SD_KBUFFER) {
        set_error("rsd_sd_trace: ReservoirSampling is a raster-only implementation");
        return RSD_ERR_UNSUPPORTED;
    }
    if (p->hit_order > RSD_HIT_ORDER_WAVEFRONT) {
        set_error("rsd_sd_trace: hit_order must be RSD_HIT_ORDER_CANONICAL, _TRAVERSAL or _WAVEFRONT");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->use_16bit && N > 4) {
        // StochasticDepthMapRT.cpp:199 throws for 16-bit maps with more than 4 samples
        set_error("rsd_sd_trace: Use16Bit supports SampleCount 1, 2 and 4 only");
        return RSD_ERR_UNSUPPORTED;
    }
    if (p->max_count == 0 && p->implementation != RSD_SD_COVERAGE_MASK) {
        set_error("rsd_sd_trace: MaxCount must be >= 1");
        return RSD_ERR_INVALID_ARG;
    }
    if (2 * p->guard_band >= (int32_t)sd_w || 2 * p->guard_band >= (int32_t)sd_h || p->guard_band < 0) {
        set_error("rsd_sd_trace: GuardBand leaves no interior");
        return RSD_ERR_INVALID_ARG;
    }
    if (scene->triangle_count == 0) {
        // no geometry: every texel keeps DEFAULT_DEPTH
        const float def = p->normalize ? 1.0f : 3.40282347e+37f;
        const size_t n = (size_t)sd_w * sd_h * (N < 4 ? N : 4) * ((N + 3) / 4);
        std::vector<float> h(n, def);
        std::vector<uint16_t> h16(n, p->normalize ? (uint16_t)0x3c00u : (uint16_t)0x7c00u);  // 1.0 / +inf
        if (p->use_16bit)
            RSD_HIP(hipMemcpyAsync(d_sd_out, h16.data(), n * 2, hipMemcpyHostToDevice, (hipStream_t)stream));
        else
            RSD_HIP(hipMemcpyAsync(d_sd_out, h.data(), n * 4, hipMemcpyHostToDevice, (hipStream_t)stream));
        RSD_HIP(hipStreamSynchronize((hipStream_t)stream));
        if (consume) {
            rsd_status cs = rsd_svao_clear_intervals(d_ray_min, d_ray_max, sd_w * sd_h, stream);
            if (cs != RSD_OK) return cs;
        }
        if (counters) { *counters = rsd_counters{}; counters->rays_dispatched = (uint64_t)sd_w * sd_h; }
        return RSD_OK;
    }
    SDArgs a{};
    a.nodes = scene->d_nodes;
    {
        const char* pEnv = std::getenv("RSD_TRACE_PRIO");  // A/B runs: the trace's waves ahead of other frames' passes
        a.prio = pEnv && std::string(pEnv) == "on" ? 1u : 0u;
    }
    a.tris = scene->d_tris;
    a.triOff = scene->tri_offset;
    a.cam = *cam;
    a.linearZ = d_linear_z;
    a.zW = (int)z_w;
    a.zH = (int)z_h;
    a.rayMin = d_ray_min;
    a.rayMax = d_ray_max;
    a.sd = d_sd_out;
    a.sdW = (int)sd_w;
    a.sdH = (int)sd_h;
    a.guard = p->guard_band;
    a.impl = p->implementation;
    a.maxCount = p->max_count;
    a.jitter = p->jitter;
    a.normalize = p->normalize;
    a.rayInterval = p->ray_interval;
    a.cull = p->cull_mode;
    a.alpha = p->alpha;
    a.lutIdx = nullptr;
    a.lut = nullptr;
    a.counters = nullptr;
    a.bandStart = (int)start;
    a.bandStep = (int)step;
    a.bandN = (int)n;
    a.alphaTest = p->alpha_test && scene->d_alpha ? 1u : 0u;
    a.f16 = p->use_16bit ? 1u : 0u;
    a.deadFast = 0u;
    a.consume = consume ? 1u : 0u;
    a.rayMinW = d_ray_min;
    a.rayMaxW = d_ray_max;
    // Lower bound of dot(normalize(W), normalize(cam_dir)) over every texel centre of the map
    // (guard band included, +-1 texel): the cosine of every SD ray's direction to the view axis
    double cosLower = 0.0;
    {
        const int dimx = (int)sd_w - 2 * p->guard_band, dimy = (int)sd_h - 2 * p->guard_band;
        auto ndcMax = [](double lo, double hi) { return std::max(std::fabs(2.0 * lo - 1.0), std::fabs(2.0 * hi - 1.0)); };
        const double nx = ndcMax((-p->guard_band + 0.5) / dimx - cam->jitterX - 1.0 / dimx,
                                 ((int)sd_w - p->guard_band) / (double)dimx - cam->jitterX + 1.0 / dimx);
        const double ny = ndcMax((-p->guard_band + 0.5) / dimy + cam->jitterY - 1.0 / dimy,
                                 ((int)sd_h - p->guard_band) / (double)dimy + cam->jitterY + 1.0 / dimy);
        auto len = [](const float* v) { return std::sqrt((double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2]); };
        const double lw = len(cam->W);
        auto dotw = [&](const float* v) { return ((double)v[0] * cam->W[0] + (double)v[1] * cam->W[1] + (double)v[2] * cam->W[2]) / lw; };
        const double num = dotw(cam->W) - nx * std::fabs(dotw(cam->U)) - ny * std::fabs(dotw(cam->V));
        const double den = nx * len(cam->U) + ny * len(cam->V) + lw;
        if (dimx > 0 && dimy > 0 && den > 0.0) cosLower = num / den;
    }
    // if farZ / bound is far below FLT_MAX, TMax < FLT_MAX for every texel, so rayMin ==
    // asuint(FLT_MAX) means TMin >= FLT_MAX > TMax (dead)
    if (p->ray_interval && d_ray_min && cosLower > 1e-3 && (double)cam->farZ / (0.5 * cosLower) < 1e37)
        a.deadFast = 1u;
    a.raster = 0u;
    a.lpt = 0u;
    a.lptLen = 0.0f;
    {
        // RSD_TRACE_SPREAD=on: the static first rays dealt row-major over the waves (SDArgs.spread; A/B)
        const char* spreadEnv = std::getenv("RSD_TRACE_SPREAD");
        a.spread = spreadEnv && std::string(spreadEnv) == "on" ? 1u : 0u;
        const char* qrEnv = std::getenv("RSD_TRACE_QRANGE");
        a.qrange = qrEnv && std::string(qrEnv) == "long" ? 1u : qrEnv && std::string(qrEnv) == "short" ? 2u : 0u;
        const char* dgEnv = std::getenv("RSD_SETUP_DIAG");  // diagnostics: skip / nolive (results wrong by design)
        a.diag = dgEnv && std::string(dgEnv) == "skip" ? 1u : dgEnv && std::string(dgEnv) == "nolive" ? 2u : 0u;
    }
    // clean tiles: the stamp names what DEFAULT_DEPTH looks like in this map (value, storage, layers)
    a.tileState = p->d_tile_state;
    a.tileSig = 1u | (p->normalize ? 2u : 0u) | (p->use_16bit ? 4u : 0u) | ((uint32_t)N << 3);
    a.tileCount = ((sd_w + kTile - 1) / kTile) * ((sd_h + kTile - 1) / kTile);
    a.primRec = scene->d_prim_rec;
    a.entOn = 0u;
    a.entSlots = static_cast<const uint4*>(scene->d_entry);
    a.entItems = scene->d_entry ? reinterpret_cast<const float4*>(static_cast<const char*>(scene->d_entry) +
                                                                   scene->entry_items_off)
                                : nullptr;
    a.entBits = scene->entry_bits;
    a.entProbe = scene->entry_probe;
    a.entRmax = (int)scene->entry_rmax;
    for (int k = 0; k < 3; ++k) a.entOrigin[k] = scene->entry_origin[k];
    a.entExtent = scene->entry_extent;
    a.entQ = nullptr;
    a.rayLog = nullptr;
    a.alphaData = scene->alpha;
    a.alphaData.spread = rsd_ray_cone_spread(cam->focalLength, sd_h);  // default texture dims = SD map
    if (p->implementation == RSD_SD_COVERAGE_MASK) {
        rsd_status s = ensure_lut(scene->dev->hip_device, N, &a.lutIdx, &a.lut);
        if (s != RSD_OK) return s;
    }
    hipStream_t s = (hipStream_t)stream;
    SdWorkspace* ws = nullptr;
    {
        rsd_status st = sd_workspace(scene, s, &ws);
        if (st != RSD_OK) return st;
    }
    {
        // per-frame-size ray terms (recomputed when the SD map size, guard band or jitter change)
        RayTabCache& rt = ws->raytab;
        const RayTabCache key{(int)sd_w, (int)sd_h, p->guard_band, p->jitter, cam->jitterX, cam->jitterY,
                              {cam->W[0], cam->W[1], cam->W[2]}, scene->dev->hip_device};
        const size_t need = (6 * (size_t)sd_w + 6 * (size_t)sd_h + 3) * sizeof(float);
        if (!rt.same(key) || rt.cap < need) {
            if (rt.cap < need) {
                RSD_HIP(hipStreamSynchronize(s));
                (void)hipFree(rt.d);
                rt.d = nullptr;
                rt.cap = 0;
                RSD_HIP(hipMalloc(&rt.d, need));
                rt.cap = need;
            }
            const int n = (int)std::max(sd_w, sd_h);
            hipLaunchKernelGGL(ray_table_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rt.d, (int)sd_w, (int)sd_h,
                               p->guard_band, p->jitter, cam->jitterX, cam->jitterY, f3{cam->W[0], cam->W[1], cam->W[2]});
            hipError_t te = hipGetLastError();
            if (te != hipSuccess) return hip_fail(te, "ray_table_kernel launch");
            rt.setKey(key);
        }
        a.rayTab = rt.d;
    }
    if (counters) {
        // per (scene, stream): concurrent instrumented traces on other streams keep their own
        RSD_HIP(hipMemsetAsync(ws->counters, 0, 32 * sizeof(unsigned long long), s));
        a.counters = ws->counters;
    }
    const char* rayLogPath = counters ? std::getenv("RSD_TRACE_RAYLOG") : nullptr;  // diagnostics only
    const uint32_t tiles = (sd_h + kTile - 1) / kTile;
    dim3 grid((sd_w + kTile - 1) / kTile, consume ? tiles : n);
    // k = the MAX_COUNT nearest keys decide Default and KBuffer; coverage mask streams chunks
    const uint32_t need = p->implementation == RSD_SD_COVERAGE_MASK ? 8u : p->max_count;
    const uint32_t setupBlocks = grid.x * grid.y;
    a.partCap = (setupBlocks + kQueueParts - 1) / kQueueParts * (uint32_t)kBlock;
    // the two-pass setup's touched-texel lists: a partition holds the texels of its classify workgroups (and its
    // queue partition those texels' rays: partCap covers both)
    constexpr uint32_t kClassTilesPerBlock = kClassWaves * kClassTiles;
    const uint32_t classBlocks = (grid.x + kClassTilesPerBlock - 1) / kClassTilesPerBlock * grid.y;
    const uint32_t touchCap = (classBlocks + kQueueParts - 1) / kQueueParts * (kClassTilesPerBlock * (uint32_t)kBlock);
    a.partCap = std::max(a.partCap, touchCap + 2u * (uint32_t)kBlock * kQueueParts);
    // live-ray queue workspace (grow-only; the first call of a larger map allocates)
    const size_t need_q = std::max(((size_t)(sd_w + kTile - 1) / kTile * ((sd_h + kTile - 1) / kTile) + kQueueParts) * kBlock,
                                   (size_t)a.partCap * kQueueParts);
    const uint32_t K = need <= 4 ? 4u : (need <= 8 ? 8u : 16u);
    // split walk (trace -> keys -> resolve) when one chunk of K keys decides every texel
    const bool split = p->implementation != RSD_SD_COVERAGE_MASK && p->max_count <= K;
    const size_t queueBytes = need_q * 32, keyBytes = split ? need_q * K * sizeof(uint2) : 0;
    const size_t entBytes = scene->d_entry ? need_q * kEntryCap * sizeof(uint32_t) : 0;
    const size_t touchBytes = (size_t)touchCap * kQueueParts * sizeof(uint32_t);
    if (ws->queue_cap < queueBytes + keyBytes + entBytes + touchBytes) {
        RSD_HIP(hipStreamSynchronize(s));
        (void)hipFree(ws->queue);
        ws->queue = nullptr;
        ws->queue_cap = 0;
        RSD_HIP(hipMalloc(&ws->queue, queueBytes + keyBytes + entBytes + touchBytes));
        ws->queue_cap = queueBytes + keyBytes + entBytes + touchBytes;
    }
    uint32_t* touchList = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws->queue) + queueBytes + keyBytes + entBytes);
    float4* queue = reinterpret_cast<float4*>(ws->queue);
    uint2* keys = reinterpret_cast<uint2*>(reinterpret_cast<char*>(ws->queue) + queueBytes);
    if (entBytes) a.entQ = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws->queue) + queueBytes + keyBytes);
    const size_t rayLogBytes = rayLogPath && *rayLogPath ? need_q * 8 * sizeof(uint32_t) : 0;
    if (rayLogBytes) {
        RSD_HIP(hipMalloc(&a.rayLog, rayLogBytes));
        RSD_HIP(hipMemsetAsync(a.rayLog, 0, rayLogBytes, s));
    }
    // double-buffered queue control (sd_setup_kernel); both buffers are reset on first use and
    // after a failed launch sequence
    if (ws->qctl_dirty) {
        RSD_HIP(hipMemsetAsync(ws->qctl, 0, 2 * kQctlWords * sizeof(uint32_t), s));
        ws->qctl_dirty = false;
    }
    uint32_t* qctl = ws->qctl + (ws->qctl_gen & 1u) * kQctlWords;
    a.qctlNext = ws->qctl + ((ws->qctl_gen + 1u) & 1u) * kQctlWords;
    // traversal walk: row-parallel (default) unless the tree is too deep for its LDS pool
    // bound (kPoolCap >= poolSoft + 48 + 3 * depth), or RSD_TRACE_WALK=quad asks for the
    // depth-first quad walk (A/B measurements)
    const int depth = (int)std::max(1u, scene->stats.wide_depth);
    a.quadStack = quad_stack_entries((uint32_t)depth);
    // the row walk's LDS pool: 128 entries per ray (8 KB per wave) wherever the tree depth allows it
    // (the pool bound above), else 256; with the specialised walk the smaller pool measured faster alone
    // (75.7 vs 78.3 us at configs[1]) and leaves more LDS to the other frames' passes
    // (profiles/round3/ab/trace_pool/).  RSD_TRACE_POOL=256 forces the large pool (A/B runs); the
    // instrumented (counters) walk always uses 256.
    static const char* poolEnv = std::getenv("RSD_TRACE_POOL");
    // (the wavefront stream's order depends on the pool bound: always the 256-entry pool, soft bound below)
    int pool = (poolEnv && std::atoi(poolEnv) == 256) || counters || p->hit_order == RSD_HIT_ORDER_WAVEFRONT
                   ? kPoolCap : 128;
    if (pool - 48 - 3 * depth < 16) pool = kPoolCap;
    a.poolSoft = std::min(pool - 48 - 3 * depth, 160);
    const char* walkEnv = std::getenv("RSD_TRACE_WALK");  // read per call: tests cover every walk
    const std::string walkName = walkEnv ? walkEnv : "";
    // The row walk wins when few rays are live (the launch is the slowest ray's chain); with
    // more SD texels the live rays fill the machine and the quad walk's lane utilisation wins
    // (rsd_sd_trace, row vs quad: 1080p/4 0.43 M texels 92 vs 133 us; 4K/4 1.0 M texels 443 vs
    // 327 us; 1080p full 6.9 M texels 688 vs 294 us -- DESIGN.md section 4)
    const uint64_t bandTexels = (uint64_t)sd_w * std::min<uint64_t>((uint64_t)n * kTile, sd_h);
    // RSD_SD_THROUGHPUT (frames in flight) no longer changes the walk: round 1 measured the quad walk
    // ahead with frames in flight (108 vs 118 us per frame), but with the segment entry grid and the
    // longest-first queue the row walk is ahead at every F (20-frame bench, configs[1]: F = 2/3/4/6
    // -> 169/157/154/161 vs 200/172/162/171 us; profiles/round3/ab/walk_*.json)
    (void)throughput;
    const bool rowWalk = a.poolSoft >= 16 && walkName != "quad" &&
                         (walkName == "fused" || walkName == "split" || bandTexels <= 600000u);
    // default: the fused row walk; RSD_TRACE_WALK=split|quad for A/B runs
    // raster walk: triangles -> per-texel K nearest keys (split-eligible canonical traces; the near
    // clip needs the cosine bound)
    const bool rasterOk = split && p->hit_order == RSD_HIT_ORDER_CANONICAL && cosLower > 1e-3 && scene->d_prim_rec;
    const bool raster = rasterOk && walkName == "raster";
    // the fused row walk carries every key's hit terms from its leaf test, so it needs no resolve
    // pass; RSD_TRACE_WALK=split keeps the key-list + resolve-kernel variant for A/B runs
    if (p->hit_order == RSD_HIT_ORDER_WAVEFRONT && a.poolSoft < 16) {
        set_error("rsd_sd_trace: the BVH is too deep for the wavefront order's LDS pool");
        return RSD_ERR_UNSUPPORTED;
    }
    int walk = p->hit_order == RSD_HIT_ORDER_TRAVERSAL ? 3 : p->hit_order == RSD_HIT_ORDER_WAVEFRONT ? 5
                     : raster ? 4 : !rowWalk ? 0
                     : (split && walkName == "split") ? 2 : 1;
    // segment entry grid: canonical walks (row, quad, split) start from the frontier of each ray's
    // segment; RSD_TRACE_ENTRY=off walks every ray from the root (A/B runs)
    if ((walk == 0 || walk == 1 || walk == 2) && a.entQ) {
        const char* entEnv = std::getenv("RSD_TRACE_ENTRY");
        a.entOn = entEnv && std::string(entEnv) == "off" ? 0u : 1u;
    }
    if (walk == 1 || walk == 0 || walk == 5) {
        // longest-first queue: rays whose interval exceeds 0.1 x TMin are dequeued first (configs[1]:
        // 90 -> 84 us); RSD_TRACE_LPT = off | a threshold (> 0 absolute, < 0 relative to TMin).  (The
        // traversal-order walk reads the split queue too, but measured no gain from it: 150.7 vs 147.3 us at
        // configs[1], profiles/round5/trace_ab/lpt_ordered_c1.json -- its rays start at the root.)
        const char* lptEnv = std::getenv("RSD_TRACE_LPT");
        const bool off = lptEnv && std::string(lptEnv) == "off";
        a.lpt = off ? 0u : 1u;
        a.lptLen = lptEnv && *lptEnv && !off ? (float)std::atof(lptEnv) : -0.1f;
    }
    // two-pass setup (sd_classify_kernel + sd_live_kernel) for the full-resolution maps, where the one-pass setup's
    // live-ray chains pass through the machine in tens of rounds: configs[2] setup 66 -> 45 us, trace 177 -> 154 us;
    // configs[4] 202 -> 152 us, 551 -> 487 us at the static pose, 0.989 -> 0.922 ms along the orbit
    // (profiles/round6/setup_twopass/).  The 1/4-resolution maps keep the one-pass setup: configs[1] 67 -> 72 us (one
    // round of the chain there: the second launch costs more than it saves), configs[3] (1.0 M texels) 197 -> 215 us
    // (the setup flat, the hybrid walk slower with the listed order of its rays).  Above 2 M texels;
    // RSD_SETUP_TWOPASS = on | off overrides (A/B runs, tests of small maps).
    {
        const char* tpEnv = std::getenv("RSD_SETUP_TWOPASS");
        const bool force = tpEnv && std::string(tpEnv) == "on", never = tpEnv && std::string(tpEnv) == "off";
        if (a.deadFast && walk != 4 && a.diag == 0u && !never && (force || bandTexels > 2000000u)) {
            a.touchList = touchList;
            a.touchCap = touchCap;
            // the resident grid: 5 workgroups of 4 waves per CU (92-94 VGPRs: 5 waves per SIMD), rounded to the partitions
            const uint32_t perCu = RSD_LIVE_WAVES > 5 ? (uint32_t)RSD_LIVE_WAVES : 5u;
            a.liveBlocks = ((uint32_t)std::max(1, scene->dev->cu_count) * perCu + kQueueParts - 1) / kQueueParts * kQueueParts;
        }
    }
    if (walk == 4) {
        const uint32_t tilesW = (sd_w + kTile - 1) / kTile, tilesH = (sd_h + kTile - 1) / kTile;
        const size_t slotBytes = (size_t)sd_w * sd_h * 4, tileBytes = (size_t)tilesW * tilesH * 8;
        const size_t keys64Bytes = (size_t)a.partCap * kQueueParts * K * 8;
        const size_t liveBytes = (size_t)tilesW * tilesH * 4;
        const size_t rb = slotBytes + tileBytes + liveBytes + keys64Bytes + 256;
        if (ws->raster_cap < rb) {
            RSD_HIP(hipStreamSynchronize(s));
            (void)hipFree(ws->raster);
            ws->raster = nullptr;
            ws->raster_cap = 0;
            RSD_HIP(hipMalloc(&ws->raster, rb));
            ws->raster_cap = rb;
        }
        char* base = static_cast<char*>(ws->raster);
        a.raster = 1u;
        a.keysK = K;
        a.nTris = scene->triangle_count;
        a.keys64 = reinterpret_cast<unsigned long long*>(base);
        a.slotMap = reinterpret_cast<int32_t*>(base + keys64Bytes);
        a.tileRec = reinterpret_cast<float2*>(base + keys64Bytes + slotBytes);
        a.liveTiles = reinterpret_cast<uint32_t*>(base + keys64Bytes + slotBytes + tileBytes);
        a.primRec = scene->d_prim_rec;
        a.tilesW = (int)tilesW;
        auto dot3h = [](const float* u, const float* v) { return (double)u[0] * v[0] + (double)u[1] * v[1] + (double)u[2] * v[2]; };
        const double uu = dot3h(cam->U, cam->U), vv = dot3h(cam->V, cam->V), ww = dot3h(cam->W, cam->W);
        for (int k = 0; k < 3; ++k) {
            a.projU[k] = (float)(cam->U[k] / uu);
            a.projV[k] = (float)(cam->V[k] / vv);
            a.projW[k] = (float)(cam->W[k] / ww);
            a.camWn[k] = (float)(cam->W[k] / std::sqrt(ww));
        }
        // every valid hit has t >= TMin >= 0.1 nearZ (initRayDesc eps) and cos >= cosLower, i.e. a
        // view depth >= 0.1 nearZ cosLower = w |W|: clip at half of that
        a.wClip = (float)(0.5 * 0.1 * cam->nearZ * cosLower / std::sqrt(ww));
    }
    // persistent waves: 8 per CU.  At 1080p/4 every row gets one of the ~22 K live rays in its
    // static first slot and the launch lasts as long as the slowest ray; 16 waves per CU (the
    // split walk holds < 128 VGPRs) measured no faster (tools/sd_time.py sweep)
    // The quad walk keeps its keys distributed over the quad since round 5 (QuadKeys: 177 -> 115 VGPRs at K = 16,
    // 96 at K = 8), and the full-resolution maps it serves are throughput-bound: 16 waves per CU, the register
    // limit at K = 16 once its LDS stack is sized to the tree (quad_stack_entries: the fixed 96-entry stack held
    // residency to 13; configs[4] 827 -> 713 us at 12, 699 -> 671 us from 12 to 16), and at K <= 8 (configs[2]
    // 263 -> 257 us; 20 measured the same, as did configs[3]); profiles/round5/trace_ab/wpc_*, r5p/.  The row walk
    // stays at 8 (latency-bound: 10 / 12 / 16 measured no faster).
    const char* wpcEnv = std::getenv("RSD_TRACE_WAVES_PER_CU");  // experiments only (read per call: A/B runs)
    const uint32_t wavesPerCu = wpcEnv ? (uint32_t)std::max(1, std::atoi(wpcEnv)) : (walk == 0 ? 16u : 8u);
    uint32_t pb = ((uint32_t)std::max(1, scene->dev->cu_count) * wavesPerCu + kQueueParts - 1) / kQueueParts *
                  kQueueParts;
    // The hybrid walk (round 5): a trace whose longest-first rays -- the ones whose chains set the launch: configs[3]'s
    // quad walk over them alone is 261 of its 268 us -- take the row walk (8 items per step) in the same launch
    // (sd_trace_hybrid_kernel: its first blocks run the row walk over the longest-first end of each queue partition,
    // the others the quad walk over the rest), where the fused row walk (configs[1]: 74 -> 66 us) or the quad walk
    // (configs[3] 268 -> 195 us, configs[2] 236 -> 177 us) would walk every ray alike.  Only for 8-lane rows
    // (K <= 8: with K = 16 the 16-lane row walk is the slower one).  With frames in flight (RSD_SD_THROUGHPUT) it
    // replaces the fused row walk of the small maps (configs[1]: 0.0834-0.0860 -> 0.0815-0.0840 ms per frame, three
    // alternating pairs, profiles/round6/hybrid_in_flight/), but not the quad walk of the full-resolution maps: there
    // the machine is already full of other frames' work and the quad walk's lane use wins (RSD_TRACE_HYBRID=all:
    // configs[2] 0.188-0.191 -> 0.202-0.206 ms per frame, configs[3] 0.308-0.317 -> 0.327-0.347;
    // profiles/round5/hybrid/in_flight/).  RSD_TRACE_HYBRID=off disables it, =all takes it for every walk;
    // RSD_TRACE_HYBRID_ROWWPC / RSD_TRACE_WAVES_PER_CU set the row / quad blocks per CU (A/B runs).
    const char* hyEnv = std::getenv("RSD_TRACE_HYBRID");
    // K = 16 (round 6, RSD_TRACE_HYBRID16=on; off by default): the row blocks walk 8-lane rows holding two keys per lane
    // (row_insert2).  Same bits, but slower at configs[4]: 555 -> 688 us static, 0.987 -> 1.597 ms along the orbit
    // (profiles/round6/hybrid16/).  Its long rays are many (the quad walk over them alone takes 411 of its 547 us: the
    // set is throughput-bound, where 8 lanes per ray lose to 4), and one launch gives every block the row walk's 191
    // VGPRs: 8 waves per CU instead of the quad walk's 16 (the quad walk alone at 4 per CU: 972 us).
    const char* hy16Env = std::getenv("RSD_TRACE_HYBRID16");
    const bool hybridK = K <= 8 || (hy16Env && std::string(hy16Env) == "on");
    const bool hybridOk = (walk == 0 || walk == 1) && hybridK && a.lpt && a.poolSoft >= 16 &&
                          (!throughput || walk == 1 || (hyEnv && std::string(hyEnv) == "all")) &&
                          !(hyEnv && std::string(hyEnv) == "off") && !a.alphaTest && a.impl != 1u && a.impl != 3u &&
                          a.maxCount <= (uint32_t)K && !(specEnvOff());
    if (hybridOk && !counters) {
        const char* rwEnv = std::getenv("RSD_TRACE_HYBRID_ROWWPC");
        const uint32_t rw = rwEnv ? (uint32_t)std::max(1, std::atoi(rwEnv)) : 4u, qw = wpcEnv ? wavesPerCu : 8u;
        const uint32_t cus = (uint32_t)std::max(1, scene->dev->cu_count);
        a.hybridRowBlocks = (cus * rw + kQueueParts - 1) / kQueueParts * kQueueParts;
        const char* prEnv = std::getenv("RSD_TRACE_ROWPRIO");
        a.rowPrio = prEnv && std::string(prEnv) == "on" ? 1u : 0u;
        pb = a.hybridRowBlocks + (cus * qw + kQueueParts - 1) / kQueueParts * kQueueParts;
        walk = 6;
    }
    hipError_t e = hipSuccess;
    if (grid.y == 0) {}
    else if (K == 4) e = launch_sd_k<4>(a, N, grid, pb, queue, qctl, keys, walk, pool, s);
    else if (K == 8) e = launch_sd_k<8>(a, N, grid, pb, queue, qctl, keys, walk, pool, s);
    else e = launch_sd_k<16>(a, N, grid, pb, queue, qctl, keys, walk, pool, s);
    if (e != hipSuccess) {
        ws->qctl_dirty = true;
        return hip_fail(e, "sd_trace_kernel launch");
    }
    if (grid.y != 0) ws->qctl_gen++;
    if (counters) {
        unsigned long long h[32];
        RSD_HIP(hipMemcpyAsync(h, ws->counters, sizeof(h), hipMemcpyDeviceToHost, s));
        RSD_HIP(hipStreamSynchronize(s));
        counters->rays_dispatched = h[0];
        counters->rays_active = h[1];
        counters->nodes_visited = h[2];
        counters->tris_tested = h[3];
        counters->hits_delivered = h[4];
        counters->max_nodes_per_ray = h[5];
        counters->max_steps_per_ray = h[6];
        counters->sum_ray_clocks = h[7];
        counters->max_ray_clocks = h[8];
        counters->leaves_visited = h[9];
        // walk: the hybrid an uninstrumented trace of this call takes (the kernels a caller's timed traces ran);
        // walk_instrumented: the walk this instrumented launch ran (its step clocks), never the hybrid
        counters->walk = (uint64_t)((walk == 0 || walk == 1) && hybridOk ? 6 : walk);
        counters->walk_instrumented = (uint64_t)walk;
        counters->entry_lookups = h[19];
        counters->entry_items = h[20];
        // row walk (instrumented): per-step clock sums and the clock of the instrumented launch
        counters->step_fetch_clocks = h[16];
        counters->step_compute_clocks = h[17];
        counters->step_pool_clocks = h[18];
        counters->row_steps = h[14];
        counters->texels_clean = h[25];
        counters->shader_clock_mhz = h[22] ? (double)h[21] / ((double)h[22] * 0.01) : 0.0;  // 100 MHz realtime
        if (const char* dbg = std::getenv("RSD_TRACE_PHASES"))
            if (*dbg) std::fprintf(stderr, "[rsd] row walk phase clocks: fetch %llu step %llu resolve %llu steps %llu loops %llu"
                                   " | step split: mem %llu compute %llu pool %llu | compute split: box+sort %llu"
                                   " tri-tests %llu merge+push %llu\n",
                                   h[11], h[12], h[13], h[14], h[15], h[16], h[17], h[18], h[23], h[24],
                                   h[17] - h[23] - h[24]);
        if (a.rayLog) {
            std::vector<uint32_t> lg(rayLogBytes / 4);
            RSD_HIP(hipMemcpy(lg.data(), a.rayLog, rayLogBytes, hipMemcpyDeviceToHost));
            (void)hipFree(a.rayLog);
            if (FILE* f = std::fopen(rayLogPath, "wb")) {
                std::fwrite(lg.data(), 4, lg.size(), f);
                std::fclose(f);
            }
        }
        if (h[10]) {  // the pool bound was violated: results of this trace are not reliable
            set_error("rsd_sd_trace: traversal pool overflow (BVH deeper than the row walk supports)");
            return RSD_ERR_HIP;
        }
    }
    return RSD_OK;
}

}  // namespace

extern "C" rsd_status rsd_sd_trace_band_ex(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* p,
                                           const float* d_linear_z, uint32_t z_w, uint32_t z_h, uint32_t* d_ray_min,
                                           uint32_t* d_ray_max, float* d_sd_out, uint32_t sd_w, uint32_t sd_h,
                                           uint32_t band_index, uint32_t band_count, uint32_t flags,
                                           rsd_counters* counters, rsd_stream stream) {
    if (band_count == 0 || band_index >= band_count) {
        set_error("rsd_sd_trace_band: band_index must be < band_count");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t tiles = (sd_h + kTile - 1) / kTile;
    const uint32_t n = tiles > band_index ? (tiles - band_index + band_count - 1) / band_count : 0u;
    return sd_trace_impl(scene, cam, p, d_linear_z, z_w, z_h, d_ray_min, d_ray_max, d_sd_out, sd_w, sd_h, band_index,
                         band_count, n, flags, counters, stream);
}

extern "C" rsd_status rsd_sd_trace_rows(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* p,
                                        const float* d_linear_z, uint32_t z_w, uint32_t z_h, uint32_t* d_ray_min,
                                        uint32_t* d_ray_max, float* d_sd_out, uint32_t sd_w, uint32_t sd_h,
                                        uint32_t row0, uint32_t row1, uint32_t flags, rsd_counters* counters,
                                        rsd_stream stream) {
    if (row0 > row1 || row1 > sd_h || row0 % kTile != 0u || (row1 % kTile != 0u && row1 != sd_h)) {
        set_error("rsd_sd_trace_rows: rows must satisfy row0 <= row1 <= sd_h, multiples of 8 (row1 may be sd_h)");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t t0 = row0 / kTile, t1 = (row1 + kTile - 1) / kTile;
    return sd_trace_impl(scene, cam, p, d_linear_z, z_w, z_h, d_ray_min, d_ray_max, d_sd_out, sd_w, sd_h, t0, 1u,
                         t1 - t0, flags, counters, stream);
}

extern "C" rsd_status rsd_sd_trace_band(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* p,
                                        const float* d_linear_z, uint32_t z_w, uint32_t z_h,
                                        const uint32_t* d_ray_min, const uint32_t* d_ray_max, float* d_sd_out,
                                        uint32_t sd_w, uint32_t sd_h, uint32_t band_index, uint32_t band_count,
                                        rsd_counters* counters, rsd_stream stream) {
    return rsd_sd_trace_band_ex(scene, cam, p, d_linear_z, z_w, z_h, const_cast<uint32_t*>(d_ray_min),
                                const_cast<uint32_t*>(d_ray_max), d_sd_out, sd_w, sd_h, band_index, band_count, 0u,
                                counters, stream);
}

extern "C" uint32_t rsd_sd_tile_state_count(uint32_t sd_w, uint32_t sd_h) {
    // per 8x8 tile a stamp word, then (ABI v8) per tile the two words of its 64-texel DEFAULT mask
    return 3u * ((sd_w + kTile - 1) / kTile) * ((sd_h + kTile - 1) / kTile);
}

extern "C" rsd_status rsd_sd_trace(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* p,
                                   const float* d_linear_z, uint32_t z_w, uint32_t z_h, const uint32_t* d_ray_min,
                                   const uint32_t* d_ray_max, float* d_sd_out, uint32_t sd_w, uint32_t sd_h,
                                   rsd_counters* counters, rsd_stream stream) {
    return rsd_sd_trace_band(scene, cam, p, d_linear_z, z_w, z_h, d_ray_min, d_ray_max, d_sd_out, sd_w, sd_h, 0, 1,
                             counters, stream);
}

extern "C" rsd_status rsd_gbuffer(rsd_scene* scene, const rsd_camera* cam, uint32_t width, uint32_t height,
                                  uint32_t cull_mode, float* d_linear_z, uint16_t* d_normals, rsd_stream stream) {
    if (!scene || !cam || !d_linear_z || !d_normals || width == 0 || height == 0) {
        set_error("rsd_gbuffer: null argument or empty extent");
        return RSD_ERR_INVALID_ARG;
    }
    if (cull_mode > 2) {
        set_error("rsd_gbuffer: cull_mode must be 0, 1 or 2");
        return RSD_ERR_INVALID_ARG;
    }
    hipStream_t s = (hipStream_t)stream;
    if (scene->triangle_count == 0) {
        std::vector<float> z((size_t)width * height, cam->farZ);
        RSD_HIP(hipMemcpyAsync(d_linear_z, z.data(), z.size() * 4, hipMemcpyHostToDevice, s));
        RSD_HIP(hipMemsetAsync(d_normals, 0, (size_t)width * height * 2, s));
        RSD_HIP(hipStreamSynchronize(s));
        return RSD_OK;
    }
    GBArgs a{scene->d_nodes, scene->d_tris, scene->tri_offset, *cam, (int)width, (int)height, cull_mode, d_linear_z,
             d_normals, nullptr, scene->d_alpha ? 1u : 0u, scene->alpha};
    dim3 grid((width + kTile - 1) / kTile, (height + kTile - 1) / kTile);
    hipLaunchKernelGGL(gbuffer_kernel, grid, dim3(kBlock), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "gbuffer_kernel launch");
    return RSD_OK;
}

extern "C" rsd_status rsd_gbuffer_raster(rsd_scene* scene, const rsd_camera* cam, uint32_t width, uint32_t height,
                                         uint32_t cull_mode, float* d_depth, float* d_normal_w, rsd_stream stream) {
    if (!scene || !cam || !d_depth || !d_normal_w || width == 0 || height == 0 || cull_mode > 2) {
        set_error("rsd_gbuffer_raster: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    hipStream_t s = (hipStream_t)stream;
    if (scene->triangle_count == 0) {
        std::vector<float> z((size_t)width * height, 1.0f);
        RSD_HIP(hipMemcpyAsync(d_depth, z.data(), z.size() * 4, hipMemcpyHostToDevice, s));
        RSD_HIP(hipMemsetAsync(d_normal_w, 0, (size_t)width * height * 16, s));
        RSD_HIP(hipStreamSynchronize(s));
        return RSD_OK;
    }
    GBArgs a{scene->d_nodes, scene->d_tris, scene->tri_offset, *cam, (int)width, (int)height, cull_mode, d_depth,
             nullptr, reinterpret_cast<float4*>(d_normal_w), scene->d_alpha ? 1u : 0u, scene->alpha};
    dim3 grid((width + kTile - 1) / kTile, (height + kTile - 1) / kTile);
    hipLaunchKernelGGL(gbuffer_kernel, grid, dim3(kBlock), 0, s, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "gbuffer_kernel launch");
}

namespace rsd {
void release_sd_workspaces(rsd_scene* scene) {
    for (SdWorkspace* w : scene->sd_ws) {
        (void)hipFree(w->qctl);
        (void)hipFree(w->queue);
        (void)hipFree(w->raytab.d);
        (void)hipFree(w->counters);
        delete w;
    }
    scene->sd_ws.clear();
}
}  // namespace rsd
