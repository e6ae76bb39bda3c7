// svao_rt.hip -- SVAO "AO 2" in SecondaryDepthMode::Raytraced (the ground-truth AO of
// scripts/SVAO_depth.py / SAVO_record.py): every stencilled direction is
// refined by tracing the scene instead of reading the stochastic depth map.
//
// Reference: calcAO2 DEPTH_MODE_RAYTRACING (SVAO/Common.slang:598-651), traceAORay
// (SVAORaster2.ps.slang:9-46 RayQuery, Ray.rt.slang:46-58 TraceRay) and aoAnyHit
// (Common.slang:679-718); dispatch SVAO.cpp:408-455.  Both AO kernels and both primary depth modes:
// the raster sample p of a refined direction comes from evalPrimaryVisibility, or with DualDepth from
// evalDualVisibility(data, true) (Common.slang:555-558).
//
// HBAO (Common.slang:622-628, 646-650): the ray spans [sphereStart, sphereEnd] (TMin raised to the
// depth buffer + epsilon on screen) WITHOUT RAY_FLAG_FORCE_NON_OPAQUE, so opaque triangles commit as
// closest hits directly and alpha-masked ones pass aoAnyHit (alpha test, then ACCEPT whatever the face,
// Common.slang:695-697, 715-717): tFirst = the nearest non-culled hit that passes the alpha test (0 when
// the ray misses, SVAORaster2.ps.slang:42-45 / Ray.rt.slang:37-43), and the sample point
// mul(viewMat, posW + dir tFirst) goes through addSample (max of saturate(HBAOKernel / pdf)).  The
// traversal below finds that hit with tCRS = -inf: every accepted hit then terminates, so A = tFirst.
//
// Any-hit order.  As for the SD trace, the hit stream is canonical: ascending t, each
// triangle once.  aoAnyHit over that stream (accepted = front face, or double-sided, or
// alpha-masked; culled triangles and, with USE_ALPHA_TEST, alpha-masked triangles failing the
// alpha test at LOD 0 never arrive):
//     t <= tSphereStart:  halo = max(halo, t); end the query if t >= tConstRadiusStart
//     t >  tSphereStart:  inside = min(inside, t); commit (TMax = t) -- nothing nearer follows
// The query therefore ends at the first accepted hit A with term(A) = (A > tSphereStart ||
// A >= tConstRadiusStart), a predicate monotone in t, and every accepted hit before A is
// a halo update.  So the result is:  halo = max(halo0, B, A if A <= tSphereStart),
// inside = A if A > tSphereStart else inside0, with A the nearest terminating and B the
// farthest non-terminating accepted hit in [TMin, TMax] -- which one traversal with the
// upper bound min(TMax, A) collects in any order.  (The RayQuery's "t < halo: skip" test
// never fires in ascending order: TMin >= halo0.)  The CPU oracle replays the ascending
// stream literally (oracle/rsd_oracle.c ocpu_svao_pass2_rt_band).
#include <cfloat>

#include "bvh_traverse.h"
#include "rsd_device.h"
#include "rsd_internal.h"
#include "svao_math.h"

namespace rsd {

struct RtArgs {
    SvaoArgs s;
    const float4* nodes;  // BVH base (wide nodes, then triangle records)
    uint32_t triOff;
    uint32_t cull;
    uint32_t rayPipeline;  // 1: ray-pipeline dispatch extent (SVAO.cpp:429-430), 0: compute (:452-453)
    float invView[9];      // float3x3(inverse(viewMat)), row-major
    uint32_t alphaTest;    // USE_ALPHA_TEST and the scene has alpha data
    AlphaData alpha;
};

// The aoAnyHit stream of one AO ray reduced to (A, B), see the file header.
__device__ __forceinline__ void trace_ao(const float4* __restrict__ bvh, uint32_t triOff, const RayCtx& r, float tmin,
                                         float tmax, uint32_t cull, float tCRS, float tSS, float& A, float& B,
                                         uint32_t* __restrict__ ldsItem, float* __restrict__ ldsT, bool alphaOn,
                                         const AlphaData& alpha, bool anyFace) {
    A = INFINITY;
    B = -INFINITY;
    uint32_t spillItem[kStackTotal - kLdsStack];
    float spillT[kStackTotal - kLdsStack];
    int sp = 0;
    uint32_t item = 0;  // root node
    while (true) {
        const float4* p = bvh + (item & kOffMask);
        float4 q[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) q[j] = p[j];
        uint32_t next = kNoItem;
        const float thi = fminf(tmax, A);
        if (item & kLeafBit) {
            const uint32_t cnt = ((item >> 29) & 3u) + 1u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if ((uint32_t)j >= cnt) continue;
                float t, bu, bv, det;
                if (!intersect_tri(r, q[3 * j], q[3 * j + 1], q[3 * j + 2], t, bu, bv, det)) continue;
                if (!(t >= tmin && t <= thi)) continue;
                const uint32_t flags = __float_as_uint(q[3 * j + 1].w);
                if (culled(det, flags, cull)) continue;
                // aoAnyHit: frontFace || isDoubleSided || isAlphaTested (Common.slang:695-697); HBAO's opaque
                // triangles never reach it (closest hit without RAY_FLAG_FORCE_NON_OPAQUE)
                const bool front = (det > 0.0f) != ((flags & RSD_TRI_FRONT_CW) != 0u);
                if (!anyFace && !(front || (flags & (RSD_TRI_DOUBLE_SIDED | RSD_TRI_ALPHA_MASK)))) continue;
                // USE_ALPHA_TEST: alpha test at LOD 0 (Common.slang:683-691) -> AO_HIT_IGNORE
                if (alphaOn && (flags & RSD_TRI_ALPHA_MASK) &&
                    alpha_test_fails(alpha, __float_as_uint(q[3 * j].w), q[3 * j], q[3 * j + 1], q[3 * j + 2], bu, bv,
                                     false, t, r.d))
                    continue;
                if (t > tSS || t >= tCRS) A = fminf(A, t);
                else B = fmaxf(B, t);
            }
        } else {
            const uint4 rf = make_uint4(__float_as_uint(q[6].x), __float_as_uint(q[6].y), __float_as_uint(q[6].z),
                                        __float_as_uint(q[6].w));
            const uint4 ct = make_uint4(__float_as_uint(q[7].x), __float_as_uint(q[7].y), __float_as_uint(q[7].z),
                                        __float_as_uint(q[7].w));
            float k0, k1, k2, k3;
            bool h0 = rf.x != kNoItem && box_hit(r, q[0].x, q[1].x, q[2].x, q[3].x, q[4].x, q[5].x, tmin, thi, k0);
            bool h1 = rf.y != kNoItem && box_hit(r, q[0].y, q[1].y, q[2].y, q[3].y, q[4].y, q[5].y, tmin, thi, k1);
            bool h2 = rf.z != kNoItem && box_hit(r, q[0].z, q[1].z, q[2].z, q[3].z, q[4].z, q[5].z, tmin, thi, k2);
            bool h3 = rf.w != kNoItem && box_hit(r, q[0].w, q[1].w, q[2].w, q[3].w, q[4].w, q[5].w, tmin, thi, k3);
            auto mkitem = [&](uint32_t ref, uint32_t cnt) {
                return cnt ? (kLeafBit | ((cnt - 1u) << 29) | (triOff + 3u * ref)) : 8u * ref;
            };
            uint32_t c0 = h0 ? mkitem(rf.x, ct.x) : kNoItem, c1 = h1 ? mkitem(rf.y, ct.y) : kNoItem;
            uint32_t c2 = h2 ? mkitem(rf.z, ct.z) : kNoItem, c3 = h3 ? mkitem(rf.w, ct.w) : kNoItem;
            k0 = h0 ? k0 : INFINITY;
            k1 = h1 ? k1 : INFINITY;
            k2 = h2 ? k2 : INFINITY;
            k3 = h3 ? k3 : INFINITY;
            cswap(k0, c0, k1, c1);
            cswap(k2, c2, k3, c3);
            cswap(k0, c0, k2, c2);
            cswap(k1, c1, k3, c3);
            cswap(k1, c1, k2, c2);
#define RSD_PUSH(c, k)                                                                  \
    if ((c) != kNoItem) {                                                               \
        if (sp < kLdsStack) { ldsItem[sp * 64] = (c); ldsT[sp * 64] = (k); }            \
        else { spillItem[sp - kLdsStack] = (c); spillT[sp - kLdsStack] = (k); }         \
        ++sp;                                                                           \
    }
            RSD_PUSH(c3, k3)
            RSD_PUSH(c2, k2)
            RSD_PUSH(c1, k1)
#undef RSD_PUSH
            next = c0;
        }
        if (next == kNoItem) {
            const float hi = fminf(tmax, A);
            while (sp > 0) {
                --sp;
                const uint32_t it = sp < kLdsStack ? ldsItem[sp * 64] : spillItem[sp - kLdsStack];
                const float tt = sp < kLdsStack ? ldsT[sp * 64] : spillT[sp - kLdsStack];
                if (tt <= hi) { next = it; break; }
            }
            if (next == kNoItem) break;
        }
        item = next;
    }
}

// One refined direction of a pixel: primary visibility p (subtracted) and the traced
// visibility r (added), Common.slang:598-651.
__device__ __forceinline__ void rt_dir(const RtArgs& ra, const Basic& b, float u, float v, int i, float& p, float& rOut,
                                       uint32_t* __restrict__ ldsItem, float* __restrict__ ldsT) {
    const SvaoArgs& a = ra.s;
    const rsd_vao_data& d = a.d;
    const f3 camPos = mk(a.cam.posW[0], a.cam.posW[1], a.cam.posW[2]);
    const float* M = ra.invView;
    Sample s;
    bool ssrAbove;
    sample_init(a, u, v, b, i, s, ssrAbove);
    if (a.dualDepth) eval_dual(a, b, s, ssrAbove, true);  // Common.slang:555-558 (force init)
    else eval_primary(a, b, s);
    p = s.visibility;
    // getSnappedUV (Common.slang:116-125), not clamped: rays may leave the screen
    const float su = (floorf(s.su * d.resolution[0]) + 0.5f) / d.resolution[0];
    const float sv = (floorf(s.sv * d.resolution[1]) + 0.5f) / d.resolution[1];
    const f3 dv = normalize(uv_to_view(a, su, sv, 1.0f));
    const f3 dw = mk(M[0] * dv.x + M[1] * dv.y + M[2] * dv.z, M[3] * dv.x + M[4] * dv.y + M[5] * dv.z,
                     M[6] * dv.x + M[7] * dv.y + M[8] * dv.z);
    const float initLen = length(s.ip);
    const float pl = b.posVLength;
    if (a.k.hbao) {  // Common.slang:622-628, 637-638, 646-650
        float TMin = (pl - s.sphereStart) * initLen / pl;
        const float TMax = (pl - s.sphereEnd) * initLen / pl;
        if (!s.isInScreen) { s.visibility = 0.0f; s.objectSpaceZ = 3.402823466e+38f; }  // resetSample (HBAO)
        const float eps = b.radius * 0.01f;
        if (s.isInScreen) TMin = hmax(TMin, (pl - s.objectSpaceZ) * initLen / pl + eps);
        float tFirst = 0.0f;
        if (TMin <= TMax) {
            RayCtx r;
            ray_setup(r, camPos, dw);
            float A, B;
            trace_ao(ra.nodes, ra.triOff, r, TMin, TMax, ra.cull, -INFINITY, INFINITY, A, B, ldsItem, ldsT,
                     ra.alphaTest != 0u, ra.alpha, true);
            if (A != INFINITY) tFirst = A;
        }
        // samplePosW = ray.Origin + ray.Direction tFirst; samplePosV = mul(viewMat, float4(samplePosW, 1))
        const f3 pw = mk(camPos.x + dw.x * tFirst, camPos.y + dw.y * tFirst, camPos.z + dw.z * tFirst);
        const float* V = a.cam.viewMat;
        const f3 pv = mk(((V[0] * pw.x + V[1] * pw.y) + V[2] * pw.z) + V[3],
                         ((V[4] * pw.x + V[5] * pw.y) + V[6] * pw.z) + V[7],
                         ((V[8] * pw.x + V[9] * pw.y) + V[10] * pw.z) + V[11]);
        add_sample(a, b, s, pv, false);
        rOut = s.visibility;
        return;
    }
    const float tHalo0 = (pl - s.sphereStart - b.radius - d.thickness * b.radius) * initLen / pl;
    const float tInside0 = (pl - s.sphereEnd) * initLen / pl;
    const float tCRS = (pl - b.radius - d.thickness * b.radius) * initLen / pl;
    const float tSS = (pl - s.sphereStart) * initLen / pl;
    float TMin = hmax(tHalo0, 0.0f);
    const float TMax = tInside0;
    if (!s.isInScreen) { s.visibility = 1.0f; s.objectSpaceZ = 3.402823466e+38f; }  // resetSample
    const float eps = b.radius * 0.01f;
    if (s.isInScreen) TMin = hmax(TMin, (pl - s.objectSpaceZ) * initLen / pl + eps);
    float halo = tHalo0, inside = tInside0;
    if (TMin <= TMax) {
        RayCtx r;
        ray_setup(r, camPos, dw);
        float A, B;
        trace_ao(ra.nodes, ra.triOff, r, TMin, TMax, ra.cull, tCRS, tSS, A, B, ldsItem, ldsT, ra.alphaTest != 0u,
                 ra.alpha, false);
        if (B != -INFINITY) halo = hmax(halo, B);
        if (A != INFINITY) {
            if (A <= tSS) halo = hmax(halo, A);
            else inside = hmin(inside, A);
        }
    }
    const float sphereVis = calc_visibility(d, pl - inside * pl / initLen, s.sphereStart, s.sphereEnd, s.pdf,
                                            b.radius);
    const float haloVis = calc_halo_visibility(d, pl - halo * pl / initLen, s.sphereStart, s.sphereEnd, s.pdf,
                                               b.radius);
    rOut = hmin(s.visibility, hmin(sphereVis, haloVis));
}

// SVAORaster2.ps.slang:48-65 / Ray.rt.slang:60-75 -> calcAO2 (Common.slang:523-663), Raytraced
// branch.  An 8 x 8 pixel tile per 64-lane workgroup: the tile's (pixel, direction) pairs of
// non-zero stencil are listed in LDS (grouped per pixel, direction order) and every lane
// traces one AO ray at a time; each pixel's vis = (vis - p_i) + r_i is then applied in
// direction order (the per-pixel loop's exact float sequence).
__global__ void __launch_bounds__(64) svao_pass2_rt_kernel(RtArgs ra) {
    __shared__ uint32_t sItem[kLdsStack * 64];
    __shared__ float sT[kLdsStack * 64];
    __shared__ uint32_t sPix[64];                    // slot: local pixel
    __shared__ uint16_t sPair[kMaxDirections * 64];  // slot << 5 | direction
    __shared__ uint16_t sFirst[64];
    __shared__ float sAcc[64], sAccD[64], sP[64], sR[64];  // bright / dark (DUAL_AO) sums
    __shared__ uint32_t sNPix, sNPair;
    const SvaoArgs& a = ra.s;
    const rsd_vao_data& d = a.d;
    const uint32_t lane = threadIdx.x;
    // band: 8-row tiles of the 32-row groups g (counted from the first visible row) with
    // g % bandCount == bandIndex
    const uint32_t by = blockIdx.y;
    const uint32_t tileRow = ((by / 4u) * a.bandCount + a.bandIndex) * 4u + by % 4u;
    const uint32_t x0 = a.guard + blockIdx.x * 8u, y0 = a.guard + tileRow * 8u;
    const uint32_t xEnd = ra.rayPipeline ? (uint32_t)a.W : (uint32_t)a.W - a.guard;
    const uint32_t yEnd = ra.rayPipeline ? (uint32_t)a.H : (uint32_t)a.H - a.guard;
    if (lane == 0) { sNPix = 0u; sNPair = 0u; }
    __syncthreads();
    {
        const uint32_t px = x0 + lane % 8u, py = y0 + lane / 8u;
        const uint32_t m = (px < xEnd && py < yEnd) ? stencil_load(a, (size_t)py * a.W + px) : 0u;
        if (m) {
            const uint32_t slot = atomicAdd(&sNPix, 1u), base = atomicAdd(&sNPair, (uint32_t)__popc(m));
            sPix[slot] = lane;
            sFirst[slot] = (uint16_t)base;
            sAcc[slot] = 0.0f;
            sAccD[slot] = 0.0f;
            uint32_t j = base;
            for (int i = 0; i < (int)a.k.nd; ++i)
                if (m & (1u << i)) sPair[j++] = (uint16_t)(slot << 5 | i);
        }
    }
    __syncthreads();
    const uint32_t nPix = sNPix, nPair = sNPair;
    for (uint32_t c = 0; c < nPair; c += 64u) {
        const uint32_t k = c + lane;
        uint32_t slot = 0;
        if (k < nPair) {
            const uint32_t e = sPair[k];
            slot = e >> 5;
            const uint32_t lp = sPix[slot] & 63u;
            const float u = ((float)(x0 + lp % 8u) + 0.5f) * d.invResolution[0];
            const float v = ((float)(y0 + lp / 8u) + 0.5f) * d.invResolution[1];
            Basic b;
            basic_init(a, u, v, b);
            float p, r;
            rt_dir(ra, b, u, v, (int)(e & 31u), p, r, &sItem[lane], &sT[lane]);
            sP[lane] = p;
            sR[lane] = r;
        }
        __syncthreads();
        if (k < nPair && k == max((uint32_t)sFirst[slot], c)) {
            float acc = sAcc[slot], accD = sAccD[slot];
            for (uint32_t j = k; j < nPair && j < c + 64u && (uint32_t)(sPair[j] >> 5) == slot; ++j) {
                acc = (acc - sP[j - c]) + sR[j - c];
                accD = accD + sR[j - c];
            }
            sAcc[slot] = acc;
            sAccD[slot] = accD;
        }
        __syncthreads();
    }
    if (lane < nPix) {
        const uint32_t lp = sPix[lane] & 63u;
        const size_t o = (size_t)(y0 + lp / 8u) * a.W + (x0 + lp % 8u);
        const uchar2 prev = a.dual ? reinterpret_cast<const uchar2*>(a.ao)[o] : make_uchar2(a.ao[o], 0);
        ao_finish(a, o, sAcc[lane], sAccD[lane], prev);
    }
}

}  // namespace rsd

using namespace rsd;

extern "C" rsd_status rsd_svao_pass2_raytraced_band(rsd_scene* scene, const rsd_camera* cam, const rsd_vao_data* vao,
                                                    const rsd_svao_params* p, const float* d_depth,
                                                    const uint16_t* d_normals, uint32_t W, uint32_t H,
                                                    const uint8_t* d_stencil, uint8_t* d_ao, uint32_t cull_mode,
                                                    uint32_t ray_pipeline, uint32_t alpha_test, uint32_t band_index,
                                                    uint32_t band_count, rsd_stream stream) {
    if (band_count == 0 || band_index >= band_count) {
        set_error("rsd_svao_pass2_raytraced_band: band_index must be < band_count");
        return RSD_ERR_INVALID_ARG;
    }
    rsd_status st = check_common(cam, vao, p, d_depth, d_normals, W, H, "rsd_svao_pass2_raytraced");
    if (st != RSD_OK) return st;
    if (!scene || !d_stencil || !d_ao || cull_mode > 2) {
        set_error("rsd_svao_pass2_raytraced: null argument or bad cull mode");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->ao_kernel > RSD_AO_KERNEL_HBAO || p->primary_depth_mode > 1u || (p->primary_depth_mode == 1u && !p->d_depth2)) {
        set_error("rsd_svao_pass2_raytraced: ao_kernel must be VAO or HBAO, primary_depth_mode 0 or 1 (DualDepth needs "
                  "d_depth2)");
        return RSD_ERR_INVALID_ARG;
    }
    RtArgs ra{};
    SvaoArgs& a = ra.s;
    a.cam = *cam;
    a.d = *vao;
    fill_consts(a.k, a.d, p->num_directions, p->ao_kernel);
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
    a.guard = p->guard_band;
    a.secondary = 3u;
    a.dual = p->dual_ao ? 1u : 0u;
    a.bandIndex = band_index;
    a.bandCount = band_count;
    a.dualDepth = p->primary_depth_mode == 1u ? 1u : 0u;
    a.depth2 = p->d_depth2;
    ra.nodes = scene->d_nodes;
    ra.triOff = scene->tri_offset;
    ra.cull = cull_mode;
    ra.rayPipeline = ray_pipeline ? 1u : 0u;
    ra.alphaTest = alpha_test && scene->d_alpha ? 1u : 0u;
    ra.alpha = scene->alpha;
    // float3x3(inverse(viewMat)): the view matrix is a rotation + translation, so the rotation
    // part of its inverse is the transpose (exact; Falcor's general inverse rounds it)
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) ra.invView[r * 3 + c] = cam->viewMat[c * 4 + r];
    const uint32_t xEnd = ra.rayPipeline ? W : W - p->guard_band, yEnd = ra.rayPipeline ? H : H - p->guard_band;
    const uint32_t tilesX = (xEnd - p->guard_band + 7u) / 8u;
    const uint32_t groups = (yEnd - p->guard_band + 31u) / 32u;
    const uint32_t bandGroups = groups > band_index ? (groups - band_index + band_count - 1) / band_count : 0u;
    if (bandGroups == 0 || tilesX == 0) return RSD_OK;
    hipLaunchKernelGGL(svao_pass2_rt_kernel, dim3(tilesX, 4 * bandGroups), dim3(64), 0, (hipStream_t)stream, ra);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "svao_pass2_rt_kernel launch");
}

extern "C" rsd_status rsd_svao_pass2_raytraced(rsd_scene* scene, const rsd_camera* cam, const rsd_vao_data* vao,
                                               const rsd_svao_params* p, const float* d_depth,
                                               const uint16_t* d_normals, uint32_t W, uint32_t H,
                                               const uint8_t* d_stencil, uint8_t* d_ao, uint32_t cull_mode,
                                               uint32_t ray_pipeline, uint32_t alpha_test, rsd_stream stream) {
    return rsd_svao_pass2_raytraced_band(scene, cam, vao, p, d_depth, d_normals, W, H, d_stencil, d_ao, cull_mode,
                                         ray_pipeline, alpha_test, 0, 1, stream);
}
