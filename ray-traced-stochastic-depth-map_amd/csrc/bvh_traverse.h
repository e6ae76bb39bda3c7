// bvh_traverse.h -- BVH traversal primitives shared by librsd's ray kernels (the SD trace,
// the primary-visibility G-buffer and the Raytraced secondary mode of SVAO pass 2).
//
// Reference: IntersectionHelpers.slang:109-180 (watertight triangle test), the DXR triangle
// culling of the instance flags (Scene.cpp:3446-3452), Camera.slang:46-90 (pinhole rays).
// BVH layout: csrc/bvh_build.h.
#pragma once
#include "rsd_device.h"
#include "../../include/rsd.h"
#include "alpha_test.h"

namespace rsd {

constexpr int kTile = 8;               // 8x8 texels per wave
constexpr uint32_t kQueueParts = 32;   // live-ray queue partitions (counter sharding)
constexpr int kBlock = kTile * kTile;  // 64 threads
constexpr int kLdsStack = 16;
constexpr int kStackTotal = 96;        // 4-wide: <= 3 pushes per level, <= 30 levels

struct RayCtx {
    f3 o, d;
    int kx, ky, kz;
    float Sx, Sy, Sz;
    f3 invd, oinvd;
};

__device__ __forceinline__ float comp(f3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

__device__ __forceinline__ void ray_setup(RayCtx& r, f3 o, f3 d) {
    r.o = o;
    r.d = d;
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int axis = 0;
    if (ay > ax && ay > az) axis = 1;
    if (az > ax && az > ay) axis = 2;
    r.kz = axis;
    r.kx = axis == 2 ? 0 : axis + 1;
    r.ky = r.kx == 2 ? 0 : r.kx + 1;
    if (comp(d, r.kz) < 0.0f) { int s = r.kx; r.kx = r.ky; r.ky = s; }
    float dz = comp(d, r.kz);
    r.Sx = comp(d, r.kx) / dz;
    r.Sy = comp(d, r.ky) / dz;
    r.Sz = 1.0f / dz;
    // box test reciprocal: avoid 0 * inf = NaN for axis-parallel rays
    auto safe = [](float v) { return fabsf(v) > 1e-20f ? v : copysignf(1e-20f, v); };
    r.invd = mk(1.0f / safe(d.x), 1.0f / safe(d.y), 1.0f / safe(d.z));
    r.oinvd = mk(o.x * r.invd.x, o.y * r.invd.y, o.z * r.invd.z);
}

// IntersectionHelpers.slang:109-180 -- bit-identical to the oracle (no contraction).
__device__ __forceinline__ bool intersect_tri(const RayCtx& r, float4 a, float4 b, float4 c, float& t, float& bu,
                                              float& bv, float& detOut) {
    f3 A = mk(a.x - r.o.x, a.y - r.o.y, a.z - r.o.z);
    f3 B = mk(b.x - r.o.x, b.y - r.o.y, b.z - r.o.z);
    f3 C = mk(c.x - r.o.x, c.y - r.o.y, c.z - r.o.z);
    const float Akz = comp(A, r.kz), Bkz = comp(B, r.kz), Ckz = comp(C, r.kz);
    const float Ax = comp(A, r.kx) - r.Sx * Akz;
    const float Ay = comp(A, r.ky) - r.Sy * Akz;
    const float Bx = comp(B, r.kx) - r.Sx * Bkz;
    const float By = comp(B, r.ky) - r.Sy * Bkz;
    const float Cx = comp(C, r.kx) - r.Sx * Ckz;
    const float Cy = comp(C, r.ky) - r.Sy * Ckz;
    float U = Cx * By - Cy * Bx;
    float V = Ax * Cy - Ay * Cx;
    float W = Bx * Ay - By * Ax;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        double CxBy = (double)Cx * (double)By, CyBx = (double)Cy * (double)Bx;
        U = (float)(CxBy - CyBx);
        double AxCy = (double)Ax * (double)Cy, AyCx = (double)Ay * (double)Cx;
        V = (float)(AxCy - AyCx);
        double BxAy = (double)Bx * (double)Ay, ByAx = (double)By * (double)Ax;
        W = (float)(BxAy - ByAx);
    }
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return false;
    const float det = U + V + W;
    if (det == 0.0f) return false;
    const float Az = r.Sz * Akz, Bz = r.Sz * Bkz, Cz = r.Sz * Ckz;
    const float T = U * Az + V * Bz + W * Cz;
    const float rcpDet = 1.0f / det;
    t = T * rcpDet;
    bu = V * rcpDet;
    bv = W * rcpDet;
    detOut = det;
    return true;
}

// det > 0 <=> counter-clockwise seen from the ray origin = Falcor front face (unless
// the mesh is frontFaceCW); double-sided disables culling (Scene.cpp:3446-3452).
__device__ __forceinline__ bool culled(float det, uint32_t flags, uint32_t cull) {
    if (cull == 0u || (flags & 1u)) return false;
    const bool front = (det > 0.0f) != ((flags & 2u) != 0u);
    return cull == 1u ? !front : front;
}

// Conservative slab test: entry/exit widened by a relative 1e-5 so that a node is skipped
// only if it cannot hold a reported hit in [tlo, thi].
__device__ __forceinline__ bool box_hit(const RayCtx& r, float lox, float hix, float loy, float hiy, float loz,
                                        float hiz, float tlo, float thi, float& tnear) {
    float x0 = fmaf(lox, r.invd.x, -r.oinvd.x), x1 = fmaf(hix, r.invd.x, -r.oinvd.x);
    float y0 = fmaf(loy, r.invd.y, -r.oinvd.y), y1 = fmaf(hiy, r.invd.y, -r.oinvd.y);
    float z0 = fmaf(loz, r.invd.z, -r.oinvd.z), z1 = fmaf(hiz, r.invd.z, -r.oinvd.z);
    float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    float m = 1e-5f * (fabsf(tn) + fabsf(tf));
    tn -= m;
    tf += m;
    tnear = tn;
    return fmaxf(tn, tlo) <= fminf(tf, thi);
}

__device__ __forceinline__ bool key_less(float ta, uint32_t pa, float tb, uint32_t pb) {
    return ta < tb || (ta == tb && pa < pb);
}

template <int K>
struct KList {
    float t[K];
    uint32_t p[K];
    uint32_t l[K];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int j = 0; j < K; ++j) { t[j] = INFINITY; p[j] = 0xffffffffu; l[j] = 0u; }
    }
    // insert keeping ascending (t, prim) order; the largest key falls off the end
    __device__ __forceinline__ void insert(float nt, uint32_t np, uint32_t nl) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool lt = key_less(nt, np, t[j], p[j]);
            const float tt = t[j];
            const uint32_t pp = p[j], ll = l[j];
            t[j] = lt ? nt : tt;
            p[j] = lt ? np : pp;
            l[j] = lt ? nl : ll;
            nt = lt ? tt : nt;
            np = lt ? pp : np;
            nl = lt ? ll : nl;
        }
    }
};

struct TraceStats {
    uint32_t nodes, tris, leaves;
};

__device__ __forceinline__ void cswap(float& ta, uint32_t& ra, float& tb, uint32_t& rb) {
    const bool s = tb < ta;
    const float t = ta;
    const uint32_t r = ra;
    ta = s ? tb : ta;
    ra = s ? rb : ra;
    tb = s ? t : tb;
    rb = s ? r : rb;
}

// Work items of the traversal: one 32-bit word.  bit31 = leaf, bits 29-30 = leaf triangle
// count - 1, bits 0-28 = offset in 16-B units from the BVH base (wide nodes and triangle
// records share one allocation).  Every step fetches 12 x 16 B at the item's offset -- a
// 128-B node (+ 64 B ignored) or a whole leaf of <= 4 48-B triangle records -- with the
// same instructions, so a wave whose lanes mix node steps and leaf steps still pays ONE
// memory latency per step.  The SD trace is latency-bound (few active rays, long tails).
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kOffMask = 0x1fffffffu;
constexpr uint32_t kNoItem = 0xffffffffu;

// Collects the K smallest keys (t, prim) with tmin <= t <= tmax, key > (lbT, lbP) when
// useLB, culling applied.  Returns the number of keys found (<= K).  Children are visited
// nearest-first; the others go to a per-lane LDS stack with their entry distance, and a
// popped item is dropped without a fetch once the k-th key is nearer than its box.
// alphaOn: alpha-masked triangles that fail the alpha test at LOD 0 are ignored
// (closest hit with IgnoreHit in the any-hit shader, GBufferRaster useAlphaTest).
template <int K>
__device__ __forceinline__ int trace_knearest(const float4* __restrict__ bvh, uint32_t triOff, const RayCtx& r,
                                              float tmin, float tmax, uint32_t cull, bool useLB, float lbT,
                                              uint32_t lbP, KList<K>& kl, uint32_t* __restrict__ ldsItem,
                                              float* __restrict__ ldsT, TraceStats& st, bool alphaOn,
                                              const AlphaData& alpha) {
    kl.clear();
    uint32_t spillItem[kStackTotal - kLdsStack];
    float spillT[kStackTotal - kLdsStack];
    int sp = 0;
    int found = 0;
    uint32_t item = 0;  // root node
    const float tlo = useLB ? fmaxf(tmin, lbT) : tmin;
    while (true) {
        const float4* p = bvh + (item & kOffMask);
        float4 q[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) q[j] = p[j];
        uint32_t next = kNoItem;
        if (item & kLeafBit) {
            const uint32_t cnt = ((item >> 29) & 3u) + 1u;
            const uint32_t first = ((item & kOffMask) - triOff) / 3u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if ((uint32_t)j >= cnt) continue;
                st.tris++;
                float t, bu, bv, det;
                if (!intersect_tri(r, q[3 * j], q[3 * j + 1], q[3 * j + 2], t, bu, bv, det)) continue;
                if (!(t >= tmin && t <= tmax)) continue;
                const uint32_t prim = __float_as_uint(q[3 * j].w);
                if (culled(det, __float_as_uint(q[3 * j + 1].w), cull)) continue;
                if (useLB && !key_less(lbT, lbP, t, prim)) continue;
                if (!key_less(t, prim, kl.t[K - 1], kl.p[K - 1])) continue;
                if (alphaOn && (__float_as_uint(q[3 * j + 1].w) & 4u) &&
                    alpha_test_fails(alpha, prim, q[3 * j], q[3 * j + 1], q[3 * j + 2], bu, bv, false, t, r.d))
                    continue;
                kl.insert(t, prim, first + (uint32_t)j);
                found = found < K ? found + 1 : K;
            }
        } else {
            st.nodes++;
            const float thi = fminf(tmax, kl.t[K - 1]);
            const uint4 rf = make_uint4(__float_as_uint(q[6].x), __float_as_uint(q[6].y), __float_as_uint(q[6].z),
                                        __float_as_uint(q[6].w));
            const uint4 ct = make_uint4(__float_as_uint(q[7].x), __float_as_uint(q[7].y), __float_as_uint(q[7].z),
                                        __float_as_uint(q[7].w));
            float k0, k1, k2, k3;
            bool h0 = rf.x != kNoItem && box_hit(r, q[0].x, q[1].x, q[2].x, q[3].x, q[4].x, q[5].x, tlo, thi, k0);
            bool h1 = rf.y != kNoItem && box_hit(r, q[0].y, q[1].y, q[2].y, q[3].y, q[4].y, q[5].y, tlo, thi, k1);
            bool h2 = rf.z != kNoItem && box_hit(r, q[0].z, q[1].z, q[2].z, q[3].z, q[4].z, q[5].z, tlo, thi, k2);
            bool h3 = rf.w != kNoItem && box_hit(r, q[0].w, q[1].w, q[2].w, q[3].w, q[4].w, q[5].w, tlo, thi, k3);
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
#define RSD_PUSH(c, k)                                                 \
    if ((c) != kNoItem) {                                              \
        if (sp < kLdsStack) { ldsItem[sp * kBlock] = (c); ldsT[sp * kBlock] = (k); } \
        else { spillItem[sp - kLdsStack] = (c); spillT[sp - kLdsStack] = (k); }      \
        ++sp;                                                          \
    }
            RSD_PUSH(c3, k3)
            RSD_PUSH(c2, k2)
            RSD_PUSH(c1, k1)
#undef RSD_PUSH
            next = c0;
        }
        if (next == kNoItem) {
            const float thi = fminf(tmax, kl.t[K - 1]);
            while (sp > 0) {
                --sp;
                const uint32_t it = sp < kLdsStack ? ldsItem[sp * kBlock] : spillItem[sp - kLdsStack];
                const float tt = sp < kLdsStack ? ldsT[sp * kBlock] : spillT[sp - kLdsStack];
                if (tt <= thi) { next = it; break; }
            }
            if (next == kNoItem) break;
        }
        item = next;
    }
    return found;
}


__device__ __forceinline__ f3 cam_dir(const rsd_camera& c, float px, float py) {
    const float ndcx = 2.0f * px + -1.0f;
    const float ndcy = -2.0f * py + 1.0f;
    return mk(ndcx * c.U[0] + ndcy * c.V[0] + c.W[0], ndcx * c.U[1] + ndcy * c.V[1] + c.W[1],
              ndcx * c.U[2] + ndcy * c.V[2] + c.W[2]);
}

}  // namespace rsd
