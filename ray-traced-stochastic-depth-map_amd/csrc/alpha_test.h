// alpha_test.h -- the alpha test of alpha-masked materials on the device.
//
// Reference: MaterialFactory::alphaTest (Scene/Material/MaterialFactory.slang:124-151),
// StandardMaterial::evalOpacity (Rendering/Materials/StandardMaterial.slang:128-132, the
// base-colour alpha), evalBasicAlphaTest (Scene/Material/AlphaTest.slang:81-84: alpha <
// threshold fails), Scene::computeVertexData (Scene/Scene.slang:444-480: texC and face normal
// interpolation), ray-cone LOD (StochasticDepthMapRT.rt.slang:31-37, TexLODHelpers.slang:97-129,
// ExplicitRayConesLodTextureSampler TextureSampler.slang:81-97; coneTexLODValue is 0 for
// getVertexData).  Sampling (librsd's definition, DESIGN.md "Alpha test"): trilinear over the
// host-built 2x2 box mip chain, wrap addressing, 8 sub-texel bits and 8 LOD-fraction bits;
// log2 evaluated in double and rounded once.  The CPU oracle restates exactly this.
#pragma once
#include "rsd_device.h"
#include "rsd_internal.h"

namespace rsd {

__device__ __forceinline__ float alpha_texel(const uint8_t* __restrict__ lvl, int w, int h, int x, int y) {
    x %= w;
    y %= h;
    x += x < 0 ? w : 0;
    y += y < 0 ? h : 0;
    return (float)lvl[(size_t)y * w + x] / 255.0f;
}

// bilinear, wrap, 8 sub-texel bits (the linearZ sampler convention of rsd_device.h)
__device__ __forceinline__ float alpha_bilinear(const uint8_t* __restrict__ lvl, int w, int h, float u, float v) {
    const float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    float qx = floorf((x - fx0) * 256.0f + 0.5f), qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) { ix += 1; qx = 0.0f; }
    if (qy >= 256.0f) { iy += 1; qy = 0.0f; }
    const float wx = qx * (1.0f / 256.0f), wy = qy * (1.0f / 256.0f);
    const float t00 = alpha_texel(lvl, w, h, ix, iy), t10 = alpha_texel(lvl, w, h, ix + 1, iy);
    const float t01 = alpha_texel(lvl, w, h, ix, iy + 1), t11 = alpha_texel(lvl, w, h, ix + 1, iy + 1);
    const float r0 = t00 * (1.0f - wx) + t10 * wx;
    const float r1 = t01 * (1.0f - wx) + t11 * wx;
    return r0 * (1.0f - wy) + r1 * wy;
}

// SampleLevel(uv, level): trilinear between the two nearest mips, LOD clamped to the chain
__device__ __forceinline__ float alpha_sample(const AlphaData& A, uint32_t texIndex, float u, float v, float level) {
    const uint4 tx = A.textures[texIndex];
    const int mips = (int)tx.z;
    float lod = level != level ? 0.0f : fminf(fmaxf(level, 0.0f), (float)(mips - 1));
    int l0 = (int)floorf(lod);
    float qf = floorf((lod - (float)l0) * 256.0f + 0.5f);
    if (qf >= 256.0f) { l0 += 1; qf = 0.0f; }
    const float f = qf * (1.0f / 256.0f);
    size_t off = tx.w;
    int w = (int)tx.x, h = (int)tx.y;
    for (int m = 0; m < l0; ++m) {
        off += (size_t)w * h;
        w = max(1, w >> 1);
        h = max(1, h >> 1);
    }
    const float s0 = alpha_bilinear(A.texels + off, w, h, u, v);
    if (qf == 0.0f || l0 + 1 >= mips) return s0;
    const float s1 = alpha_bilinear(A.texels + off + (size_t)w * h, max(1, w >> 1), max(1, h >> 1), u, v);
    return s0 * (1.0f - f) + s1 * f;
}

// MaterialFactory::alphaTest: true = the hit is discarded.  (bu, bv) = DXR barycentrics;
// lodRayCone: the ray-cone LOD with the hit distance t and direction d, else LOD 0.
__device__ __forceinline__ bool alpha_test_fails(const AlphaData& A, uint32_t prim, float4 v0, float4 v1, float4 v2,
                                                 float bu, float bv, bool lodRayCone, float t, f3 d) {
    const uint32_t mat = A.triMat[prim];
    const float4 m = A.materials[mat];
    const uint32_t tex = __float_as_uint(m.z);
    float alpha = m.y;
    if (tex != 0xffffffffu) {
        const float* uv = A.triUV + 6 * (size_t)prim;
        const float b0 = 1.0f - bu - bv;  // TriangleHit::getBarycentricWeights
        float tu = uv[0] * b0, tv = uv[1] * b0;
        tu += uv[2] * bu;
        tv += uv[3] * bu;
        tu += uv[4] * bv;
        tv += uv[5] * bv;
        float level = 0.0f;
        if (lodRayCone) {
            const uint4 tx = A.textures[tex];
            const f3 e1 = mk(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z), e2 = mk(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z);
            const f3 n = normalize(cross(e1, e2));
            const float width = A.spread * t + 0.0f;  // RayCone(0, spread).propagateDistance(t)
            const float lambda = 0.0f + (float)log2((double)(fabsf(width) / fabsf(dot(d, n))));
            level = 0.5f * (float)log2((double)(float)(tx.x * tx.y)) + lambda;  // + 0.5 log2(w h)
        }
        alpha = alpha_sample(A, tex, tu, tv, level);
    }
    return alpha < m.x;  // evalBasicAlphaTest
}

}  // namespace rsd
