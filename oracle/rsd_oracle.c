/*
 * rsd_oracle.c -- CPU ORACLE (test infrastructure only; see rsd_oracle.h).
 *
 * Scalar C restatement of the Ray-SD + SVAO reference shaders.  Compile with
 * -ffp-contract=off: every float expression below is evaluated operation by
 * operation, in the order written, like the product kernels.
 *
 * Numerics contract shared with the product (DESIGN.md "Numerics"):
 *  - float ops are IEEE binary32, round-to-nearest, no contraction;
 *  - normalize(v) = v * (1 / sqrt(dot(v,v)))  (Falcor VectorMath.h:1731 rsqrt form);
 *  - sin/cos/pow of a float argument = (float)libm(double)  ("accurate" transcendental;
 *    HLSL leaves the precision of sin/pow implementation-defined);
 *  - bilinear filtering uses 8 fractional sub-texel bits (D3D11_SUBTEXEL_FRACTIONAL_BIT_COUNT);
 *  - any-hit calls arrive in ascending (t, primitive id) order, at most once per triangle.
 */
#include "rsd_oracle.h"
#include <math.h>
#include <float.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define O_FLT_MAX 3.402823466e+38f

/* ------------------------------------------------------------------ vector helpers */
static inline float o_dot(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void o_cross(const float a[3], const float b[3], float r[3])
{
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
}
static inline void o_normalize(const float v[3], float r[3])
{
    float inv = 1.0f / sqrtf(o_dot(v, v));
    r[0] = v[0] * inv; r[1] = v[1] * inv; r[2] = v[2] * inv;
}
static inline float o_len(const float v[3]) { return sqrtf(o_dot(v, v)); }
/* HLSL saturate/min/max: a NaN operand yields the other operand (saturate(NaN) = 0) */
static inline float o_saturate(float x) { return !(x > 0.0f) ? 0.0f : (x > 1.0f ? 1.0f : x); }
static inline float o_sin(float x) { return (float)sin((double)x); }
static inline float o_cos(float x) { return (float)cos((double)x); }
static inline float o_pow(float x, float y) { return (float)pow((double)x, (double)y); }
static inline float o_max(float a, float b) { return fmaxf(a, b); }
static inline float o_min(float a, float b) { return fminf(a, b); }
static inline uint32_t o_asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float o_asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* R8Unorm store: saturate, round to nearest (D3D FLOAT->UNORM); NaN -> 0 */
static inline uint8_t o_unorm8(float x)
{
    if (x != x) return 0;
    x = o_saturate(x);
    return (uint8_t)floorf(x * 255.0f + 0.5f);
}
static inline float o_unorm8_to_float(uint8_t c) { return (float)c / 255.0f; }

/* ------------------------------------------------------------------ constant tables */
/* Jitter.slangh:20 -- sobol 2d jitter table, indexed (y%4)*4 + x%4 */
static const float k_jitter[16][2] = {
    {0.6483604982495308f, 0.914070401340723f},   {0.7279119342565536f, 0.1037941575050354f},
    {0.48886989802122116f, 0.699178121984005f},  {0.3848271369934082f, 0.25951504334807396f},
    {0.1555836834013462f, 0.8020274639129639f},  {0.2205628715455532f, 0.2412630058825016f},
    {0.9962188489735126f, 0.5846633277833462f},  {0.8776040785014629f, 0.3954884633421898f},
    {0.9271227307617664f, 0.831196017563343f},   {0.9490576796233654f, 0.14202157780528069f},
    {0.20916065946221352f, 0.5476771481335163f}, {0.16468944773077965f, 0.4869129806756973f},
    {0.43544455617666245f, 0.9515445046126842f}, {0.44085410237312317f, 0.011881716549396515f},
    {0.7173641100525856f, 0.6695209294557571f},  {0.6563677340745926f, 0.35924511030316353f},
};

/* SVAO/Common.slang:52-58 -- VAO sample radii for NUM_DIRECTIONS = 8, 16, 32 (the shader's float
 * constants; the 16 / 32 tables are double literals there, rounded to float like these) */
static const float k_radius8[8] = {0.917883f, 0.564429f, 0.734504f, 0.359545f,
                                   0.820004f, 0.470149f, 0.650919f, 0.205215f};
static const float k_radius16[16] = {
    0.949098221604059, 0.5865639019441775, 0.7554681720909893, 0.3895439574863043,
    0.8425560503012255, 0.4948003867747738, 0.6719196866381647, 0.25203100417434543,
    0.8908588816103737, 0.5418210823278604, 0.7136427497994143, 0.32724136087586453,
    0.7980920320691521, 0.4445340224611676, 0.6297373536812639, 0.1447182620692375,
};
static const float k_radius32[32] = {
    0.9682458365518543, 0.5974803093982587, 0.7660169295429302, 0.4038472576817624,
    0.8541535023444914, 0.5068159098187986, 0.6823727109604635, 0.2726076670970059,
    0.904018191941786, 0.5531894754180758, 0.7240656647095169, 0.34372202910162664,
    0.8089818132350507, 0.45747336127867605, 0.640354849019649, 0.17748061996818404,
    0.9327350969376332, 0.5755500192397054, 0.7449678114312224, 0.37479566486456295,
    0.8311856199411515, 0.4825843210309559, 0.6614378277661477, 0.22975243551455923,
    0.878233108646881, 0.5303115209931901, 0.7032256306171377, 0.3099952198410562,
    0.7873133907642258, 0.43130429537268, 0.6190581352335289, 0.10219580968897692,
};
/* SVAO/Common.slang:60-66 -- HBAO sample radii (AO_KERNEL == AO_KERNEL_HBAO), double literals there */
static const float k_hbao8[8] = {0.019897607325877215, 0.3239192018939078, 0.15013283288204182, 0.5608856339193332,
                                 0.07874804859295396, 0.4306374970658152, 0.23159241868180838, 0.74770696488701};
static const float k_hbao16[16] = {
    0.008364792005390745, 0.29968419137477154, 0.13131974798930376, 0.5251597224509892,
    0.06264063727314514, 0.40226410430222115, 0.21027995621089465, 0.6906178807859765,
    0.03303993608633204, 0.34903099295095424, 0.16956281924775551, 0.5996160679614535,
    0.09559795810145842, 0.46040865279052423, 0.25357218870257175, 0.8218290863578166,
};
static const float k_hbao32[32] = {
    0.0035168784979124203, 0.28787249889929795, 0.12214740408236834, 0.5082189968610005,
    0.05489041689357717, 0.38854375322009427, 0.19986558164830323, 0.6656225173745592,
    0.02630214826181389, 0.33636038195532914, 0.15977097044845298, 0.579825376399601,
    0.08708424832212604, 0.44533522627083877, 0.24249692822679572, 0.7816464549941924,
    0.013886447731081395, 0.3116969449839127, 0.14064876764650994, 0.5426920213922799,
    0.07059703986067731, 0.41628837439340993, 0.22085459126773643, 0.7177502077720759,
    0.04006955250785802, 0.36194276200351894, 0.17950859741413544, 0.6203897476558216,
    0.10428292232859922, 0.47588885313824597, 0.2648228762567681, 0.8740952987729764,
};
static const float* o_radius_table_k(uint32_t nd, uint32_t kernel)
{
    if (kernel == 1) return nd == 32 ? k_hbao32 : nd == 16 ? k_hbao16 : k_hbao8;
    return nd == 32 ? k_radius32 : nd == 16 ? k_radius16 : k_radius8;
}
static const float* o_radius_table(uint32_t nd) { return o_radius_table_k(nd, 0); }

/* Jitter.slangh:27-50 randomJitter */
void ocpu_jitter(uint32_t x, uint32_t y, float* jx, float* jy)
{
    uint32_t idx = (y % 4u) * 4u + (x % 4u);
    *jx = k_jitter[idx][0];
    *jy = k_jitter[idx][1];
}

float ocpu_sample_radius(uint32_t num_directions, uint32_t i)
{
    if ((num_directions == 8 || num_directions == 16 || num_directions == 32) && i < num_directions)
        return o_radius_table(num_directions)[i];
    return 0.0f;
}

/* the sample radius of direction i for AO_KERNEL `kernel` (0 VAO, 1 HBAO) */
float ocpu_sample_radius_kernel(uint32_t num_directions, uint32_t i, uint32_t kernel)
{
    if ((num_directions == 8 || num_directions == 16 || num_directions == 32) && i < num_directions && kernel <= 1)
        return o_radius_table_k(num_directions, kernel)[i];
    return 0.0f;
}

/* SVAO.cpp:663-688 genNoiseTexture: 4x4 Bayer dither -> R8Unorm bytes */
void ocpu_noise_texture(uint8_t out[16])
{
    static const float dither[16] = {0.0f, 8.0f, 2.0f, 10.0f, 12.0f, 4.0f, 14.0f, 6.0f,
                                     3.0f, 11.0f, 1.0f, 9.0f, 15.0f, 7.0f, 13.0f, 5.0f};
    for (int i = 0; i < 16; ++i) out[i] = (uint8_t)(dither[i] / 16.0f * 255.0f);
}

/* StochasticDepthMapRT.cpp:79-124: binomial-ordered popcount look-up table */
static int o_binomial(int n, int k)
{
    int C[64];
    memset(C, 0, sizeof(C));
    C[0] = 1;
    for (int i = 1; i <= n; i++)
        for (int j = (i < k ? i : k); j > 0; j--) C[j] = C[j] + C[j - 1];
    return C[k];
}
void ocpu_stratified_lut(int n, int32_t* indices, uint32_t* lut)
{
    uint32_t maxEntries = 1u << n;
    indices[0] = 0;
    for (int i = 1; i <= n; i++) indices[i] = o_binomial(n, i - 1) + indices[i - 1];
    int32_t cur[33];
    for (int i = 0; i <= n; i++) cur[i] = indices[i];
    lut[0] = 0;
    for (uint32_t i = 1; i < maxEntries; i++) {
        int pc = __builtin_popcount(i);
        lut[cur[pc]] = i;
        cur[pc]++;
    }
}

/* Common.slangh:36-39 -- hash from "Improved Alpha Testing Using Hashed Sampling" */
float ocpu_hash(float x, float y)
{
    float a = 17.0f * x + 0.1f * y;
    float b = 13.0f * y + x;
    float r = 1.0e4f * o_sin(a) * (0.1f + fabsf(o_sin(b)));
    return r - floorf(r); /* frac */
}

/* ------------------------------------------------------------------ normal packing */
/* FormatConversion.slang:49-53 */
static int o_float_to_snorm8(float v)
{
    v = (v != v) ? 0.0f : o_min(o_max(v, -1.0f), 1.0f);
    return (int)truncf(v * 127.0f + (v >= 0.0f ? 0.5f : -0.5f));
}
/* MathHelpers.slang:156-159 */
static void o_oct_wrap(const float v[2], float r[2])
{
    r[0] = (1.0f - fabsf(v[1])) * (v[0] >= 0.0f ? 1.0f : -1.0f);
    r[1] = (1.0f - fabsf(v[0])) * (v[1] >= 0.0f ? 1.0f : -1.0f);
}
/* PackedFormats.slang:35-39 + MathHelpers.slang:166-172 + FormatConversion.slang:91-95 */
uint32_t ocpu_encode_normal_2x8(const float n[3])
{
    float s = 1.0f / (fabsf(n[0]) + fabsf(n[1]) + fabsf(n[2]));
    float p[2] = {n[0] * s, n[1] * s};
    if (n[2] < 0.0f) {
        float w[2];
        o_oct_wrap(p, w);
        p[0] = w[0]; p[1] = w[1];
    }
    return ((uint32_t)o_float_to_snorm8(p[0]) & 0xffu) | (((uint32_t)o_float_to_snorm8(p[1]) << 8) & 0xff00u);
}
/* PackedFormats.slang:44-48 + FormatConversion.slang:81-86 + MathHelpers.slang:186-191 */
void ocpu_decode_normal_2x8(uint32_t packed, float out[3])
{
    int bx = (int)(int8_t)(uint8_t)(packed & 0xffu);
    int by = (int)(int8_t)(uint8_t)((packed >> 8) & 0xffu);
    float p[2] = {o_max((float)bx / 127.0f, -1.0f), o_max((float)by / 127.0f, -1.0f)};
    float n[3] = {p[0], p[1], 1.0f - fabsf(p[0]) - fabsf(p[1])};
    if (n[2] < 0.0f) {
        float w[2];
        o_oct_wrap(n, w);
        n[0] = w[0]; n[1] = w[1];
    }
    o_normalize(n, out);
}

/* ------------------------------------------------------------------ camera */
/* Camera.cpp:99-185 (calculateCameraParameters), MatrixMath.h:686-712 (RightHanded look-at),
 * FalcorMath.h:123-126 (focalLengthToFovY).  preserveHeight = true. */
void ocpu_camera_look_at(const float pos[3], const float target[3], const float up[3],
                         float focalLength, float frameHeight, float aspectRatio,
                         float nearZ, float farZ, float focalDistance, ocam* c)
{
    memset(c, 0, sizeof(*c));
    for (int i = 0; i < 3; ++i) c->posW[i] = pos[i];
    c->nearZ = nearZ;
    c->farZ = farZ;
    c->focalLength = focalLength;
    c->frameHeight = frameHeight;
    c->aspectRatio = aspectRatio;
    c->frameWidth = frameHeight * aspectRatio;
    float fovY = focalLength == 0.0f ? 0.0f : 2.0f * atanf(0.5f * frameHeight / focalLength);

    /* view matrix */
    float emc[3] = {pos[0] - target[0], pos[1] - target[1], pos[2] - target[2]};
    float f[3], r[3], u[3], t[3];
    o_normalize(emc, f);
    o_cross(up, f, t);
    o_normalize(t, r);
    o_cross(f, r, u);
    float* m = c->viewMat;
    for (int i = 0; i < 16; ++i) m[i] = 0.0f;
    m[0] = r[0]; m[1] = r[1]; m[2] = r[2]; m[3] = -o_dot(r, pos);
    m[4] = u[0]; m[5] = u[1]; m[6] = u[2]; m[7] = -o_dot(u, pos);
    m[8] = f[0]; m[9] = f[1]; m[10] = f[2]; m[11] = -o_dot(f, pos);
    m[15] = 1.0f;

    /* ray tracing basis */
    float tmp[3] = {target[0] - pos[0], target[1] - pos[1], target[2] - pos[2]};
    float w[3];
    o_normalize(tmp, w);
    for (int i = 0; i < 3; ++i) c->W[i] = w[i] * focalDistance;
    float cu[3], cv[3];
    o_cross(c->W, up, tmp);
    o_normalize(tmp, cu);
    o_cross(cu, c->W, tmp);
    o_normalize(tmp, cv);
    float ulen = focalDistance * tanf(fovY * 0.5f) * aspectRatio;
    float vlen = focalDistance * tanf(fovY * 0.5f);
    for (int i = 0; i < 3; ++i) { c->U[i] = cu[i] * ulen; c->V[i] = cv[i] * vlen; }
}

/* Camera.slang:73-90 computeNonNormalizedRayDirPinhole: p in [0,1] screen space */
static void o_ray_dir(const ocam* c, float px, float py, float out[3])
{
    float ndcx = 2.0f * px + -1.0f;
    float ndcy = -2.0f * py + 1.0f;
    for (int i = 0; i < 3; ++i) out[i] = ndcx * c->U[i] + ndcy * c->V[i] + c->W[i];
}

/* ------------------------------------------------------------------ textures */
/* Linear filtering of an R32F texture at uv, D3D conventions, 8 sub-texel bits.
 * wrap = 1: AddressMode::Wrap (Falcor Sampler default, StochasticDepthMapRT S sampler)
 * wrap = 0: AddressMode::Clamp (SVAO gTextureSampler, SVAO.cpp:76). */
static inline int o_addr(int i, int n, int wrap)
{
    if (wrap) { i %= n; return i < 0 ? i + n : i; }
    return i < 0 ? 0 : (i >= n ? n - 1 : i);
}
static float o_bilinear(const float* tex, int W, int H, float u, float v, int wrap)
{
    float x = u * (float)W - 0.5f;
    float y = v * (float)H - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float qx = floorf((x - fx0) * 256.0f + 0.5f);
    float qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) { ix += 1; qx = 0.0f; }
    if (qy >= 256.0f) { iy += 1; qy = 0.0f; }
    float wx = qx * (1.0f / 256.0f), wy = qy * (1.0f / 256.0f);
    int x0 = o_addr(ix, W, wrap), x1 = o_addr(ix + 1, W, wrap);
    int y0 = o_addr(iy, H, wrap), y1 = o_addr(iy + 1, H, wrap);
    float t00 = tex[(size_t)y0 * W + x0], t10 = tex[(size_t)y0 * W + x1];
    float t01 = tex[(size_t)y1 * W + x0], t11 = tex[(size_t)y1 * W + x1];
    float r0 = t00 * (1.0f - wx) + t10 * wx;
    float r1 = t01 * (1.0f - wx) + t11 * wx;
    return r0 * (1.0f - wy) + r1 * wy;
}

/* ------------------------------------------------------------------ intersection */
/* Pre-computed per-ray data of the watertight test (IntersectionHelpers.slang:114-133) */
typedef struct {
    float o[3], d[3];
    int kx, ky, kz;
    float Sx, Sy, Sz;
} oray;

static void o_ray_setup(oray* r, const float o[3], const float d[3])
{
    for (int i = 0; i < 3; ++i) { r->o[i] = o[i]; r->d[i] = d[i]; }
    float ax = fabsf(d[0]), ay = fabsf(d[1]), az = fabsf(d[2]);
    int axis = 0;
    if (ay > ax && ay > az) axis = 1;
    if (az > ax && az > ay) axis = 2;
    r->kz = axis;
    r->kx = (axis + 1) % 3;
    r->ky = (r->kx + 1) % 3;
    if (d[r->kz] < 0.0f) { int s = r->kx; r->kx = r->ky; r->ky = s; }
    r->Sx = d[r->kx] / d[r->kz];
    r->Sy = d[r->ky] / d[r->kz];
    r->Sz = 1.0f / d[r->kz];
}

/* IntersectionHelpers.slang:109-180.  Returns 1 on hit, t, DXR barycentrics (V,W)/det, det */
static int o_intersect_tri(const oray* r, const float v0[3], const float v1[3], const float v2[3],
                           float* t, float* bu, float* bv, float* detOut)
{
    float A[3], B[3], C[3];
    for (int i = 0; i < 3; ++i) { A[i] = v0[i] - r->o[i]; B[i] = v1[i] - r->o[i]; C[i] = v2[i] - r->o[i]; }
    const int kx = r->kx, ky = r->ky, kz = r->kz;
    float Ax = A[kx] - r->Sx * A[kz];
    float Ay = A[ky] - r->Sy * A[kz];
    float Bx = B[kx] - r->Sx * B[kz];
    float By = B[ky] - r->Sy * B[kz];
    float Cx = C[kx] - r->Sx * C[kz];
    float Cy = C[ky] - r->Sy * C[kz];
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
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return 0;
    float det = U + V + W;
    if (det == 0.0f) return 0;
    float Az = r->Sz * A[kz], Bz = r->Sz * B[kz], Cz = r->Sz * C[kz];
    float T = U * Az + V * Bz + W * Cz;
    float rcpDet = 1.0f / det;
    *t = T * rcpDet;
    *bu = V * rcpDet;
    *bv = W * rcpDet;
    *detOut = det;
    return 1;
}

int ocpu_intersect(const float o[3], const float d[3], const float v0[3], const float v1[3],
                   const float v2[3], float* t, float* u, float* v, float* det)
{
    oray r;
    o_ray_setup(&r, o, d);
    return o_intersect_tri(&r, v0, v1, v2, t, u, v, det);
}

/* Culling (RtAccelerationStructure instance flags, Scene.cpp:3446-3452; ray flags
 * CULL_BACK/FRONT_FACING_TRIANGLES).  det > 0 <=> vertices counter-clockwise seen from
 * the ray origin (right-handed), which is Falcor's front face unless frontFaceCW. */
static int o_culled(float det, uint32_t flags, uint32_t cull_mode)
{
    if (cull_mode == 0 || (flags & 1u)) return 0;
    int front = (det > 0.0f) != ((flags & 2u) != 0);
    return cull_mode == 1 ? !front : front;
}

/* ------------------------------------------------------------------ oracle BVH (object median) */
typedef struct { float lo[3], hi[3]; uint32_t left, right, first, count; } onode;

struct oscene {
    uint32_t nt;
    float* tri;        /* nt * 9 floats (v0,v1,v2), original primitive order */
    uint32_t* flags;   /* nt */
    uint32_t* order;   /* leaf order -> primitive id */
    onode* nodes;
    uint32_t nnodes;
    /* alpha-masked materials (ocpu_scene_set_alpha); uv == NULL: none */
    float* uv;          /* nt * 6: texture coordinates of v0, v1, v2 */
    uint32_t* mat;      /* nt */
    float* mthr;        /* alpha threshold, float16-rounded */
    float* malpha;      /* constant alpha */
    uint32_t* mtex;     /* texture or 0xffffffff */
    uint32_t nm, ntex;
    uint32_t* tw; uint32_t* th; uint32_t* tmips;
    size_t* toff;       /* first texel of mip 0 */
    uint8_t* texels;    /* mip chains, R8 */
};

static float* g_cent; /* centroid array used by the select routine */

static void o_bounds(const oscene* s, const uint32_t* idx, uint32_t n, float lo[3], float hi[3])
{
    for (int k = 0; k < 3; ++k) { lo[k] = FLT_MAX; hi[k] = -FLT_MAX; }
    for (uint32_t i = 0; i < n; ++i) {
        const float* v = s->tri + (size_t)idx[i] * 9;
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) {
                if (v[j * 3 + k] < lo[k]) lo[k] = v[j * 3 + k];
                if (v[j * 3 + k] > hi[k]) hi[k] = v[j * 3 + k];
            }
    }
}

/* 3-way-partition quickselect: afterwards idx[k] holds the k-th smallest centroid along
 * `axis`, smaller ones before it and larger ones after it. */
static void o_select(uint32_t* idx, uint32_t n, uint32_t k, int axis)
{
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        float a = g_cent[(size_t)idx[lo] * 3 + axis];
        float b = g_cent[(size_t)idx[(lo + hi) / 2] * 3 + axis];
        float c = g_cent[(size_t)idx[hi - 1] * 3 + axis];
        float pivot = a < b ? (b < c ? b : (a < c ? c : a)) : (a < c ? a : (b < c ? c : b));
        uint32_t lt = lo, i = lo, gt = hi;
        while (i < gt) {
            float v = g_cent[(size_t)idx[i] * 3 + axis];
            if (v < pivot) { uint32_t t = idx[lt]; idx[lt] = idx[i]; idx[i] = t; lt++; i++; }
            else if (v > pivot) { gt--; uint32_t t = idx[gt]; idx[gt] = idx[i]; idx[i] = t; }
            else i++;
        }
        if (k < lt) hi = lt;
        else if (k >= gt) lo = gt;
        else return;
    }
}

static uint32_t o_build(oscene* s, uint32_t* idx, uint32_t first, uint32_t n)
{
    uint32_t me = s->nnodes++;
    onode* nd = &s->nodes[me];
    o_bounds(s, idx + first, n, nd->lo, nd->hi);
    if (n <= 4) {
        nd->left = nd->right = 0;
        nd->first = first;
        nd->count = n;
        return me;
    }
    float clo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, chi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (uint32_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            float c = g_cent[(size_t)idx[first + i] * 3 + k];
            if (c < clo[k]) clo[k] = c;
            if (c > chi[k]) chi[k] = c;
        }
    int axis = 0;
    float ext = chi[0] - clo[0];
    if (chi[1] - clo[1] > ext) { axis = 1; ext = chi[1] - clo[1]; }
    if (chi[2] - clo[2] > ext) axis = 2;
    uint32_t half = n / 2;
    o_select(idx + first, n, half, axis);
    uint32_t l = o_build(s, idx, first, half);
    uint32_t r = o_build(s, idx, first + half, n - half);
    nd = &s->nodes[me];
    nd->left = l;
    nd->right = r;
    nd->count = 0;
    return me;
}

oscene* ocpu_scene_create(const float* pos, uint32_t nv, const uint32_t* ind, uint32_t nt, const uint32_t* flags)
{
    (void)nv;
    oscene* s = (oscene*)calloc(1, sizeof(oscene));
    s->nt = nt;
    s->tri = (float*)malloc(sizeof(float) * 9 * (size_t)(nt ? nt : 1));
    s->flags = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(nt ? nt : 1));
    s->order = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(nt ? nt : 1));
    g_cent = (float*)malloc(sizeof(float) * 3 * (size_t)(nt ? nt : 1));
    for (uint32_t i = 0; i < nt; ++i) {
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) s->tri[(size_t)i * 9 + j * 3 + k] = pos[(size_t)ind[(size_t)i * 3 + j] * 3 + k];
        s->flags[i] = flags ? flags[i] : 0u;
        s->order[i] = i;
        for (int k = 0; k < 3; ++k) {
            const float* v = s->tri + (size_t)i * 9;
            g_cent[(size_t)i * 3 + k] = (v[k] + v[3 + k] + v[6 + k]) * (1.0f / 3.0f);
        }
    }
    s->nodes = (onode*)calloc(2 * (size_t)(nt ? nt : 1) + 1, sizeof(onode));
    if (nt) o_build(s, s->order, 0, nt);
    free(g_cent);
    g_cent = NULL;
    return s;
}

void ocpu_scene_destroy(oscene* s)
{
    if (!s) return;
    free(s->tri); free(s->flags); free(s->order); free(s->nodes);
    free(s->uv); free(s->mat); free(s->mthr); free(s->malpha); free(s->mtex);
    free(s->tw); free(s->th); free(s->tmips); free(s->toff); free(s->texels);
    free(s);
}

/* ------------------------------------------------------------------ alpha test
 * MaterialFactory::alphaTest (Scene/Material/MaterialFactory.slang:124-151) with the
 * base-colour alpha of StandardMaterial (StandardMaterial.slang:128-132) and the basic test
 * (AlphaTest.slang:81-84): the hit is discarded when alpha < threshold.  The threshold is
 * a float16 in MaterialHeader (MaterialData.slang:99).  Texture coordinate interpolation:
 * Scene::computeVertexData (Scene.slang:444-480).  Sampling follows librsd's definition
 * (DESIGN.md "Alpha test"): 2x2 box mips (a+b+c+d+2)/4, wrap, bilinear with 8 sub-texel
 * bits, trilinear with the LOD fraction quantised to 8 bits. */

/* float -> IEEE half (round to nearest even) -> float, through the half's bit pattern */
static float o_half_round(float f)
{
    uint32_t x = o_asuint(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t e = (x >> 23) & 0xffu, m = x & 0x7fffffu;
    uint32_t h;
    if (e == 0xffu) h = sign | 0x7c00u | (m ? 0x200u : 0u);
    else {
        int he = (int)e - 127 + 15;
        if (he >= 31) h = sign | 0x7c00u;
        else if (he <= 0) {
            if (he < -10) h = sign;
            else {
                uint32_t mm = m | 0x800000u;
                int shift = 14 - he;            /* 24-bit significand -> subnormal half */
                uint32_t q = mm >> shift, rem = mm & ((1u << shift) - 1u), half = 1u << (shift - 1);
                if (rem > half || (rem == half && (q & 1u))) q++;
                h = sign | q;
            }
        } else {
            uint32_t q = ((uint32_t)he << 10) | (m >> 13), rem = m & 0x1fffu;
            if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++; /* may carry into inf */
            h = sign | q;
        }
    }
    /* half -> float */
    uint32_t hs = (h & 0x8000u) << 16, he2 = (h >> 10) & 0x1fu, hm = h & 0x3ffu;
    if (he2 == 0x1fu) return o_asfloat(hs | 0x7f800000u | (hm << 13));
    if (he2 == 0) {
        float v = (float)hm * (1.0f / 16777216.0f); /* hm 2^-24, exact */
        return hs ? -v : v;
    }
    return o_asfloat(hs | ((he2 - 15 + 127) << 23) | (hm << 13));
}

void ocpu_scene_set_alpha(oscene* s, const uint32_t* ind, const float* texcoords, const uint32_t* triMat,
                          uint32_t nm, const float* thr, const float* alpha, const uint32_t* tex,
                          uint32_t ntex, const uint32_t* tex_w, const uint32_t* tex_h, const uint8_t* mip0)
{
    const uint32_t nt = s->nt;
    s->uv = (float*)malloc(sizeof(float) * 6 * (size_t)(nt ? nt : 1));
    s->mat = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(nt ? nt : 1));
    for (uint32_t i = 0; i < nt; ++i) {
        for (int k = 0; k < 3; ++k) {
            const uint32_t v = ind[(size_t)i * 3 + k];
            s->uv[(size_t)i * 6 + 2 * k] = texcoords[2 * (size_t)v];
            s->uv[(size_t)i * 6 + 2 * k + 1] = texcoords[2 * (size_t)v + 1];
        }
        s->mat[i] = triMat[i];
    }
    s->nm = nm;
    s->mthr = (float*)malloc(sizeof(float) * nm);
    s->malpha = (float*)malloc(sizeof(float) * nm);
    s->mtex = (uint32_t*)malloc(sizeof(uint32_t) * nm);
    for (uint32_t i = 0; i < nm; ++i) {
        s->mthr[i] = o_half_round(thr[i]);
        s->malpha[i] = alpha[i];
        s->mtex[i] = tex[i];
    }
    s->ntex = ntex;
    s->tw = (uint32_t*)malloc(sizeof(uint32_t) * (ntex ? ntex : 1));
    s->th = (uint32_t*)malloc(sizeof(uint32_t) * (ntex ? ntex : 1));
    s->tmips = (uint32_t*)malloc(sizeof(uint32_t) * (ntex ? ntex : 1));
    s->toff = (size_t*)malloc(sizeof(size_t) * (ntex ? ntex : 1));
    /* total texels of all chains */
    size_t total = 0;
    for (uint32_t i = 0; i < ntex; ++i) {
        uint32_t w = tex_w[i], h = tex_h[i];
        for (;;) {
            total += (size_t)w * h;
            if (w == 1 && h == 1) break;
            w = w > 1 ? w / 2 : 1;
            h = h > 1 ? h / 2 : 1;
        }
    }
    s->texels = (uint8_t*)malloc(total ? total : 1);
    size_t at = 0, src0 = 0;
    for (uint32_t i = 0; i < ntex; ++i) {
        uint32_t w = tex_w[i], h = tex_h[i];
        s->tw[i] = w; s->th[i] = h; s->toff[i] = at;
        memcpy(s->texels + at, mip0 + src0, (size_t)w * h);
        src0 += (size_t)w * h;
        uint32_t mips = 1;
        while (w > 1 || h > 1) {
            const uint8_t* src = s->texels + at;
            uint8_t* dst = s->texels + at + (size_t)w * h;
            const uint32_t nw = w > 1 ? w / 2 : 1, nh = h > 1 ? h / 2 : 1;
            for (uint32_t y = 0; y < nh; ++y)
                for (uint32_t x = 0; x < nw; ++x) {
                    uint32_t xa = 2 * x < w ? 2 * x : w - 1, xb = 2 * x + 1 < w ? 2 * x + 1 : w - 1;
                    uint32_t ya = 2 * y < h ? 2 * y : h - 1, yb = 2 * y + 1 < h ? 2 * y + 1 : h - 1;
                    uint32_t sum = (uint32_t)src[(size_t)ya * w + xa] + src[(size_t)ya * w + xb] +
                                   src[(size_t)yb * w + xa] + src[(size_t)yb * w + xb];
                    dst[(size_t)y * nw + x] = (uint8_t)((sum + 2u) >> 2);
                }
            at += (size_t)w * h;
            w = nw; h = nh;
            mips++;
        }
        at += (size_t)w * h;
        s->tmips[i] = mips;
    }
}

static float o_alpha_texel(const uint8_t* lvl, int w, int h, int x, int y)
{
    x = ((x % w) + w) % w;
    y = ((y % h) + h) % h;
    return (float)lvl[(size_t)y * w + x] / 255.0f;
}

/* one bilinear tap, wrap addressing, weights quantised to 1/256 */
static float o_alpha_bilinear(const uint8_t* lvl, int w, int h, float u, float v)
{
    float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    float x0 = floorf(x), y0 = floorf(y);
    int ix = (int)x0, iy = (int)y0;
    float qx = floorf((x - x0) * 256.0f + 0.5f), qy = floorf((y - y0) * 256.0f + 0.5f);
    if (qx >= 256.0f) { qx = 0.0f; ix++; }
    if (qy >= 256.0f) { qy = 0.0f; iy++; }
    float wx = qx * (1.0f / 256.0f), wy = qy * (1.0f / 256.0f);
    float top = o_alpha_texel(lvl, w, h, ix, iy) * (1.0f - wx) + o_alpha_texel(lvl, w, h, ix + 1, iy) * wx;
    float bot = o_alpha_texel(lvl, w, h, ix, iy + 1) * (1.0f - wx) + o_alpha_texel(lvl, w, h, ix + 1, iy + 1) * wx;
    return top * (1.0f - wy) + bot * wy;
}

/* Texture2D.SampleLevel(uv, level), trilinear, LOD clamped to [0, mips - 1], NaN -> 0 */
static float o_alpha_sample(const oscene* s, uint32_t ti, float u, float v, float level)
{
    const int mips = (int)s->tmips[ti];
    float lod = level;
    if (lod != lod) lod = 0.0f;
    if (lod < 0.0f) lod = 0.0f;
    if (lod > (float)(mips - 1)) lod = (float)(mips - 1);
    int l = (int)floorf(lod);
    float qf = floorf((lod - (float)l) * 256.0f + 0.5f);
    if (qf >= 256.0f) { qf = 0.0f; l++; }
    size_t off = s->toff[ti];
    int w = (int)s->tw[ti], h = (int)s->th[ti];
    for (int m = 0; m < l; ++m) {
        off += (size_t)w * h;
        w = w > 1 ? w / 2 : 1;
        h = h > 1 ? h / 2 : 1;
    }
    float a = o_alpha_bilinear(s->texels + off, w, h, u, v);
    if (qf == 0.0f || l + 1 >= mips) return a;
    float b = o_alpha_bilinear(s->texels + off + (size_t)w * h, w > 1 ? w / 2 : 1, h > 1 ? h / 2 : 1, u, v);
    float f = qf * (1.0f / 256.0f);
    return a * (1.0f - f) + b * f;
}

/* Camera::computeScreenSpacePixelSpreadAngle (Camera.cpp:296-301) with focalLengthToFovY at
 * the 24 mm default frame height (FalcorMath.h:123-126), as the "%f" text of the shader
 * define RAY_CONE_SPREAD (StochasticDepthMapRT.cpp:266-267) read back as a float */
float ocpu_ray_cone_spread(float focal, uint32_t height)
{
    float fov = 2.0f * atanf(0.5f * 24.0f / focal);
    float ang = atanf(2.0f * tanf(fov * 0.5f) / (float)height);
    char txt[64];
    snprintf(txt, sizeof(txt), "%f", (double)ang);
    return strtof(txt, NULL);
}

/* 1 = the alpha test discards the hit.  lodRayCone: computeLod of StochasticDepthMapRT.rt.slang:
 * 31-37 (RayCone(0, spread).propagateDistance(t).computeLOD(0, dir, faceNormalW),
 * TexLODHelpers.slang:97-129) plus 0.5 log2(w h) (TextureSampler.slang:90-96); else LOD 0.
 * log2 in double, rounded once (numerics contract). */
float ocpu_alpha_value(const oscene* s, uint32_t prim, float bu, float bv, int lodRayCone, float t,
                       const float d[3], float spread)
{
    const uint32_t m = s->mat[prim];
    float alpha = s->malpha[m];
    const uint32_t ti = s->mtex[m];
    if (ti != 0xffffffffu) {
        const float* uv = s->uv + (size_t)prim * 6;
        const float w0 = 1.0f - bu - bv;
        float tu = uv[0] * w0 + uv[2] * bu + uv[4] * bv;
        float tv = uv[1] * w0 + uv[3] * bu + uv[5] * bv;
        float level = 0.0f;
        if (lodRayCone) {
            const float* v = s->tri + (size_t)prim * 9;
            float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
            float e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
            float cr[3], n[3];
            o_cross(e1, e2, cr);
            o_normalize(cr, n);
            float width = spread * t + 0.0f;
            float lambda = 0.0f + (float)log2((double)(fabsf(width) / fabsf(o_dot(d, n))));
            float dims = (float)(s->tw[ti] * s->th[ti]);
            level = 0.5f * (float)log2((double)dims) + lambda;
        }
        alpha = o_alpha_sample(s, ti, tu, tv, level);
    }
    return alpha;
}

int ocpu_alpha_fails(const oscene* s, uint32_t prim, float bu, float bv, int lodRayCone, float t,
                     const float d[3], float spread)
{
    return ocpu_alpha_value(s, prim, bu, bv, lodRayCone, t, d, spread) < s->mthr[s->mat[prim]];
}

float ocpu_alpha_threshold(const oscene* s, uint32_t material) { return s->mthr[material]; }

static inline int o_alpha_masked(const oscene* s, uint32_t prim) { return s->uv && (s->flags[prim] & 4u); }
uint32_t ocpu_scene_node_count(const oscene* s) { return s->nnodes; }

/* Conservative slab test in double precision with a relative margin: a node is
 * skipped only when it certainly holds no triangle hit with t in [tmin, tmax]. */
static int o_box(const oray* r, const onode* n, double tmin, double tmax)
{
    double t0 = -INFINITY, t1 = INFINITY;
    for (int k = 0; k < 3; ++k) {
        double o = r->o[k], d = r->d[k];
        if (d == 0.0) {
            if (o < n->lo[k] || o > n->hi[k]) return 0;
            continue;
        }
        double a = (n->lo[k] - o) / d, b = (n->hi[k] - o) / d;
        if (a > b) { double t = a; a = b; b = t; }
        if (a > t0) t0 = a;
        if (b < t1) t1 = b;
    }
    double m = 1e-5 * (fabs(t0) + fabs(t1)) + 1e-30;
    t0 -= m; t1 += m;
    if (t0 < tmin) t0 = tmin;
    if (t1 > tmax) t1 = tmax;
    return t0 <= t1;
}

/* ------------------------------------------------------------------ hit collection */
typedef struct { float t, u, v; uint32_t prim; float det; } ohit;

typedef struct {
    ohit* h;
    uint32_t n, cap;
    uint32_t limit; /* keep only the `limit` smallest (t,prim); 0 = keep all */
} ohits;

static inline int o_key_less(float ta, uint32_t pa, float tb, uint32_t pb)
{
    return ta < tb || (ta == tb && pa < pb);
}

static void o_hits_push(ohits* hs, ohit x)
{
    if (hs->limit && hs->n == hs->limit) {
        ohit* last = &hs->h[hs->n - 1];
        if (!o_key_less(x.t, x.prim, last->t, last->prim)) return;
        hs->n--; /* drop the largest */
    }
    if (hs->n == hs->cap) {
        hs->cap = hs->cap ? hs->cap * 2 : 16;
        hs->h = (ohit*)realloc(hs->h, sizeof(ohit) * hs->cap);
    }
    /* insertion keeps the list sorted by (t, prim) */
    uint32_t i = hs->n++;
    while (i > 0 && o_key_less(x.t, x.prim, hs->h[i - 1].t, hs->h[i - 1].prim)) {
        hs->h[i] = hs->h[i - 1];
        i--;
    }
    hs->h[i] = x;
}

/* all hits with TMin <= t <= TMax, culling applied, ascending (t, prim) order */
static void o_collect(const oscene* s, const oray* r, float TMin, float TMax, uint32_t cull, int alpha0, ohits* hs)
{
    if (!s->nt || !(TMin <= TMax)) return;
    uint32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const onode* n = &s->nodes[stack[--sp]];
        float bound = TMax;
        if (hs->limit && hs->n == hs->limit && hs->h[hs->n - 1].t < bound) bound = hs->h[hs->n - 1].t;
        if (!o_box(r, n, TMin, bound)) continue;
        if (n->count) {
            for (uint32_t i = 0; i < n->count; ++i) {
                uint32_t prim = s->order[n->first + i];
                const float* v = s->tri + (size_t)prim * 9;
                float t, u, vv, det;
                if (!o_intersect_tri(r, v, v + 3, v + 6, &t, &u, &vv, &det)) continue;
                if (!(t >= TMin && t <= TMax)) continue;
                if (o_culled(det, s->flags[prim], cull)) continue;
                /* any-hit IgnoreHit of an alpha-masked triangle failing at LOD 0 */
                if (alpha0 && o_alpha_masked(s, prim) && ocpu_alpha_fails(s, prim, u, vv, 0, t, r->d, 0.0f)) continue;
                ohit x = {t, u, vv, prim, det};
                o_hits_push(hs, x);
            }
        } else {
            stack[sp++] = n->left;
            stack[sp++] = n->right;
        }
    }
}

/* ------------------------------------------------------------------ G-buffer */
typedef struct {
    const oscene* s; const ocam* c; uint32_t W, H, cull;
    float* z; uint16_t* n;
    float* nw; /* raster mode (GBufferRaster): z = non-linear depth, nw = RGBA32F world face normal */
    uint32_t y0, y1;
} ogb_job;

static void* o_gbuffer_rows(void* arg)
{
    ogb_job* j = (ogb_job*)arg;
    const ocam* c = j->c;
    float wn[3];
    o_normalize(c->W, wn);
    for (uint32_t y = j->y0; y < j->y1; ++y)
        for (uint32_t x = 0; x < j->W; ++x) {
            /* Camera.slang:46-59 computeRayPinhole (camera jitter applied) */
            float px = ((float)x + 0.5f) / (float)j->W + -c->jitterX;
            float py = ((float)y + 0.5f) / (float)j->H + c->jitterY;
            float dn[3], d[3];
            o_ray_dir(c, px, py, dn);
            o_normalize(dn, d);
            float invCos = 1.0f / o_dot(wn, d);
            float tmin = c->nearZ * invCos, tmax = c->farZ * invCos;
            oray r;
            o_ray_setup(&r, c->posW, d);
            ohits hs = {0};
            hs.limit = 1;
            o_collect(j->s, &r, tmin, tmax, j->cull, 1, &hs); /* GBufferRaster useAlphaTest */
            size_t o = (size_t)y * j->W + x;
            if (hs.n == 0) {
                if (j->nw) { /* cleared depth buffer / zero normal */
                    j->z[o] = 1.0f;
                    for (int k = 0; k < 4; ++k) j->nw[o * 4 + k] = 0.0f;
                } else {
                    j->z[o] = c->farZ;
                    j->n[o] = 0;
                }
            } else {
                const float zlin = hs.h[0].t * o_dot(wn, d);
                const float* v = j->s->tri + (size_t)hs.h[0].prim * 9;
                float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
                float e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
                float cr[3], nw[3], nv[3];
                o_cross(e1, e2, cr);
                o_normalize(cr, nw);
                if (j->nw) {
                    /* D3D [0,1] depth of the right-handed perspective projection
                     * (Camera.cpp:164 perspective(), depth range [0,1]): far (z - near) / (z (far - near)) */
                    j->z[o] = c->farZ * (zlin - c->nearZ) / (zlin * (c->farZ - c->nearZ));
                    j->nw[o * 4 + 0] = nw[0]; j->nw[o * 4 + 1] = nw[1]; j->nw[o * 4 + 2] = nw[2];
                    j->nw[o * 4 + 3] = 0.0f;
                    free(hs.h);
                    continue;
                }
                j->z[o] = zlin;
                const float* m = c->viewMat;
                for (int k = 0; k < 3; ++k) nv[k] = m[k * 4 + 0] * nw[0] + m[k * 4 + 1] * nw[1] + m[k * 4 + 2] * nw[2];
                j->n[o] = (uint16_t)ocpu_encode_normal_2x8(nv);
            }
            free(hs.h);
        }
    return NULL;
}

static void o_run_rows(void* (*fn)(void*), void* jobs, size_t jobsz, uint32_t y0, uint32_t y1, int nthreads,
                       void (*setrows)(void*, uint32_t, uint32_t))
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    uint32_t rows = y1 - y0;
    for (int i = 0; i < nthreads; ++i) {
        void* job = (char*)jobs + jobsz * i;
        setrows(job, y0 + (uint32_t)((uint64_t)rows * i / nthreads), y0 + (uint32_t)((uint64_t)rows * (i + 1) / nthreads));
        pthread_create(&th[i], NULL, fn, job);
    }
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
}

static void o_gb_setrows(void* j, uint32_t a, uint32_t b) { ((ogb_job*)j)->y0 = a; ((ogb_job*)j)->y1 = b; }

void ocpu_gbuffer(const oscene* s, const ocam* cam, uint32_t W, uint32_t H, uint32_t cull,
                  float* linearZ, uint16_t* normals, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    ogb_job* jobs = (ogb_job*)calloc((size_t)nthreads, sizeof(ogb_job));
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].s = s; jobs[i].c = cam; jobs[i].W = W; jobs[i].H = H; jobs[i].cull = cull;
        jobs[i].z = linearZ; jobs[i].n = normals;
    }
    o_run_rows(o_gbuffer_rows, jobs, sizeof(ogb_job), 0, H, nthreads, o_gb_setrows);
    free(jobs);
}

void ocpu_gbuffer_raster(const oscene* s, const ocam* cam, uint32_t W, uint32_t H, uint32_t cull,
                         float* depth, float* normalW, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    ogb_job* jobs = (ogb_job*)calloc((size_t)nthreads, sizeof(ogb_job));
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].s = s; jobs[i].c = cam; jobs[i].W = W; jobs[i].H = H; jobs[i].cull = cull;
        jobs[i].z = depth; jobs[i].nw = normalW;
    }
    o_run_rows(o_gbuffer_rows, jobs, sizeof(ogb_job), 0, H, nthreads, o_gb_setrows);
    free(jobs);
}

/* LinearizeDepth/Linearize.ps.slang:11-16 */
void ocpu_linearize_depth(const float* d, float* z, size_t n, float zn, float zf)
{
    for (size_t i = 0; i < n; ++i) z[i] = zn * zf / (zf + d[i] * (zn - zf));
}

/* CompressNormals/CompressNormals.ps.slang:11-23 (viewSpace, use16Bit) */
void ocpu_compress_normals(const float* nw, uint16_t* out, size_t n, const ocam* c)
{
    const float* m = c->viewMat;
    for (size_t i = 0; i < n; ++i) {
        const float* v = nw + i * 4;
        float nv[3];
        for (int k = 0; k < 3; ++k) nv[k] = m[k * 4 + 0] * v[0] + m[k * 4 + 1] * v[1] + m[k * 4 + 2] * v[2];
        out[i] = (uint16_t)ocpu_encode_normal_2x8(nv);
    }
}

/* ------------------------------------------------------------------ SD trace */
/* initRayDesc, Common.slangh:65-92 (+ Camera.slang:46-90).  Returns TMin/TMax, the
 * normalized jittered direction d and cosT = dot(normalize(cameraW), d). */
static void o_sd_ray(const ocam* c, const osd_params* p, const float* z, uint32_t zW, uint32_t zH,
                     const uint32_t* rmin, const uint32_t* rmax, uint32_t sdW, uint32_t sdH,
                     uint32_t x, uint32_t y, float d[3], float* TMinOut, float* TMaxOut, float* cosTOut)
{
    const int G = p->guard_band;
    const int dimx = (int)sdW - 2 * G, dimy = (int)sdH - 2 * G;
    float wn[3];
    o_normalize(c->W, wn);
    int sx = (int)x - G, sy = (int)y - G;
    float pcx = ((float)sx + 0.5f) / (float)dimx + -c->jitterX;
    float pcy = ((float)sy + 0.5f) / (float)dimy + c->jitterY;
    float dn[3], dc[3];
    o_ray_dir(c, pcx, pcy, dn);
    o_normalize(dn, dc);
    float invCos = 1.0f / o_dot(wn, dc);
    float TMax = c->farZ * invCos; /* computeRayPinhole tMax (pixel centre) */
    float jx = 0.5f, jy = 0.5f;
    if (p->jitter) ocpu_jitter(x, y, &jx, &jy);
    float pjx = ((float)sx + jx) / (float)dimx;
    float pjy = ((float)sy + jy) / (float)dimy;
    o_ray_dir(c, pjx, pjy, dn);
    o_normalize(dn, d);
    float eps = 0.1f * c->nearZ;
    float depth = 0.0f;
    if (sx >= 0 && sy >= 0 && sx < dimx && sy < dimy)
        depth = o_bilinear(z, (int)zW, (int)zH, ((float)sx + 0.5f) / (float)dimx,
                           ((float)sy + 0.5f) / (float)dimy, 1);
    float cosT = o_dot(wn, d);
    float TMin = depth / cosT + eps;
    if (p->ray_interval) {
        size_t o = (size_t)y * sdW + x;
        uint32_t iMin = rmin ? rmin[o] : 0u;
        if (iMin != 0u) TMin = o_max(o_asfloat(iMin), TMin);
        uint32_t iMax = rmax ? rmax[o] : 0u;
        if (iMax != 0u) TMax = o_min(o_asfloat(iMax), TMax);
    }
    *TMinOut = TMin; *TMaxOut = TMax; *cosTOut = cosT;
}

void ocpu_sd_ray(const ocam* c, const osd_params* p, const float* z, uint32_t zW, uint32_t zH,
                 const uint32_t* rmin, const uint32_t* rmax, uint32_t sdW, uint32_t sdH, uint32_t x, uint32_t y,
                 float out[6] /* o.xyz, d.xyz */, float* tmin, float* tmax, float* cosT)
{
    float d[3];
    o_sd_ray(c, p, z, zW, zH, rmin, rmax, sdW, sdH, x, y, d, tmin, tmax, cosT);
    for (int i = 0; i < 3; ++i) { out[i] = c->posW[i]; out[3 + i] = d[i]; }
}

/* anyHit -> algorithm (Common.slangh:102-254) for ONE delivered hit: rng = hash(barycentrics),
 * t = (normalized) view depth, af = the alpha test failed.  Returns the commit decision (the
 * any-hit shader does not IgnoreHit: DXR accepts the hit, TMax = t). */
static int o_any_hit(const osd_params* p, uint32_t N, const int32_t* lutIdx, const uint32_t* lut,
                     float* depths, uint32_t* count, float rng, float t, int af)
{
    if (p->implementation == 1) { /* CoverageMask, Common.slangh:117-131, 189-209 */
        int R = (int)floorf(p->alpha * (float)N + rng);
        uint32_t mask = 0;
        if (R >= (int)N) mask = 0xffffu;
        else if (R != 0) {
            float rng2 = ocpu_hash(rng, t); /* hash3D(float3(bary, t)) */
            float a = (float)lutIdx[R], b = (float)lutIdx[R + 1];
            int index = (int)(a + rng2 * (b - a));
            mask = lut[index];
        }
        if (af) return *count >= p->max_count; /* alpha test failed: ignore (count stays 0) */
        float maxT = 0.0f;
        for (uint32_t i = 0; i < N; ++i) {
            if (mask & (1u << i))
                if (t < depths[i]) depths[i] = t;
            maxT = o_max(maxT, depths[i]);
        }
        return !(t < maxT);
    } else if (p->implementation == 3) { /* KBuffer, Common.slangh:132-135, 211-232 */
        if (t >= depths[N - 1]) return 1;
        (*count)++;
        if (af) return *count >= p->max_count;
        float rayT = t;
        for (uint32_t i = 0; i < N; ++i)
            if (t < depths[i]) { float tmp = depths[i]; depths[i] = t; t = tmp; }
        return (depths[N - 1] == rayT) ? 1 : (*count >= p->max_count);
    } else { /* Default: reservoir, Common.slangh:136-153, 234-247 */
        uint32_t slot = (*count)++;
        if (*count > N) slot = (uint32_t)(rng * (float)*count);
        if (slot < N && !(depths[slot] <= t) && !af) depths[slot] = t;
        return *count >= p->max_count;
    }
}

/* ---- traversal-order any-hit stream (rsd.h RSD_HIT_ORDER_TRAVERSAL) ----------------------
 * DXR's any-hit order is the driver's traversal order (third-party, not in the reference), so
 * librsd DEFINES one: a depth-first walk of its own 4-wide BVH (exported by rsd_scene_export_bvh),
 * children nearest entry distance first, leaf triangles in record order, each triangle once; a
 * committed hit sets TMax = t and later candidates must satisfy t < TMax (RayTCurrent()).  This
 * restates that definition (librsd csrc/sd_trace.hip sd_trace_ordered_ray, box test
 * csrc/bvh_traverse.h box_hit) over the same tree, so the GPU result is checked bit for bit;
 * the per-hit algorithm is the reference's (o_any_hit). */
typedef struct { float invd[3], oinvd[3]; } obox_ray;

static void o_box_setup(obox_ray* b, const float o[3], const float d[3])
{
    for (int i = 0; i < 3; ++i) {
        const float v = fabsf(d[i]) > 1e-20f ? d[i] : copysignf(1e-20f, d[i]); /* axis-parallel rays */
        b->invd[i] = 1.0f / v;
        b->oinvd[i] = o[i] * b->invd[i];
    }
}

/* conservative slab test, entry/exit widened by a relative 1e-5 (librsd box_hit) */
static int o_box4(const obox_ray* b, float lox, float hix, float loy, float hiy, float loz, float hiz, float tlo,
                  float thi, float* tnear)
{
    const float x0 = fmaf(lox, b->invd[0], -b->oinvd[0]), x1 = fmaf(hix, b->invd[0], -b->oinvd[0]);
    const float y0 = fmaf(loy, b->invd[1], -b->oinvd[1]), y1 = fmaf(hiy, b->invd[1], -b->oinvd[1]);
    const float z0 = fmaf(loz, b->invd[2], -b->oinvd[2]), z1 = fmaf(hiz, b->invd[2], -b->oinvd[2]);
    float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    const float m = 1e-5f * (fabsf(tn) + fabsf(tf));
    tn -= m;
    tf += m;
    *tnear = tn;
    return fmaxf(tn, tlo) <= fminf(tf, thi);
}

static void o_cswap4(float* k, uint32_t* it, int a, int b)
{
    if (k[b] < k[a]) {
        const float t = k[a]; k[a] = k[b]; k[b] = t;
        const uint32_t u = it[a]; it[a] = it[b]; it[b] = u;
    }
}

/* Walks one SD ray; returns the number of hits delivered to the any-hit algorithm. */
static uint64_t o_ordered_walk(const oscene* s, const float* bvh, uint32_t triOff, const ocam* c,
                               const osd_params* p, const float d[3], float TMin, float TMax, float cosT,
                               float spread, const int32_t* lutIdx, const uint32_t* lut, float* depths,
                               uint32_t* count)
{
    const uint32_t LEAF = 0x80000000u, OFF = 0x1fffffffu, NONE = 0xffffffffu;
    const uint32_t N = p->sample_count;
    oray r;
    o_ray_setup(&r, c->posW, d);
    obox_ray b;
    o_box_setup(&b, c->posW, d);
    uint32_t stItem[128];
    float stT[128];
    int sp = 0, committed = 0;
    float tCur = TMax;
    uint64_t delivered = 0;
    uint32_t item = 0; /* root */
    for (;;) {
        const uint32_t off = item & OFF;
        uint32_t next = NONE;
        if (item & LEAF) {
            const uint32_t n = ((item >> 29) & 3u) + 1u;
            for (uint32_t q = 0; q < n; ++q) {
                const float* tp = bvh + 4u * (off + 3u * q); /* {v0, prim}{v1, flags}{v2, 0} */
                float t, bu, bv, det;
                if (!o_intersect_tri(&r, tp, tp + 4, tp + 8, &t, &bu, &bv, &det)) continue;
                if (!(t >= TMin) || (committed ? !(t < tCur) : !(t <= tCur))) continue;
                const uint32_t prim = o_asuint(tp[3]), flags = o_asuint(tp[7]);
                if (o_culled(det, flags, p->cull_mode)) continue; /* ray flags: before any-hit */
                delivered++;
                const float rng = ocpu_hash(bu, bv);
                float z = t * cosT; /* RayToViewDepth */
                if (p->normalize) z = o_saturate((z - c->nearZ) / (c->farZ - c->nearZ));
                const int af = p->alpha_test && o_alpha_masked(s, prim) &&
                               ocpu_alpha_fails(s, prim, bu, bv, 1, t, d, spread);
                if (o_any_hit(p, N, lutIdx, lut, depths, count, rng, z, af)) {
                    tCur = t; /* AcceptHit: TMax = t */
                    committed = 1;
                }
            }
        } else {
            const float* nb = bvh + 4u * off; /* lo.x[4] hi.x[4] lo.y[4] hi.y[4] lo.z[4] hi.z[4] ref[4] cnt[4] */
            float k[4];
            uint32_t it[4];
            int m = 0;
            for (int q = 0; q < 4; ++q) {
                const uint32_t ref = o_asuint(nb[24 + q]), cnt = o_asuint(nb[28 + q]);
                float tn = 0.0f;
                const int hit = ref != NONE && o_box4(&b, nb[q], nb[4 + q], nb[8 + q], nb[12 + q], nb[16 + q],
                                                      nb[20 + q], TMin, tCur, &tn);
                k[q] = hit ? tn : INFINITY;
                it[q] = hit ? (cnt ? (LEAF | ((cnt - 1u) << 29) | (triOff + 3u * ref)) : 8u * ref) : NONE;
                m += hit;
            }
            o_cswap4(k, it, 0, 1); o_cswap4(k, it, 2, 3);
            o_cswap4(k, it, 0, 2); o_cswap4(k, it, 1, 3);
            o_cswap4(k, it, 1, 2);
            next = it[0];
            for (int q = m - 1; q >= 1; --q) { /* the nearest of the rest on top */
                if (sp >= 128) abort();
                stItem[sp] = it[q];
                stT[sp] = k[q];
                ++sp;
            }
        }
        if (next == NONE) {
            while (sp > 0) {
                --sp;
                if (stT[sp] <= tCur) { next = stItem[sp]; break; }
            }
            if (next == NONE) break;
        }
        item = next;
    }
    return delivered;
}

/* ---- wavefront any-hit stream (rsd.h RSD_HIT_ORDER_WAVEFRONT) -------------------------------
 * The other order librsd defines (librsd csrc/sd_trace.hip sd_trace_wavefront_kernel): the canonical row walk's
 * traversal of the exported 4-wide BVH, 8 work items per step.  Per step every held item is tested against the
 * TMax of the step's start (a node's 4 children, sorted by entry distance with the 5-exchange network; a leaf's
 * triangles); the step's candidate hits go to any-hit in lane order, a leaf's triangles in record order, each
 * against the current TMax with the commit rule of o_ordered_walk; then each lane's children with entry
 * distance <= TMax are pushed, lane after lane, nearest on top of its own group, onto a LIFO pool, and the next
 * step pops min(pool, pool <= soft ? 8 : 1) entries into lanes 0.. (an entry beyond TMax pops as nothing).
 * The walk starts with the root in lane 0 and ends when the pool and the lanes are empty. */
static uint64_t o_wavefront_walk(const oscene* s, const float* bvh, uint32_t triOff, uint32_t soft, const ocam* c,
                                 const osd_params* p, const float d[3], float TMin, float TMax, float cosT,
                                 float spread, const int32_t* lutIdx, const uint32_t* lut, float* depths,
                                 uint32_t* count)
{
    enum { LANES = 8, POOL = 256 };
    const uint32_t LEAF = 0x80000000u, OFF = 0x1fffffffu, NONE = 0xffffffffu;
    const uint32_t N = p->sample_count;
    oray r;
    o_ray_setup(&r, c->posW, d);
    obox_ray b;
    o_box_setup(&b, c->posW, d);
    uint32_t poolItem[POOL];
    float poolT[POOL];
    int pool = 0, committed = 0;
    float tCur = TMax;
    uint64_t delivered = 0;
    uint32_t item[LANES];
    for (int l = 0; l < LANES; ++l) item[l] = NONE;
    item[0] = 0; /* root */
    for (;;) {
        const float thi0 = tCur;
        float ck[LANES][4];
        uint32_t ci[LANES][4];
        int nc[LANES];
        for (int l = 0; l < LANES; ++l) {
            nc[l] = 0;
            for (int j = 0; j < 4; ++j) { ck[l][j] = INFINITY; ci[l][j] = NONE; }
            if (item[l] == NONE || (item[l] & LEAF)) continue;
            const float* nb = bvh + 4u * (item[l] & OFF);
            for (int q = 0; q < 4; ++q) {
                const uint32_t ref = o_asuint(nb[24 + q]), cnt = o_asuint(nb[28 + q]);
                float tn = 0.0f;
                const int hit = ref != NONE && o_box4(&b, nb[q], nb[4 + q], nb[8 + q], nb[12 + q], nb[16 + q],
                                                      nb[20 + q], TMin, thi0, &tn);
                ck[l][q] = hit ? tn : INFINITY;
                ci[l][q] = hit ? (cnt ? (LEAF | ((cnt - 1u) << 29) | (triOff + 3u * ref)) : 8u * ref) : NONE;
                nc[l] += hit;
            }
            o_cswap4(ck[l], ci[l], 0, 1); o_cswap4(ck[l], ci[l], 2, 3);
            o_cswap4(ck[l], ci[l], 0, 2); o_cswap4(ck[l], ci[l], 1, 3);
            o_cswap4(ck[l], ci[l], 1, 2);
        }
        /* the step's leaf candidates, tested against thi0, delivered lane by lane */
        for (int l = 0; l < LANES; ++l) {
            if (item[l] == NONE || !(item[l] & LEAF)) continue;
            const uint32_t off = item[l] & OFF, n = ((item[l] >> 29) & 3u) + 1u;
            float ct[4], cr[4], cz[4];
            int cv[4], caf[4];
            for (uint32_t q = 0; q < 4; ++q) {
                cv[q] = 0;
                if (q >= n) continue;
                const float* tp = bvh + 4u * (off + 3u * q);
                float t, bu, bv, det;
                if (!o_intersect_tri(&r, tp, tp + 4, tp + 8, &t, &bu, &bv, &det)) continue;
                if (!(t >= TMin) || !(t <= thi0)) continue;
                const uint32_t prim = o_asuint(tp[3]), flags = o_asuint(tp[7]);
                if (o_culled(det, flags, p->cull_mode)) continue; /* ray flags: before any-hit */
                cv[q] = 1;
                ct[q] = t;
                cr[q] = ocpu_hash(bu, bv);
                float z = t * cosT; /* RayToViewDepth */
                if (p->normalize) z = o_saturate((z - c->nearZ) / (c->farZ - c->nearZ));
                cz[q] = z;
                caf[q] = p->alpha_test && o_alpha_masked(s, prim) && ocpu_alpha_fails(s, prim, bu, bv, 1, t, d, spread);
            }
            for (uint32_t q = 0; q < 4; ++q) {
                if (!cv[q] || (committed ? !(ct[q] < tCur) : !(ct[q] <= tCur))) continue;
                delivered++;
                if (o_any_hit(p, N, lutIdx, lut, depths, count, cr[q], cz[q], caf[q])) {
                    tCur = ct[q]; /* AcceptHit: TMax = t */
                    committed = 1;
                }
            }
        }
        /* push: lane l's kept children above lanes 0..l-1's, its nearest child on top of its group */
        const float thi = tCur;
        int pre = 0;
        for (int l = 0; l < LANES; ++l) {
            int keep = 0;
            for (int j = 0; j < 4; ++j) keep += (j < nc[l] && ck[l][j] <= thi) ? 1 : 0;
            if (pool + pre + keep > POOL) abort(); /* librsd's pool bound makes this unreachable */
            for (int j = 0; j < keep; ++j) {
                poolItem[pool + pre + (keep - 1 - j)] = ci[l][j];
                poolT[pool + pre + (keep - 1 - j)] = ck[l][j];
            }
            pre += keep;
        }
        pool += pre;
        /* pop */
        const int lim = pool <= (int)soft ? LANES : 1, take = pool < lim ? pool : lim;
        int any = 0;
        for (int l = 0; l < LANES; ++l) {
            item[l] = NONE;
            if (l < take) {
                const uint32_t it = poolItem[pool - 1 - l];
                item[l] = poolT[pool - 1 - l] <= thi ? it : NONE;
            }
            any |= item[l] != NONE;
        }
        pool -= take;
        if (pool == 0 && !any) break;
    }
    return delivered;
}

typedef struct {
    const oscene* s; const ocam* c; const osd_params* p;
    const float* z; uint32_t zW, zH;
    const uint32_t* rmin; const uint32_t* rmax;
    float* sd; uint32_t sdW, sdH;
    uint32_t y0, y1;
    uint32_t bi, bc; /* band: 8-row tile rows t with t % bc == bi */
    uint64_t active, hits;
    const float* bvh; uint32_t triOff; /* p->hit_order 1 / 2: librsd's exported BVH */
    uint32_t soft;                      /* p->hit_order 2: librsd's pool bound (rsd.h WAVEFRONT) */
} osd_job;

static void* o_sd_rows(void* arg)
{
    osd_job* j = (osd_job*)arg;
    const ocam* c = j->c;
    const osd_params* p = j->p;
    const uint32_t N = p->sample_count;
    const float DEFAULT = p->normalize ? 1.0f : 3.40282347e+37f; /* Common.slangh:16 */
    const uint32_t ch = N < 4 ? N : 4, layers = (N + 3) / 4;
    const float spread = ocpu_ray_cone_spread(c->focalLength, j->sdH); /* default dims = SD map */

    int32_t lutIdx[33];
    uint32_t* lut = NULL;
    if (p->implementation == 1) {
        lut = (uint32_t*)malloc(sizeof(uint32_t) << N);
        ocpu_stratified_lut((int)N, lutIdx, lut);
    }

    for (uint32_t y = j->y0; y < j->y1; ++y)
        for (uint32_t x = 0; x < j->sdW; ++x) {
            if ((y / 8u) % j->bc != j->bi) break;
            float d[3], TMin, TMax, cosT;
            o_sd_ray(c, p, j->z, j->zW, j->zH, j->rmin, j->rmax, j->sdW, j->sdH, x, y, d, &TMin, &TMax, &cosT);

            /* ---- rayGen payload init, StochasticDepthMapRT.rt.slang:74-80 ---- */
            float depths[16];
            for (uint32_t i = 0; i < N; ++i) depths[i] = DEFAULT;
            uint32_t count = 0;

            if (TMin <= TMax && p->hit_order == 2) {
                j->active++;
                j->hits += o_wavefront_walk(j->s, j->bvh, j->triOff, j->soft, c, p, d, TMin, TMax, cosT, spread, lutIdx,
                                            lut, depths, &count);
            } else if (TMin <= TMax && p->hit_order == 1) {
                j->active++;
                j->hits += o_ordered_walk(j->s, j->bvh, j->triOff, c, p, d, TMin, TMax, cosT, spread, lutIdx, lut,
                                          depths, &count);
            } else if (TMin <= TMax) {
                j->active++;
                oray r;
                o_ray_setup(&r, c->posW, d);
                ohits hs = {0};
                /* Default / KBuffer always commit by the MAX_COUNT-th hit */
                hs.limit = (p->implementation == 1) ? 0u : (p->max_count ? p->max_count : 1u);
                o_collect(j->s, &r, TMin, TMax, p->cull_mode, 0, &hs);
                /* ---- anyHit -> algorithm, Common.slangh:102-254, ascending (t, prim) ---- */
                for (uint32_t k = 0; k < hs.n; ++k) {
                    j->hits++;
                    float rng = ocpu_hash(hs.h[k].u, hs.h[k].v);
                    float t = hs.h[k].t * cosT; /* RayToViewDepth */
                    if (p->normalize) t = o_saturate((t - c->nearZ) / (c->farZ - c->nearZ));
                    /* USE_ALPHA_TEST, Common.slangh:155-175: ray-cone LOD at RayTCurrent() */
                    const int af = p->alpha_test && o_alpha_masked(j->s, hs.h[k].prim) &&
                                   ocpu_alpha_fails(j->s, hs.h[k].prim, hs.h[k].u, hs.h[k].v, 1, hs.h[k].t, d, spread);
                    if (o_any_hit(p, N, lutIdx, lut, depths, &count, rng, t, af))
                        break; /* committed hit: TMax = t, stream ends */
                }
                free(hs.h);
            }

            /* ---- store, StochasticDepthMapRT.rt.slang:90-104 ---- */
            for (uint32_t l = 0; l < layers; ++l)
                for (uint32_t k = 0; k < ch; ++k) {
                    size_t o = (((size_t)l * j->sdH + y) * j->sdW + x) * ch + k;
                    j->sd[o] = depths[l * 4 + k];
                }
        }
    free(lut);
    return NULL;
}

static void o_sd_setrows(void* j, uint32_t a, uint32_t b) { ((osd_job*)j)->y0 = a; ((osd_job*)j)->y1 = b; }

void ocpu_sd_trace(const oscene* s, const ocam* cam, const osd_params* p,
                   const float* linearZ, uint32_t zW, uint32_t zH,
                   const uint32_t* rayMin, const uint32_t* rayMax,
                   float* sd, uint32_t sdW, uint32_t sdH,
                   uint32_t row0, uint32_t row1, int nthreads, uint64_t* stats)
{
    ocpu_sd_trace_band(s, cam, p, linearZ, zW, zH, rayMin, rayMax, sd, sdW, sdH, row0, row1, 0, 1, nthreads, stats);
}

static void o_sd_trace_impl(const oscene* s, const float* bvh, uint32_t triOff, uint32_t soft, const ocam* cam,
                            const osd_params* p, const float* linearZ, uint32_t zW, uint32_t zH,
                            const uint32_t* rayMin, const uint32_t* rayMax, float* sd, uint32_t sdW, uint32_t sdH,
                            uint32_t row0, uint32_t row1, uint32_t band_index, uint32_t band_count, int nthreads,
                            uint64_t* stats);

void ocpu_sd_trace_band(const oscene* s, const ocam* cam, const osd_params* p,
                        const float* linearZ, uint32_t zW, uint32_t zH,
                        const uint32_t* rayMin, const uint32_t* rayMax,
                        float* sd, uint32_t sdW, uint32_t sdH,
                        uint32_t row0, uint32_t row1, uint32_t band_index, uint32_t band_count,
                        int nthreads, uint64_t* stats)
{
    osd_params q = *p;
    q.hit_order = 0; /* the canonical stream (ocpu_sd_trace_ordered for the traversal order) */
    o_sd_trace_impl(s, NULL, 0, 0, cam, &q, linearZ, zW, zH, rayMin, rayMax, sd, sdW, sdH, row0, row1, band_index,
                    band_count, nthreads, stats);
}

void ocpu_sd_trace_ordered(const oscene* s, const float* bvh, uint32_t tri_offset, const ocam* cam,
                           const osd_params* p, const float* linearZ, uint32_t zW, uint32_t zH,
                           const uint32_t* rayMin, const uint32_t* rayMax, float* sd, uint32_t sdW, uint32_t sdH,
                           uint32_t row0, uint32_t row1, uint32_t band_index, uint32_t band_count, int nthreads,
                           uint64_t* stats)
{
    osd_params q = *p;
    q.hit_order = 1;
    o_sd_trace_impl(s, bvh, tri_offset, 0, cam, &q, linearZ, zW, zH, rayMin, rayMax, sd, sdW, sdH, row0, row1,
                    band_index, band_count, nthreads, stats);
}

void ocpu_sd_trace_wavefront(const oscene* s, const float* bvh, uint32_t tri_offset, uint32_t pool_soft,
                             const ocam* cam, const osd_params* p, const float* linearZ, uint32_t zW, uint32_t zH,
                             const uint32_t* rayMin, const uint32_t* rayMax, float* sd, uint32_t sdW, uint32_t sdH,
                             uint32_t row0, uint32_t row1, uint32_t band_index, uint32_t band_count, int nthreads,
                             uint64_t* stats)
{
    osd_params q = *p;
    q.hit_order = 2;
    o_sd_trace_impl(s, bvh, tri_offset, pool_soft, cam, &q, linearZ, zW, zH, rayMin, rayMax, sd, sdW, sdH, row0, row1,
                    band_index, band_count, nthreads, stats);
}

static void o_sd_trace_impl(const oscene* s, const float* bvh, uint32_t triOff, uint32_t soft, const ocam* cam,
                            const osd_params* p, const float* linearZ, uint32_t zW, uint32_t zH,
                            const uint32_t* rayMin, const uint32_t* rayMax, float* sd, uint32_t sdW, uint32_t sdH,
                            uint32_t row0, uint32_t row1, uint32_t band_index, uint32_t band_count, int nthreads,
                            uint64_t* stats)
{
    if (nthreads < 1) nthreads = 1;
    osd_job* jobs = (osd_job*)calloc((size_t)nthreads, sizeof(osd_job));
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].s = s; jobs[i].c = cam; jobs[i].p = p;
        jobs[i].z = linearZ; jobs[i].zW = zW; jobs[i].zH = zH;
        jobs[i].rmin = rayMin; jobs[i].rmax = rayMax;
        jobs[i].sd = sd; jobs[i].sdW = sdW; jobs[i].sdH = sdH;
        jobs[i].bi = band_index; jobs[i].bc = band_count ? band_count : 1;
        jobs[i].bvh = bvh; jobs[i].triOff = triOff; jobs[i].soft = soft;
    }
    if (row1 > sdH) row1 = sdH;
    o_run_rows(o_sd_rows, jobs, sizeof(osd_job), row0, row1, nthreads, o_sd_setrows);
    if (stats) {
        stats[0] = stats[1] = 0;
        for (int i = 0; i < nthreads; ++i) { stats[0] += jobs[i].active; stats[1] += jobs[i].hits; }
    }
    free(jobs);
}

/* ------------------------------------------------------------------ SVAO */
typedef struct {
    const ocam* c; const ovao* d; const osvao_params* p;
    const float* depth; const uint16_t* normals; uint32_t W, H;
    float sinNoise[16], cosNoise[16];
    uint32_t nd;  /* NUM_DIRECTIONS: 8, 16, 32 */
    float sinDir[32], cosDir[32];
    uint32_t hbao;  /* AO_KERNEL == AO_KERNEL_HBAO */
    uint32_t dual;  /* PRIMARY_DEPTH_MODE == DEPTH_MODE_DUAL (gDepthTex2 = p->depth2) */
    float hbaoPdf[32]; /* HBAO pdf of direction i: 0.9 * pow(1 - sampleRadius[i], 1.5) (Common.slang:364) */
} octx;

/* the SVAO stencil texel (SVAO.cpp:132-134): R8Uint / R16Uint / R32Uint for 8 / 16 / 32 directions,
 * NUM_DIRECTIONS / 8 bytes per pixel, little-endian */
static uint32_t o_stencil_get(const uint8_t* st, size_t i, uint32_t nd)
{
    if (nd == 32) { uint32_t v; memcpy(&v, st + 4 * i, 4); return v; }
    if (nd == 16) { uint16_t v; memcpy(&v, st + 2 * i, 2); return v; }
    return st[i];
}
static void o_stencil_set(uint8_t* st, size_t i, uint32_t nd, uint32_t v)
{
    if (nd == 32) memcpy(st + 4 * i, &v, 4);
    else if (nd == 16) { uint16_t h = (uint16_t)v; memcpy(st + 2 * i, &h, 2); }
    else st[i] = (uint8_t)v;
}

typedef struct {
    float posV[3]; float posVLength;
    float normal[3], tangent[3], bitangent[3], normalO[3], normalV[3];
    float radiusInPixels, radius;
} obasic;

typedef struct {
    float sphereStart, sphereEnd, pdf;
    int isInScreen;
    float samplePosUV[2], rasterSamplePosUV[2];
    float visibility, objectSpaceZ;
    float initialSamplePosLength, radius;
    float initialSamplePosV[3];
    float screenSpaceRadius;
} osample;

static void o_ctx_init(octx* x, const ocam* c, const ovao* d, const osvao_params* p,
                       const float* depth, const uint16_t* normals, uint32_t W, uint32_t H)
{
    x->c = c; x->d = d; x->p = p; x->depth = depth; x->normals = normals; x->W = W; x->H = H;
    uint8_t noise[16];
    ocpu_noise_texture(noise);
    for (int i = 0; i < 16; ++i) {
        float rr = o_unorm8_to_float(noise[i]) * 2.0f * 3.141f; /* Common.slang:311 */
        x->sinNoise[i] = o_sin(rr);
        x->cosNoise[i] = o_cos(rr);
    }
    x->nd = p->num_directions == 16 || p->num_directions == 32 ? p->num_directions : 8u;
    x->hbao = p->ao_kernel == 1;
    x->dual = p->primary_depth_mode == 1 && p->depth2;
    for (uint32_t i = 0; i < x->nd; ++i) {
        float a = ((float)i / (float)x->nd) * 2.0f * 3.141f; /* Common.slang:357 */
        x->sinDir[i] = o_sin(a);
        x->cosDir[i] = o_cos(a);
        x->hbaoPdf[i] = 0.9f * o_pow(1.0f - o_radius_table_k(x->nd, 1)[i], 1.5f);
    }
}

/* Common.slang:139-144 */
static void o_uv_to_view(const octx* x, float u, float v, float z, float out[3])
{
    float ndcx = u * 2.0f - 1.0f, ndcy = (1.0f - v) * 2.0f - 1.0f;
    float isx = 0.5f * (x->c->frameWidth / x->c->focalLength);
    float isy = 0.5f * (x->c->frameHeight / x->c->focalLength);
    out[0] = ndcx * z * isx;
    out[1] = ndcy * z * isy;
    out[2] = -z;
}
/* Common.slang:148-153 */
static void o_view_to_uv(const octx* x, const float p[3], float uv[2])
{
    float isx = 0.5f * (x->c->frameWidth / x->c->focalLength);
    float isy = 0.5f * (x->c->frameHeight / x->c->focalLength);
    float ndcx = p[0] / (isx * p[2]), ndcy = p[1] / (isy * p[2]);
    uv[0] = ndcx * -0.5f + 0.5f;
    uv[1] = ndcy * 0.5f + 0.5f;
}

static float o_depth_sample(const octx* x, float u, float v)
{
    return o_bilinear(x->depth, (int)x->W, (int)x->H, u, v, 0);
}

/* Common.slang:285-324 BasicAOData::Init */
static int o_basic_init(const octx* x, float u, float v, obasic* b)
{
    const ovao* d = x->d;
    float z = o_depth_sample(x, u, v);
    /* GetAORadiusInPixels, Common.slang:247-261 */
    float rux = (d->radius * x->c->focalLength) / (x->c->frameWidth * z);
    float ruy = (d->radius * x->c->focalLength) / (x->c->frameHeight * z);
    float a = rux * d->resolution[0], bb = ruy * d->resolution[1];
    b->radiusInPixels = a + 0.5f * (bb - a); /* lerp(a, b, 0.5) */
    b->radius = d->radius;
    float maxRadius = d->ssMaxRadius;
    if (b->radiusInPixels > maxRadius) {
        b->radius = b->radius / b->radiusInPixels * maxRadius;
        b->radiusInPixels = maxRadius;
    }
    if (b->radiusInPixels < 0.5f) return 0;
    o_uv_to_view(x, u, v, z, b->posV);
    b->posVLength = o_len(b->posV);
    /* loadNormal, Common.slang:98-103: integer load at uint2(texC * resolution) */
    uint32_t ix = (uint32_t)(u * d->resolution[0]), iy = (uint32_t)(v * d->resolution[1]);
    uint32_t packed = (ix < x->W && iy < x->H) ? x->normals[(size_t)iy * x->W + ix] : 0u;
    ocpu_decode_normal_2x8(packed, b->normalV);
    if (o_dot(b->posV, b->normalV) > 0.0f)
        for (int k = 0; k < 3; ++k) b->normalV[k] = -b->normalV[k];
    /* noise: point sampler, wrap, 4x4 texture at texC * noiseScale */
    float nu = u * d->noiseScale[0], nv = v * d->noiseScale[1];
    int ni = ((int)floorf(nu * 4.0f)) & 3, nj = ((int)floorf(nv * 4.0f)) & 3;
    float rd[3] = {x->sinNoise[nj * 4 + ni], x->cosNoise[nj * 4 + ni], 0.0f};
    float il = 1.0f / b->posVLength; (void)il;
    for (int k = 0; k < 3; ++k) b->normal[k] = -b->posV[k] / b->posVLength;
    float t[3];
    o_cross(b->normal, rd, t);
    o_normalize(t, b->bitangent);
    o_cross(b->bitangent, b->normal, b->tangent);
    b->normalO[0] = o_dot(b->normalV, b->tangent);
    b->normalO[1] = o_dot(b->normalV, b->bitangent);
    b->normalO[2] = o_dot(b->normalV, b->normal);
    return 1;
}

/* Common.slang:170-174 */
static float o_make_nonzero(float v, float eps)
{
    float a = o_max(fabsf(v), eps);
    return v >= 0.0f ? a : -a;
}

/* Common.slang:354-399 SampleAOData::Init (VAO kernel) */
static int o_sample_init(const octx* x, float u, float v, const obasic* b, uint32_t i, osample* s)
{
    const ovao* d = x->d;
    s->radius = o_radius_table_k(x->nd, x->hbao)[i] * b->radius;
    float dir[2] = {s->radius * x->sinDir[i], s->radius * x->cosDir[i]};
    float sphereHeight = sqrtf(b->radius * b->radius - s->radius * s->radius);
    s->pdf = x->hbao ? x->hbaoPdf[i] : 2.0f * sphereHeight; /* Common.slang:362-365 */
    s->sphereStart = sphereHeight;
    s->sphereEnd = -sphereHeight;
    float zi = -(dir[0] * b->normalO[0] + dir[1] * b->normalO[1]) / o_make_nonzero(b->normalO[2], 0.0001f);
    float zc = o_min(o_max(zi, -sphereHeight), sphereHeight);
    s->sphereEnd = zc;
    if ((s->sphereStart - s->sphereEnd) / (2.0f * sphereHeight) <= 0.1f) return 0;
    for (int k = 0; k < 3; ++k) s->initialSamplePosV[k] = b->posV[k] + b->tangent[k] * dir[0] + b->bitangent[k] * dir[1];
    s->initialSamplePosLength = o_len(s->initialSamplePosV);
    o_view_to_uv(x, s->initialSamplePosV, s->samplePosUV);
    s->visibility = 0.0f;
    s->objectSpaceZ = 0.0f;
    float dd[2] = {(u - s->samplePosUV[0]) * d->resolution[0], (v - s->samplePosUV[1]) * d->resolution[1]};
    s->screenSpaceRadius = sqrtf(dd[0] * dd[0] + dd[1] * dd[1]);
    float su = o_saturate(s->samplePosUV[0]), sv = o_saturate(s->samplePosUV[1]);
    s->isInScreen = (s->samplePosUV[0] == su) && (s->samplePosUV[1] == sv);
    /* getSnappedUV, Common.slang:116-120 */
    s->rasterSamplePosUV[0] = (floorf(su * d->resolution[0]) + 0.5f) / d->resolution[0];
    s->rasterSamplePosUV[1] = (floorf(sv * d->resolution[1]) + 0.5f) / d->resolution[1];
    return 1;
}

/* Common.slang:180-196 */
static float o_calc_visibility(const ovao* d, float oz, float ss, float se, float pdf, float radius)
{
    float sphere = o_max(ss - o_max(se, oz), 0.0f) / pdf;
    float halo = o_saturate((oz - (1.0f + d->thickness) * radius) / ss) * (ss - se) / pdf;
    return sphere + halo;
}

/* Common.slang:421-430 HBAOKernel (gData.radius: the VAOData radius, not the pixel's clamped one) */
static float o_hbao_kernel(const octx* x, const obasic* b, const float S[3])
{
    float V[3] = {S[0] - b->posV[0], S[1] - b->posV[1], S[2] - b->posV[2]};
    const float NdotVBias = 0.1f;
    float nV[3];
    o_normalize(V, nV);
    float angleTerm = o_saturate(o_dot(b->normalV, nV) - NdotVBias);
    float distanceTerm = o_saturate(1.0f - o_dot(V, V) / (x->d->radius * x->d->radius));
    return angleTerm * distanceTerm;
}

/* Common.slang:463-483 addSample: VAO (min of calcVisibility) or HBAO (max of the kernel / pdf) */
static void o_add_sample(const octx* x, const obasic* b, osample* s, const float spV[3], int init)
{
    float diff[3] = {spV[0] - b->posV[0], spV[1] - b->posV[1], spV[2] - b->posV[2]};
    float oz = o_dot(diff, b->normal);
    s->objectSpaceZ = init ? oz : o_min(s->objectSpaceZ, oz);
    if (x->hbao) {
        float v = o_saturate(o_hbao_kernel(x, b, spV) / s->pdf);
        s->visibility = init ? v : o_max(s->visibility, v);
        return;
    }
    float vis = o_calc_visibility(x->d, oz, s->sphereStart, s->sphereEnd, s->pdf, b->radius);
    s->visibility = init ? vis : o_min(s->visibility, vis);
}

/* Common.slang:455-461 requireRay (VAO with CONST_RADIUS, Common.slang:37; HBAO) */
static int o_require_ray(const octx* x, const obasic* b, const osample* s)
{
    const ovao* d = x->d;
    if (x->hbao)
        return s->objectSpaceZ > o_max(s->sphereStart, b->radius * 0.1f) && s->screenSpaceRadius > d->ssRadiusCutoff;
    float constRadius = (1.0f + d->thickness) * b->radius - s->sphereStart;
    return s->objectSpaceZ > s->sphereStart + constRadius && s->screenSpaceRadius > d->ssRadiusCutoff;
}

/* Common.slang:492-496 evalPrimaryVisibility */
static void o_eval_primary(const octx* x, const obasic* b, osample* s)
{
    float z = o_depth_sample(x, s->rasterSamplePosUV[0], s->rasterSamplePosUV[1]);
    float spV[3];
    o_uv_to_view(x, s->rasterSamplePosUV[0], s->rasterSamplePosUV[1], z, spV);
    o_add_sample(x, b, s, spV, 1);
}

/* Common.slang:498-505 evalDualVisibility: the second depth layer (gDepthTex2) at the same texel,
 * only where the sample still requires a ray */
static void o_eval_dual(const octx* x, const obasic* b, osample* s, int init)
{
    if (!o_require_ray(x, b, s)) return;
    float z = o_bilinear(x->p->depth2, (int)x->W, (int)x->H, s->rasterSamplePosUV[0], s->rasterSamplePosUV[1], 0);
    float spV[3];
    o_uv_to_view(x, s->rasterSamplePosUV[0], s->rasterSamplePosUV[1], z, spV);
    o_add_sample(x, b, s, spV, init);
}

/* Common.slang:326-330 finalize */
static float o_finalize(const octx* x, float avgAO)
{
    if (x->hbao) avgAO = o_saturate(1.0f - 2.0f * avgAO);
    return o_pow(avgAO, x->d->exponent);
}

/* Common.slang:164-168 UVToSDPixel */
static void o_uv_to_sd_pixel(const ovao* d, const float uv[2], int out[2])
{
    for (int k = 0; k < 2; ++k) {
        int px = (int)floorf(uv[k] * d->lowResolution[k]) + d->sdGuard;
        int hi = (int)d->lowResolution[k] + d->sdGuard * 2 - 1;
        out[k] = px < 0 ? 0 : (px > hi ? hi : px);
    }
}

void ocpu_svao_clear(uint32_t* rayMin, uint32_t* rayMax, uint32_t n)
{
    /* SVAO.cpp:334-340 */
    for (uint32_t i = 0; i < n; ++i) { rayMax[i] = 0u; rayMin[i] = o_asuint(FLT_MAX); }
}

/* SVAORaster.ps.slang:29-122 */
void ocpu_svao_pass1(const ocam* cam, const ovao* d, const osvao_params* p,
                     const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                     uint8_t* ao, uint8_t* stencil, uint32_t* rayMin, uint32_t* rayMax,
                     uint32_t sdW, uint32_t sdH)
{
    ocpu_svao_pass1_band(cam, d, p, depth, normals, W, H, ao, stencil, rayMin, rayMax, sdW, sdH, 0, 1);
}

static void o_pass1_impl(const ocam* cam, const ovao* d, const osvao_params* p,
                         const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                         uint8_t* ao, uint8_t* stencil, uint32_t* rayMin, uint32_t* rayMax,
                         uint32_t sdW, uint32_t sdH, uint32_t band_index, uint32_t band_count,
                         uint32_t row0, uint32_t row1);

void ocpu_svao_pass1_band(const ocam* cam, const ovao* d, const osvao_params* p,
                          const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                          uint8_t* ao, uint8_t* stencil, uint32_t* rayMin, uint32_t* rayMax,
                          uint32_t sdW, uint32_t sdH, uint32_t band_index, uint32_t band_count)
{
    o_pass1_impl(cam, d, p, depth, normals, W, H, ao, stencil, rayMin, rayMax, sdW, sdH, band_index, band_count, 0,
                 0xffffffffu);
}

/* visible rows [row0, row1) counted from the first visible row (multiples of 32, a
 * contiguous screen band: librsd rsd_svao_pass1_rows) */
void ocpu_svao_pass1_rows(const ocam* cam, const ovao* d, const osvao_params* p,
                          const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                          uint8_t* ao, uint8_t* stencil, uint32_t* rayMin, uint32_t* rayMax,
                          uint32_t sdW, uint32_t sdH, uint32_t row0, uint32_t row1)
{
    o_pass1_impl(cam, d, p, depth, normals, W, H, ao, stencil, rayMin, rayMax, sdW, sdH, 0, 1, row0, row1);
}

static void o_pass1_impl(const ocam* cam, const ovao* d, const osvao_params* p,
                         const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                         uint8_t* ao, uint8_t* stencil, uint32_t* rayMin, uint32_t* rayMax,
                         uint32_t sdW, uint32_t sdH, uint32_t band_index, uint32_t band_count,
                         uint32_t row0, uint32_t row1)
{
    if (!band_count) band_count = 1;
    octx x;
    o_ctx_init(&x, cam, d, p, depth, normals, W, H);
    const uint32_t g = p->guard_band;
    /* SVAO.cpp:347-350: dispatch roundup32(dims - 2 guardBand); the 2x2 group interleave
     * (SVAORaster.ps.slang:36) is a bijection of that range, so iterate it directly. */
    uint32_t nx = ((W - 2 * g) + 31u) / 32u * 32u, ny = ((H - 2 * g) + 31u) / 32u * 32u;
    for (uint32_t oy = row0; oy < ny && oy < row1; ++oy)
        for (uint32_t ox = 0; ox < nx; ++ox) {
            if ((oy / 32u) % band_count != band_index) break;
            uint32_t px = ox + g, py = oy + g;
            float u = ((float)px + 0.5f) * d->invResolution[0];
            float v = ((float)py + 0.5f) * d->invResolution[1];
            float aoOut = 0.0f, aoD = 0.0f; /* ao_t: bright, dark (DUAL_AO, SVAORaster.ps.slang:13) */
            uint32_t st = 0;
            obasic b;
            if (!o_basic_init(&x, u, v, &b)) {
                aoOut = aoD = 1.0f;
            } else {
                for (uint32_t i = 0; i < x.nd; ++i) {
                    osample s;
                    if (!o_sample_init(&x, u, v, &b, i, &s)) continue;
                    /* isSamePixel, Common.slang:129-134 */
                    if (fabsf(u - s.rasterSamplePosUV[0]) < d->invResolution[0] * 0.9f &&
                        fabsf(v - s.rasterSamplePosUV[1]) < d->invResolution[1] * 0.9f) {
                        if (!x.hbao) { /* SVAORaster.ps.slang:57-58: HBAO adds 0 */
                            float w = (s.sphereStart - s.sphereEnd) / s.pdf;
                            aoOut += w;
                            aoD += w;
                        }
                        continue;
                    }
                    /* SVAORaster.ps.slang:62-66: Raytraced mode with TRACE_OUT_OF_SCREEN (SVAO.h:104) */
                    int forceRay = p->secondary_depth_mode == 3 && !s.isInScreen;
                    o_eval_primary(&x, &b, &s);
                    if (x.dual) o_eval_dual(&x, &b, &s, 0); /* SVAORaster.ps.slang:69-70 */
                    aoOut += s.visibility;
                    if (!s.isInScreen && d->sdGuard > 0) {
                        forceRay = 1;
                        s.objectSpaceZ = O_FLT_MAX;
                    }
                    int req = o_require_ray(&x, &b, &s);
                    if (req || forceRay) {
                        st |= 1u << i;
                        if (p->secondary_depth_mode == 2) {
                            int pix[2];
                            o_uv_to_sd_pixel(d, s.samplePosUV, pix);
                            size_t o = (size_t)pix[1] * sdW + pix[0];
                            if (p->ray_interval) {
                                /* SVAORaster.ps.slang:90-91 */
                                float osMin = x.hbao ? o_min(s.objectSpaceZ, s.sphereStart)
                                                     : o_min(s.objectSpaceZ, b.radius + d->thickness * b.radius + s.sphereStart);
                                uint32_t rmin = o_asuint(o_max(b.posVLength - osMin, 0.0f));
                                uint32_t rmax = o_asuint(o_max(b.posVLength - s.sphereEnd, 0.0f));
                                if (rmin < rayMin[o]) rayMin[o] = rmin;
                                if (rmax > rayMax[o]) rayMax[o] = rmax;
                            } else {
                                rayMax[o] = 1u;
                            }
                        }
                    } else {
                        aoD += s.visibility; /* darkmap, SVAORaster.ps.slang:101-104 */
                    }
                }
                aoOut *= 1.0f / (float)x.nd;  /* SVAORaster.ps.slang:108-109 (x 2: VAO only) */
                aoD *= 1.0f / (float)x.nd;
                if (!x.hbao) {
                    aoOut *= 2.0f;
                    aoD *= 2.0f;
                }
                if (p->secondary_depth_mode == 0 || st == 0) {
                    aoOut = o_finalize(&x, aoOut);
                    aoD = o_finalize(&x, aoD);
                }
            }
            if (px < W && py < H) {
                if (p->dual_ao) {
                    ao[2 * ((size_t)py * W + px)] = o_unorm8(aoOut);
                    ao[2 * ((size_t)py * W + px) + 1] = o_unorm8(aoD);
                } else {
                    ao[(size_t)py * W + px] = o_unorm8(aoOut);
                }
                o_stencil_set(stencil, (size_t)py * W + px, x.nd, st);
            }
        }
    (void)sdH;
}

/* SVAORaster2.ps.slang:60-64: the direction sums * 2 / NUM_DIRECTIONS (Common.slang:660-661) plus
 * the pass-1 AO, dark = min(bright, dark) (DUAL_AO), finalize, store */
static void o_ao_finish(const octx* x, uint8_t* ao, size_t o, float vis, float visD)
{
    vis *= 1.0f / (float)x->nd;
    if (!x->hbao) vis *= 2.0f; /* Common.slang:660-661 */
    if (!x->p->dual_ao) {
        vis += o_unorm8_to_float(ao[o]);
        ao[o] = o_unorm8(o_finalize(x, vis));
        return;
    }
    visD *= 1.0f / (float)x->nd;
    if (!x->hbao) visD *= 2.0f;
    vis += o_unorm8_to_float(ao[2 * o]);
    visD += o_unorm8_to_float(ao[2 * o + 1]);
    visD = o_min(vis, visD);
    ao[2 * o] = o_unorm8(o_finalize(x, vis));
    ao[2 * o + 1] = o_unorm8(o_finalize(x, visD));
}

/* SVAORaster2.ps.slang:48-65 -> calcAO2 (Common.slang:523-663), stochastic branch */
typedef struct {
    const octx* x; const uint8_t* stencil; const float* sd; uint32_t sdW, sdH; uint8_t* ao;
    uint32_t y0, y1;
    uint32_t bi, bc; /* band: 32-row groups of visible rows */
} op2_job;

static void* o_pass2_rows(void* arg)
{
    op2_job* j = (op2_job*)arg;
    const octx* x = j->x;
    const ovao* d = x->d;
    const uint32_t g = x->p->guard_band, W = x->W, N = x->p->sd_samples;
    const uint32_t ch = N < 4 ? N : 4;
    const float depthRange = x->c->farZ - x->c->nearZ, depthOffset = x->c->nearZ;
    for (uint32_t py = j->y0; py < j->y1; ++py)
        for (uint32_t px = g; px < W - g; ++px) {
            if (((py - g) / 32u) % j->bc != j->bi) break;
            size_t o = (size_t)py * W + px;
            uint32_t mask = o_stencil_get(j->stencil, o, x->nd);
            if (mask == 0) continue;
            float u = ((float)px + 0.5f) * d->invResolution[0];
            float v = ((float)py + 0.5f) * d->invResolution[1];
            obasic b;
            o_basic_init(x, u, v, &b);
            float vis = 0.0f, visD = 0.0f; /* bright, dark (DUAL_AO) */
            for (uint32_t i = 0; i < x->nd; ++i) {
                if (!(mask & (1u << i))) continue;
                osample s;
                o_sample_init(x, u, v, &b, i, &s);
                if (x->dual) o_eval_dual(x, &b, &s, 1); /* Common.slang:555-558 (force init) */
                else o_eval_primary(x, &b, &s);
                vis -= s.visibility;
                if (x->p->secondary_depth_mode != 2) {
                    /* secondary DualDepth: calcAO2 has no branch for it (Common.slang:562-651) */
                    vis += s.visibility;
                    visD += s.visibility;
                    continue;
                }
                int pc[2];
                o_uv_to_sd_pixel(d, s.samplePosUV, pc);
                float jx = 0.5f, jy = 0.5f;
                if (x->p->sd_jitter) ocpu_jitter((uint32_t)pc[0], (uint32_t)pc[1], &jx, &jy);
                float su = ((float)(pc[0] - d->sdGuard) + jx) / d->lowResolution[0];
                float sv = ((float)(pc[1] - d->sdGuard) + jy) / d->lowResolution[1];
                if (!s.isInScreen) { s.visibility = x->hbao ? 0.0f : 1.0f; s.objectSpaceZ = O_FLT_MAX; } /* resetSample */
                for (uint32_t k = 0; k < N; ++k) {
                    size_t so = ((((size_t)(k / 4) * j->sdH) + (size_t)pc[1]) * j->sdW + (size_t)pc[0]) * ch + (k % 4);
                    float lz = j->sd[so] * depthRange + depthOffset;
                    float spV[3];
                    o_uv_to_view(x, su, sv, lz, spV);
                    o_add_sample(x, &b, &s, spV, 0);
                }
                vis += s.visibility;
                visD += s.visibility;
            }
            o_ao_finish(x, j->ao, o, vis, visD);
        }
    return NULL;
}

static void o_p2_setrows(void* j, uint32_t a, uint32_t b) { ((op2_job*)j)->y0 = a; ((op2_job*)j)->y1 = b; }

void ocpu_svao_pass2(const ocam* cam, const ovao* d, const osvao_params* p,
                     const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                     const uint8_t* stencil, const float* sd, uint32_t sdW, uint32_t sdH,
                     uint8_t* ao, int nthreads)
{
    ocpu_svao_pass2_band(cam, d, p, depth, normals, W, H, stencil, sd, sdW, sdH, ao, 0, 1, nthreads);
}

/* visible rows [row0, row1) from the first visible row (librsd rsd_svao_pass2_rows) */
void ocpu_svao_pass2_rows(const ocam* cam, const ovao* d, const osvao_params* p,
                          const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                          const uint8_t* stencil, const float* sd, uint32_t sdW, uint32_t sdH,
                          uint8_t* ao, uint32_t row0, uint32_t row1, int nthreads)
{
    octx x;
    o_ctx_init(&x, cam, d, p, depth, normals, W, H);
    if (nthreads < 1) nthreads = 1;
    op2_job* jobs = (op2_job*)calloc((size_t)nthreads, sizeof(op2_job));
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].x = &x; jobs[i].stencil = stencil; jobs[i].sd = sd;
        jobs[i].sdW = sdW; jobs[i].sdH = sdH; jobs[i].ao = ao;
        jobs[i].bi = 0; jobs[i].bc = 1;
    }
    const uint32_t y0 = p->guard_band + row0, yEnd = H - p->guard_band;
    const uint32_t y1 = row1 < yEnd - p->guard_band ? p->guard_band + row1 : yEnd;
    if (y0 < y1) o_run_rows(o_pass2_rows, jobs, sizeof(op2_job), y0, y1, nthreads, o_p2_setrows);
    free(jobs);
}

void ocpu_svao_pass2_band(const ocam* cam, const ovao* d, const osvao_params* p,
                          const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                          const uint8_t* stencil, const float* sd, uint32_t sdW, uint32_t sdH,
                          uint8_t* ao, uint32_t band_index, uint32_t band_count, int nthreads)
{
    octx x;
    o_ctx_init(&x, cam, d, p, depth, normals, W, H);
    if (nthreads < 1) nthreads = 1;
    op2_job* jobs = (op2_job*)calloc((size_t)nthreads, sizeof(op2_job));
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].x = &x; jobs[i].stencil = stencil; jobs[i].sd = sd;
        jobs[i].sdW = sdW; jobs[i].sdH = sdH; jobs[i].ao = ao;
        jobs[i].bi = band_index; jobs[i].bc = band_count ? band_count : 1;
    }
    o_run_rows(o_pass2_rows, jobs, sizeof(op2_job), p->guard_band, H - p->guard_band, nthreads, o_p2_setrows);
    free(jobs);
}

/* ------------------------------------------------------------------ SVAO pass 2, Raytraced */
/* calcAO2 DEPTH_MODE_RAYTRACING (Common.slang:598-651), traceAORay (SVAORaster2.ps.slang:9-46,
 * Ray.rt.slang:46-58) and aoAnyHit (Common.slang:679-718), replayed literally over the canonical any-hit
 * stream: every hit in [TMin, TMax] (culling applied) in ascending (t, prim) order, TMax shrinking on a
 * commit.  VAO and HBAO kernels; SingleDepth or DualDepth primary visibility. */
typedef struct {
    const oscene* s; const octx* x; const uint8_t* stencil; uint8_t* ao;
    uint32_t cull, rayPipeline, alphaTest;
    float invView[9];
    uint32_t y0, y1, bi, bc;
} ort_job;

static void* o_pass2_rt_rows(void* arg)
{
    ort_job* j = (ort_job*)arg;
    const octx* x = j->x;
    const ovao* d = x->d;
    const ocam* c = x->c;
    const uint32_t g = x->p->guard_band, W = x->W, H = x->H;
    const uint32_t xEnd = j->rayPipeline ? W : W - g; /* SVAO.cpp:429-430 vs :452-453 */
    (void)H;
    for (uint32_t py = j->y0; py < j->y1; ++py)
        for (uint32_t px = g; px < xEnd; ++px) {
            if (((py - g) / 32u) % j->bc != j->bi) break;
            size_t o = (size_t)py * W + px;
            uint32_t mask = o_stencil_get(j->stencil, o, x->nd);
            if (mask == 0) continue;
            float u = ((float)px + 0.5f) * d->invResolution[0];
            float v = ((float)py + 0.5f) * d->invResolution[1];
            obasic b;
            o_basic_init(x, u, v, &b);
            float vis = 0.0f, visD = 0.0f; /* bright, dark (DUAL_AO) */
            for (uint32_t i = 0; i < x->nd; ++i) {
                if (!(mask & (1u << i))) continue;
                osample s;
                o_sample_init(x, u, v, &b, i, &s);
                if (x->dual) o_eval_dual(x, &b, &s, 1); /* Common.slang:555-558 (force init) */
                else o_eval_primary(x, &b, &s);
                vis -= s.visibility;
                /* getSnappedUV(samplePosUV): Common.slang:116-125, no clamp */
                float suv[2] = {(floorf(s.samplePosUV[0] * d->resolution[0]) + 0.5f) / d->resolution[0],
                                (floorf(s.samplePosUV[1] * d->resolution[1]) + 0.5f) / d->resolution[1]};
                float pv[3], dv[3], dw[3];
                o_uv_to_view(x, suv[0], suv[1], 1.0f, pv);
                o_normalize(pv, dv);
                for (int k = 0; k < 3; ++k)
                    dw[k] = j->invView[k * 3 + 0] * dv[0] + j->invView[k * 3 + 1] * dv[1] + j->invView[k * 3 + 2] * dv[2];
                const float L = s.initialSamplePosLength, pl = b.posVLength;
                if (x->hbao) {
                    /* Common.slang:622-628: the ray spans [sphereStart, sphereEnd]; no RAY_FLAG_FORCE_NON_OPAQUE, so
                     * opaque triangles commit as closest hits and alpha-masked ones pass aoAnyHit (alpha test, then
                     * ACCEPT whatever the face, :695-697, 715-717): tFirst = the nearest hit of the stream */
                    float TMin = (pl - s.sphereStart) * L / pl;
                    const float TMax = (pl - s.sphereEnd) * L / pl;
                    if (!s.isInScreen) { s.visibility = 0.0f; s.objectSpaceZ = O_FLT_MAX; } /* resetSample (HBAO) */
                    const float eps = b.radius * 0.01f;
                    if (s.isInScreen) TMin = o_max(TMin, (pl - s.objectSpaceZ) * L / pl + eps);
                    float tFirst = 0.0f; /* rayData.tFirst = 0.0: a miss leaves the ray origin */
                    if (TMin <= TMax) {
                        oray r;
                        o_ray_setup(&r, c->posW, dw);
                        ohits hs = {0};
                        hs.limit = 1; /* the nearest hit only */
                        o_collect(j->s, &r, TMin, TMax, j->cull, (int)j->alphaTest, &hs);
                        if (hs.n) tFirst = hs.h[0].t; /* CommittedRayT (SVAORaster2.ps.slang:42-45) */
                        free(hs.h);
                    }
                    /* Common.slang:647-649: samplePosW = origin + dir tFirst, samplePosV = mul(viewMat, (samplePosW, 1)) */
                    float pw[3], pv[3];
                    for (int k = 0; k < 3; ++k) pw[k] = c->posW[k] + dw[k] * tFirst;
                    for (int k = 0; k < 3; ++k)
                        pv[k] = ((c->viewMat[k * 4 + 0] * pw[0] + c->viewMat[k * 4 + 1] * pw[1]) + c->viewMat[k * 4 + 2] * pw[2]) +
                                c->viewMat[k * 4 + 3];
                    o_add_sample(x, &b, &s, pv, 0);
                    vis += s.visibility;
                    visD += s.visibility;
                    continue;
                }
                /* RayData init, Common.slang:614-620 */
                float halo = (pl - s.sphereStart - b.radius - d->thickness * b.radius) * L / pl;
                float inside = (pl - s.sphereEnd) * L / pl;
                const float tCRS = (pl - b.radius - d->thickness * b.radius) * L / pl;
                const float tSS = (pl - s.sphereStart) * L / pl;
                float TMin = o_max(halo, 0.0f), TMax = inside;
                if (!s.isInScreen) { s.visibility = x->hbao ? 0.0f : 1.0f; s.objectSpaceZ = O_FLT_MAX; } /* resetSample */
                const float eps = b.radius * 0.01f;
                if (s.isInScreen) TMin = o_max(TMin, (pl - s.objectSpaceZ) * L / pl + eps);
                if (TMin <= TMax) {
                    oray r;
                    o_ray_setup(&r, c->posW, dw);
                    ohits hs = {0};
                    o_collect(j->s, &r, TMin, TMax, j->cull, (int)j->alphaTest, &hs);
                    for (uint32_t k = 0; k < hs.n; ++k) {
                        const float t = hs.h[k].t;
                        if (t > TMax) break;          /* beyond a committed hit */
                        if (t < halo) continue;       /* SVAORaster2.ps.slang:27-28 */
                        const uint32_t fl = j->s->flags[hs.h[k].prim];
                        const int front = (hs.h[k].det > 0.0f) != ((fl & 2u) != 0u);
                        if (!(front || (fl & 1u) || (fl & 4u))) continue; /* Common.slang:695-697 */
                        if (t <= tSS) {
                            halo = o_max(halo, t);
                            if (t >= tCRS) break;     /* AO_HIT_ACCEPT_AND_END */
                        } else {
                            inside = o_min(inside, t); /* AO_HIT_ACCEPT: commit */
                            TMax = t;
                        }
                    }
                    free(hs.h);
                }
                /* Common.slang:641-644 */
                float sphereVis = o_calc_visibility(d, pl - inside * pl / L, s.sphereStart, s.sphereEnd, s.pdf, b.radius);
                float haloVis = o_saturate((pl - halo * pl / L - (1.0f + d->thickness) * b.radius) / s.sphereStart) *
                                (s.sphereStart - s.sphereEnd) / s.pdf;
                s.visibility = o_min(s.visibility, o_min(sphereVis, haloVis));
                vis += s.visibility;
                visD += s.visibility;
            }
            o_ao_finish(x, j->ao, o, vis, visD);
        }
    return NULL;
}

static void o_rt_setrows(void* j, uint32_t a, uint32_t b) { ((ort_job*)j)->y0 = a; ((ort_job*)j)->y1 = b; }

void ocpu_svao_pass2_rt_band(const oscene* sc, const ocam* cam, const ovao* d, const osvao_params* p,
                             const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                             const uint8_t* stencil, uint8_t* ao, uint32_t cull, uint32_t ray_pipeline,
                             uint32_t alpha_test, uint32_t band_index, uint32_t band_count, int nthreads)
{
    octx x;
    o_ctx_init(&x, cam, d, p, depth, normals, W, H);
    if (nthreads < 1) nthreads = 1;
    ort_job* jobs = (ort_job*)calloc((size_t)nthreads, sizeof(ort_job));
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].s = sc; jobs[i].x = &x; jobs[i].stencil = stencil; jobs[i].ao = ao;
        jobs[i].cull = cull; jobs[i].rayPipeline = ray_pipeline; jobs[i].alphaTest = alpha_test;
        /* float3x3(inverse(viewMat)) = transpose of the view rotation (rigid view matrix) */
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) jobs[i].invView[r * 3 + k] = cam->viewMat[k * 4 + r];
        jobs[i].bi = band_index; jobs[i].bc = band_count ? band_count : 1;
    }
    const uint32_t g = p->guard_band, yEnd = ray_pipeline ? H : H - g;
    o_run_rows(o_pass2_rt_rows, jobs, sizeof(ort_job), g, yEnd, nthreads, o_rt_setrows);
    free(jobs);
}

/* ------------------------------------------------------------------ CrossBilateralBlur
 * CrossBilateralBlur.ps.slang:1-88 / CrossBilateralBlur.cpp:113-149: x pass into the
 * ping-pong image, y pass into dst, point sampling (clamp) at texC + d * dir / size clamped
 * to the guard band's uv bounds (GuardBand.cpp:62-63), writes inside the scissor only. */
static int o_point(float uv, int n)
{
    int t = (int)floorf(uv * (float)n);
    return t < 0 ? 0 : (t > n - 1 ? n - 1 : t);
}

static void o_blur_pass(const uint8_t* src, const float* z, int zW, int zH, uint8_t* dst, int W, int H, int g,
                        int R, int better, float dirX, float dirY)
{
    const float uvMinX = ((float)g + 0.5f) / (float)W, uvMinY = ((float)g + 0.5f) / (float)H;
    const float uvMaxX = ((float)W - ((float)g + 0.5f)) / (float)W;
    const float uvMaxY = ((float)H - ((float)g + 0.5f)) / (float)H;
    const float sigma = ((float)R + 1.0f) * 0.5f;
    const float falloff = 1.0f / (2.0f * sigma * sigma);
    float zc[41], ac[41];
    for (int y = g; y < H - g; ++y)
        for (int x = g; x < W - g; ++x) {
            const float tx = ((float)x + 0.5f) / (float)W, ty = ((float)y + 0.5f) / (float)H;
            const float ux = (1.0f / (float)W) * dirX, uy = (1.0f / (float)H) * dirY;
            for (int d = -R; d <= R; ++d) {
                float u = o_min(o_max(tx + (float)d * ux, uvMinX), uvMaxX);
                float v = o_min(o_max(ty + (float)d * uy, uvMinY), uvMaxY);
                zc[R + d] = z[(size_t)o_point(v, zH) * zW + o_point(u, zW)];
                ac[R + d] = o_unorm8_to_float(src[(size_t)o_point(v, H) * W + o_point(u, W)]);
            }
            float ao = ac[R], ws = 1.0f;
            float left = zc[R] - zc[R - 1], right = zc[R + 1] - zc[R];
            float minSlope = fabsf(left) < fabsf(right) ? left : right;
            for (int side = 0; side < 2; ++side) { /* BlurDirection(+1, minSlope), (-1, -minSlope) */
                int sgn = side ? -1 : 1;
                float slope = side ? -minSlope : minSlope;
                for (int d = 1; d <= R; ++d) {
                    float a = ac[R + sgn * d], sz = zc[R + sgn * d];
                    if (d == 1 && !better) slope = sz - zc[R];
                    sz -= slope * (float)d; /* AddSample */
                    float dz = fabsf(sz - zc[R]) * 16.0f;
                    dz = dz * 12.0f / zc[R];
                    float w = (float)exp2((double)(-(float)(d * d) * falloff - dz * dz));
                    ao += w * a;
                    ws += w;
                }
            }
            dst[(size_t)y * W + x] = o_unorm8(ao / ws);
        }
}

void ocpu_cross_bilateral_blur(const uint8_t* src, const float* z, uint32_t zW, uint32_t zH, uint8_t* pingpong,
                               uint8_t* dst, uint32_t W, uint32_t H, uint32_t g, uint32_t R, uint32_t better)
{
    o_blur_pass(src, z, (int)zW, (int)zH, pingpong, (int)W, (int)H, (int)g, (int)R, (int)better, 1.0f, 0.0f);
    o_blur_pass(pingpong, z, (int)zW, (int)zH, dst, (int)W, (int)H, (int)g, (int)R, (int)better, 0.0f, 1.0f);
}

/* ------------------------------------------------------------------ TemporalAO
 * TemporalAO.ps.slang:55-101 (TemporalAO.cpp:113-163, enabled).  gDepth / gMotionVec / gAO are
 * sampled at the pixel centre (= the texel); the previous AO is a clamped bilinear R8Unorm
 * fetch at texC + mvec (TemporalAO.cpp:73-77); prevDepth / prevHistory are loaded at the pixel
 * UVToPixel(texC + mvec); writes only inside the guard-band scissor (TemporalAO.cpp:144). */
static float o_bilinear_u8(const uint8_t* t, int W, int H, float u, float v)
{
    float x = u * (float)W - 0.5f, y = v * (float)H - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float qx = floorf((x - fx0) * 256.0f + 0.5f), qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) { ix += 1; qx = 0.0f; }
    if (qy >= 256.0f) { iy += 1; qy = 0.0f; }
    float wx = qx * (1.0f / 256.0f), wy = qy * (1.0f / 256.0f);
    int x0 = o_addr(ix, W, 0), x1 = o_addr(ix + 1, W, 0), y0 = o_addr(iy, H, 0), y1 = o_addr(iy + 1, H, 0);
    float t00 = o_unorm8_to_float(t[(size_t)y0 * W + x0]), t10 = o_unorm8_to_float(t[(size_t)y0 * W + x1]);
    float t01 = o_unorm8_to_float(t[(size_t)y1 * W + x0]), t11 = o_unorm8_to_float(t[(size_t)y1 * W + x1]);
    float r0 = t00 * (1.0f - wx) + t10 * wx, r1 = t01 * (1.0f - wx) + t11 * wx;
    return r0 * (1.0f - wy) + r1 * wy;
}

void ocpu_temporal_ao(const uint8_t* aoIn, const float* z, const float* mvec, const float* prevZ,
                      const uint8_t* prevAo, const uint8_t* prevN, const uint8_t* stable, uint32_t W_,
                      uint32_t H_, uint32_t g_, const ocam* cam, const float m[16], uint8_t* aoOut,
                      uint8_t* nOut)
{
    const int W = (int)W_, H = (int)H_, g = (int)g_;
    const float uvMinX = ((float)g + 0.5f) / (float)W, uvMinY = ((float)g + 0.5f) / (float)H;
    const float uvMaxX = ((float)W - ((float)g + 0.5f)) / (float)W;
    const float uvMaxY = ((float)H - ((float)g + 0.5f)) / (float)H;
    const float isx = 0.5f * (cam->frameWidth / cam->focalLength), isy = 0.5f * (cam->frameHeight / cam->focalLength);
    for (int y = g; y < H - g; ++y)
        for (int x = g; x < W - g; ++x) {
            const size_t o = (size_t)y * W + x;
            const float tu = ((float)x + 0.5f) / (float)W, tv = ((float)y + 0.5f) / (float)H;
            const float depth = z[o];
            float ao = o_unorm8_to_float(aoIn[o]);
            uint32_t n = 1;
            const float pu = tu + mvec[2 * o], pv = tv + mvec[2 * o + 1];
            if (pu >= uvMinX && pu <= uvMaxX && pv >= uvMinY && pv <= uvMaxY) { /* isInValidArea */
                int qx = (int)floorf(pu * (float)W), qy = (int)floorf(pv * (float)H); /* UVToPixel */
                qx = qx < 0 ? 0 : (qx > W - 1 ? W - 1 : qx);
                qy = qy < 0 ? 0 : (qy > H - 1 ? H - 1 : qy);
                const size_t po = (size_t)qy * W + qx;
                const float prevRaw = prevZ[po];
                const float ndcx = pu * 2.0f - 1.0f, ndcy = (1.0f - pv) * 2.0f - 1.0f; /* UVToViewSpace */
                const float vx = ndcx * prevRaw * isx, vy = ndcy * prevRaw * isy, vz = -prevRaw;
                const float pz = m[8] * vx + m[9] * vy + m[10] * vz + m[11];
                const float prevDepth = -pz;
                const int isStable = stable && stable[o] != 0;
                if (fabsf(1.0f - prevDepth / depth) < 0.1f && !isStable) { /* RelativeDepth */
                    const float pa = o_bilinear_u8(prevAo, W, H, pu, pv);
                    const uint32_t pn = prevN[po];
                    ao = ((float)pn * pa + ao) / (float)(pn + 1u);
                    n = pn + 1u < 30u ? pn + 1u : 30u;
                }
            }
            aoOut[o] = o_unorm8(ao);
            nOut[o] = (uint8_t)n;
        }
}

/* GBufferRaster.mvec for a static scene and a moving camera (librsd's definition, rsd_graph.h):
 * the pixel-centre primary hit from the linear depth, projected with the previous camera.
 * Background (linear depth >= farZ) -> (0, 0): GBufferRaster clears mvec (GBufferRaster.cpp:176)
 * and writes it for rasterized geometry only (GBufferRaster.3d.slang:117). */
void ocpu_motion_vectors(const ocam* c, const ocam* prev, const float* z, uint32_t W_, uint32_t H_, float* mvec)
{
    const int W = (int)W_, H = (int)H_;
    float pU[3], pV[3], pW[3], wn[3];
    const double uu = (double)prev->U[0] * prev->U[0] + (double)prev->U[1] * prev->U[1] + (double)prev->U[2] * prev->U[2];
    const double vv = (double)prev->V[0] * prev->V[0] + (double)prev->V[1] * prev->V[1] + (double)prev->V[2] * prev->V[2];
    const double ww = (double)prev->W[0] * prev->W[0] + (double)prev->W[1] * prev->W[1] + (double)prev->W[2] * prev->W[2];
    for (int k = 0; k < 3; ++k) {
        pU[k] = (float)(prev->U[k] / uu);
        pV[k] = (float)(prev->V[k] / vv);
        pW[k] = (float)(prev->W[k] / ww);
    }
    o_normalize(c->W, wn);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float u = ((float)x + 0.5f) / (float)W, v = ((float)y + 0.5f) / (float)H;
            float dn[3], d[3], rel[3];
            if (!(z[(size_t)y * W + x] < c->farZ)) {
                mvec[2 * ((size_t)y * W + x)] = 0.0f;
                mvec[2 * ((size_t)y * W + x) + 1] = 0.0f;
                continue;
            }
            for (int k = 0; k < 3; ++k) dn[k] = (2.0f * u + -1.0f) * c->U[k] + (-2.0f * v + 1.0f) * c->V[k] + c->W[k];
            o_normalize(dn, d);
            const float t = z[(size_t)y * W + x] / o_dot(wn, d);
            for (int k = 0; k < 3; ++k) rel[k] = c->posW[k] + t * d[k] - prev->posW[k];
            const float pa = o_dot(rel, pU), pb = o_dot(rel, pV), pw = o_dot(rel, pW);
            float mx = 2.0f, my = 2.0f;
            if (pw > 0.0f) { mx = (pa / pw + 1.0f) * 0.5f - u; my = (1.0f - pb / pw) * 0.5f - v; }
            mvec[2 * ((size_t)y * W + x)] = mx;
            mvec[2 * ((size_t)y * W + x) + 1] = my;
        }
}

/* rsd_motion_vectors_raster: GBufferRaster's non-linear depth linearised like LinearizeDepth, the
 * cleared depth (d >= 1, GBufferRaster.cpp:176) classified as background on the raw value */
void ocpu_motion_vectors_raster(const ocam* c, const ocam* prev, const float* d, uint32_t W, uint32_t H, float* mvec)
{
    const size_t n = (size_t)W * H;
    float* z = (float*)malloc(n * sizeof(float));
    for (size_t i = 0; i < n; ++i)
        z[i] = d[i] < 1.0f ? c->nearZ * c->farZ / (c->farZ + d[i] * (c->nearZ - c->farZ)) : INFINITY;
    ocpu_motion_vectors(c, prev, z, W, H, mvec);
    free(z);
}

/* ------------------------------------------------------------------ TAA
 * TAA.ps.slang:78-150 (TAA.cpp:99-124); librsd's definitions where HLSL leaves them open:
 * lerp(x, y, s) = x + s * (y - x), Load outside the texture = 0, gSampler = linear + wrap with
 * 8-bit sub-texel weights (all four taps), min / max / clamp return the non-NaN operand. */
static void o_ycgco(const float* c, float out[3])
{
    out[0] = c[0] * 0.25f + c[1] * 0.50f + c[2] * 0.25f;
    out[1] = c[0] * -0.25f + c[1] * 0.50f + c[2] * -0.25f;
    out[2] = c[0] * 0.50f + c[1] * 0.00f + c[2] * -0.50f;
}

static void o_bilinear_rgb_wrap(const float* t, int W, int H, float u, float v, float out[3])
{
    float x = u * (float)W - 0.5f, y = v * (float)H - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float qx = floorf((x - fx0) * 256.0f + 0.5f), qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) { ix += 1; qx = 0.0f; }
    if (qy >= 256.0f) { iy += 1; qy = 0.0f; }
    float wx = qx * (1.0f / 256.0f), wy = qy * (1.0f / 256.0f);
    int x0 = o_addr(ix, W, 1), x1 = o_addr(ix + 1, W, 1), y0 = o_addr(iy, H, 1), y1 = o_addr(iy + 1, H, 1);
    const float *a = t + 4 * ((size_t)y0 * W + x0), *b = t + 4 * ((size_t)y0 * W + x1);
    const float *c = t + 4 * ((size_t)y1 * W + x0), *d = t + 4 * ((size_t)y1 * W + x1);
    for (int k = 0; k < 3; ++k) {
        float r0 = a[k] * (1.0f - wx) + b[k] * wx, r1 = c[k] * (1.0f - wx) + d[k] * wx;
        out[k] = r0 * (1.0f - wy) + r1 * wy;
    }
}

void ocpu_taa(const float* color, const float* mvec, const float* prev, uint32_t W_, uint32_t H_, float alpha,
              float sigma, uint32_t antiFlicker, float* out)
{
    static const int ox[8] = {-1, -1, 1, 1, 1, 0, 0, -1}, oy[8] = {-1, 1, -1, 1, 0, -1, 1, 0};
    const int W = (int)W_, H = (int)H_;
    const float inv[2] = {1.0f / (float)W, 1.0f / (float)H};
    static const float zero4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float tu = ((float)x + 0.5f) / (float)W, tv = ((float)y + 0.5f) / (float)H;
            float col[3], avg[3], var[3];
            o_ycgco(color + 4 * ((size_t)y * W + x), col);
            for (int k = 0; k < 3; ++k) { avg[k] = col[k]; var[k] = col[k] * col[k]; }
            for (int n = 0; n < 8; ++n) {
                const int xx = x + ox[n], yy = y + oy[n];
                const float* src = (xx < 0 || yy < 0 || xx >= W || yy >= H) ? zero4 : color + 4 * ((size_t)yy * W + xx);
                float c[3];
                o_ycgco(src, c);
                for (int k = 0; k < 3; ++k) { avg[k] = avg[k] + c[k]; var[k] = var[k] + c[k] * c[k]; }
            }
            const float nine = 1.0f / 9.0f;
            float cmin[3], cmax[3];
            for (int k = 0; k < 3; ++k) {
                avg[k] = avg[k] * nine;
                var[k] = var[k] * nine;
                const float sg = sqrtf(o_max(0.0f, var[k] - avg[k] * avg[k]));
                cmin[k] = avg[k] - sigma * sg;
                cmax[k] = avg[k] + sigma * sg;
            }
            float mx = mvec[2 * ((size_t)y * W + x)], my = mvec[2 * ((size_t)y * W + x) + 1];
            for (int n = 0; n < 8; ++n) {
                const int xx = x + ox[n], yy = y + oy[n];
                float m0 = 0.0f, m1 = 0.0f;
                if (!(xx < 0 || yy < 0 || xx >= W || yy >= H)) {
                    m0 = mvec[2 * ((size_t)yy * W + xx)];
                    m1 = mvec[2 * ((size_t)yy * W + xx) + 1];
                }
                if (m0 * m0 + m1 * m1 > mx * mx + my * my) { mx = m0; my = m1; }
            }
            const float sp[2] = {(tu + mx) * (float)W, (tv + my) * (float)H};
            float w0[2], w12[2], w3[2], c0[2], c12[2], c3[2];
            for (int k = 0; k < 2; ++k) {
                const float tc = floorf(sp[k] - 0.5f) + 0.5f;
                const float f = sp[k] - tc, f2 = f * f, f3 = f2 * f;
                const float q0 = f2 - 0.5f * (f3 + f);
                const float q1 = 1.5f * f3 - 2.5f * f2 + 1.0f;
                const float q3 = 0.5f * (f3 - f2);
                const float q2 = 1.0f - q0 - q1 - q3;
                w0[k] = q0;
                w12[k] = q1 + q2;
                w3[k] = q3;
                c0[k] = (tc - 1.0f) * inv[k];
                c12[k] = (tc + q2 / w12[k]) * inv[k];
                c3[k] = (tc + 2.0f) * inv[k];
            }
            const float xs[3] = {c0[0], c12[0], c3[0]}, ys[3] = {c0[1], c12[1], c3[1]};
            const float wxs[3] = {w0[0], w12[0], w3[0]}, wys[3] = {w0[1], w12[1], w3[1]};
            float h[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    float t[3];
                    o_bilinear_rgb_wrap(prev, W, H, xs[i], ys[j], t);
                    const float w = wxs[i] * wys[j];
                    for (int k = 0; k < 3; ++k) h[k] = (i == 0 && j == 0) ? t[k] * w : h[k] + t[k] * w;
                }
            float hist[3];
            o_ycgco(h, hist);
            float al = alpha;
            if (antiFlicker) {
                const float dist = o_min(fabsf(cmin[0] - hist[0]), fabsf(cmax[0] - hist[0]));
                al = o_min(o_max((alpha * dist) / (dist + cmax[0] - cmin[0]), 0.0f), 1.0f);
            }
            float l[3];
            for (int k = 0; k < 3; ++k) {
                const float hc = o_min(o_max(hist[k], cmin[k]), cmax[k]);
                l[k] = hc + al * (col[k] - hc);
            }
            const float tmp = l[0] - l[1];
            float* o = out + 4 * ((size_t)y * W + x);
            o[0] = tmp + l[2];
            o[1] = l[0] + l[1];
            o[2] = tmp - l[2];
            o[3] = 1.0f;
        }
}

/* ------------------------------------------------------------------ AOFlickerMask
 * AOFlickerMask.ps.slang:43-63: Loads outside the image read 0; min returns the non-NaN operand. */
static void o_px_view(int i, int j, int W, int H, float d, float isx, float isy, float out[3])
{
    float u = o_saturate(((float)i + 0.5f) / (float)W), v = o_saturate(((float)j + 0.5f) / (float)H);
    float ndcx = u * 2.0f - 1.0f, ndcy = (1.0f - v) * 2.0f - 1.0f;
    out[0] = ndcx * d * isx;
    out[1] = ndcy * d * isy;
    out[2] = -d;
}

void ocpu_ao_flicker_mask(const float* z, const float* nw, uint32_t W_, uint32_t H_, const ocam* cam, uint8_t* mask)
{
    const int W = (int)W_, H = (int)H_;
    const float isx = 0.5f * (cam->frameWidth / cam->focalLength), isy = 0.5f * (cam->frameHeight / cam->focalLength);
    const float* m = cam->viewMat;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
#define LD(i, j) (((i) < 0 || (j) < 0 || (i) >= W || (j) >= H) ? 0.0f : z[(size_t)(j) * W + (i)])
            const float* n = nw + 4 * ((size_t)y * W + x);
            float nv[3] = {m[0] * n[0] + m[1] * n[1] + m[2] * n[2], m[4] * n[0] + m[5] * n[1] + m[6] * n[2],
                           m[8] * n[0] + m[9] * n[1] + m[10] * n[2]};
            float P[3];
            o_px_view(x, y, W, H, LD(x, y), isx, isy, P);
            const int nx[4] = {x + 1, x - 1, x, x}, ny[4] = {y, y, y + 1, y - 1};
            float pd[4];
            for (int k = 0; k < 4; ++k) {
                float q[3], dlt[3], dn[3];
                o_px_view(nx[k], ny[k], W, H, LD(nx[k], ny[k]), isx, isy, q);
                for (int c = 0; c < 3; ++c) dlt[c] = P[c] - q[c];
                o_normalize(dlt, dn);
                pd[k] = fabsf(o_dot(dn, nv));
            }
#undef LD
            const float dx = o_min(pd[0], pd[1]), dy = o_min(pd[2], pd[3]);
            mask[(size_t)y * W + x] = (dx <= 0.1f && dy <= 0.1f) ? 1u : 0u;
        }
}

/* ------------------------------------------------------------------ BinaryDilation
 * BinaryDilation.ps.slang:13-43: OP over five Gather footprints (librsd's bilinear footprint,
 * wrap addressing). */
static uint32_t o_gather_op(const uint8_t* t, int W, int H, float u, float v, int mx)
{
    float x = u * (float)W - 0.5f, y = v * (float)H - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float qx = floorf((x - fx0) * 256.0f + 0.5f), qy = floorf((y - fy0) * 256.0f + 0.5f);
    int ix = (int)fx0, iy = (int)fy0;
    if (qx >= 256.0f) ix += 1;
    if (qy >= 256.0f) iy += 1;
    int x0 = o_addr(ix, W, 1), x1 = o_addr(ix + 1, W, 1), y0 = o_addr(iy, H, 1), y1 = o_addr(iy + 1, H, 1);
    uint32_t v4[4] = {t[(size_t)y1 * W + x0], t[(size_t)y1 * W + x1], t[(size_t)y0 * W + x1], t[(size_t)y0 * W + x0]};
    uint32_t r = v4[0];
    for (int k = 1; k < 4; ++k) r = mx ? (v4[k] > r ? v4[k] : r) : (v4[k] < r ? v4[k] : r);
    return r;
}

void ocpu_binary_dilation(const uint8_t* in, uint32_t W_, uint32_t H_, uint32_t opMax, uint8_t* out)
{
    const int W = (int)W_, H = (int)H_, mx = opMax != 0u;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float u = ((float)x + 0.5f) / (float)W, v = ((float)y + 0.5f) / (float)H;
            const float dx = 0.5f / (float)W, dy = 0.5f / (float)H;
            uint32_t r[5] = {o_gather_op(in, W, H, u + dx, v + 3.0f * dy, mx),
                             o_gather_op(in, W, H, u + 3.0f * dx, v + -dy, mx),
                             o_gather_op(in, W, H, u + -dx, v + -3.0f * dy, mx),
                             o_gather_op(in, W, H, u + -3.0f * dx, v + dy, mx), o_gather_op(in, W, H, u, v, mx)};
            uint32_t o = r[0];
            for (int k = 1; k < 5; ++k) o = mx ? (r[k] > o ? r[k] : o) : (r[k] < o ? r[k] : o);
            out[(size_t)y * W + x] = (uint8_t)o;
        }
}
