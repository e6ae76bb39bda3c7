/*
 * rsd_oracle.h -- CPU ORACLE for the Ray-SD + SVAO hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (librsd / the HIP kernels /
 * the render-graph host) includes, links or calls this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it, and only as
 * the checker (or the timed CPU baseline), never as the thing measured.
 *
 * It is a scalar, plain-C restatement of the reference shaders:
 *   StochasticDepthMapRT/Common.slangh:16-254, Jitter.slangh:20-50,
 *   StochasticDepthMapRT.rt.slang:63-105, StochasticDepthMapRT.cpp:79-124,
 *   Camera.slang:46-90, Camera.cpp:99-185,303-324,
 *   Utils/Geometry/IntersectionHelpers.slang:109-180,
 *   SVAO/Common.slang:98-663, SVAORaster.ps.slang:29-122, SVAORaster2.ps.slang:48-65,
 *   SVAO.cpp:143-190,327-455,663-723, PackedFormats.slang:35-48,
 *   MathHelpers.slang:156-194, FormatConversion.slang:49-95.
 *
 * It deliberately shares NO code with the product: it has its own camera
 * builder, its own (object-median) BVH and its own traversal.  Because the
 * any-hit stream is defined in canonical (t, primitive-id) order (DESIGN.md
 * "Any-hit order"), results are BVH-independent, so product == oracle
 * bit-for-bit is a meaningful check of the product's BVH as well.
 *
 * Parity pinning: the reference (Falcor + Slang + DXR) cannot be built or run
 * in this container.  The oracle's constant tables are pinned
 * against data extracted from the reference sources (tests/golden/); the
 * per-hit / per-pixel arithmetic is a restatement ("parity partially
 * unpinned": no reference output images exist for this path).
 */
#ifndef RSD_ORACLE_H
#define RSD_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same memory layout as rsd_camera in include/rsd.h (32 floats). */
typedef struct {
    float posW[3];  float nearZ;
    float U[3];     float farZ;
    float V[3];     float focalLength;
    float W[3];     float frameHeight;
    float frameWidth; float jitterX; float jitterY; float aspectRatio;
    float viewMat[16];  /* row-major, Falcor matrixFromLookAt (RightHanded) */
} ocam;

/* Same layout as rsd_sd_params. */
typedef struct {
    uint32_t sample_count;   /* N: 1,2,4,8,16 (16 = documented extension) */
    uint32_t implementation; /* 0 Default(reservoir), 1 CoverageMask, 3 KBuffer */
    uint32_t max_count;      /* MAX_COUNT */
    int32_t  guard_band;     /* GUARD_BAND (SD texels) */
    uint32_t jitter;         /* SD_JITTER */
    uint32_t normalize;      /* NORMALIZE */
    uint32_t ray_interval;   /* USE_RAY_INTERVAL */
    uint32_t cull_mode;      /* 0 None, 1 Back, 2 Front */
    uint32_t alpha_test;     /* USE_ALPHA_TEST (opaque scenes: no-op) */
    float    alpha;          /* ALPHA (coverage mask) */
    uint32_t hit_order;      /* rsd_hit_order: 0 canonical (ocpu_sd_trace), 1 traversal (ocpu_sd_trace_ordered),
                                2 wavefront (ocpu_sd_trace_wavefront) */
    uint32_t use_16bit;      /* not read by the oracle (tests round the f32 map to binary16 in numpy) */
} osd_params;

/* Same layout as rsd_vao_data: mirror of VAOData.slang:33-45 */
typedef struct {
    float noiseScale[2];
    float resolution[2];
    float lowResolution[2];
    float invResolution[2];
    float radius;
    float exponent;
    float thickness;
    int32_t sdGuard;
    float ssRadiusCutoff;
    float ssMaxRadius;
} ovao;

/* Same layout as rsd_svao_params */
typedef struct {
    uint32_t num_directions;   /* NUM_DIRECTIONS: 8, 16, 32 */
    uint32_t sd_samples;       /* MSAA_SAMPLES */
    uint32_t secondary_depth_mode; /* 0 Single, 2 Stochastic */
    uint32_t ray_interval;     /* USE_RAY_INTERVAL */
    uint32_t sd_jitter;        /* SD_JITTER */
    uint32_t guard_band;       /* frame-buffer guard band (GuardBand pass) */
    uint32_t dual_ao;          /* DUAL_AO: ao is RG8Unorm (bright, dark), 2 bytes per pixel */
    /* the layout of librsd's rsd_svao_params continues (tests copy the common prefix): */
    void* tile_flags_unused;   /* librsd's busy-tile flags (device only) */
    uint32_t numerics_unused;  /* librsd's fast / exact arithmetic (the oracle is the exact one) */
    uint32_t ao_kernel;        /* AO_KERNEL (SVAO.cpp:233, AOKernel.h): 0 VAO, 1 HBAO */
    uint32_t primary_depth_mode; /* PRIMARY_DEPTH_MODE (DepthMode.h): 0 SingleDepth, 1 DualDepth */
    const float* depth2;       /* DualDepth: gDepthTex2, the second linear-depth layer (W x H) */
} osvao_params;

typedef struct oscene oscene;

/* scene: positions float3[nv], indices uint32[3*nt], flags uint32[nt]
 * (bit0 double-sided, bit1 front-face-CW, bit2 alpha-masked). */
oscene* ocpu_scene_create(const float* positions, uint32_t nv, const uint32_t* indices,
                          uint32_t nt, const uint32_t* flags);
void ocpu_scene_destroy(oscene* s);
/* alpha-masked materials (rsd_alpha_desc restated): texcoords float2[nv], per-triangle
 * material, per-material threshold / constant alpha / texture (0xffffffff: none), textures
 * as their mip-0 R8 texels concatenated (the oracle builds its own mip chains) */
void ocpu_scene_set_alpha(oscene* s, const uint32_t* indices, const float* texcoords, const uint32_t* triMat,
                          uint32_t nm, const float* threshold, const float* alpha, const uint32_t* texture,
                          uint32_t ntex, const uint32_t* tex_w, const uint32_t* tex_h, const uint8_t* mip0);
int ocpu_alpha_fails(const oscene* s, uint32_t prim, float bu, float bv, int lodRayCone, float t,
                     const float d[3], float spread);
float ocpu_alpha_value(const oscene* s, uint32_t prim, float bu, float bv, int lodRayCone, float t,
                       const float d[3], float spread);
float ocpu_alpha_threshold(const oscene* s, uint32_t material);
float ocpu_ray_cone_spread(float focal_length, uint32_t height);
uint32_t ocpu_scene_node_count(const oscene* s);

void ocpu_camera_look_at(const float pos[3], const float target[3], const float up[3],
                         float focalLength, float frameHeight, float aspectRatio,
                         float nearZ, float farZ, float focalDistance, ocam* out);

/* primary visibility: linear view depth (R32F) + view-space octahedral 2x8 normal (R16Uint) */
void ocpu_gbuffer(const oscene* s, const ocam* cam, uint32_t W, uint32_t H, uint32_t cull_mode,
                  float* linearZ, uint16_t* normals, int nthreads);
/* GBufferRaster.depth (non-linear [0,1], cleared 1) + faceNormalW (RGBA32F, cleared 0) */
void ocpu_gbuffer_raster(const oscene* s, const ocam* cam, uint32_t W, uint32_t H, uint32_t cull_mode,
                         float* depth, float* normalW, int nthreads);
void ocpu_linearize_depth(const float* d, float* z, size_t n, float near_z, float far_z);
void ocpu_compress_normals(const float* normalW, uint16_t* out, size_t n, const ocam* cam);

/* SD trace for rows [row0,row1) of the SD map.  sd layout: [layer][y][x][ch],
 * ch = min(N,4), layers = ceil(N/4).  rayMin/rayMax may be NULL.
 * stats (optional): [0] active rays, [1] hits delivered to the any-hit stream. */
void ocpu_sd_trace(const oscene* s, const ocam* cam, const osd_params* p,
                   const float* linearZ, uint32_t zW, uint32_t zH,
                   const uint32_t* rayMin, const uint32_t* rayMax,
                   float* sd, uint32_t sdW, uint32_t sdH,
                   uint32_t row0, uint32_t row1, int nthreads, uint64_t* stats);

/* The same SD trace with librsd's traversal-order any-hit stream (rsd.h RSD_HIT_ORDER_TRAVERSAL)
 * over librsd's own BVH: bvh = the rsd_scene_export_bvh bytes, tri_offset in float4 units.
 * s supplies the alpha-masked materials (by primitive id).  Rows [row0, row1), band of tile rows. */
void ocpu_sd_trace_ordered(const oscene* s, const float* bvh, uint32_t tri_offset, const ocam* cam,
                           const osd_params* p, const float* linearZ, uint32_t zW, uint32_t zH,
                           const uint32_t* rayMin, const uint32_t* rayMax, float* sd, uint32_t sdW, uint32_t sdH,
                           uint32_t row0, uint32_t row1, uint32_t band_index, uint32_t band_count, int nthreads,
                           uint64_t* stats);
/* The wavefront any-hit stream (rsd.h RSD_HIT_ORDER_WAVEFRONT) over librsd's exported BVH; pool_soft =
 * min(208 - 3 wide_depth, 160) as librsd computes it (rsd_scene_info.wide_depth). */
void ocpu_sd_trace_wavefront(const oscene* s, const float* bvh, uint32_t tri_offset, uint32_t pool_soft,
                             const ocam* cam, const osd_params* p, const float* linearZ, uint32_t zW, uint32_t zH,
                             const uint32_t* rayMin, const uint32_t* rayMax, float* sd, uint32_t sdW, uint32_t sdH,
                             uint32_t row0, uint32_t row1, uint32_t band_index, uint32_t band_count, int nthreads,
                             uint64_t* stats);

/* the SD ray of texel (x, y): origin+direction, TMin, TMax and cosT (for tests) */
void ocpu_sd_ray(const ocam* c, const osd_params* p, const float* z, uint32_t zW, uint32_t zH,
                 const uint32_t* rmin, const uint32_t* rmax, uint32_t sdW, uint32_t sdH, uint32_t x, uint32_t y,
                 float out[6], float* tmin, float* tmax, float* cosT);

void ocpu_svao_clear(uint32_t* rayMin, uint32_t* rayMax, uint32_t n);
/* contiguous screen bands: visible rows [row0, row1) counted from the first visible row */
void ocpu_svao_pass1_rows(const ocam* cam, const ovao* d, const osvao_params* p,
                          const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                          uint8_t* ao, uint8_t* stencil, uint32_t* rayMin, uint32_t* rayMax,
                          uint32_t sdW, uint32_t sdH, uint32_t row0, uint32_t row1);
void ocpu_svao_pass2_rows(const ocam* cam, const ovao* d, const osvao_params* p,
                          const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                          const uint8_t* stencil, const float* sd, uint32_t sdW, uint32_t sdH,
                          uint8_t* ao, uint32_t row0, uint32_t row1, int nthreads);
void ocpu_svao_pass1(const ocam* cam, const ovao* d, const osvao_params* p,
                     const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                     uint8_t* ao, uint8_t* stencil, uint32_t* rayMin, uint32_t* rayMax,
                     uint32_t sdW, uint32_t sdH);
void ocpu_svao_pass2(const ocam* cam, const ovao* d, const osvao_params* p,
                     const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                     const uint8_t* stencil, const float* sd, uint32_t sdW, uint32_t sdH,
                     uint8_t* ao, int nthreads);

/* screen-band variants (multi-GPU sharding, same band rules as rsd.h) */
void ocpu_sd_trace_band(const oscene* s, const ocam* cam, const osd_params* p,
                        const float* linearZ, uint32_t zW, uint32_t zH,
                        const uint32_t* rayMin, const uint32_t* rayMax,
                        float* sd, uint32_t sdW, uint32_t sdH,
                        uint32_t row0, uint32_t row1, uint32_t band_index, uint32_t band_count,
                        int nthreads, uint64_t* stats);
void ocpu_svao_pass1_band(const ocam* cam, const ovao* d, const osvao_params* p,
                          const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                          uint8_t* ao, uint8_t* stencil, uint32_t* rayMin, uint32_t* rayMax,
                          uint32_t sdW, uint32_t sdH, uint32_t band_index, uint32_t band_count);
void ocpu_svao_pass2_band(const ocam* cam, const ovao* d, const osvao_params* p,
                          const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                          const uint8_t* stencil, const float* sd, uint32_t sdW, uint32_t sdH,
                          uint8_t* ao, uint32_t band_index, uint32_t band_count, int nthreads);

/* constant tables / helpers exposed for golden-vector tests */
float ocpu_hash(float x, float y);
void ocpu_jitter(uint32_t x, uint32_t y, float* jx, float* jy);
void ocpu_stratified_lut(int n, int32_t* indices /* n+1 */, uint32_t* lut /* 2^n */);
void ocpu_noise_texture(uint8_t out[16]);
float ocpu_sample_radius(uint32_t num_directions, uint32_t i);
float ocpu_sample_radius_kernel(uint32_t num_directions, uint32_t i, uint32_t kernel); /* 0 VAO, 1 HBAO */
uint32_t ocpu_encode_normal_2x8(const float n[3]);
void ocpu_decode_normal_2x8(uint32_t packed, float out[3]);
/* returns 1 on hit; outputs t, DXR barycentrics (u,v) and det */
int ocpu_intersect(const float o[3], const float d[3], const float v0[3], const float v1[3],
                   const float v2[3], float* t, float* u, float* v, float* det);

/* SVAO pass 2 in SecondaryDepthMode::Raytraced (Common.slang:598-651, aoAnyHit :679-718) */
void ocpu_svao_pass2_rt_band(const oscene* sc, const ocam* cam, const ovao* d, const osvao_params* p,
                             const float* depth, const uint16_t* normals, uint32_t W, uint32_t H,
                             const uint8_t* stencil, uint8_t* ao, uint32_t cull, uint32_t ray_pipeline,
                             uint32_t alpha_test, uint32_t band_index, uint32_t band_count, int nthreads);

/* CrossBilateralBlur (x then y through pingpong; dst written inside the guard band only) */
void ocpu_cross_bilateral_blur(const uint8_t* src, const float* z, uint32_t zW, uint32_t zH, uint8_t* pingpong,
                               uint8_t* dst, uint32_t W, uint32_t H, uint32_t guard, uint32_t radius,
                               uint32_t better_slope);
void ocpu_temporal_ao(const uint8_t* aoIn, const float* z, const float* mvec, const float* prevZ,
                      const uint8_t* prevAo, const uint8_t* prevN, const uint8_t* stable, uint32_t W,
                      uint32_t H, uint32_t g, const ocam* cam, const float m[16], uint8_t* aoOut,
                      uint8_t* nOut);
void ocpu_motion_vectors(const ocam* c, const ocam* prev, const float* z, uint32_t W, uint32_t H, float* mvec);
void ocpu_motion_vectors_raster(const ocam* c, const ocam* prev, const float* depth, uint32_t W, uint32_t H,
                                float* mvec);
void ocpu_ao_flicker_mask(const float* z, const float* nw, uint32_t W, uint32_t H, const ocam* cam, uint8_t* mask);
void ocpu_binary_dilation(const uint8_t* in, uint32_t W, uint32_t H, uint32_t opMax, uint8_t* out);
void ocpu_taa(const float* color, const float* mvec, const float* prev, uint32_t W, uint32_t H, float alpha,
              float sigma, uint32_t antiFlicker, float* out);

#ifdef __cplusplus
}
#endif
#endif
