/*
 * rsd.h -- C ABI of librsd, the MI355X-native Ray-SD + SVAO hot path.
 *
 * This is the drop-in boundary.  In the reference the hot path is reached through
 * Falcor's plugin ABI (Plugin.cpp:56-91 dlopen + registerPlugin) and the RenderPass
 * virtuals (RenderPass.h:119-259); each pass's execute() records DXR / compute
 * dispatches.  librsd exports those dispatches as plain C entry points: device
 * pointers, sizes and a HIP stream, no C++ or torch types.  The C++ RenderPass
 * mirror (csrc/host/) and the Python graph front end (falcor/) call exactly these.
 *
 * Conventions:
 *   - every entry point returns rsd_status; never throws across the ABI;
 *     rsd_last_error() gives a thread-local message for the last failure;
 *   - the caller owns every d_* buffer (device memory);
 *   - compute entry points are asynchronous and ordered on the given stream
 *     (rsd_stream = hipStream_t; NULL = the legacy default stream);
 *   - one rsd_device per GPU per host thread; scenes are bound to a device;
 *   - SD traces of one scene may run concurrently on DIFFERENT streams (frames in flight):
 *     librsd keeps the trace's scratch per (scene, stream); calls on one stream are ordered.
 */
#ifndef RSD_H
#define RSD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSD_ABI_VERSION 8

typedef enum {
    RSD_OK = 0,
    RSD_ERR_INVALID_ARG = 1,
    RSD_ERR_UNSUPPORTED = 2,
    RSD_ERR_HIP = 3,
    RSD_ERR_OUT_OF_MEMORY = 4,
    RSD_ERR_NO_DEVICE = 5,
} rsd_status;

typedef struct rsd_device rsd_device;
typedef struct rsd_scene rsd_scene;
typedef void* rsd_stream; /* hipStream_t */

/* Scene ingest (replaces Scene::initGeomDesc/buildBlas/buildTlas, Scene.cpp:2688-2830,
 * 3091, 3628-3739).  A world-space triangle soup; triangle_flags per triangle:
 *   bit0 double-sided (TriangleFacingCullDisable, Scene.cpp:3452)
 *   bit1 front face clockwise (TriangleFrontCounterClockwise, Scene.cpp:3451)
 *   bit2 alpha-masked material (AlphaMode::Mask): alpha-tested, see rsd_scene_upload_alpha
 * Primitive id = triangle index in this array.                                        */
#define RSD_TRI_DOUBLE_SIDED 1u
#define RSD_TRI_FRONT_CW 2u
#define RSD_TRI_ALPHA_MASK 4u

typedef struct {
    const float* positions;   /* float3[vertex_count] (host) */
    uint32_t vertex_count;
    const uint32_t* indices;  /* uint32[3 * triangle_count] (host) */
    uint32_t triangle_count;
    const uint32_t* triangle_flags; /* uint32[triangle_count] or NULL (all 0) */
} rsd_scene_desc;

typedef struct {
    uint32_t triangle_count;
    uint32_t node_count;      /* 4-wide BVH nodes (128 B each) */
    uint32_t max_depth;
    uint32_t leaf_count;
    double sah_cost;
    double build_ms;          /* host build wall time: BVH + segment entry grid */
    uint64_t device_bytes;
    uint32_t build_threads;   /* host threads of the build (the process's CPU affinity, or RSD_BUILD_THREADS) */
    uint32_t entry_cells;     /* cells of the segment entry grid (RSD_ENTRY_CELLS bounds it, 0 = none) */
    uint32_t wide_depth;      /* 4-wide nodes on the longest root-to-leaf path (sizes the walks' LDS stacks) */
} rsd_scene_info;

/* Alpha-masked materials (MaterialFactory.slang:124-151, AlphaTest.slang:54-84,
 * StandardMaterial.slang:128-132): the opacity of a triangle flagged RSD_TRI_ALPHA_MASK is the
 * alpha of its material's base-colour texture at the interpolated texture coordinate (or the
 * material's constant alpha); the hit is alpha-tested away when opacity < alpha_threshold
 * (the threshold is stored as float16 like MaterialHeader, MaterialData.slang:99).
 * Textures are R8 (alpha only), row-major, mip 0; librsd builds the 2x2 box-filter mip chain.
 * Sampling: trilinear, wrap, 8 sub-texel / LOD-fraction bits (DESIGN.md "Alpha test"). */
#define RSD_NO_TEXTURE 0xffffffffu
typedef struct {
    uint32_t width, height;
    const uint8_t* alpha; /* width * height texels (host) */
} rsd_alpha_texture;
typedef struct {
    float alpha_threshold; /* MaterialHeader alpha threshold (default 0.5) */
    float alpha;           /* constant alpha (baseColor.a) when texture == RSD_NO_TEXTURE */
    uint32_t texture;      /* index into rsd_alpha_desc.textures or RSD_NO_TEXTURE */
} rsd_material;
typedef struct {
    const float* texcoords;            /* float2[vertex_count] (indexed like the positions) */
    const uint32_t* triangle_material; /* uint32[triangle_count] */
    const rsd_material* materials;
    uint32_t material_count;
    const rsd_alpha_texture* textures;
    uint32_t texture_count;
} rsd_alpha_desc;

/* Camera data mirror (CameraData.slang:35-68 subset), 32 floats. */
typedef struct {
    float posW[3];  float nearZ;
    float U[3];     float farZ;
    float V[3];     float focalLength;
    float W[3];     float frameHeight;
    float frameWidth; float jitterX; float jitterY; float aspectRatio;
    float viewMat[16]; /* row-major */
} rsd_camera;

/* StochasticDepthMapRT Properties -> shader defines (StochasticDepthMapRT.cpp:262-276) */
typedef enum { RSD_SD_DEFAULT = 0, RSD_SD_COVERAGE_MASK = 1, RSD_SD_RESERVOIR_SAMPLING = 2, RSD_SD_KBUFFER = 3 } rsd_sd_impl;
typedef enum { RSD_CULL_NONE = 0, RSD_CULL_BACK = 1, RSD_CULL_FRONT = 2 } rsd_cull_mode;

typedef struct {
    uint32_t sample_count;   /* SampleCount N: 1, 2, 4, 8 (reference) or 16 (extension) */
    uint32_t implementation; /* rsd_sd_impl (ReservoirSampling is raster-only -> unsupported) */
    uint32_t max_count;      /* MaxCount (MAX_COUNT) */
    int32_t guard_band;      /* GuardBand (GUARD_BAND), SD texels */
    uint32_t jitter;         /* Jitter (SD_JITTER) */
    uint32_t normalize;      /* normalize (NORMALIZE) */
    uint32_t ray_interval;   /* RayInterval (USE_RAY_INTERVAL) */
    uint32_t cull_mode;      /* CullMode (CULL_MODE_RAY_FLAG) */
    uint32_t alpha_test;     /* AlphaTest (USE_ALPHA_TEST) */
    float alpha;             /* Alpha (ALPHA), coverage-mask implementation */
    uint32_t hit_order;      /* any-hit delivery order: rsd_hit_order (librsd extension) */
    uint32_t use_16bit;      /* Use16Bit (StochasticDepthMapRT.cpp:192-198): store R16F / RG16F / RGBA16F,
                                N <= 4; d_sd_out then holds IEEE binary16 (round to nearest even) */
    uint32_t* d_tile_state;  /* NULL, or rsd_sd_tile_state_count(sd_w, sd_h) device words owned with d_sd_out
                                (librsd extension, DESIGN.md 4 "clean tiles"): the trace records per 8x8 SD tile
                                whether it left every texel of the tile it wrote at DEFAULT_DEPTH -- since ABI v8
                                also which texels (a 64-bit mask per tile after the tiles' stamps) -- and does not
                                rewrite those texels while they have no live ray.  The caller zeroes the words when
                                it allocates the map, writes the map itself, or changes which texels its traces
                                own (a band split); the map's bits are those of a trace without it. */
} rsd_sd_params;

/* Any-hit order of the SD trace.  DXR calls any-hit in an implementation-defined traversal order
 * (Common.slangh:136-153 under RAY_FLAG_FORCE_NON_OPAQUE, StochasticDepthMapRT.rt.slang:83-88),
 * so three orders are defined:
 *   CANONICAL  ascending (t, primitive id), each triangle once -- independent of the BVH; the
 *              result depends only on the MAX_COUNT nearest hits (Default == KBuffer on opaque
 *              geometry: the reservoir never replaces a slot).
 *   TRAVERSAL  the order of a depth-first walk of the scene's 4-wide BVH: children nearest entry
 *              distance first (ties: child slot), leaf triangles in record order, each triangle
 *              once; a committed hit (algorithm returns true = DXR AcceptHit) shrinks the ray's
 *              TMax to its t and later hits must be nearer (t < TMax), like DXR's RayTCurrent().
 *              The reservoir samples stochastically; the result depends on the BVH
 *              (rsd_scene_export_bvh gives the oracle the same tree).
 *   WAVEFRONT  the order of an 8-wide wavefront walk of the same tree (round 5, the canonical row walk's
 *              traversal): per step up to 8 items, each tested by its own lane against the TMax of the
 *              step's start; the step's leaf hits go to any-hit in lane order, a leaf's triangles in
 *              record order, with the same commit rule (t < TMax after a commit); surviving children
 *              are pushed nearest-on-top per lane (lanes in order) onto a LIFO pool, from which the next
 *              step pops up to 8 items (one while the pool holds more than min(208 - 3 depth, 160) items,
 *              depth = rsd_scene_info.wide_depth).  Stochastic like TRAVERSAL; about the canonical
 *              walk's speed instead of half of it. */
typedef enum { RSD_HIT_ORDER_CANONICAL = 0, RSD_HIT_ORDER_TRAVERSAL = 1, RSD_HIT_ORDER_WAVEFRONT = 2 } rsd_hit_order;

/* VAOData.slang:33-45 mirror */
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
} rsd_vao_data;

/* SVAO compile-time defines (SVAO.cpp:221-237) + the per-frame guardBand */
typedef struct {
    uint32_t num_directions;       /* NUM_DIRECTIONS: 8 (default), 16 or 32 */
    uint32_t sd_samples;           /* MSAA_SAMPLES = SD N */
    uint32_t secondary_depth_mode; /* DepthMode: 0 SingleDepth, 2 StochasticDepth, 3 Raytraced */
    uint32_t ray_interval;         /* USE_RAY_INTERVAL */
    uint32_t sd_jitter;            /* SD_JITTER */
    uint32_t guard_band;           /* dict["guardBand"] from the GuardBand pass */
    uint32_t dual_ao;              /* DUAL_AO (SVAO dualAO, SVAO.cpp:130): d_ao is RG8Unorm -- R bright, G dark
                                      (SVAORaster.ps.slang:103, SVAORaster2.ps.slang:62), 2 bytes per pixel */
    uint8_t* tile_flags;           /* ABI v4 (layout v5), optional (NULL = none): busy-tile state of the 16x16
                                      tiles of the visible region, rsd_svao_tile_count bytes, caller-owned,
                                      zeroed once.  Pass 1 flags every tile holding a stencilled pixel and
                                      appends it to a list; a whole-frame pass 2 walks the list (no workgroup
                                      for an empty tile), a band / row-range pass 2 visits the flagged tiles
                                      of its rows; both clear what they consumed, so the buffer is clean for
                                      the next pass 1 (the reference's pass 2 returns on aoMask == 0,
                                      SVAORaster2.ps.slang:50-52).  Pass 2 must get the buffer of the pass 1
                                      that wrote d_stencil. */
    uint32_t numerics;             /* ABI v5: rsd_numerics of pass 1 and pass 2 (DESIGN.md 2 "Numerics") */
    uint32_t ao_kernel;            /* ABI v5: AO_KERNEL (SVAO.cpp:233, AOKernel.h): rsd_ao_kernel */
    uint32_t primary_depth_mode;   /* ABI v5: PRIMARY_DEPTH_MODE (SVAO.cpp:222, DepthMode.h): 0 SingleDepth,
                                      1 DualDepth (the second depth layer d_depth2 refines the raster samples,
                                      SVAORaster.ps.slang:69-70, Common.slang:498-505, :555-558) */
    const float* d_depth2;         /* ABI v5: DualDepth: gDepthTex2, linear depth of the second layer
                                      (DepthPeeling / TemporalDepthPeel), width x height R32F */
} rsd_svao_params;
/* SVAO's AO kernel (SVAO::mKernel, a UI dropdown in the reference, SVAO.cpp:615-620):
 *   VAO   volumetric obscurance: visibility = min over the samples of the sphere + halo terms (default);
 *   HBAO  horizon-based: visibility = max over the samples of saturate(HBAOKernel / pdf), pdf =
 *         0.9 (1 - r_i)^1.5, AO = saturate(1 - 2 avg)^exponent (Common.slang:60-66, 326-330, 362-365,
 *         421-430, 455-488).  The reference's UI scales the world radius by 1.5 on switching to HBAO
 *         (SVAO.cpp:617-620); callers pass the radius they want.  Every secondary mode takes either kernel
 *         (Raytraced HBAO: a closest-hit ray over [sphereStart, sphereEnd], Common.slang:622-650). */
typedef enum { RSD_AO_KERNEL_VAO = 0, RSD_AO_KERNEL_HBAO = 1 } rsd_ao_kernel;
/* Arithmetic of the SVAO passes ("AO 1", "AO 2"; the SD trace is always exact).
 *   FAST   FMA contraction, v_rcp_f32-based division, hardware sqrt / rsq, float32 denormals flushed, no
 *          NaN operands assumed: what D3D allows the reference's HLSL (mad may fuse, '/' within 2.5 ulp,
 *          denormals flushed, min / max without signalling-NaN quieting).
 *          Graded against the CPU oracle by BASELINE.md section 4's AO tolerance (MAE <= 1/255 over the
 *          visible pixels, |diff| <= 2/255 on >= 99.5 %).  The default (zero-initialised params).
 *   EXACT  binary32 round-to-nearest operation by operation, correctly rounded '/' and sqrt: bit-identical
 *          to the CPU oracle (oracle/rsd_oracle.c), at a higher instruction count. */
typedef enum { RSD_NUMERICS_FAST = 0, RSD_NUMERICS_EXACT = 1 } rsd_numerics;
/* Bytes of rsd_svao_params.tile_flags for a width x height frame buffer with guard_band: for the T 16x16
 * tiles of the visible region rounded up to 32 rows (the padded pass-1 dispatch, SVAO.cpp:347-350), T flag
 * words, a 16-byte list header (two list counts: frames alternate between them, so no pass resets the
 * list on the device) and T list entries (8 T + 16 bytes; ABI v4 had T bytes). */
uint32_t rsd_svao_tile_count(uint32_t width, uint32_t height, uint32_t guard_band);
/* librsd keeps one generation counter per tile_flags buffer on the host (pass 1 / pass 2 alternate the list
 * counts by it; pass 1 stamps a busy tile's flag with it, so a flag a pass 2 did not consume -- a pass 1
 * whose rows no pass 2 covered -- never keeps its tile out of a later list).  An owner that frees the buffer
 * calls this, so a new buffer at the same address starts from a fresh counter (with its zeroed memory). */
void rsd_svao_tile_flags_release(const void* tile_flags);

/* Traversal counters of the last instrumented trace (roofline bytes) */
typedef struct {
    uint64_t rays_dispatched;
    uint64_t rays_active;     /* TMin <= TMax after the ray interval */
    uint64_t nodes_visited;   /* 128-B 4-wide BVH nodes fetched */
    uint64_t tris_tested;     /* 48-B triangle records fetched */
    uint64_t hits_delivered;  /* any-hit invocations (sorted stream) */
    uint64_t max_nodes_per_ray; /* longest traversal (latency tail of the launch) */
    uint64_t max_steps_per_ray; /* node + leaf steps of the longest traversal */
    uint64_t sum_ray_clocks;    /* shader clocks (s_memtime) spent in live rays */
    uint64_t max_ray_clocks;    /* the slowest live ray */
    uint64_t leaves_visited;    /* leaf steps (<= 4 triangle records each) */
    uint64_t walk;              /* traversal walk of the trace: RSD_WALK_* */
    uint64_t entry_lookups;     /* segment entry-grid lookups (one 16-B hash slot each, first probe) */
    uint64_t entry_items;       /* frontier items tested by the setup kernel (32 B each) */
    /* ABI v5, the instrumented row walk (RSD_WALK_FUSED; 0 for the other walks): per row-step clock
     * sums of lane 0 of every row -- the step's dependent fetch (the instrumented build waits for it),
     * its box / triangle tests and merges, its LDS pool pops and pushes -- and the steps walked; the
     * s_memtime rate of the launch (MHz) converts them to time.  Latency roofline of the walk (bench.py
     * roofline.latency_floor_us): max_steps_per_ray x the mean step time. */
    uint64_t step_fetch_clocks;
    uint64_t step_compute_clocks;
    uint64_t step_pool_clocks;
    uint64_t row_steps;
    double shader_clock_mhz;
    uint64_t texels_clean;   /* SD texels of clean tiles the setup did not rewrite (rsd_sd_params.d_tile_state) */
    /* ABI v7: the walk the instrumented launch itself ran (RSD_WALK_*).  `walk` names the walk an uninstrumented
     * trace of the same call takes (the kernels a caller's timed traces ran); the step clocks above belong to
     * walk_instrumented (the hybrid walk is instrumented through its row or quad walk alone). */
    uint64_t walk_instrumented;
} rsd_counters;
/* rsd_counters.walk: which kernels an rsd_sd_trace launched (besides sd_setup_kernel) */
#define RSD_WALK_QUAD 0u   /* sd_trace_queue_kernel: depth-first, 4 lanes per ray */
#define RSD_WALK_FUSED 1u  /* sd_trace_row_kernel with the algorithm in-kernel */
#define RSD_WALK_SPLIT 2u  /* sd_trace_row_kernel (K nearest keys) + sd_resolve_row_kernel */
#define RSD_WALK_ORDERED 3u /* sd_trace_ordered_kernel: RSD_HIT_ORDER_TRAVERSAL */
#define RSD_WALK_WAVEFRONT 5u /* sd_trace_wavefront_kernel: RSD_HIT_ORDER_WAVEFRONT */
#define RSD_WALK_HYBRID 6u /* one frame in flight with K <= 8 (the canonical stream): sd_trace_hybrid_kernel, whose
                              first blocks row-walk the longest-first rays and whose others quad-walk the rest; an
                              instrumented trace reports it but walks the single walk (fused or quad) */
#define RSD_WALK_RASTER 4u  /* sd_raster_kernel (triangles -> K nearest keys per texel) + sd_resolve_row_kernel */

/* --- library / device ------------------------------------------------------------ */
uint32_t rsd_abi_version(void);
const char* rsd_last_error(void);
rsd_status rsd_device_open(int hip_device, rsd_device** out);
void rsd_device_close(rsd_device* dev);

/* --- scene (BVH2 build on the host, upload to HBM) --------------------------------- */
rsd_status rsd_scene_upload(rsd_device* dev, const rsd_scene_desc* desc, rsd_scene** out);
/* The same with alpha-masked materials (alpha may be NULL = all opaque).  The SD trace applies
 * the alpha test when rsd_sd_params.alpha_test is set (ray-cone LOD, StochasticDepthMapRT.rt.slang:
 * 31-37, RAY_CONE_SPREAD of the SD map height); the G-buffer (GBufferRaster useAlphaTest) and the
 * Raytraced SVAO pass (alphaTest, LOD 0, Common.slang:684-693) test at LOD 0. */
rsd_status rsd_scene_upload_alpha(rsd_device* dev, const rsd_scene_desc* desc, const rsd_alpha_desc* alpha,
                                  rsd_scene** out);
rsd_status rsd_scene_info_get(const rsd_scene* scene, rsd_scene_info* out);
/* Copy of the scene's device BVH (host memory): 4-wide nodes (128 B: SoA lo.x[4] hi.x[4] lo.y[4]
 * hi.y[4] lo.z[4] hi.z[4] ref[4] count[4]), then 48-B triangle records {v0, prim}{v1, flags}{v2, 0}
 * from float4 offset *tri_offset.  dst == NULL: only *bytes.  Synchronous. */
rsd_status rsd_scene_export_bvh(const rsd_scene* scene, void* dst, uint64_t capacity, uint64_t* bytes,
                                uint32_t* tri_offset);
/* The same bytes without a GPU: the host build rsd_scene_upload would upload for `desc`
 * (deterministic: same desc, same tree).  dst == NULL: only *bytes. */
rsd_status rsd_bvh_build(const rsd_scene_desc* desc, void* dst, uint64_t capacity, uint64_t* bytes,
                         uint32_t* tri_offset);
void rsd_scene_release(rsd_scene* scene);

/* --- host helpers (no GPU work) ---------------------------------------------------- */
/* RAY_CONE_SPREAD of the SD pass (StochasticDepthMapRT.cpp:266-267): Camera::
 * computeScreenSpacePixelSpreadAngle(height) (Camera.cpp:296-301) with the fovY of the 24 mm
 * default frame height, passed through std::to_string ("%f") like the shader define. */
float rsd_ray_cone_spread(float focal_length, uint32_t height);
/* Camera::calculateCameraParameters (Camera.cpp:99-185), preserveHeight = true */
rsd_status rsd_camera_look_at(const float pos[3], const float target[3], const float up[3],
                              float focal_length, float frame_height, float aspect_ratio,
                              float near_z, float far_z, float focal_distance, rsd_camera* out);
/* SVAO::compile / getStochMapSize / getExtraGuardBand (SVAO.cpp:143-150, 700-723):
 * fb_w x fb_h frame buffer, divisor, SD guard band in full-res pixels (mStochMapGuardBand). */
rsd_status rsd_svao_make_vao_data(uint32_t fb_w, uint32_t fb_h, uint32_t divisor, int32_t sd_guard_px,
                                  float radius, float exponent, float thickness,
                                  rsd_vao_data* out, uint32_t* sd_w, uint32_t* sd_h);

/* --- GPU passes (stream-ordered, asynchronous) ------------------------------------- */
/* Primary visibility (GBufferRaster -> LinearizeDepth -> CompressNormals):
 * linear view depth (R32F) and view-space octahedral 2x8 face normal (R16Uint). */
rsd_status rsd_gbuffer(rsd_scene* scene, const rsd_camera* cam, uint32_t width, uint32_t height,
                       uint32_t cull_mode, float* d_linear_z, uint16_t* d_normals, rsd_stream stream);

/* The raster-style G-buffer of scripts/SVAO.py, for the render-graph host:
 * GBufferRaster.depth (non-linear [0,1] depth, R32F) + GBufferRaster.faceNormalW (RGBA32F),
 * LinearizeDepth (Linearize.ps.slang) and CompressNormals (CompressNormals.ps.slang,
 * view space, 2x8 octahedral). */
rsd_status rsd_gbuffer_raster(rsd_scene* scene, const rsd_camera* cam, uint32_t width, uint32_t height,
                              uint32_t cull_mode, float* d_depth, float* d_normal_w, rsd_stream stream);
rsd_status rsd_linearize_depth(const float* d_depth, float* d_linear_z, uint32_t count, float near_z, float far_z,
                               rsd_stream stream);
rsd_status rsd_compress_normals(const float* d_normal_w, uint16_t* d_packed, uint32_t count,
                                const rsd_camera* cam, rsd_stream stream);

/* StochasticDepthMapRT::execute (StochasticDepthMapRT.cpp:231-331) + rayGen/anyHit
 * (StochasticDepthMapRT.rt.slang:39-105).  d_sd_out layout = Texture2DArray:
 * [layer][y][x][ch], ch = min(N,4), layers = ceil(N/4).  d_ray_min / d_ray_max may be
 * NULL (no interval).  If `counters` is non-NULL, an instrumented kernel fills it
 * (synchronises the stream). */
rsd_status rsd_sd_trace(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* params,
                        const float* d_linear_z, uint32_t z_w, uint32_t z_h,
                        const uint32_t* d_ray_min, const uint32_t* d_ray_max,
                        float* d_sd_out, uint32_t sd_w, uint32_t sd_h,
                        rsd_counters* counters, rsd_stream stream);

/* SVAO.cpp:330-341: rayMax <- 0, rayMin <- asuint(FLT_MAX) */
/* Words of rsd_sd_params.d_tile_state for an sd_w x sd_h map: three per 8x8 tile (a stamp; since ABI v8 a texel mask). */
uint32_t rsd_sd_tile_state_count(uint32_t sd_w, uint32_t sd_h);
rsd_status rsd_svao_clear_intervals(uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t count, rsd_stream stream);

/* "AO 1": SVAORaster.ps.slang:29-122, dispatched as SVAO.cpp:344-350.
 * params->num_directions (NUM_DIRECTIONS) is 8, 16 or 32 (Common.slang:51-58); the stencil texel is
 * R8Uint / R16Uint / R32Uint accordingly (SVAO.cpp:132-134): d_stencil holds width * height texels of
 * num_directions / 8 bytes (the same for every pass that takes a stencil). */
rsd_status rsd_svao_pass1(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* params,
                          const float* d_depth, const uint16_t* d_normals, uint32_t width, uint32_t height,
                          uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                          uint32_t sd_w, uint32_t sd_h, rsd_stream stream);

/* "AO 2": SVAORaster2.ps.slang:48-65 / calcAO2 (Common.slang:523-663), SVAO.cpp:450-454 */
rsd_status rsd_svao_pass2(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* params,
                          const float* d_depth, const uint16_t* d_normals, uint32_t width, uint32_t height,
                          const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                          uint8_t* d_ao, rsd_stream stream);

/* "AO 2" in SecondaryDepthMode::Raytraced (the ground-truth AO of
 * scripts/SVAO_depth.py and SAVO_record.py): calcAO2 DEPTH_MODE_RAYTRACING (Common.slang:598-651)
 * with aoAnyHit (:679-718) over the canonical ascending hit stream.  Replaces the RayQuery
 * compute pass (SVAORaster2.ps.slang:9-65, SVAO.cpp:432-455; ray_pipeline = 0: visible pixels)
 * and the ray pipeline (Ray.rt.slang, SVAO.cpp:408-431; ray_pipeline = 1: the rayGen grid covers
 * the frame from the guard band to the right/bottom edge).  Pass 1 must have run with
 * secondary_depth_mode = 3.  cull_mode: SVAO's CULL_MODE_RAY_FLAG (rsd_cull_mode). */
rsd_status rsd_svao_pass2_raytraced(rsd_scene* scene, const rsd_camera* cam, const rsd_vao_data* vao,
                                    const rsd_svao_params* params, const float* d_depth, const uint16_t* d_normals,
                                    uint32_t width, uint32_t height, const uint8_t* d_stencil, uint8_t* d_ao,
                                    uint32_t cull_mode, uint32_t ray_pipeline, uint32_t alpha_test, rsd_stream stream);

/* --- screen-band sharding (multi-GPU) ----------------------------------
 * Band b of B owns: pass-1/pass-2 rows whose 32-row group g (counted from the first
 * visible row, SVAORaster.ps.slang:36 interleave) has g % B == b, and SD-map 8-row tile
 * rows t with t % B == b.  The union over b = 0..B-1 is exactly the full-frame call;
 * the functions above are band 0 of 1.  Interleaving balances sky vs. geometry. */
rsd_status rsd_sd_trace_band(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* params,
                             const float* d_linear_z, uint32_t z_w, uint32_t z_h,
                             const uint32_t* d_ray_min, const uint32_t* d_ray_max,
                             float* d_sd_out, uint32_t sd_w, uint32_t sd_h,
                             uint32_t band_index, uint32_t band_count, rsd_counters* counters, rsd_stream stream);
/* The same with flags.  RSD_SD_CONSUME_INTERVALS (needs RayInterval): the trace resets every
 * texel of d_ray_min / d_ray_max (rayMin = asuint(FLT_MAX), rayMax = 0) after reading it --
 * the whole map, not only the band -- so the next frame's pass 1 may run without
 * rsd_svao_clear_intervals (SVAO.cpp:334-340 folded into the trace's first kernel). */
#define RSD_SD_CONSUME_INTERVALS 1u
/* RSD_SD_THROUGHPUT: the caller overlaps this trace with other GPU work (frames in flight).  A hint:
 * librsd measured the row walk (8 lanes per ray) ahead of the depth-first quad walk there too since
 * the segment entry grid, so it currently picks the same walk either way.
 * Same result bits whatever the walk. */
#define RSD_SD_THROUGHPUT 2u
rsd_status rsd_sd_trace_band_ex(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* params,
                                const float* d_linear_z, uint32_t z_w, uint32_t z_h,
                                uint32_t* d_ray_min, uint32_t* d_ray_max,
                                float* d_sd_out, uint32_t sd_w, uint32_t sd_h,
                                uint32_t band_index, uint32_t band_count, uint32_t flags,
                                rsd_counters* counters, rsd_stream stream);
rsd_status rsd_svao_pass1_band(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* params,
                               const float* d_depth, const uint16_t* d_normals, uint32_t width, uint32_t height,
                               uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                               uint32_t sd_w, uint32_t sd_h, uint32_t band_index, uint32_t band_count,
                               rsd_stream stream);
rsd_status rsd_svao_pass2_band(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* params,
                               const float* d_depth, const uint16_t* d_normals, uint32_t width, uint32_t height,
                               const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                               uint8_t* d_ao, uint32_t band_index, uint32_t band_count, rsd_stream stream);

/* Contiguous screen bands (the halo-exchange split, rsd/shard.py HaloFrame): pass 1 / pass 2 of the
 * visible rows [row0, row1) counted from the first visible row (multiples of 32: the 2x2 group
 * interleave of SVAORaster.ps.slang:36 stays inside 32-row groups; row1 may end the frame), and
 * the SD trace of the SD-map rows [row0, row1) (multiples of 8; row1 may be sd_h).  Same kernels
 * and bits as the band calls; flags as rsd_sd_trace_band_ex (CONSUME resets the whole map). */
rsd_status rsd_svao_pass1_rows(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* params,
                               const float* d_depth, const uint16_t* d_normals, uint32_t width, uint32_t height,
                               uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                               uint32_t sd_w, uint32_t sd_h, uint32_t row0, uint32_t row1, rsd_stream stream);
rsd_status rsd_svao_pass2_rows(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* params,
                               const float* d_depth, const uint16_t* d_normals, uint32_t width, uint32_t height,
                               const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                               uint8_t* d_ao, uint32_t row0, uint32_t row1, rsd_stream stream);
rsd_status rsd_sd_trace_rows(rsd_scene* scene, const rsd_camera* cam, const rsd_sd_params* params,
                             const float* d_linear_z, uint32_t z_w, uint32_t z_h,
                             uint32_t* d_ray_min, uint32_t* d_ray_max,
                             float* d_sd_out, uint32_t sd_w, uint32_t sd_h,
                             uint32_t row0, uint32_t row1, uint32_t flags, rsd_counters* counters, rsd_stream stream);

/* --- sparse halo exchange of the band split (rsd/shard.py HaloFrame) ----------
 * Device-side steps around the point-to-point transfers, one call each instead of a dozen small torch
 * ops per peer (the host issue cost of an N > 1 frame).  No host synchronisation.
 *
 * rsd_halo_compact: for each region r, the touched texels (rayMin != asuint(FLT_MAX) or rayMax != 0;
 * SVAO.cpp:334-340's cleared state) are written as int32 triples -- texel index, rayMin bits, rayMax
 * bits -- to out[r] (three rows of `stride` int32: out[r][0 .. n), out[r][stride ..], out[r][2 stride ..];
 * stride >= the region's texel count) in an unspecified order, and their number to *count[r] (int64,
 * overwritten; regions may share an output and a count).  The merge below is order-independent
 * (min / max), so the order does not change a result bit.
 * A region is SD rows [row0, row1) (period <= 1), or (period > 1; row0 a multiple of 8) the 8-row SD
 * tiles t = row0 / 8 + j period that start below row1 -- one rank's tiles when the SD trace's tiles
 * are dealt round-robin to the ranks (rsd_sd_trace_band_ex with band_count = period). */
typedef struct {
    uint32_t row0, row1;  /* SD-map rows of the region */
    int32_t* out;         /* 3 x stride int32 (device) */
    uint32_t stride;
    uint32_t period;      /* 0 / 1: rows [row0, row1); > 1: every period-th 8-row tile from row0 */
    int64_t* count;       /* device int64, overwritten */
} rsd_halo_region;
rsd_status rsd_halo_compact(const uint32_t* d_ray_min, const uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h,
                            const rsd_halo_region* regions, uint32_t n_regions, rsd_stream stream);
/* rsd_halo_merge: atomicMin / atomicMax of received triples (per list: n triples in three rows of `stride`
 * int32, as above) into the interval maps -- the exact union (non-negative float bit patterns order like
 * the floats); ray_interval = 0 (no RayInterval): rayMin is not merged.  All lists in one launch. */
typedef struct {
    const int32_t* triples;
    uint32_t n;
    uint32_t stride;
} rsd_halo_list;
rsd_status rsd_halo_merge(uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h,
                          const rsd_halo_list* lists, uint32_t n_lists, uint32_t ray_interval, rsd_stream stream);
/* rsd_halo_sd_gather / _scatter: the SD depths of n texels per list (int32 texel indices of the sd_w x sd_h
 * plane) between the map (layers x texels x ch floats, Texture2DArray order) and the list's packed buffer
 * (layers x n x ch floats) -- the sparse SD halo's reply.  All lists in one launch; at most 64 lists. */
typedef struct {
    const int32_t* idx;
    float* buf;
    uint32_t n;
    uint32_t pad;
} rsd_halo_sd_list;
rsd_status rsd_halo_sd_gather(const float* d_sd, uint32_t layers, uint32_t sd_w, uint32_t sd_h, uint32_t ch,
                              const rsd_halo_sd_list* lists, uint32_t n_lists, rsd_stream stream);
rsd_status rsd_halo_sd_scatter(float* d_sd, uint32_t layers, uint32_t sd_w, uint32_t sd_h, uint32_t ch,
                               const rsd_halo_sd_list* lists, uint32_t n_lists, rsd_stream stream);

rsd_status rsd_svao_pass2_raytraced_band(rsd_scene* scene, const rsd_camera* cam, const rsd_vao_data* vao,
                                         const rsd_svao_params* params, const float* d_depth,
                                         const uint16_t* d_normals, uint32_t width, uint32_t height,
                                         const uint8_t* d_stencil, uint8_t* d_ao, uint32_t cull_mode,
                                         uint32_t ray_pipeline, uint32_t alpha_test, uint32_t band_index,
                                         uint32_t band_count, rsd_stream stream);

/* --- one whole frame per call (SVAO::execute, SVAO.cpp:192-456) ---------------------
 * The frame's dispatch sequence on one stream, issued from C++: the interval clear (SVAO.cpp:
 * 330-341; skipped with RSD_FRAME_INTERVALS_CLEAR when the previous frame's trace on these maps
 * consumed them) -> "AO 1" -> (StochasticDepth) the SD trace, which consumes the interval maps when
 * RayInterval is on -> "AO 2"; (Raytraced) "AO 1" -> the Raytraced "AO 2"; (SingleDepth) "AO 1".
 * The same kernels and bits as the separate calls; one ABI crossing per frame instead of four
 * (the host issue cost of a frame).
 * events: NULL or 4 hipEvent_t (each may be NULL) recorded on the stream before "AO 1", before the
 * SD trace, after the SD trace and after "AO 2" (per-pass timing without host round trips). */
typedef struct {
    rsd_scene* scene;               /* StochasticDepth / Raytraced modes */
    const rsd_camera* cam;
    const rsd_vao_data* vao;
    const rsd_svao_params* svao;    /* secondary_depth_mode selects the sequence */
    const rsd_sd_params* sd;        /* the nested SD pass (StochasticDepth); cull_mode / alpha_test of the
                                       Raytraced pass */
    const float* d_depth;           /* linear Z, width x height */
    const uint16_t* d_normals;      /* 2x8 octahedral view-space normals */
    uint32_t width, height;
    uint8_t* d_ao;
    uint8_t* d_stencil;
    uint32_t* d_ray_min;            /* sd_w x sd_h (StochasticDepth) */
    uint32_t* d_ray_max;
    float* d_sd;                    /* the SD map (StochasticDepth) */
    uint32_t sd_w, sd_h;
    uint32_t ray_pipeline;          /* Raytraced mode: SVAO rayPipeline (rsd_svao_pass2_raytraced) */
} rsd_svao_frame_desc;
#define RSD_FRAME_INTERVALS_CLEAR 4u  /* the interval maps hold the cleared state: no clear launch */
#define RSD_FRAME_KEEP_INTERVALS 8u   /* the trace leaves the interval maps as pass 1 wrote them (no consume) */
/* flags: RSD_FRAME_INTERVALS_CLEAR | RSD_FRAME_KEEP_INTERVALS | RSD_SD_THROUGHPUT */
rsd_status rsd_svao_frame(const rsd_svao_frame_desc* frame, uint32_t flags, void* const* events, rsd_stream stream);

/* --- communicators of the band frame (ABI v6; multi-GPU) ---------------
 * The exchanges of a screen-band frame, stream-ordered (no host wait for the GPU):
 *   RCCL   one process per GPU (north_star: "final AO image all-gathered over RCCL/xGMI"): ncclAllGather,
 *          ncclSend / ncclRecv in one ncclGroupStart / End on the caller's stream.  librccl.so.1 is loaded
 *          on first use (the copy torch loaded, when it did).  rsd_comm_rccl_create is collective: every
 *          rank calls it with the id rank 0 got from rsd_comm_rccl_unique_id, on its own GPU (the HIP
 *          device current on the calling thread).
 *   LOCAL  `world` host threads of one process sharing a GPU, one stream each (one-GPU tests of the N > 1
 *          frame): device-to-device copies ordered by events; a hub is the threads' rendezvous.
 * The reference renders on one GPU (no counterpart); the split's geometry follows SVAO.cpp:700-723 and
 * VAOData.slang:44. */
typedef struct rsd_comm rsd_comm;
typedef struct rsd_comm_hub rsd_comm_hub;
#define RSD_COMM_UNIQUE_ID_BYTES 128
#define RSD_COMM_RCCL 1u
#define RSD_COMM_LOCAL 2u
#define RSD_COMM_NULL 3u   /* moves nothing: host-cost probes of one rank's frame (diagnostics only) */
/* ABI v7: RSD_OK when librccl.so.1 loads with every symbol the RCCL communicator uses (no RCCL call, no
 * socket: every rank may ask, so that the ranks can agree on the native path before the collective create) */
rsd_status rsd_comm_rccl_available(void);
rsd_status rsd_comm_rccl_unique_id(uint8_t id[RSD_COMM_UNIQUE_ID_BYTES]);
rsd_status rsd_comm_rccl_create(const uint8_t id[RSD_COMM_UNIQUE_ID_BYTES], uint32_t world, uint32_t rank,
                                rsd_comm** out);
rsd_status rsd_comm_hub_create(uint32_t world, rsd_comm_hub** out);
void rsd_comm_hub_release(rsd_comm_hub* hub); /* after every rsd_comm of the hub */
rsd_status rsd_comm_local_create(rsd_comm_hub* hub, uint32_t rank, rsd_comm** out);
rsd_status rsd_comm_null_create(uint32_t world, uint32_t rank, rsd_comm** out);
void rsd_comm_release(rsd_comm* comm);
rsd_status rsd_comm_info(const rsd_comm* comm, uint32_t* kind, uint32_t* rank, uint32_t* world);
/* d_recv = world x bytes (rank k's d_send at offset k x bytes) */
rsd_status rsd_comm_all_gather(rsd_comm* comm, const void* d_send, void* d_recv, uint64_t bytes, rsd_stream stream);
/* One group of point-to-point transfers (sizes agreed beforehand; a peer may be the rank itself) */
typedef struct {
    void* buf;
    uint64_t bytes;
    uint32_t peer;
    uint32_t pad;
} rsd_comm_xfer;
rsd_status rsd_comm_exchange(rsd_comm* comm, const rsd_comm_xfer* sends, uint32_t n_sends, const rsd_comm_xfer* recvs,
                             uint32_t n_recvs, rsd_stream stream);

/* --- the screen-band frame (ABI v6) ---------------------------------
 * One rank's share of SVAO::execute (SVAO.cpp:192-456) split into contiguous screen bands, issued from
 * C++ on the caller's stream.  Rank r of the communicator's world:
 *   front  the interval clear (skipped when the previous trace of this object consumed them) -> "AO 1" of
 *          its visible rows (rsd_svao_pass1_rows) -> the SD texels its samples touched inside every other
 *          rank's SD share, compacted on the device as (texel, rayMin, rayMax) triples -> an all-gather of
 *          the per-peer counts (+ this object's previous frame time) -> an async copy of the count matrix
 *          to pinned host memory;
 *   back   the host reads the counts (one event; with frames in flight it completed long before) ->
 *          point-to-point transfer of the triples -> atomic min / max merge (the exact 1-GPU interval
 *          union on the rank's SD share) -> the SD trace of its share (round-robin 8-row tiles, or the SD
 *          rows under its band: rsd_band_params.sd_split) -> the depths of exactly the texels each peer
 *          sent come back to it -> "AO 2" of its rows -> its AO band to every other rank, theirs into d_ao
 *          (point-to-point, image to image).
 * Every SD texel and AO pixel is produced by exactly one rank with the same kernels: each rank's AO
 * image and its own SD share are bit-identical to the 1-GPU frame (rsd_svao_frame), whatever the split.
 * The split of the 32-row groups is re-balanced every fourth frame from the ranks' measured pass-1 +
 * trace + pass-2 times (same decision on every rank): frame 4j + 1 is timed, its time is read in the back() of
 * frame 4j + 2 (after that frame's counts arrived, so without waiting), travels with the counts of frame
 * 4j + 3, whose back() decides, and front() of frame 4j + 4 applies the new split.  A camera whose focal
 * length or frame height differs from the previous frame's re-plans the halo windows (the sample reach).  The count matrix reaches the host through pinned
 * memory written by a kernel (a sequence word the host polls): front and back of a frame must be issued on
 * the same stream.  The frame description's buffers are used in
 * place; its camera / params structs are copied (rsd_band_frame_front may pass a new camera).
 * StochasticDepth mode with RayInterval only (the north_star's path). */
#define RSD_SD_SPLIT_AUTO 0u   /* tiles for reduced-resolution SD maps (divisor > 1), rows at full resolution */
#define RSD_SD_SPLIT_TILES 1u  /* the SD map's 8-row tiles dealt round-robin (tile t to rank t mod world) */
#define RSD_SD_SPLIT_ROWS 2u   /* the SD rows under each rank's pass-1 band */
typedef struct {
    uint32_t divisor;     /* stochMapDivisor of the SD map (SVAO.cpp:143-150) */
    uint32_t sd_split;    /* RSD_SD_SPLIT_* */
    uint32_t rebalance;   /* 1: re-split from the measured per-rank time (needs world > 1) */
    uint32_t throughput;  /* 1: traces flagged RSD_SD_THROUGHPUT (this frame overlaps others) */
} rsd_band_params;
typedef struct rsd_band_frame rsd_band_frame;
rsd_status rsd_band_frame_create(const rsd_svao_frame_desc* frame, const rsd_band_params* params, rsd_comm* comm,
                                 rsd_band_frame** out);
/* ABI v7: a split chosen by the caller (split[0] = 0 < split[1] < ... < split[world] = rsd_band_stats.groups;
 * the same on every rank), applied by the next front(): e.g. a skewed start that the re-balancing corrects.
 * It does not count as a re-split in rsd_band_stats.resplits. */
rsd_status rsd_band_frame_set_split(rsd_band_frame* bf, const uint32_t* split, uint32_t n);
/* cam: NULL or the camera of this frame (an animated camera; copied) */
rsd_status rsd_band_frame_front(rsd_band_frame* bf, const rsd_camera* cam, rsd_stream stream);
/* events: NULL or 2 hipEvent_t (each may be NULL) recorded before and after this rank's SD trace */
rsd_status rsd_band_frame_back(rsd_band_frame* bf, void* const* events, rsd_stream stream);
typedef struct {
    uint32_t rank, world;
    uint32_t sd_split;          /* RSD_SD_SPLIT_TILES or _ROWS (resolved) */
    uint32_t groups;            /* 32-row groups of the visible rows */
    uint32_t split[65];         /* group boundaries of the current split: rank k owns [split[k], split[k+1]) */
    uint32_t sd_row0, sd_row1;  /* SD rows under this rank's band (sd_split ROWS: the rows it traces) */
    uint32_t halo_px;           /* vertical reach of a sample in frame-buffer pixels (the window's margin) */
    uint64_t frames;            /* back() calls */
    uint64_t blocked_waits;     /* back() calls whose counts had not reached the host yet */
    uint64_t resplits;          /* applied re-splits */
    uint64_t bytes_intervals;   /* bytes sent so far: interval triples, SD replies, AO band (to every peer) */
    uint64_t bytes_sd;
    uint64_t bytes_ao;
    uint64_t dense_intervals;   /* what the dense halo (whole candidate regions) would send per frame */
    uint64_t dense_sd;
    uint64_t growth_syncs;      /* exchange buffers grown (each waits for this stream once) */
    uint64_t host_front_ns;     /* host time inside rsd_band_frame_front / _back so far (issue cost), and the */
    uint64_t host_back_ns;      /*   part of _back spent waiting for the count matrix (0 with frames in flight */
    uint64_t host_wait_ns;      /*   once the counts are long complete) */
} rsd_band_stats;
rsd_status rsd_band_frame_stats(const rsd_band_frame* bf, rsd_band_stats* out);
void rsd_band_frame_release(rsd_band_frame* bf); /* waits for the frame's stream work to finish */

#ifdef __cplusplus
}
#endif
#endif /* RSD_H */
