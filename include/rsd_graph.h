/* rsd_graph.h -- C ABI of the librsd render-graph host (csrc/host/graph.h).
 *
 * This is the surface a graph script binds (Falcor's Python RenderGraph API,
 * RenderGraph.cpp / RenderGraphScripting): scripts/SVAO*.py call
 *   RenderGraph(name)              -> rsd_graph_create        (RenderGraph.cpp:55 create)
 *   g.create_pass(n, type, dict)   -> rsd_graph_create_pass   (RenderGraph.cpp:101 createPass)
 *   g.add_edge(src, dst)           -> rsd_graph_add_edge      (RenderGraph.cpp:249 addEdge)
 *   g.mark_output(name)            -> rsd_graph_mark_output   (RenderGraph.cpp:525 markOutput)
 * and the application drives it with
 *   setScene / compile / execute / getOutput / setInput
 *                                  -> rsd_graph_set_scene / _compile / _execute / _get_output / _set_input
 *                                     (RenderGraph.cpp:158, 336, 420, 470, 444)
 * Pass types come from the plugin registry (Plugin.cpp:45-91): built-ins (GuardBand,
 * GBufferRaster, LinearizeDepth, CompressNormals, StochasticDepthMapRT, SVAO), then
 * dlopen("<plugin dir>/<Type>.so") with extern "C" registerPlugin, else a no-op stub.
 * Properties travel as a flat JSON object ({"radius": 0.2, "cull": "Back", ...}).
 *
 * Every call returns rsd_status and never throws; rsd_last_error() has the message.
 */
#ifndef RSD_GRAPH_H
#define RSD_GRAPH_H
#include <stddef.h>
#include <stdint.h>

#include "rsd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rsd_graph rsd_graph;

/* resource formats of graph textures (graph.h Format) */
typedef enum {
    RSD_FMT_R32F = 0, RSD_FMT_RG32F = 1, RSD_FMT_RGBA32F = 2, RSD_FMT_R16U = 3,
    RSD_FMT_R8U = 4, RSD_FMT_R8UNORM = 5, RSD_FMT_R32U = 6, RSD_FMT_UNKNOWN = 7,
    RSD_FMT_R16F = 8, RSD_FMT_RG16F = 9, RSD_FMT_RGBA16F = 10, /* StochasticDepthMapRT Use16Bit */
    RSD_FMT_RG8UNORM = 11                                      /* SVAO ao with dualAO */
} rsd_format;

typedef struct {
    void* ptr;        /* device pointer, [layer][y][x][texel] */
    uint32_t width, height, layers;
    uint32_t format;  /* rsd_format */
    uint64_t bytes;
} rsd_texture;

rsd_status rsd_graph_create(const char* name, rsd_graph** out);
void rsd_graph_destroy(rsd_graph* g);
rsd_status rsd_graph_create_pass(rsd_graph* g, const char* pass_name, const char* type, const char* props_json);
rsd_status rsd_graph_add_edge(rsd_graph* g, const char* src, const char* dst);
rsd_status rsd_graph_mark_output(rsd_graph* g, const char* name);
/* scene + camera of the frame; call again with a new camera each frame (the camera is copied) */
rsd_status rsd_graph_set_scene(rsd_graph* g, rsd_scene* scene, const rsd_camera* cam);
/* external input bound to "pass.field" (caller-owned device memory) */
rsd_status rsd_graph_set_input(rsd_graph* g, const char* name, const rsd_texture* tex);
rsd_status rsd_graph_compile(rsd_graph* g, uint32_t width, uint32_t height, rsd_stream stream);
rsd_status rsd_graph_execute(rsd_graph* g, rsd_stream stream);
/* compile without device work: culling, execution order and the resource table only
 * (RenderGraphCompiler.cpp:48-172); lets a script be validated on a host without a GPU */
rsd_status rsd_graph_plan(rsd_graph* g, uint32_t width, uint32_t height);
/* resource table of the last plan/compile: "pass.field width height layers format\n" lines */
rsd_status rsd_graph_resources(const rsd_graph* g, char* buf, size_t cap, size_t* needed);
/* "pass.field" of a compiled graph (graph-owned memory, valid until the next compile) */
rsd_status rsd_graph_get_output(rsd_graph* g, const char* name, rsd_texture* out);
/* device-to-device (or to host) copy of a graph resource, exactly its size in bytes */
rsd_status rsd_graph_copy_output(rsd_graph* g, const char* name, void* dst, uint64_t bytes, rsd_stream stream);
/* pass names in execution order, '\n'-separated; *needed receives the full length + 1 */
rsd_status rsd_graph_execution_order(const rsd_graph* g, char* buf, size_t cap, size_t* needed);
/* per-pass GPU time (ms) of the last execute, in execution order (synchronises the stream) */
rsd_status rsd_graph_pass_times(rsd_graph* g, float* ms, uint32_t cap, uint32_t* count);
/* graph dictionary entry (RenderData::getDictionary), e.g. "guardBand" */
rsd_status rsd_graph_get_dict_int(const rsd_graph* g, const char* key, int64_t* out);
rsd_status rsd_graph_pass_count(const rsd_graph* g, uint32_t* passes, uint32_t* edges);

/* --- image passes after SVAO in the graph scripts ------------------ */
/* CrossBilateralBlur (CrossBilateralBlur.ps.slang:1-88, CrossBilateralBlur.cpp:113-149):
 * R8Unorm AO -> x blur into d_pingpong -> y blur into d_dst, KERNEL_RADIUS 1..20 (default 4),
 * betterSlope (default 1); writes only inside the guard band (scissor). */
rsd_status rsd_cross_bilateral_blur(const uint8_t* d_src, const float* d_linear_z, uint32_t z_w, uint32_t z_h,
                                    uint8_t* d_pingpong, uint8_t* d_dst, uint32_t width, uint32_t height,
                                    uint32_t guard_band, uint32_t kernel_radius, uint32_t better_slope,
                                    rsd_stream stream);
/* RayMinMaxLength (RayMinMaxLength.ps.slang:4-16): the SD ray interval length per texel,
 * max(0, asfloat(rayMax) - asfloat(rayMin)) / 32, and 0 where rayMax is 0 (R32Float). */
rsd_status rsd_ray_min_max_length(const uint32_t* d_ray_min, const uint32_t* d_ray_max, uint32_t width,
                                  uint32_t height, float* d_out, rsd_stream stream);
/* DeinterleaveTexture (Deinterleave.slang, DeinterleaveTexture.cpp:143-158): a width x height
 * texture of texel_bytes-byte texels -> 16 layers of ceil(width/4) x ceil(height/4), layer
 * (dy * 4 + dx) holding src[4y + dy][4x + dx] (0 outside the source).  InterleaveTexture
 * (Interleave.slang): the inverse, width x height (the full-size image) from the 16 layers. */
rsd_status rsd_deinterleave(const void* d_src, uint32_t width, uint32_t height, uint32_t texel_bytes, void* d_dst,
                            rsd_stream stream);
rsd_status rsd_interleave(const void* d_src, uint32_t width, uint32_t height, uint32_t texel_bytes, void* d_dst,
                          rsd_stream stream);
/* AOFlickerMask (AOFlickerMask.cpp:73-86, AOFlickerMask.ps.slang:43-63): 1 where the pixel's
 * x and y neighbours lie in its view-space normal plane (|dot| <= 0.1), else 0 (R8Uint).
 * d_normal_w: world-space normals, RGBA32F (GBufferRaster.faceNormalW). */
rsd_status rsd_ao_flicker_mask(const float* d_linear_z, const float* d_normal_w, uint32_t width, uint32_t height,
                               const rsd_camera* cam, uint8_t* d_mask, rsd_stream stream);
/* BinaryDilation (BinaryDilation.ps.slang:13-43): min (op_max 0) or max (op_max 1) over the
 * five 2x2 Gather footprints of the pixel (R8Uint in and out, not in place). */
rsd_status rsd_binary_dilation(const uint8_t* d_in, uint32_t width, uint32_t height, uint32_t op_max, uint8_t* d_out,
                               rsd_stream stream);
/* TAA (TAA.cpp:99-124, TAA.ps.slang:78-150): colour-box clamped, motion-compensated history
 * blend.  Colours RGBA32F (the output's alpha is 1), motion vectors RG32F in uv units; the
 * caller keeps d_prev_color = the previous output (TAA.cpp:123 blit; zeros on the first frame).
 * TAA.h defaults: alpha 0.1, color_box_sigma 1.0, anti_flicker 1.  d_color_out must not alias
 * d_prev_color. */
rsd_status rsd_taa(const float* d_color_in, const float* d_mvec, const float* d_prev_color, uint32_t width,
                   uint32_t height, float alpha, float color_box_sigma, uint32_t anti_flicker, float* d_color_out,
                   rsd_stream stream);
/* TemporalAO enabled (TemporalAO.cpp:113-163, TemporalAO.ps.slang:55-101): reproject the previous
 * frame's AO along the motion vectors (RG32F, uv units), reject on > 10 % relative depth change or
 * a non-zero stable-mask pixel (d_stable_mask may be NULL: none), accumulate up to 30 frames.
 * prev_view_to_cur_view = viewMat * inverse(prevViewMat), row-major (TemporalAO.cpp:156).
 * Writes AO (R8Unorm) and the history count (R8Uint) inside the guard-band scissor; the caller
 * keeps the previous frame's linear depth, AO output and history (the pass's blits, :165-168). */
rsd_status rsd_temporal_ao(const uint8_t* d_ao_in, const float* d_linear_z, const float* d_mvec,
                           const float* d_prev_linear_z, const uint8_t* d_prev_ao, const uint8_t* d_prev_history,
                           const uint8_t* d_stable_mask, uint32_t width, uint32_t height, uint32_t guard_band,
                           const rsd_camera* cam, const float prev_view_to_cur_view[16], uint8_t* d_ao_out,
                           uint8_t* d_history_out, rsd_stream stream);
/* GBufferRaster.mvec for a static scene and a moving camera (librsd definition): the pixel-centre
 * primary hit (from the linear depth) projected with the previous camera, prevUV - uv (RG32F). */
rsd_status rsd_motion_vectors(const rsd_camera* cam, const rsd_camera* prev_cam, const float* d_linear_z,
                              uint32_t width, uint32_t height, float* d_mvec, rsd_stream stream);
/* The same from GBufferRaster's non-linear depth (the GBufferRaster pass's mvec channel): linearised
 * in-kernel like rsd_linearize_depth, background classified on the raw value (d >= 1, the cleared
 * depth, GBufferRaster.cpp:176) -> mvec (0, 0) whatever near / far do to its linearisation. */
rsd_status rsd_motion_vectors_raster(const rsd_camera* cam, const rsd_camera* prev_cam, const float* d_depth,
                                     uint32_t width, uint32_t height, float* d_mvec, rsd_stream stream);
/* ImageEquation (ImageEquation.cpp:134-160, ImageEquation.ps.slang): `formula` is the HLSL
 * expression of `float4 result = (FORMULA)` over I0..I3[xy].  Compile on the host (syntax
 * errors -> RSD_ERR_INVALID_ARG, message in rsd_last_error), run on a stream: inputs[4]
 * (ptr NULL = unbound), output RGBA32F / RG32F / R32F / R8Unorm. */
typedef struct rsd_image_program rsd_image_program;
rsd_status rsd_image_equation_compile(const char* formula, rsd_image_program** out);
rsd_status rsd_image_equation_info(const rsd_image_program* prog, uint32_t* instructions, uint32_t* texture_mask);
rsd_status rsd_image_equation_run(const rsd_image_program* prog, const rsd_texture* inputs, const rsd_texture* out,
                                  rsd_stream stream);
void rsd_image_equation_release(rsd_image_program* prog);

/* plugin registry */
rsd_status rsd_plugin_set_dir(const char* dir);
/* registered pass types, '\n'-separated */
rsd_status rsd_plugin_types(char* buf, size_t cap, size_t* needed);

#ifdef __cplusplus
}
#endif
#endif /* RSD_GRAPH_H */
