"""ctypes binding of librsd's C ABI (include/rsd.h).

This is the binding a Python host (Falcor's scripting layer, a test, the bench)
uses; it mirrors the header one to one.  There is no fallback: if librsd.so is
missing or a call fails, a RuntimeError is raised with rsd_last_error().
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parents[1]
# RSD_LIB_VARIANT=<name>: load librsd_<name>.so built beside it (A/B builds of one kernel option;
# experiments only -- the product and the tests load librsd.so)
LIB_PATH = PKG_DIR / (f"librsd_{os.environ['RSD_LIB_VARIANT']}.so" if os.environ.get("RSD_LIB_VARIANT") else "librsd.so")

RSD_OK = 0
ERR_INVALID_ARG, ERR_UNSUPPORTED, ERR_HIP = 1, 2, 3
STATUS_NAMES = {0: "RSD_OK", 1: "RSD_ERR_INVALID_ARG", 2: "RSD_ERR_UNSUPPORTED", 3: "RSD_ERR_HIP",
                4: "RSD_ERR_OUT_OF_MEMORY", 5: "RSD_ERR_NO_DEVICE"}

TRI_DOUBLE_SIDED = 1
TRI_FRONT_CW = 2
TRI_ALPHA_MASK = 4

SD_DEFAULT, SD_COVERAGE_MASK, SD_RESERVOIR_SAMPLING, SD_KBUFFER = 0, 1, 2, 3
DEPTH_SINGLE, DEPTH_DUAL, DEPTH_STOCHASTIC, DEPTH_RAYTRACED = 0, 1, 2, 3  # VAO/DepthMode.h
CULL_NONE, CULL_BACK, CULL_FRONT = 0, 1, 2


class SceneDesc(C.Structure):
    _fields_ = [("positions", C.c_void_p), ("vertex_count", C.c_uint32), ("indices", C.c_void_p),
                ("triangle_count", C.c_uint32), ("triangle_flags", C.c_void_p)]


NO_TEXTURE = 0xFFFFFFFF


class AlphaTexture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("alpha", C.c_void_p)]


class Material(C.Structure):
    _fields_ = [("alpha_threshold", C.c_float), ("alpha", C.c_float), ("texture", C.c_uint32)]


class AlphaDesc(C.Structure):
    _fields_ = [("texcoords", C.c_void_p), ("triangle_material", C.c_void_p), ("materials", C.POINTER(Material)),
                ("material_count", C.c_uint32), ("textures", C.POINTER(AlphaTexture)), ("texture_count", C.c_uint32)]


class SceneInfo(C.Structure):
    _fields_ = [("triangle_count", C.c_uint32), ("node_count", C.c_uint32), ("max_depth", C.c_uint32),
                ("leaf_count", C.c_uint32), ("sah_cost", C.c_double), ("build_ms", C.c_double),
                ("device_bytes", C.c_uint64), ("build_threads", C.c_uint32), ("entry_cells", C.c_uint32),
                ("wide_depth", C.c_uint32)]


class Camera(C.Structure):
    _fields_ = [("posW", C.c_float * 3), ("nearZ", C.c_float),
                ("U", C.c_float * 3), ("farZ", C.c_float),
                ("V", C.c_float * 3), ("focalLength", C.c_float),
                ("W", C.c_float * 3), ("frameHeight", C.c_float),
                ("frameWidth", C.c_float), ("jitterX", C.c_float), ("jitterY", C.c_float),
                ("aspectRatio", C.c_float), ("viewMat", C.c_float * 16)]


class SDParams(C.Structure):
    _fields_ = [("sample_count", C.c_uint32), ("implementation", C.c_uint32), ("max_count", C.c_uint32),
                ("guard_band", C.c_int32), ("jitter", C.c_uint32), ("normalize", C.c_uint32),
                ("ray_interval", C.c_uint32), ("cull_mode", C.c_uint32), ("alpha_test", C.c_uint32),
                ("alpha", C.c_float), ("hit_order", C.c_uint32), ("use_16bit", C.c_uint32),
                ("d_tile_state", C.c_void_p)]


class VAOData(C.Structure):
    _fields_ = [("noiseScale", C.c_float * 2), ("resolution", C.c_float * 2),
                ("lowResolution", C.c_float * 2), ("invResolution", C.c_float * 2),
                ("radius", C.c_float), ("exponent", C.c_float), ("thickness", C.c_float),
                ("sdGuard", C.c_int32), ("ssRadiusCutoff", C.c_float), ("ssMaxRadius", C.c_float)]


class SVAOParams(C.Structure):
    _fields_ = [("num_directions", C.c_uint32), ("sd_samples", C.c_uint32),
                ("secondary_depth_mode", C.c_uint32), ("ray_interval", C.c_uint32),
                ("sd_jitter", C.c_uint32), ("guard_band", C.c_uint32), ("dual_ao", C.c_uint32),
                ("tile_flags", C.c_void_p),  # ABI v4: busy 16x16 tiles (pass 1 sets, pass 2 consumes)
                ("numerics", C.c_uint32),    # ABI v5: rsd_numerics of pass 1 / pass 2
                ("ao_kernel", C.c_uint32),   # ABI v5: rsd_ao_kernel (VAO / HBAO)
                ("primary_depth_mode", C.c_uint32),  # ABI v5: 0 SingleDepth, 1 DualDepth
                ("d_depth2", C.c_void_p)]    # ABI v5: DualDepth's second depth layer
AO_KERNEL_VAO, AO_KERNEL_HBAO = 0, 1  # rsd.h rsd_ao_kernel
AO_KERNELS = {"vao": AO_KERNEL_VAO, "hbao": AO_KERNEL_HBAO}


NUMERICS_FAST, NUMERICS_EXACT = 0, 1  # rsd.h rsd_numerics
NUMERICS = {"fast": NUMERICS_FAST, "exact": NUMERICS_EXACT}


class HaloRegion(C.Structure):  # rsd_halo_region
    _fields_ = [("row0", C.c_uint32), ("row1", C.c_uint32), ("out", C.c_void_p), ("stride", C.c_uint32),
                ("period", C.c_uint32), ("count", C.c_void_p)]


class HaloList(C.Structure):  # rsd_halo_list
    _fields_ = [("triples", C.c_void_p), ("n", C.c_uint32), ("stride", C.c_uint32)]


class HaloSdList(C.Structure):  # rsd_halo_sd_list
    _fields_ = [("idx", C.c_void_p), ("buf", C.c_void_p), ("n", C.c_uint32), ("pad", C.c_uint32)]


class FrameDesc(C.Structure):  # rsd_svao_frame_desc
    _fields_ = [("scene", C.c_void_p), ("cam", C.c_void_p), ("vao", C.c_void_p), ("svao", C.c_void_p),
                ("sd", C.c_void_p), ("d_depth", C.c_void_p), ("d_normals", C.c_void_p), ("width", C.c_uint32),
                ("height", C.c_uint32), ("d_ao", C.c_void_p), ("d_stencil", C.c_void_p), ("d_ray_min", C.c_void_p),
                ("d_ray_max", C.c_void_p), ("d_sd", C.c_void_p), ("sd_w", C.c_uint32), ("sd_h", C.c_uint32),
                ("ray_pipeline", C.c_uint32)]


class CommXfer(C.Structure):  # rsd_comm_xfer
    _fields_ = [("buf", C.c_void_p), ("bytes", C.c_uint64), ("peer", C.c_uint32), ("pad", C.c_uint32)]


COMM_RCCL, COMM_LOCAL, COMM_NULL = 1, 2, 3  # rsd.h RSD_COMM_*
COMM_UNIQUE_ID_BYTES = 128
SD_SPLIT_AUTO, SD_SPLIT_TILES, SD_SPLIT_ROWS = 0, 1, 2  # rsd.h RSD_SD_SPLIT_*
SD_SPLITS = {"auto": SD_SPLIT_AUTO, "tiles": SD_SPLIT_TILES, "rows": SD_SPLIT_ROWS}


class BandParams(C.Structure):  # rsd_band_params
    _fields_ = [("divisor", C.c_uint32), ("sd_split", C.c_uint32), ("rebalance", C.c_uint32),
                ("throughput", C.c_uint32)]


class BandStats(C.Structure):  # rsd_band_stats
    _fields_ = [("rank", C.c_uint32), ("world", C.c_uint32), ("sd_split", C.c_uint32), ("groups", C.c_uint32),
                ("split", C.c_uint32 * 65), ("sd_row0", C.c_uint32), ("sd_row1", C.c_uint32),
                ("halo_px", C.c_uint32), ("frames", C.c_uint64), ("blocked_waits", C.c_uint64),
                ("resplits", C.c_uint64), ("bytes_intervals", C.c_uint64), ("bytes_sd", C.c_uint64),
                ("bytes_ao", C.c_uint64), ("dense_intervals", C.c_uint64), ("dense_sd", C.c_uint64),
                ("growth_syncs", C.c_uint64), ("host_front_ns", C.c_uint64), ("host_back_ns", C.c_uint64),
                ("host_wait_ns", C.c_uint64)]


FRAME_INTERVALS_CLEAR = 4  # rsd.h RSD_FRAME_INTERVALS_CLEAR
FRAME_KEEP_INTERVALS = 8   # rsd.h RSD_FRAME_KEEP_INTERVALS


class Counters(C.Structure):
    _fields_ = [("rays_dispatched", C.c_uint64), ("rays_active", C.c_uint64), ("nodes_visited", C.c_uint64),
                ("tris_tested", C.c_uint64), ("hits_delivered", C.c_uint64), ("max_nodes_per_ray", C.c_uint64),
                ("max_steps_per_ray", C.c_uint64), ("sum_ray_clocks", C.c_uint64), ("max_ray_clocks", C.c_uint64),
                ("leaves_visited", C.c_uint64), ("walk", C.c_uint64), ("entry_lookups", C.c_uint64),
                ("entry_items", C.c_uint64), ("step_fetch_clocks", C.c_uint64), ("step_compute_clocks", C.c_uint64),
                ("step_pool_clocks", C.c_uint64), ("row_steps", C.c_uint64), ("shader_clock_mhz", C.c_double),
                ("texels_clean", C.c_uint64), ("walk_instrumented", C.c_uint64)]


WALK_QUAD, WALK_FUSED, WALK_SPLIT, WALK_ORDERED, WALK_RASTER, WALK_WAVEFRONT, WALK_HYBRID = 0, 1, 2, 3, 4, 5, 6
WALK_NAMES = {WALK_QUAD: "quad", WALK_FUSED: "fused", WALK_SPLIT: "split", WALK_ORDERED: "ordered", WALK_RASTER: "raster",
              WALK_WAVEFRONT: "wavefront", WALK_HYBRID: "hybrid"}
HIT_ORDER_CANONICAL, HIT_ORDER_TRAVERSAL, HIT_ORDER_WAVEFRONT = 0, 1, 2
# kernels of one rsd_sd_trace per walk (rsd_counters.walk)
WALK_KERNELS = {WALK_QUAD: ("sd_setup_kernel", "sd_trace_queue_kernel"),
                WALK_FUSED: ("sd_setup_kernel", "sd_trace_row_kernel"),
                WALK_SPLIT: ("sd_setup_kernel", "sd_trace_row_kernel", "sd_resolve_row_kernel"),
                WALK_ORDERED: ("sd_setup_kernel", "sd_trace_ordered_kernel"),
                WALK_RASTER: ("sd_setup_kernel", "sd_raster_kernel", "sd_resolve_row_kernel"),
                WALK_WAVEFRONT: ("sd_setup_kernel", "sd_trace_wavefront_kernel"),
                WALK_HYBRID: ("sd_setup_kernel", "sd_trace_hybrid_kernel")}


# every symbol include/rsd.h declares (checked by tests/test_abi.py)
EXPORTS = ["rsd_abi_version", "rsd_svao_tile_count", "rsd_sd_tile_state_count", "rsd_svao_tile_flags_release", "rsd_last_error", "rsd_device_open", "rsd_device_close", "rsd_scene_upload",
           "rsd_scene_info_get", "rsd_scene_release", "rsd_camera_look_at", "rsd_svao_make_vao_data",
           "rsd_gbuffer", "rsd_sd_trace", "rsd_svao_clear_intervals", "rsd_svao_pass1", "rsd_svao_pass2",
           "rsd_sd_trace_band", "rsd_svao_pass1_band", "rsd_svao_pass2_band", "rsd_gbuffer_raster",
           "rsd_linearize_depth", "rsd_compress_normals", "rsd_svao_pass2_raytraced", "rsd_svao_pass2_raytraced_band",
           "rsd_scene_upload_alpha", "rsd_ray_cone_spread", "rsd_sd_trace_band_ex", "rsd_scene_export_bvh",
           "rsd_bvh_build", "rsd_svao_pass1_rows", "rsd_svao_pass2_rows", "rsd_sd_trace_rows", "rsd_svao_frame",
           "rsd_halo_compact", "rsd_halo_merge", "rsd_halo_sd_gather", "rsd_halo_sd_scatter",
           "rsd_comm_rccl_available", "rsd_comm_rccl_unique_id", "rsd_comm_rccl_create", "rsd_comm_hub_create", "rsd_comm_hub_release",
           "rsd_comm_local_create", "rsd_comm_null_create", "rsd_comm_release", "rsd_comm_info", "rsd_comm_all_gather", "rsd_comm_exchange",
           "rsd_band_frame_create", "rsd_band_frame_front", "rsd_band_frame_back", "rsd_band_frame_stats",
           "rsd_band_frame_release", "rsd_band_frame_set_split"]

SD_CONSUME_INTERVALS = 1
SD_THROUGHPUT = 2  # frames in flight: the work-efficient traversal (rsd.h RSD_SD_THROUGHPUT)

# every symbol include/rsd_graph.h declares
GRAPH_EXPORTS = ["rsd_graph_create", "rsd_graph_destroy", "rsd_graph_create_pass", "rsd_graph_add_edge",
                 "rsd_graph_mark_output", "rsd_graph_set_scene", "rsd_graph_set_input", "rsd_graph_compile",
                 "rsd_graph_execute", "rsd_graph_plan", "rsd_graph_resources", "rsd_graph_get_output",
                 "rsd_graph_copy_output", "rsd_graph_execution_order", "rsd_graph_pass_times",
                 "rsd_graph_get_dict_int", "rsd_graph_pass_count", "rsd_plugin_set_dir", "rsd_plugin_types",
                 "rsd_cross_bilateral_blur", "rsd_image_equation_compile", "rsd_image_equation_info",
                 "rsd_image_equation_run", "rsd_image_equation_release", "rsd_temporal_ao",
                 "rsd_motion_vectors", "rsd_motion_vectors_raster", "rsd_taa", "rsd_ao_flicker_mask", "rsd_binary_dilation",
                 "rsd_deinterleave", "rsd_interleave", "rsd_ray_min_max_length"]

FMT_R32F, FMT_RG32F, FMT_RGBA32F, FMT_R16U, FMT_R8U, FMT_R8UNORM, FMT_R32U, FMT_UNKNOWN = range(8)
FMT_R16F, FMT_RG16F, FMT_RGBA16F, FMT_RG8UNORM = 8, 9, 10, 11


class Texture(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32), ("layers", C.c_uint32),
                ("format", C.c_uint32), ("bytes", C.c_uint64)]

_lib = None


def lib():
    """Load librsd.so (in-tree).  Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"librsd.so not found at {LIB_PATH}: build it with `make -C {PKG_DIR}` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)  # global: render-pass plugins resolve the host's symbols
        vp, u32, i32, f32, st = C.c_void_p, C.c_uint32, C.c_int32, C.c_float, C.c_int
        L.rsd_abi_version.restype = u32
        L.rsd_svao_tile_count.restype = u32
        L.rsd_svao_tile_count.argtypes = [u32, u32, u32]
        L.rsd_sd_tile_state_count.restype = u32
        L.rsd_sd_tile_state_count.argtypes = [u32, u32]
        L.rsd_svao_tile_flags_release.restype = None
        L.rsd_svao_tile_flags_release.argtypes = [vp]
        L.rsd_last_error.restype = C.c_char_p
        L.rsd_device_open.restype = st
        L.rsd_device_open.argtypes = [C.c_int, C.POINTER(vp)]
        L.rsd_device_close.argtypes = [vp]
        L.rsd_scene_upload.restype = st
        L.rsd_scene_upload.argtypes = [vp, C.POINTER(SceneDesc), C.POINTER(vp)]
        L.rsd_scene_upload_alpha.restype = st
        L.rsd_scene_upload_alpha.argtypes = [vp, C.POINTER(SceneDesc), C.POINTER(AlphaDesc), C.POINTER(vp)]
        L.rsd_ray_cone_spread.restype = f32
        L.rsd_ray_cone_spread.argtypes = [f32, u32]
        L.rsd_scene_info_get.restype = st
        L.rsd_scene_info_get.argtypes = [vp, C.POINTER(SceneInfo)]
        L.rsd_scene_release.argtypes = [vp]
        L.rsd_scene_export_bvh.restype = st
        L.rsd_scene_export_bvh.argtypes = [vp, vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(u32)]
        L.rsd_bvh_build.restype = st
        L.rsd_bvh_build.argtypes = [C.POINTER(SceneDesc), vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(u32)]
        L.rsd_camera_look_at.restype = st
        L.rsd_camera_look_at.argtypes = [vp, vp, vp, f32, f32, f32, f32, f32, f32, C.POINTER(Camera)]
        L.rsd_svao_make_vao_data.restype = st
        L.rsd_svao_make_vao_data.argtypes = [u32, u32, u32, i32, f32, f32, f32, C.POINTER(VAOData),
                                             C.POINTER(u32), C.POINTER(u32)]
        L.rsd_gbuffer.restype = st
        L.rsd_gbuffer.argtypes = [vp, C.POINTER(Camera), u32, u32, u32, vp, vp, vp]
        L.rsd_sd_trace.restype = st
        L.rsd_sd_trace.argtypes = [vp, C.POINTER(Camera), C.POINTER(SDParams), vp, u32, u32, vp, vp, vp, u32, u32,
                                   C.POINTER(Counters), vp]
        L.rsd_svao_clear_intervals.restype = st
        L.rsd_svao_clear_intervals.argtypes = [vp, vp, u32, vp]
        L.rsd_svao_pass1.restype = st
        L.rsd_svao_pass1.argtypes = [C.POINTER(Camera), C.POINTER(VAOData), C.POINTER(SVAOParams), vp, vp, u32, u32,
                                     vp, vp, vp, vp, u32, u32, vp]
        L.rsd_svao_pass2.restype = st
        L.rsd_svao_pass2.argtypes = [C.POINTER(Camera), C.POINTER(VAOData), C.POINTER(SVAOParams), vp, vp, u32, u32,
                                     vp, vp, u32, u32, vp, vp]
        L.rsd_sd_trace_band.restype = st
        L.rsd_sd_trace_band.argtypes = [vp, C.POINTER(Camera), C.POINTER(SDParams), vp, u32, u32, vp, vp, vp, u32,
                                        u32, u32, u32, C.POINTER(Counters), vp]
        L.rsd_sd_trace_band_ex.restype = st
        L.rsd_sd_trace_band_ex.argtypes = [vp, C.POINTER(Camera), C.POINTER(SDParams), vp, u32, u32, vp, vp, vp, u32,
                                           u32, u32, u32, u32, C.POINTER(Counters), vp]
        L.rsd_svao_pass1_band.restype = st
        L.rsd_svao_pass1_band.argtypes = [C.POINTER(Camera), C.POINTER(VAOData), C.POINTER(SVAOParams), vp, vp, u32,
                                          u32, vp, vp, vp, vp, u32, u32, u32, u32, vp]
        L.rsd_svao_pass2_band.restype = st
        L.rsd_svao_pass2_band.argtypes = [C.POINTER(Camera), C.POINTER(VAOData), C.POINTER(SVAOParams), vp, vp, u32,
                                          u32, vp, vp, u32, u32, vp, u32, u32, vp]
        L.rsd_svao_pass1_rows.restype = st
        L.rsd_svao_pass1_rows.argtypes = L.rsd_svao_pass1_band.argtypes
        L.rsd_svao_pass2_rows.restype = st
        L.rsd_svao_pass2_rows.argtypes = L.rsd_svao_pass2_band.argtypes
        L.rsd_sd_trace_rows.restype = st
        L.rsd_sd_trace_rows.argtypes = [vp, C.POINTER(Camera), C.POINTER(SDParams), vp, u32, u32, vp, vp, vp, u32,
                                        u32, u32, u32, u32, C.POINTER(Counters), vp]
        L.rsd_svao_frame.restype = st
        L.rsd_svao_frame.argtypes = [C.POINTER(FrameDesc), u32, vp, vp]
        L.rsd_halo_compact.restype = st
        L.rsd_halo_compact.argtypes = [vp, vp, u32, u32, C.POINTER(HaloRegion), u32, vp]
        L.rsd_halo_merge.restype = st
        L.rsd_halo_merge.argtypes = [vp, vp, u32, u32, C.POINTER(HaloList), u32, u32, vp]
        L.rsd_halo_sd_gather.restype = st
        L.rsd_halo_sd_gather.argtypes = [vp, u32, u32, u32, u32, C.POINTER(HaloSdList), u32, vp]
        L.rsd_halo_sd_scatter.restype = st
        L.rsd_halo_sd_scatter.argtypes = [vp, u32, u32, u32, u32, C.POINTER(HaloSdList), u32, vp]
        L.rsd_comm_rccl_available.restype = st
        L.rsd_comm_rccl_available.argtypes = []
        L.rsd_comm_rccl_unique_id.restype = st
        L.rsd_comm_rccl_unique_id.argtypes = [vp]
        L.rsd_comm_rccl_create.restype = st
        L.rsd_comm_rccl_create.argtypes = [vp, u32, u32, C.POINTER(vp)]
        L.rsd_comm_hub_create.restype = st
        L.rsd_comm_hub_create.argtypes = [u32, C.POINTER(vp)]
        L.rsd_comm_hub_release.restype = None
        L.rsd_comm_hub_release.argtypes = [vp]
        L.rsd_comm_local_create.restype = st
        L.rsd_comm_local_create.argtypes = [vp, u32, C.POINTER(vp)]
        L.rsd_comm_null_create.restype = st
        L.rsd_comm_null_create.argtypes = [u32, u32, C.POINTER(vp)]
        L.rsd_comm_release.restype = None
        L.rsd_comm_release.argtypes = [vp]
        L.rsd_comm_info.restype = st
        L.rsd_comm_info.argtypes = [vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]
        L.rsd_comm_all_gather.restype = st
        L.rsd_comm_all_gather.argtypes = [vp, vp, vp, C.c_uint64, vp]
        L.rsd_comm_exchange.restype = st
        L.rsd_comm_exchange.argtypes = [vp, C.POINTER(CommXfer), u32, C.POINTER(CommXfer), u32, vp]
        L.rsd_band_frame_create.restype = st
        L.rsd_band_frame_create.argtypes = [C.POINTER(FrameDesc), C.POINTER(BandParams), vp, C.POINTER(vp)]
        L.rsd_band_frame_front.restype = st
        L.rsd_band_frame_front.argtypes = [vp, C.POINTER(Camera), vp]
        L.rsd_band_frame_back.restype = st
        L.rsd_band_frame_back.argtypes = [vp, vp, vp]
        L.rsd_band_frame_stats.restype = st
        L.rsd_band_frame_stats.argtypes = [vp, C.POINTER(BandStats)]
        L.rsd_band_frame_set_split.restype = st
        L.rsd_band_frame_set_split.argtypes = [vp, C.POINTER(u32), u32]
        L.rsd_band_frame_release.restype = None
        L.rsd_band_frame_release.argtypes = [vp]
        L.rsd_svao_pass2_raytraced.restype = st
        L.rsd_svao_pass2_raytraced.argtypes = [vp, C.POINTER(Camera), C.POINTER(VAOData), C.POINTER(SVAOParams), vp, vp,
                                               u32, u32, vp, vp, u32, u32, u32, vp]
        L.rsd_svao_pass2_raytraced_band.restype = st
        L.rsd_svao_pass2_raytraced_band.argtypes = [vp, C.POINTER(Camera), C.POINTER(VAOData), C.POINTER(SVAOParams),
                                                    vp, vp, u32, u32, vp, vp, u32, u32, u32, u32, u32, vp]
        L.rsd_gbuffer_raster.restype = st
        L.rsd_gbuffer_raster.argtypes = [vp, C.POINTER(Camera), u32, u32, u32, vp, vp, vp]
        L.rsd_linearize_depth.restype = st
        L.rsd_linearize_depth.argtypes = [vp, vp, u32, f32, f32, vp]
        L.rsd_compress_normals.restype = st
        L.rsd_compress_normals.argtypes = [vp, vp, u32, C.POINTER(Camera), vp]
        cs, sz, tp = C.c_char_p, C.c_size_t, C.POINTER(Texture)
        for name, args in {
            "rsd_graph_create": [cs, C.POINTER(vp)],
            "rsd_graph_create_pass": [vp, cs, cs, cs],
            "rsd_graph_add_edge": [vp, cs, cs],
            "rsd_graph_mark_output": [vp, cs],
            "rsd_graph_set_scene": [vp, vp, C.POINTER(Camera)],
            "rsd_graph_set_input": [vp, cs, tp],
            "rsd_graph_compile": [vp, u32, u32, vp],
            "rsd_graph_execute": [vp, vp],
            "rsd_graph_plan": [vp, u32, u32],
            "rsd_graph_resources": [vp, vp, sz, C.POINTER(sz)],
            "rsd_graph_get_output": [vp, cs, tp],
            "rsd_graph_copy_output": [vp, cs, vp, C.c_uint64, vp],
            "rsd_graph_execution_order": [vp, vp, sz, C.POINTER(sz)],
            "rsd_graph_pass_times": [vp, C.POINTER(f32), u32, C.POINTER(u32)],
            "rsd_graph_get_dict_int": [vp, cs, C.POINTER(C.c_int64)],
            "rsd_graph_pass_count": [vp, C.POINTER(u32), C.POINTER(u32)],
            "rsd_plugin_set_dir": [cs],
            "rsd_plugin_types": [vp, sz, C.POINTER(sz)],
        }.items():
            fn = getattr(L, name)
            fn.restype = st
            fn.argtypes = args
        L.rsd_cross_bilateral_blur.restype = st
        L.rsd_cross_bilateral_blur.argtypes = [vp, vp, u32, u32, vp, vp, u32, u32, u32, u32, u32, vp]
        L.rsd_temporal_ao.restype = st
        L.rsd_temporal_ao.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, C.POINTER(Camera), vp, vp, vp, vp]
        L.rsd_ao_flicker_mask.restype = st
        L.rsd_ao_flicker_mask.argtypes = [vp, vp, u32, u32, C.POINTER(Camera), vp, vp]
        L.rsd_binary_dilation.restype = st
        L.rsd_binary_dilation.argtypes = [vp, u32, u32, u32, vp, vp]
        L.rsd_taa.restype = st
        L.rsd_ray_min_max_length.restype = st
        L.rsd_ray_min_max_length.argtypes = [vp, vp, u32, u32, vp, vp]
        for fn in (L.rsd_deinterleave, L.rsd_interleave):
            fn.restype = st
            fn.argtypes = [vp, u32, u32, u32, vp, vp]
        L.rsd_taa.argtypes = [vp, vp, vp, u32, u32, f32, f32, u32, vp, vp]
        L.rsd_motion_vectors.restype = st
        L.rsd_motion_vectors.argtypes = [C.POINTER(Camera), C.POINTER(Camera), vp, u32, u32, vp, vp]
        L.rsd_motion_vectors_raster.restype = st
        L.rsd_motion_vectors_raster.argtypes = [C.POINTER(Camera), C.POINTER(Camera), vp, u32, u32, vp, vp]
        L.rsd_image_equation_compile.restype = st
        L.rsd_image_equation_compile.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.rsd_image_equation_info.restype = st
        L.rsd_image_equation_info.argtypes = [vp, C.POINTER(u32), C.POINTER(u32)]
        L.rsd_image_equation_run.restype = st
        L.rsd_image_equation_run.argtypes = [vp, C.POINTER(Texture), C.POINTER(Texture), vp]
        L.rsd_image_equation_release.restype = None
        L.rsd_image_equation_release.argtypes = [vp]
        L.rsd_graph_destroy.restype = None
        L.rsd_graph_destroy.argtypes = [vp]
        _lib = L
    return _lib


class RsdError(RuntimeError):
    def __init__(self, status, where):
        msg = lib().rsd_last_error().decode(errors="replace")
        super().__init__(f"{where}: {STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


def check(status, where):
    if status != RSD_OK:
        raise RsdError(status, where)


def last_error() -> str:
    """librsd's message of the last failed call on this thread."""
    return lib().rsd_last_error().decode(errors="replace")
