// rsd_frame.cpp -- rsd_svao_frame: one SVAO frame per ABI call (include/rsd.h).
//
// SVAO::execute (SVAO.cpp:192-456) issues its dispatches from C++ in one RenderPass::execute; a host
// binding through Python / ctypes pays its interpreter and marshalling cost per dispatch instead (4
// calls of 13-16 arguments per frame).  This entry issues the whole sequence --
// interval clear (SVAO.cpp:330-341) -> "AO 1" (:344-350) -> StochasticDepthMapRT (:364-390, consuming
// the intervals) -> "AO 2" (:450-454) -- on one stream from C++, through the same entry points as the
// separate calls (same kernels, same bits), with optional timing events between the passes.
#include <hip/hip_runtime.h>

#include "rsd_internal.h"

namespace {
rsd_status record(void* const* events, int i, rsd_stream stream) {
    if (!events || !events[i]) return RSD_OK;
    hipError_t e = hipEventRecord((hipEvent_t)events[i], (hipStream_t)stream);
    return e == hipSuccess ? RSD_OK : rsd::hip_fail(e, "rsd_svao_frame: hipEventRecord");
}
}  // namespace

extern "C" rsd_status rsd_svao_frame(const rsd_svao_frame_desc* f, uint32_t flags, void* const* events,
                                     rsd_stream stream) {
    if (!f || !f->cam || !f->vao || !f->svao) {
        rsd::set_error("rsd_svao_frame: null frame description");
        return RSD_ERR_INVALID_ARG;
    }
    if (flags & ~(RSD_FRAME_INTERVALS_CLEAR | RSD_FRAME_KEEP_INTERVALS | RSD_SD_THROUGHPUT)) {
        rsd::set_error("rsd_svao_frame: unknown flag");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t mode = f->svao->secondary_depth_mode;
    if (mode > 3) {
        rsd::set_error("rsd_svao_frame: secondary_depth_mode must be 0 (SingleDepth), 1 (DualDepth), 2 (StochasticDepth)"
                       " or 3 (Raytraced)");
        return RSD_ERR_UNSUPPORTED;
    }
    if ((mode == 2 || mode == 3) && (!f->scene || !f->sd)) {
        rsd::set_error("rsd_svao_frame: the StochasticDepth and Raytraced modes need a scene and SD params");
        return RSD_ERR_INVALID_ARG;
    }
    rsd_status st = RSD_OK;
    const bool stochastic = mode == 2;
    if (stochastic && !(flags & RSD_FRAME_INTERVALS_CLEAR)) {
        st = rsd_svao_clear_intervals(f->d_ray_min, f->d_ray_max, f->sd_w * f->sd_h, stream);
        if (st != RSD_OK) return st;
    }
    if ((st = record(events, 0, stream)) != RSD_OK) return st;
    st = rsd_svao_pass1(f->cam, f->vao, f->svao, f->d_depth, f->d_normals, f->width, f->height, f->d_ao, f->d_stencil,
                        f->d_ray_min, f->d_ray_max, f->sd_w, f->sd_h, stream);
    if (st != RSD_OK) return st;
    if ((st = record(events, 1, stream)) != RSD_OK) return st;
    if (stochastic) {
        // the trace resets the interval maps it read (RayInterval): the next frame needs no clear
        const bool consume = f->sd->ray_interval && !(flags & RSD_FRAME_KEEP_INTERVALS);
        const uint32_t tf = (consume ? RSD_SD_CONSUME_INTERVALS : 0u) | (flags & RSD_SD_THROUGHPUT);
        st = rsd_sd_trace_band_ex(f->scene, f->cam, f->sd, f->d_depth, f->width, f->height, f->d_ray_min,
                                  f->d_ray_max, f->d_sd, f->sd_w, f->sd_h, 0, 1, tf, nullptr, stream);
        if (st != RSD_OK) return st;
    }
    if ((st = record(events, 2, stream)) != RSD_OK) return st;
    if (stochastic || mode == 1) {
        st = rsd_svao_pass2(f->cam, f->vao, f->svao, f->d_depth, f->d_normals, f->width, f->height, f->d_stencil,
                            f->d_sd, f->sd_w, f->sd_h, f->d_ao, stream);
    } else if (mode == 3) {
        st = rsd_svao_pass2_raytraced(f->scene, f->cam, f->vao, f->svao, f->d_depth, f->d_normals, f->width,
                                      f->height, f->d_stencil, f->d_ao, f->sd->cull_mode, f->ray_pipeline,
                                      f->sd->alpha_test, stream);
    }
    if (st != RSD_OK) return st;
    return record(events, 3, stream);
}
