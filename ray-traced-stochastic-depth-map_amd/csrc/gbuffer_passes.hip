// gbuffer_passes.hip -- the G-buffer producers of the SVAO graph, so
// scripts/SVAO.py's data flow runs on librsd end to end:
//   GBufferRaster.depth (non-linear D32 depth) + GBufferRaster.faceNormalW
//     -> LinearizeDepth.linearDepth (Linearize.ps.slang)
//     -> CompressNormals.normalOut (CompressNormals.ps.slang, viewSpace + use16Bit)
// GBufferRaster itself is the closest-hit traversal of sd_trace.hip (rsd_gbuffer_raster);
// the two converters are elementwise kernels here.
#include "rsd_device.h"
#include "rsd_internal.h"

namespace rsd {

// LinearizeDepth/Linearize.ps.slang: zNear * zFar / (zFar + d * (zNear - zFar))
__global__ void linearize_depth_kernel(const float* __restrict__ d, float* __restrict__ z, uint32_t n, float zn,
                                       float zf) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) z[i] = zn * zf / (zf + d[i] * (zn - zf));
}

// CompressNormals.ps.slang: normal = mul(float3x3(gViewMat), n); encodeNormal2x8
__global__ void compress_normals_kernel(const float4* __restrict__ nw, uint16_t* __restrict__ out, uint32_t n,
                                        rsd_camera cam) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = nw[i];
    const float* m = cam.viewMat;
    const f3 nv = mk(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
                     m[8] * v.x + m[9] * v.y + m[10] * v.z);
    out[i] = (uint16_t)encode_normal_2x8(nv);
}

}  // namespace rsd

using namespace rsd;

extern "C" rsd_status rsd_linearize_depth(const float* d_depth, float* d_linear_z, uint32_t count, float near_z,
                                          float far_z, rsd_stream stream) {
    if (!d_depth || !d_linear_z) {
        set_error("rsd_linearize_depth: null buffer");
        return RSD_ERR_INVALID_ARG;
    }
    if (!count) return RSD_OK;
    hipLaunchKernelGGL(linearize_depth_kernel, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_depth,
                       d_linear_z, count, near_z, far_z);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "linearize_depth_kernel launch");
}

extern "C" rsd_status rsd_compress_normals(const float* d_normal_w, uint16_t* d_packed, uint32_t count,
                                           const rsd_camera* cam, rsd_stream stream) {
    if (!d_normal_w || !d_packed || !cam) {
        set_error("rsd_compress_normals: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    if (!count) return RSD_OK;
    hipLaunchKernelGGL(compress_normals_kernel, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(d_normal_w), d_packed, count, *cam);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "compress_normals_kernel launch");
}
