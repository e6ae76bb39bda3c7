// rsd_internal.h -- librsd private state shared by the host entry points and the launchers.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/rsd.h"
#include "bvh_build.h"

struct rsd_device {
    int hip_device = 0;
    int cu_count = 0;
};

namespace rsd {
// Alpha-masked materials on the device (csrc/alpha_test.h); triUV == null: none uploaded
struct AlphaData {
    const float* triUV = nullptr;      // 6 floats per primitive (uv0, uv1, uv2)
    const uint32_t* triMat = nullptr;  // material per primitive
    const float4* materials = nullptr; // {threshold (float16-rounded), constant alpha, texture (bits), 0}
    const uint4* textures = nullptr;   // {width, height, mip count, first texel}
    const uint8_t* texels = nullptr;   // all mips of all textures, R8
    float spread = 0.0f;               // RAY_CONE_SPREAD of the SD pass (set per launch)
};
}  // namespace rsd

struct rsd_scene {
    rsd_device* dev = nullptr;
    float4* d_nodes = nullptr;   // one allocation: 8 x float4 per wide node, then
    float4* d_tris = nullptr;    //   3 x float4 per triangle record (d_tris = d_nodes + tri_offset)
    uint32_t tri_offset = 0;     // in float4 units
    uint32_t triangle_count = 0;
    uint32_t node_count = 0;
    rsd::BvhStats stats;
    uint64_t device_bytes = 0;
    unsigned long long* d_counters = nullptr;  // 8 x u64 scratch for instrumented traces
    uint32_t* d_qctl = nullptr;    // live-ray queue control {count[32], head[32]} x 2 (double-buffered)
    uint32_t qctl_gen = 0;         // trace calls so far: buffer qctl_gen % 2 is zero and next in line
    bool qctl_dirty = true;        // reset both buffers before the next trace (first use, failed launch)
    void* d_queue = nullptr;       // SD-trace workspace (live-ray records + K-key slots), grow-only
    size_t queue_cap = 0;          // bytes
    void* d_alpha = nullptr;       // alpha data (rsd_scene_upload_alpha), one allocation
    rsd::AlphaData alpha;          // device pointers into d_alpha
};

namespace rsd {
void set_error(const std::string& msg);
rsd_status hip_fail(hipError_t e, const char* what);
}  // namespace rsd

#define RSD_HIP(call)                                                   \
    do {                                                                \
        hipError_t e_ = (call);                                         \
        if (e_ != hipSuccess) return rsd::hip_fail(e_, #call);          \
    } while (0)
