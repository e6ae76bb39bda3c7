// rsd_internal.h -- librsd private state shared by the host entry points and the launchers.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <vector>

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

namespace rsd {
// Per-frame-size ray terms of the SD setup (ray_table_kernel), keyed by what they depend on
struct RayTabCache {
    int w = -1, h = -1, guard = 0;
    uint32_t jitter = 0;
    float jx = 0.0f, jy = 0.0f;
    float camW[3] = {0.0f, 0.0f, 0.0f};
    int device = -1;
    float* d = nullptr;
    size_t cap = 0;
    bool same(const RayTabCache& k) const {
        return w == k.w && h == k.h && guard == k.guard && jitter == k.jitter && jx == k.jx && jy == k.jy &&
               camW[0] == k.camW[0] && camW[1] == k.camW[1] && camW[2] == k.camW[2] && device == k.device;
    }
    void setKey(const RayTabCache& k) {
        w = k.w; h = k.h; guard = k.guard; jitter = k.jitter; jx = k.jx; jy = k.jy;
        camW[0] = k.camW[0]; camW[1] = k.camW[1]; camW[2] = k.camW[2]; device = k.device;
    }
};

// Mutable SD-trace state of one (scene, stream) pair.  Traces of one scene on DIFFERENT
// streams may run concurrently (frames in flight): each stream owns its queue control,
// live-ray / key workspace and ray table, so concurrent launches never share scratch.
struct SdWorkspace {
    hipStream_t stream = nullptr;
    uint32_t* qctl = nullptr;      // live-ray queue control {count[32], head[32]} x 2 (double-buffered)
    uint32_t qctl_gen = 0;         // trace calls so far: buffer qctl_gen % 2 is zero and next in line
    bool qctl_dirty = true;        // reset both buffers before the next trace (first use, failed launch)
    void* queue = nullptr;         // live-ray records + K-key slots, grow-only
    size_t queue_cap = 0;          // bytes
    RayTabCache raytab;
    unsigned long long* counters = nullptr;  // 16 x u64 scratch of instrumented traces on this stream
    void* raster = nullptr;        // raster walk: slot map, tile records, 64-bit key lists (grow-only)
    size_t raster_cap = 0;         // bytes
};
void release_sd_workspaces(rsd_scene* s);
}  // namespace rsd

struct rsd_scene {
    rsd_device* dev = nullptr;
    float4* d_nodes = nullptr;   // one allocation: 8 x float4 per wide node, then
    float4* d_tris = nullptr;    //   3 x float4 per triangle record (d_tris = d_nodes + tri_offset)
    uint32_t tri_offset = 0;     // in float4 units
    uint32_t triangle_count = 0;
    uint32_t node_count = 0;
    rsd::BvhStats stats;
    uint32_t build_threads = 0;  // host threads of the BVH build
    uint64_t device_bytes = 0;
    uint64_t bvh_bytes = 0;      // the d_nodes allocation (nodes + triangle records + pad)
    uint32_t* d_prim_rec = nullptr;  // primitive id -> triangle record index (raster walk's keys)
    std::vector<rsd::SdWorkspace*> sd_ws;  // one per stream that traced this scene (few: linear lookup)
    std::mutex ws_mutex;                   // sd_ws: host threads may trace one scene on their own streams
    void* d_alpha = nullptr;       // alpha data (rsd_scene_upload_alpha), one allocation
    rsd::AlphaData alpha;          // device pointers into d_alpha
    // segment entry grid (entry_grid.h): one allocation, hash slots (uint4) then entry items
    void* d_entry = nullptr;
    uint32_t entry_bits = 0, entry_probe = 0, entry_rmax = 0, entry_cells = 0;
    float entry_origin[3] = {0.0f, 0.0f, 0.0f}, entry_extent = 0.0f;
    uint64_t entry_items_off = 0;  // bytes from d_entry to the item array
    double entry_build_ms = 0.0;
};

namespace rsd {
void set_error(const std::string& msg);
rsd_status hip_fail(hipError_t e, const char* what);

// halo.hip: the sparse-halo steps with the band frame's options (csrc/band_frame.cpp).  ilv: interleaved
// triples {texel, rayMin, rayMax} (a peer's prefix is one contiguous transfer); the SD lists then index
// with stride 3 (their idx points at the triples).  row: a count row zeroed ([0, row_n)) with
// row[row_n] = extra in the launch that zeroes the region counts; zeroed: the counts are already zero
// (the previous frame's compaction cleared them through zero_row), so the compaction launch alone writes
// row[row_n] and clears zero_row[0, row_n].
rsd_status halo_compact_impl(const uint32_t* d_ray_min, const uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h,
                             const rsd_halo_region* regions, uint32_t n_regions, bool ilv, int64_t* row,
                             uint32_t row_n, int64_t extra, hipStream_t s, bool zeroed = false,
                             int64_t* zero_row = nullptr);
// the band frame's count matrix (n int64) to host-visible memory dst[1..n], then dst[0] = seq (system-scope
// release): the host polls dst[0] instead of waiting on an event
rsd_status publish_counts(const int64_t* d_src, int64_t* dst_host_dev, uint32_t n, int64_t seq, hipStream_t s);
rsd_status halo_merge_impl(uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h,
                           const rsd_halo_list* lists, uint32_t n_lists, uint32_t ray_interval, bool ilv,
                           hipStream_t s);
rsd_status halo_sd_impl(bool gather, float* sd, uint32_t layers, uint32_t sd_w, uint32_t sd_h, uint32_t ch,
                        const rsd_halo_sd_list* lists, uint32_t n_lists, bool ilv, hipStream_t s, const char* who);
}  // namespace rsd

#define RSD_HIP(call)                                                   \
    do {                                                                \
        hipError_t e_ = (call);                                         \
        if (e_ != hipSuccess) return rsd::hip_fail(e_, #call);          \
    } while (0)
