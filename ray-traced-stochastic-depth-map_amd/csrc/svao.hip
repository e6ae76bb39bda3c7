// svao.hip -- SVAO "AO 1" and "AO 2" compute passes on gfx950.
//
// Reference: SVAORaster.ps.slang:29-122 (pass 1), SVAORaster2.ps.slang:48-65 (pass 2),
//            SVAO/Common.slang:98-663 (BasicAOData / SampleAOData / calcAO2),
//            SVAO.cpp:327-354 (clears + pass-1 dispatch), :450-454 (pass-2 dispatch),
//            SVAO.cpp:663-688 (noise texture).
// Both passes are screen-space, HBM/L2-bound: pass 1 does ~10 depth fetches per pixel and
// two device-scope integer atomics per refined direction; pass 2 gathers popc(mask) x N
// SD depths at texels up to ssMaxRadius away.  Per-pixel transcendentals are tables
// (16 noise angles, 8 direction angles) computed on the host in double and rounded once;
// the only per-pixel libm call left is pow() in finalize (SVAO Common.slang:326-330).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "rsd_device.h"
#include "rsd_internal.h"
#include "svao_math.h"

namespace rsd {

// SVAO.cpp:334-340
__global__ void clear_intervals_kernel(uint32_t* rmin, uint32_t* rmax, uint32_t n) {
    // 4 texels per lane with 16-B stores where both buffers are 16-B aligned
    const uint32_t i = 4u * (blockIdx.x * blockDim.x + threadIdx.x);
    const bool vec = ((reinterpret_cast<uintptr_t>(rmin) | reinterpret_cast<uintptr_t>(rmax)) & 15u) == 0u;
    if (vec && i + 4u <= n) {
        reinterpret_cast<uint4*>(rmax)[i / 4u] = make_uint4(0u, 0u, 0u, 0u);
        reinterpret_cast<uint4*>(rmin)[i / 4u] = make_uint4(0x7f7fffffu, 0x7f7fffffu, 0x7f7fffffu, 0x7f7fffffu);
        return;
    }
    for (uint32_t k = i; k < n && k < i + 4u; ++k) {
        rmax[k] = 0u;
        rmin[k] = 0x7f7fffffu;  // asuint(FLT_MAX)
    }
}

}  // namespace rsd

// the kernels with the numerics contract (bit-identical to the oracle): rsd::exact
#define RSD_SVAO_NS exact
#include "svao_kernels.h"

namespace rsd {
namespace fast {  // svao_fast.hip: the same kernels with fast numerics (RSD_NUMERICS_FAST)
void launch_pass1(const SvaoArgs& a, int variant, dim3 grid, dim3 block, hipStream_t s);
void launch_pass2(const SvaoArgs& a, uint32_t N, uint32_t nd, bool spec, dim3 grid, dim3 block, hipStream_t s,
                  bool list, bool loop);
}  // namespace fast
}  // namespace rsd

namespace rsd {
namespace {
// Device-resident constant tables, cached per device for the life of the process (a few KB to
// 1 MB each, never freed: a table may still be read by kernels in flight on any stream).
// Process-wide with a lock: one rsd_device per GPU per host thread (rsd.h), any thread, any GPU.
constexpr int kMaxDevices = 64;
std::mutex g_tab_mutex;

__global__ void normal_lut_kernel(float4* lut) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 65536u) {
        const f3 n = decode_normal_2x8(i);
        lut[i] = make_float4(n.x, n.y, n.z, 0.0f);
    }
}
float4* g_nlut[kMaxDevices] = {};

struct SnapTable {
    int w, h;
    float* d;
};
std::vector<SnapTable> g_snap[kMaxDevices];  // per device: one table per frame-buffer size

int current_device(int* dev) {
    if (hipGetDevice(dev) != hipSuccess || *dev < 0 || *dev >= kMaxDevices) return -1;
    return 0;
}
}  // namespace

rsd_status normal_lut(const float4** out) {
    int dev = 0;
    if (current_device(&dev)) {
        set_error("normal_lut: no current HIP device (or device index >= 64)");
        return RSD_ERR_NO_DEVICE;
    }
    std::lock_guard<std::mutex> lock(g_tab_mutex);
    if (!g_nlut[dev]) {
        float4* d = nullptr;
        RSD_HIP(hipMalloc(&d, 65536 * sizeof(float4)));
        hipLaunchKernelGGL(normal_lut_kernel, dim3(256), dim3(256), 0, (hipStream_t)0, d);
        RSD_HIP(hipGetLastError());
        RSD_HIP(hipDeviceSynchronize());  // once per device
        g_nlut[dev] = d;
    }
    *out = g_nlut[dev];
    return RSD_OK;
}

// pixel-centre UVs (k + 0.5) / resolution of every column and row of the frame buffer
rsd_status snap_tables(const rsd_vao_data& vd, const float** u, const float** v) {
    const int w = (int)vd.resolution[0], h = (int)vd.resolution[1];
    int dev = 0;
    if (current_device(&dev)) {
        set_error("snap_tables: no current HIP device (or device index >= 64)");
        return RSD_ERR_NO_DEVICE;
    }
    std::lock_guard<std::mutex> lock(g_tab_mutex);
    for (const SnapTable& t : g_snap[dev])
        if (t.w == w && t.h == h) {
            *u = t.d;
            *v = t.d + w + 1;
            return RSD_OK;
        }
    std::vector<float> t((size_t)w + 1 + (size_t)h + 1);
    for (int k = 0; k <= w; ++k) t[k] = ((float)k + 0.5f) / vd.resolution[0];
    for (int k = 0; k <= h; ++k) t[(size_t)w + 1 + k] = ((float)k + 0.5f) / vd.resolution[1];
    float* d = nullptr;
    RSD_HIP(hipMalloc(&d, t.size() * sizeof(float)));
    RSD_HIP(hipMemcpy(d, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
    g_snap[dev].push_back({w, h, d});
    *u = d;
    *v = d + w + 1;
    return RSD_OK;
}
}  // namespace rsd

using namespace rsd;

namespace {
// fill_consts of (VAOData, NUM_DIRECTIONS), cached per host thread: the ~50 double sin / cos and the
// ssRadiusCutoff search are host work every pass-1 / pass-2 call would otherwise repeat per frame
void cached_consts(SvaoConsts& k, const rsd_vao_data& d, uint32_t nd, uint32_t kernel) {
    struct Entry {
        rsd_vao_data d;
        uint32_t nd, kernel;
        SvaoConsts k;
    };
    thread_local Entry cache[4];
    thread_local int used = 0, next = 0;
    for (int i = 0; i < used; ++i)
        if (cache[i].nd == nd && cache[i].kernel == kernel && std::memcmp(&cache[i].d, &d, sizeof(d)) == 0) {
            k = cache[i].k;
            return;
        }
    fill_consts(k, d, nd, kernel);
    Entry& e = cache[next];
    e.d = d;
    e.nd = nd;
    e.kernel = kernel;
    e.k = k;
    next = (next + 1) % 4;
    used = used < 4 ? used + 1 : 4;
}
// The busy-tile list's generation per tile buffer.  Pass 1 of generation g appends to count[g & 1] and
// zeroes count[(g + 1) & 1]; the whole-frame pass 2 walks count[g & 1]; the first pass 2 after a pass 1
// (whatever its rows) moves the buffer to g + 1.  Stream order makes every step see the previous one:
// the zeroing of pass 1 (g + 1) lands after pass 2 (g) read that count, so no kernel resets the list
// and no workgroup waits for the others (a per-workgroup completion ticket on one address serialised
// pass 2: 150-240 us at configs[1]).  Host-side state, one lock, a few entries per process.
struct TileGen {
    uint32_t gen = 0;
    bool appended = false;  // a pass 1 ran since the last pass 2
};
std::mutex g_tile_mutex;
std::vector<std::pair<const void*, TileGen>> g_tile_gen;  // per buffer; rsd_svao_tile_flags_release forgets one

TileGen& tile_gen_locked(const void* buf) {
    for (auto& e : g_tile_gen)
        if (e.first == buf) return e.second;
    g_tile_gen.push_back({buf, TileGen{}});
    return g_tile_gen.back().second;
}

// the list count pass 1 appends to (gen & 1) and its flag stamp (gen + 1, never 0)
uint32_t tile_gen_pass1(const void* buf, uint32_t* stamp) {
    *stamp = 1u;
    if (!buf) return 0u;
    std::lock_guard<std::mutex> lock(g_tile_mutex);
    TileGen& t = tile_gen_locked(buf);
    t.appended = true;
    *stamp = t.gen % 0xfffffffeu + 1u;
    return t.gen & 1u;
}

uint32_t tile_gen_pass2(const void* buf) {
    if (!buf) return 0u;
    std::lock_guard<std::mutex> lock(g_tile_mutex);
    TileGen& t = tile_gen_locked(buf);
    const uint32_t g = t.gen & 1u;
    if (t.appended) {
        ++t.gen;
        t.appended = false;
    }
    return g;
}
}  // namespace

extern "C" void rsd_svao_tile_flags_release(const void* tile_flags) {
    if (!tile_flags) return;
    std::lock_guard<std::mutex> lock(g_tile_mutex);
    for (size_t i = 0; i < g_tile_gen.size(); ++i)
        if (g_tile_gen[i].first == tile_flags) {
            g_tile_gen.erase(g_tile_gen.begin() + (long)i);
            return;
        }
}

extern "C" uint32_t rsd_svao_tile_count(uint32_t width, uint32_t height, uint32_t guard_band) {
    if (2 * guard_band >= width || 2 * guard_band >= height) return 0u;
    return tile_buffer_bytes(tiles_x(width, guard_band) * tiles_y(height, guard_band));
}

extern "C" rsd_status rsd_svao_clear_intervals(uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t count,
                                               rsd_stream stream) {
    if (!d_ray_min || !d_ray_max) {
        set_error("rsd_svao_clear_intervals: null buffer");
        return RSD_ERR_INVALID_ARG;
    }
    if (count == 0) return RSD_OK;
    hipLaunchKernelGGL(clear_intervals_kernel, dim3((count + 1023) / 1024), dim3(256), 0, (hipStream_t)stream, d_ray_min,
                       d_ray_max, count);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "clear_intervals_kernel launch");
}

static rsd_status check_band(uint32_t index, uint32_t count, const char* who) {
    if (count == 0 || index >= count) {
        set_error(std::string(who) + ": band_index must be < band_count");
        return RSD_ERR_INVALID_ARG;
    }
    return RSD_OK;
}

// 32-row groups g = start + k * step, k < n -- or, with n = ~0u, every group of an interleaved band
// (start = index, step = count) -- counted from the first visible row
namespace {
rsd_status pass1_impl(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p, const float* d_depth,
                      const uint16_t* d_normals, uint32_t W, uint32_t H, uint8_t* d_ao, uint8_t* d_stencil,
                      uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h, uint32_t start,
                      uint32_t step, uint32_t n, rsd_stream stream) {
    rsd_status st = check_common(cam, vao, p, d_depth, d_normals, W, H, "rsd_svao_pass1");
    if (st != RSD_OK) return st;
    if (!d_ao || !d_stencil || (p->secondary_depth_mode == 2 && (!d_ray_min || !d_ray_max || !sd_w || !sd_h))) {
        set_error("rsd_svao_pass1: null output buffer");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->secondary_depth_mode == 2 &&
        (sd_w != (uint32_t)vao->lowResolution[0] + 2u * (uint32_t)vao->sdGuard ||
         sd_h != (uint32_t)vao->lowResolution[1] + 2u * (uint32_t)vao->sdGuard)) {
        set_error("rsd_svao_pass1: SD map size does not match lowResolution + 2 sdGuard");
        return RSD_ERR_INVALID_ARG;
    }
    SvaoArgs a{};
    a.cam = *cam;
    a.d = *vao;
    cached_consts(a.k, a.d, p->num_directions, p->ao_kernel);
    {
        rsd_status ts = snap_tables(a.d, &a.snapU, &a.snapV);
        if (ts == RSD_OK) ts = normal_lut(&a.nlut);
        if (ts != RSD_OK) return ts;
    }
    fill_scale(a);
    a.depth = d_depth;
    a.normals = d_normals;
    a.W = (int)W;
    a.H = (int)H;
    a.ao = d_ao;
    a.stencil = d_stencil;
    a.rayMin = d_ray_min;
    a.rayMax = d_ray_max;
    a.sdW = (int)sd_w;
    a.sdH = (int)sd_h;
    a.guard = p->guard_band;
    a.secondary = p->secondary_depth_mode;
    a.dual = p->dual_ao ? 1u : 0u;
    a.rayInterval = p->ray_interval;
    a.sdJitter = p->sd_jitter;
    a.N = p->sd_samples;
    tile_layout(p->tile_flags, tiles_x(W, p->guard_band) * tiles_y(H, p->guard_band), a.tileFlags, a.tileCount,
                a.tileList);
    a.tilesX = tiles_x(W, p->guard_band);
    a.dualDepth = p->primary_depth_mode == 1u ? 1u : 0u;
    a.depth2 = p->d_depth2;
    // SVAO.cpp:347-350: nThreads = roundup32(dims - 2 guardBand), 16x16 groups
    const uint32_t nx = (W - 2 * p->guard_band + 31u) / 32u * 32u, ny = (H - 2 * p->guard_band + 31u) / 32u * 32u;
    const uint32_t groups = ny / 32u;
    const uint32_t bandGroups = std::min(n, groups > start ? (groups - start + step - 1) / step : 0u);
    a.bandIndex = start;
    a.bandCount = step;
    if (bandGroups == 0) return RSD_OK;
    a.tileGen = tile_gen_pass1(a.tileFlags, &a.tileStamp);
    {
        const char* xcdEnv = std::getenv("RSD_PASS1_XCD");  // A/B runs: workgroup chunks per XCD (0: off)
        a.xcdChunk = xcdEnv ? (uint32_t)std::max(0, std::atoi(xcdEnv)) : 0u;
    }
    // the specialised kernel for the StochasticDepth frame (every BASELINE config); RSD_PASS1=generic
    // forces the generic one (A/B runs)
    const char* p1Env = std::getenv("RSD_PASS1");
    const uint32_t allDirs = a.k.nd == 32u ? 0xffffffffu : (1u << a.k.nd) - 1u;
    const bool spec = !(p1Env && std::strcmp(p1Env, "generic") == 0) && a.secondary == 2u && a.rayInterval &&
                      !a.k.hbao && !a.dualDepth &&
                      a.k.samePixelInt && a.d.sdGuard > 0 && W <= 4096u && H <= 4096u &&
                      (a.k.fastDiv & allDirs) == allDirs && a.d.radius < 0x1p58f;
    const dim3 grid(nx / 16, 2 * bandGroups), block(16, 16);
    const int variant = spec ? (a.k.nd == 8u ? 1 : 2) : 0;
    if (p->numerics == RSD_NUMERICS_EXACT) exact::launch_pass1(a, variant, grid, block, (hipStream_t)stream);
    else fast::launch_pass1(a, variant, grid, block, (hipStream_t)stream);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "svao_pass1_kernel launch");
}
}  // namespace

extern "C" rsd_status rsd_svao_pass1_band(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                                          uint32_t sd_w, uint32_t sd_h, uint32_t band_index, uint32_t band_count,
                                          rsd_stream stream) {
    rsd_status st = check_band(band_index, band_count, "rsd_svao_pass1_band");
    if (st != RSD_OK) return st;
    return pass1_impl(cam, vao, p, d_depth, d_normals, W, H, d_ao, d_stencil, d_ray_min, d_ray_max, sd_w, sd_h,
                      band_index, band_count, ~0u, stream);
}

extern "C" rsd_status rsd_svao_pass1_rows(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                                          uint32_t sd_w, uint32_t sd_h, uint32_t row0, uint32_t row1,
                                          rsd_stream stream) {
    if (!p) {
        set_error("rsd_svao_pass1_rows: null params");
        return RSD_ERR_INVALID_ARG;
    }
    if (row0 > row1 || row0 % 32u != 0u || (row1 % 32u != 0u && row1 + 2u * (uint32_t)p->guard_band < H)) {
        set_error("rsd_svao_pass1_rows: rows must be multiples of 32 from the first visible row (row1 may end the frame)");
        return RSD_ERR_INVALID_ARG;
    }
    return pass1_impl(cam, vao, p, d_depth, d_normals, W, H, d_ao, d_stencil, d_ray_min, d_ray_max, sd_w, sd_h,
                      row0 / 32u, 1u, (row1 - row0 + 31u) / 32u, stream);
}

namespace {
rsd_status pass2_impl(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p, const float* d_depth,
                      const uint16_t* d_normals, uint32_t W, uint32_t H, const uint8_t* d_stencil, const float* d_sd,
                      uint32_t sd_w, uint32_t sd_h, uint8_t* d_ao, uint32_t start, uint32_t step, uint32_t n,
                      rsd_stream stream) {
    rsd_status st = check_common(cam, vao, p, d_depth, d_normals, W, H, "rsd_svao_pass2");
    if (st != RSD_OK) return st;
    // secondary DualDepth (1) refines nothing and reads no SD map; StochasticDepth (2) needs it
    const bool needSd = p->secondary_depth_mode != 1u;
    if (!d_stencil || !d_ao || (needSd && (!d_sd || !sd_w || !sd_h))) {
        set_error("rsd_svao_pass2: null buffer");
        return RSD_ERR_INVALID_ARG;
    }
    if (p->secondary_depth_mode != 1u && p->secondary_depth_mode != 2u) {
        set_error("rsd_svao_pass2: secondary_depth_mode must be 2 (StochasticDepth) or 1 (DualDepth); Raytraced is "
                  "rsd_svao_pass2_raytraced");
        return RSD_ERR_INVALID_ARG;
    }
    const uint32_t N = p->sd_samples;
    if (N != 1 && N != 2 && N != 4 && N != 8 && N != 16) {
        set_error("rsd_svao_pass2: MSAA_SAMPLES must be 1, 2, 4, 8 or 16");
        return RSD_ERR_UNSUPPORTED;
    }
    SvaoArgs a{};
    a.cam = *cam;
    a.d = *vao;
    cached_consts(a.k, a.d, p->num_directions, p->ao_kernel);
    {
        rsd_status ts = snap_tables(a.d, &a.snapU, &a.snapV);
        if (ts == RSD_OK) ts = normal_lut(&a.nlut);
        if (ts != RSD_OK) return ts;
    }
    fill_scale(a);
    a.depth = d_depth;
    a.normals = d_normals;
    a.W = (int)W;
    a.H = (int)H;
    a.ao = d_ao;
    a.stencil = const_cast<uint8_t*>(d_stencil);
    a.sd = d_sd;
    a.sdW = (int)sd_w;
    a.sdH = (int)sd_h;
    a.guard = p->guard_band;
    a.secondary = p->secondary_depth_mode;
    a.dual = p->dual_ao ? 1u : 0u;
    a.rayInterval = p->ray_interval;
    a.sdJitter = p->sd_jitter;
    a.N = N;
    tile_layout(p->tile_flags, tiles_x(W, p->guard_band) * tiles_y(H, p->guard_band), a.tileFlags, a.tileCount,
                a.tileList);
    a.tilesX = tiles_x(W, p->guard_band);
    a.dualDepth = p->primary_depth_mode == 1u ? 1u : 0u;
    a.depth2 = p->d_depth2;
    const uint32_t vw = W - 2 * p->guard_band, vh = H - 2 * p->guard_band;
    const uint32_t groups = (vh + 31u) / 32u;
    const uint32_t bandGroups = std::min(n, groups > start ? (groups - start + step - 1) / step : 0u);
    a.bandIndex = start;
    a.bandCount = step;
    if (bandGroups == 0) return RSD_OK;
    dim3 grid((vw + exact::kP2Tile - 1) / exact::kP2Tile, (32 / exact::kP2Tile) * bandGroups), block(exact::kP2Lanes);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t nd = a.k.nd;
    // the specialised kernel (8 directions; RSD_PASS2=generic forces the generic one for A/B runs)
    const char* p2Env = std::getenv("RSD_PASS2");
    const bool spec = !(p2Env && std::strcmp(p2Env, "generic") == 0) && nd == 8u && W <= 4096u && H <= 4096u &&
                      !a.k.hbao && !a.dualDepth && a.secondary == 2u &&
                      (a.k.fastDiv & 0xffu) == 0xffu && a.d.lowResolution[0] >= 1.0f &&
                      a.d.lowResolution[0] <= 0x1p20f && a.d.lowResolution[1] >= 1.0f && a.d.lowResolution[1] <= 0x1p20f &&
                      a.d.radius < 0x1p58f;
    // the whole frame with busy-tile flags: pass 1's list of busy tiles, list entry i in workgroup i (one
    // per tile of the frame: the count is on the device; the empty tail retires at once), instead of
    // the flag grid (RSD_PASS2_LIST=off, A/B runs)
    const uint32_t T = tiles_x(W, p->guard_band) * tiles_y(H, p->guard_band);
    const char* listEnv = std::getenv("RSD_PASS2_LIST");
    const bool list = a.tileFlags && start == 0u && step == 1u && bandGroups == groups &&
                      !(listEnv && std::strcmp(listEnv, "off") == 0);
    if (list) grid = dim3(T);
    // the specialised list strides over its tiles in the resident grid (RSD_PASS2_LOOP=off: one workgroup
    // per tile of the frame, A/B runs)
    const char* loopEnv = std::getenv("RSD_PASS2_LOOP");  // read per call: a test compares both
    const bool loop = list && spec && !(loopEnv && std::strcmp(loopEnv, "off") == 0);
    a.tileGen = tile_gen_pass2(a.tileFlags);
    if (p->numerics == RSD_NUMERICS_EXACT) exact::launch_pass2(a, N, nd, spec, grid, block, s, list, loop);
    else fast::launch_pass2(a, N, nd, spec, grid, block, s, list, loop);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, "svao_pass2_kernel launch");
}
}  // namespace

extern "C" rsd_status rsd_svao_pass2_band(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                                          uint8_t* d_ao, uint32_t band_index, uint32_t band_count, rsd_stream stream) {
    rsd_status st = check_band(band_index, band_count, "rsd_svao_pass2_band");
    if (st != RSD_OK) return st;
    return pass2_impl(cam, vao, p, d_depth, d_normals, W, H, d_stencil, d_sd, sd_w, sd_h, d_ao, band_index, band_count,
                      ~0u, stream);
}

extern "C" rsd_status rsd_svao_pass2_rows(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                          const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                          const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                                          uint8_t* d_ao, uint32_t row0, uint32_t row1, rsd_stream stream) {
    if (!p) {
        set_error("rsd_svao_pass2_rows: null params");
        return RSD_ERR_INVALID_ARG;
    }
    if (row0 > row1 || row0 % 32u != 0u || (row1 % 32u != 0u && row1 + 2u * (uint32_t)p->guard_band < H)) {
        set_error("rsd_svao_pass2_rows: rows must be multiples of 32 from the first visible row (row1 may end the frame)");
        return RSD_ERR_INVALID_ARG;
    }
    return pass2_impl(cam, vao, p, d_depth, d_normals, W, H, d_stencil, d_sd, sd_w, sd_h, d_ao, row0 / 32u, 1u,
                      (row1 - row0 + 31u) / 32u, stream);
}

extern "C" rsd_status rsd_svao_pass1(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                     const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                     uint8_t* d_ao, uint8_t* d_stencil, uint32_t* d_ray_min, uint32_t* d_ray_max,
                                     uint32_t sd_w, uint32_t sd_h, rsd_stream stream) {
    return rsd_svao_pass1_band(cam, vao, p, d_depth, d_normals, W, H, d_ao, d_stencil, d_ray_min, d_ray_max, sd_w,
                               sd_h, 0, 1, stream);
}

extern "C" rsd_status rsd_svao_pass2(const rsd_camera* cam, const rsd_vao_data* vao, const rsd_svao_params* p,
                                     const float* d_depth, const uint16_t* d_normals, uint32_t W, uint32_t H,
                                     const uint8_t* d_stencil, const float* d_sd, uint32_t sd_w, uint32_t sd_h,
                                     uint8_t* d_ao, rsd_stream stream) {
    return rsd_svao_pass2_band(cam, vao, p, d_depth, d_normals, W, H, d_stencil, d_sd, sd_w, sd_h, d_ao, 0, 1, stream);
}
