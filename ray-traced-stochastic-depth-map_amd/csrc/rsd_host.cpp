// rsd_host.cpp -- librsd host entry points: errors, devices, scene upload (BVH build +
// HBM residency), camera and SVAO constant derivation.  No GPU work besides copies.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "entry_grid.h"
#include "rsd_internal.h"

namespace rsd {
namespace {
thread_local std::string g_last_error;
}
void set_error(const std::string& msg) { g_last_error = msg; }
rsd_status hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? RSD_ERR_OUT_OF_MEMORY : RSD_ERR_HIP;
}
}  // namespace rsd

using rsd::set_error;

extern "C" uint32_t rsd_abi_version(void) { return RSD_ABI_VERSION; }

extern "C" const char* rsd_last_error(void) { return rsd::g_last_error.c_str(); }

extern "C" rsd_status rsd_device_open(int hip_device, rsd_device** out) {
    if (!out) {
        set_error("rsd_device_open: out is null");
        return RSD_ERR_INVALID_ARG;
    }
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        set_error("rsd_device_open: no HIP device available");
        return RSD_ERR_NO_DEVICE;
    }
    if (hip_device < 0 || hip_device >= n) {
        set_error("rsd_device_open: device index out of range");
        return RSD_ERR_INVALID_ARG;
    }
    RSD_HIP(hipSetDevice(hip_device));
    hipDeviceProp_t prop;
    RSD_HIP(hipGetDeviceProperties(&prop, hip_device));
    auto* d = new rsd_device;
    d->hip_device = hip_device;
    d->cu_count = prop.multiProcessorCount;
    *out = d;
    return RSD_OK;
}

extern "C" void rsd_device_close(rsd_device* dev) { delete dev; }

namespace {
// cgroup v2 CPU quota of this process ("max 100000" = none): ceil(quota / period) CPUs, or 0
unsigned cgroup_cpu_quota() {
    FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r");
    if (!f) return 0;
    char q[32] = {0};
    long long period = 0;
    const int n = std::fscanf(f, "%31s %lld", q, &period);
    std::fclose(f);
    if (n != 2 || period <= 0 || std::strcmp(q, "max") == 0) return 0;
    const long long quota = std::atoll(q);
    return quota > 0 ? (unsigned)((quota + period - 1) / period) : 0;
}

// Host threads of the BVH build: the CPUs this process may actually use -- its affinity mask (what a
// container or `taskset` grants) capped by the cgroup CPU quota (a GPU box shows 256 CPUs under a
// 16-CPU quota; bench.py's cpu_baseline counts cores the same way) -- or RSD_BUILD_THREADS.
unsigned build_threads() {
    if (const char* env = std::getenv("RSD_BUILD_THREADS"))
        if (int n = std::atoi(env); n > 0) return (unsigned)n;
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) n = (unsigned)CPU_COUNT(&set);
    if (const unsigned q = cgroup_cpu_quota()) n = std::min(n, q);
    return std::max(1u, n);
}
}  // namespace

extern "C" rsd_status rsd_scene_upload(rsd_device* dev, const rsd_scene_desc* desc, rsd_scene** out) {
    if (!dev || !desc || !out || (desc->triangle_count && (!desc->positions || !desc->indices))) {
        set_error("rsd_scene_upload: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    *out = nullptr;
    for (uint64_t i = 0; i < 3ull * desc->triangle_count; ++i)
        if (desc->indices[i] >= desc->vertex_count) {
            set_error("rsd_scene_upload: index out of range of vertex_count");
            return RSD_ERR_INVALID_ARG;
        }
    if (desc->triangle_count >= (1u << 30)) {
        set_error("rsd_scene_upload: too many triangles");
        return RSD_ERR_UNSUPPORTED;
    }
    RSD_HIP(hipSetDevice(dev->hip_device));
    const unsigned threads = build_threads();
    rsd::FlatBvh bvh = rsd::build_bvh(desc->positions, desc->vertex_count, desc->indices, desc->triangle_count,
                                      desc->triangle_flags, threads);
    auto* s = new rsd_scene;
    s->dev = dev;
    s->triangle_count = desc->triangle_count;
    s->node_count = (uint32_t)(bvh.nodes.size() / 32);
    s->stats = bvh.stats;
    s->build_threads = threads;
    // one allocation: wide nodes, then triangle records, then 12 x 16 B of padding so a
    // traversal step may always fetch 192 B (DESIGN.md "BVH layout in HBM")
    const size_t nb = bvh.nodes.size() * sizeof(float), tb = bvh.tris.size() * sizeof(float);
    const size_t total = nb + tb + 12 * 16;
    s->tri_offset = (uint32_t)(bvh.nodes.size() / 4);
    hipError_t e = hipMalloc(&s->d_nodes, total);
    if (e == hipSuccess) e = hipMemset(s->d_nodes, 0, total);
    if (e == hipSuccess) e = hipMemcpy(s->d_nodes, bvh.nodes.data(), nb, hipMemcpyHostToDevice);
    if (e == hipSuccess && tb)
        e = hipMemcpy(reinterpret_cast<char*>(s->d_nodes) + nb, bvh.tris.data(), tb, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        rsd_status st = rsd::hip_fail(e, "rsd_scene_upload");
        (void)hipFree(s->d_nodes);
        delete s;
        return st;
    }
    s->d_tris = s->d_nodes + s->tri_offset;
    s->device_bytes = total;
    s->bvh_bytes = total;
    if (desc->triangle_count) {
        // primitive id -> triangle record (record r holds prim in v0.w): the raster SD walk keys its
        // hits by (t, prim) and its resolve pass needs the record of each key
        std::vector<uint32_t> pr(desc->triangle_count, 0u);
        for (uint32_t r = 0; r < desc->triangle_count; ++r) {
            uint32_t prim;
            std::memcpy(&prim, &bvh.tris[(size_t)r * 12 + 3], 4);
            pr[prim] = r;
        }
        e = hipMalloc(&s->d_prim_rec, pr.size() * 4);
        if (e == hipSuccess) e = hipMemcpy(s->d_prim_rec, pr.data(), pr.size() * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            rsd_status st = rsd::hip_fail(e, "rsd_scene_upload (prim map)");
            (void)hipFree(s->d_prim_rec);
            (void)hipFree(s->d_nodes);
            delete s;
            return st;
        }
        s->device_bytes += pr.size() * 4;
    }
    // segment entry grid (RSD_ENTRY_CELLS bounds its cells, 0 = none)
    uint64_t maxCells = 1ull << 21;
    if (const char* env = std::getenv("RSD_ENTRY_CELLS")) maxCells = (uint64_t)std::atoll(env);
    if (desc->triangle_count && maxCells) {
        const rsd::EntryGrid g = rsd::build_entry_grid(bvh.nodes, s->tri_offset, maxCells, threads);
        if (g.cells) {
            const size_t sb = g.slots.size() * 4, ib = g.items.size() * 4;
            void* d = nullptr;
            e = hipMalloc(&d, sb + ib);
            if (e == hipSuccess) e = hipMemcpy(d, g.slots.data(), sb, hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(static_cast<char*>(d) + sb, g.items.data(), ib, hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                rsd_status st = rsd::hip_fail(e, "rsd_scene_upload (entry grid)");
                (void)hipFree(d);
                (void)hipFree(s->d_prim_rec);
                (void)hipFree(s->d_nodes);
                delete s;
                return st;
            }
            s->d_entry = d;
            s->entry_items_off = sb;
            uint32_t bits = 0;
            while ((4ull << bits) < g.slots.size()) ++bits;
            s->entry_bits = bits;
            s->entry_probe = g.max_probe;
            s->entry_rmax = g.rmax;
            s->entry_cells = g.cells;
            for (int k = 0; k < 3; ++k) s->entry_origin[k] = g.origin[k];
            s->entry_extent = g.extent;
            s->entry_build_ms = g.build_ms;
            s->device_bytes += sb + ib;
        }
    }
    *out = s;
    return RSD_OK;
}

namespace {
// MaterialHeader stores the alpha threshold as float16 (MaterialData.slang:99): round to
// nearest even at half precision, then widen.
float round_half(float f) {
    if (f != f) return f;
    const float a = std::fabs(f);
    if (a >= 65520.0f) return std::copysign(INFINITY, f);
    int e = 0;
    (void)std::frexp(a, &e);                  // a = m 2^e, m in [0.5, 1)
    const int q = std::max(e - 11, -24);      // quantum exponent: 10 fraction bits, subnormals
    return std::ldexp(std::nearbyint(std::ldexp(f, -q)), q);
}

// The 2x2 box mip chain of one R8 texture (DESIGN.md "Alpha test"): level l+1 texel (x, y)
// averages level l texels (2x..2x+1, 2y..2y+1), clamped to the level, (a+b+c+d+2)/4.
void build_mips(const rsd_alpha_texture& t, std::vector<uint8_t>& out, uint32_t& mips) {
    uint32_t w = t.width, h = t.height;
    size_t base = out.size();
    out.insert(out.end(), t.alpha, t.alpha + (size_t)w * h);
    mips = 1;
    while (w > 1 || h > 1) {
        const uint32_t nw = std::max(1u, w >> 1), nh = std::max(1u, h >> 1);
        const size_t nbase = out.size();
        out.resize(nbase + (size_t)nw * nh);
        for (uint32_t y = 0; y < nh; ++y)
            for (uint32_t x = 0; x < nw; ++x) {
                const uint32_t x0 = std::min(2 * x, w - 1), x1 = std::min(2 * x + 1, w - 1);
                const uint32_t y0 = std::min(2 * y, h - 1), y1 = std::min(2 * y + 1, h - 1);
                const uint8_t* l = out.data() + base;
                const uint32_t sum = l[(size_t)y0 * w + x0] + l[(size_t)y0 * w + x1] + l[(size_t)y1 * w + x0] +
                                     l[(size_t)y1 * w + x1] + 2;
                out[nbase + (size_t)y * nw + x] = (uint8_t)(sum / 4);
            }
        base = nbase;
        w = nw;
        h = nh;
        ++mips;
    }
}
}  // namespace

extern "C" rsd_status rsd_scene_upload_alpha(rsd_device* dev, const rsd_scene_desc* desc, const rsd_alpha_desc* alpha,
                                             rsd_scene** out) {
    if (!alpha) return rsd_scene_upload(dev, desc, out);
    if (!dev || !desc || !out || !alpha->triangle_material || !alpha->materials || alpha->material_count == 0 ||
        (desc->vertex_count && !alpha->texcoords) || (alpha->texture_count && !alpha->textures)) {
        set_error("rsd_scene_upload_alpha: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    for (uint32_t i = 0; i < alpha->texture_count; ++i) {
        const rsd_alpha_texture& t = alpha->textures[i];
        if (t.width == 0 || t.height == 0 || !t.alpha || t.width > 32768 || t.height > 32768) {
            set_error("rsd_scene_upload_alpha: texture " + std::to_string(i) + " is empty or too large");
            return RSD_ERR_INVALID_ARG;
        }
    }
    for (uint32_t i = 0; i < alpha->material_count; ++i) {
        const uint32_t tex = alpha->materials[i].texture;
        if (tex != RSD_NO_TEXTURE && tex >= alpha->texture_count) {
            set_error("rsd_scene_upload_alpha: material " + std::to_string(i) + " names a missing texture");
            return RSD_ERR_INVALID_ARG;
        }
    }
    for (uint32_t i = 0; i < desc->triangle_count; ++i)
        if (alpha->triangle_material[i] >= alpha->material_count) {
            set_error("rsd_scene_upload_alpha: triangle_material out of range of material_count");
            return RSD_ERR_INVALID_ARG;
        }
    rsd_status st = rsd_scene_upload(dev, desc, out);
    if (st != RSD_OK) return st;
    rsd_scene* s = *out;
    const uint32_t nt = desc->triangle_count, nm = alpha->material_count, nx = alpha->texture_count;
    // per-primitive texture coordinates (Scene::computeVertexData reads them per vertex)
    std::vector<float> uv(6 * (size_t)nt);
    for (size_t t = 0; t < nt; ++t)
        for (int j = 0; j < 3; ++j) {
            const uint32_t v = desc->indices[3 * t + j];
            uv[6 * t + 2 * j] = alpha->texcoords[2 * (size_t)v];
            uv[6 * t + 2 * j + 1] = alpha->texcoords[2 * (size_t)v + 1];
        }
    std::vector<float> mats(4 * (size_t)nm);
    for (uint32_t i = 0; i < nm; ++i) {
        const rsd_material& m = alpha->materials[i];
        mats[4 * i] = round_half(m.alpha_threshold);
        mats[4 * i + 1] = m.alpha;
        std::memcpy(&mats[4 * i + 2], &m.texture, 4);
        mats[4 * i + 3] = 0.0f;
    }
    std::vector<uint32_t> texs(4 * (size_t)nx);
    std::vector<uint8_t> texels;
    for (uint32_t i = 0; i < nx; ++i) {
        texs[4 * i] = alpha->textures[i].width;
        texs[4 * i + 1] = alpha->textures[i].height;
        texs[4 * i + 3] = (uint32_t)texels.size();
        build_mips(alpha->textures[i], texels, texs[4 * i + 2]);
        if (texels.size() >= (1ull << 32)) {
            rsd_scene_release(s);
            *out = nullptr;
            set_error("rsd_scene_upload_alpha: more than 4 GiB of texels");
            return RSD_ERR_UNSUPPORTED;
        }
    }
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t oUV = 0, oMat = al(uv.size() * 4), oMats = oMat + al(4 * (size_t)nt), oTex = oMats + al(mats.size() * 4),
                 oTexel = oTex + al(texs.size() * 4), total = oTexel + al(texels.size() + 16);
    char* d = nullptr;
    hipError_t e = hipMalloc(&d, total);
    if (e == hipSuccess) e = hipMemset(d, 0, total);
    if (e == hipSuccess && nt) e = hipMemcpy(d + oUV, uv.data(), uv.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && nt) e = hipMemcpy(d + oMat, alpha->triangle_material, 4 * (size_t)nt, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + oMats, mats.data(), mats.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && nx) e = hipMemcpy(d + oTex, texs.data(), texs.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && !texels.empty()) e = hipMemcpy(d + oTexel, texels.data(), texels.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        st = rsd::hip_fail(e, "rsd_scene_upload_alpha");
        (void)hipFree(d);
        rsd_scene_release(s);
        *out = nullptr;
        return st;
    }
    s->d_alpha = d;
    s->alpha.triUV = reinterpret_cast<const float*>(d + oUV);
    s->alpha.triMat = reinterpret_cast<const uint32_t*>(d + oMat);
    s->alpha.materials = reinterpret_cast<const float4*>(d + oMats);
    s->alpha.textures = reinterpret_cast<const uint4*>(d + oTex);
    s->alpha.texels = reinterpret_cast<const uint8_t*>(d + oTexel);
    s->device_bytes += total;
    return RSD_OK;
}

extern "C" float rsd_ray_cone_spread(float focal_length, uint32_t height) {
    // every SD trace asks for it with the frame's (focal length, height): keep the last answer per thread
    // (the decimal round trip below costs about as much as a kernel launch on the host)
    thread_local float lastF = -1.0f, lastS = 0.0f;
    thread_local uint32_t lastH = 0;
    if (focal_length == lastF && height == lastH) return lastS;
    const float fovY = 2.0f * std::atan(0.5f * 24.0f / focal_length);  // focalLengthToFovY(f, kDefaultFrameHeight)
    const float angle = std::atan(2.0f * std::tan(fovY * 0.5f) / (float)height);
    char buf[64];
    std::snprintf(buf, sizeof(buf), "%f", (double)angle);  // std::to_string(float)
    lastS = std::strtof(buf, nullptr);
    lastF = focal_length;
    lastH = height;
    return lastS;
}

extern "C" rsd_status rsd_scene_info_get(const rsd_scene* s, rsd_scene_info* out) {
    if (!s || !out) {
        set_error("rsd_scene_info_get: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    out->triangle_count = s->triangle_count;
    out->node_count = s->node_count;
    out->max_depth = s->stats.max_depth;
    out->wide_depth = s->stats.wide_depth;
    out->leaf_count = s->stats.leaves;
    out->sah_cost = s->stats.sah_cost;
    out->build_ms = s->stats.build_ms + s->entry_build_ms;
    out->device_bytes = s->device_bytes;
    out->build_threads = s->build_threads;
    out->entry_cells = s->entry_cells;
    return RSD_OK;
}

extern "C" rsd_status rsd_bvh_build(const rsd_scene_desc* desc, void* dst, uint64_t capacity, uint64_t* bytes,
                                    uint32_t* tri_offset) {
    if (!desc || !bytes || (desc->triangle_count && (!desc->positions || !desc->indices))) {
        set_error("rsd_bvh_build: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    for (uint64_t i = 0; i < 3ull * desc->triangle_count; ++i)
        if (desc->indices[i] >= desc->vertex_count) {
            set_error("rsd_bvh_build: index out of range of vertex_count");
            return RSD_ERR_INVALID_ARG;
        }
    rsd::FlatBvh bvh = rsd::build_bvh(desc->positions, desc->vertex_count, desc->indices, desc->triangle_count,
                                      desc->triangle_flags, build_threads());
    const size_t nb = bvh.nodes.size() * sizeof(float), tb = bvh.tris.size() * sizeof(float);
    *bytes = nb + tb + 12 * 16;  // the layout of rsd_scene_upload's allocation
    if (tri_offset) *tri_offset = (uint32_t)(bvh.nodes.size() / 4);
    if (!dst) return RSD_OK;
    if (capacity < *bytes) {
        set_error("rsd_bvh_build: capacity below the BVH size");
        return RSD_ERR_INVALID_ARG;
    }
    std::memcpy(dst, bvh.nodes.data(), nb);
    if (tb) std::memcpy(static_cast<char*>(dst) + nb, bvh.tris.data(), tb);
    std::memset(static_cast<char*>(dst) + nb + tb, 0, 12 * 16);
    return RSD_OK;
}

extern "C" rsd_status rsd_scene_export_bvh(const rsd_scene* s, void* dst, uint64_t capacity, uint64_t* bytes,
                                           uint32_t* tri_offset) {
    if (!s || !bytes) {
        set_error("rsd_scene_export_bvh: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    *bytes = s->bvh_bytes;
    if (tri_offset) *tri_offset = s->tri_offset;
    if (!dst) return RSD_OK;
    if (capacity < s->bvh_bytes) {
        set_error("rsd_scene_export_bvh: capacity below the BVH size");
        return RSD_ERR_INVALID_ARG;
    }
    if (s->bvh_bytes == 0) return RSD_OK;
    RSD_HIP(hipSetDevice(s->dev->hip_device));
    RSD_HIP(hipMemcpy(dst, s->d_nodes, s->bvh_bytes, hipMemcpyDeviceToHost));
    return RSD_OK;
}

extern "C" void rsd_scene_release(rsd_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->dev->hip_device);
    (void)hipFree(s->d_nodes);
    (void)hipFree(s->d_prim_rec);
    rsd::release_sd_workspaces(s);
    (void)hipFree(s->d_alpha);
    (void)hipFree(s->d_entry);
    delete s;
}

// ---- Camera::calculateCameraParameters, Camera.cpp:99-185 (preserveHeight), with
//      MatrixMath.h:686-712 (RightHanded look-at) and VectorMath.h:1731 normalize.
namespace {
struct v3 { float x, y, z; };
inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline v3 cross3(v3 a, v3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline v3 norm3(v3 v) {
    float inv = 1.0f / std::sqrt(dot3(v, v));
    return {v.x * inv, v.y * inv, v.z * inv};
}
}  // namespace

extern "C" rsd_status rsd_camera_look_at(const float pos[3], const float target[3], const float up[3],
                                         float focal_length, float frame_height, float aspect_ratio, float near_z,
                                         float far_z, float focal_distance, rsd_camera* c) {
    if (!pos || !target || !up || !c) {
        set_error("rsd_camera_look_at: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    std::memset(c, 0, sizeof(*c));
    const v3 P{pos[0], pos[1], pos[2]}, T{target[0], target[1], target[2]}, Up{up[0], up[1], up[2]};
    for (int i = 0; i < 3; ++i) c->posW[i] = pos[i];
    c->nearZ = near_z;
    c->farZ = far_z;
    c->focalLength = focal_length;
    c->frameHeight = frame_height;
    c->aspectRatio = aspect_ratio;
    c->frameWidth = frame_height * aspect_ratio;
    const float fovY = focal_length == 0.0f ? 0.0f : 2.0f * std::atan(0.5f * frame_height / focal_length);
    const v3 f = norm3({P.x - T.x, P.y - T.y, P.z - T.z});
    const v3 r = norm3(cross3(Up, f));
    const v3 u = cross3(f, r);
    float* m = c->viewMat;
    m[0] = r.x; m[1] = r.y; m[2] = r.z; m[3] = -dot3(r, P);
    m[4] = u.x; m[5] = u.y; m[6] = u.z; m[7] = -dot3(u, P);
    m[8] = f.x; m[9] = f.y; m[10] = f.z; m[11] = -dot3(f, P);
    m[15] = 1.0f;
    const v3 w = norm3({T.x - P.x, T.y - P.y, T.z - P.z});
    const v3 W{w.x * focal_distance, w.y * focal_distance, w.z * focal_distance};
    const v3 cu = norm3(cross3(W, Up));
    const v3 cv = norm3(cross3(cu, W));
    const float ulen = focal_distance * std::tan(fovY * 0.5f) * aspect_ratio;
    const float vlen = focal_distance * std::tan(fovY * 0.5f);
    c->W[0] = W.x; c->W[1] = W.y; c->W[2] = W.z;
    c->U[0] = cu.x * ulen; c->U[1] = cu.y * ulen; c->U[2] = cu.z * ulen;
    c->V[0] = cv.x * vlen; c->V[1] = cv.y * vlen; c->V[2] = cv.z * vlen;
    return RSD_OK;
}

// SVAO::compile (SVAO.cpp:143-150), getStochMapSize (:700-716), getExtraGuardBand (:718-723)
extern "C" rsd_status rsd_svao_make_vao_data(uint32_t fb_w, uint32_t fb_h, uint32_t divisor, int32_t sd_guard_px,
                                             float radius, float exponent, float thickness, rsd_vao_data* out,
                                             uint32_t* sd_w, uint32_t* sd_h) {
    if (!out || fb_w == 0 || fb_h == 0 || divisor == 0 || sd_guard_px < 0) {
        set_error("rsd_svao_make_vao_data: invalid argument");
        return RSD_ERR_INVALID_ARG;
    }
    rsd_vao_data d{};
    d.resolution[0] = (float)fb_w;
    d.resolution[1] = (float)fb_h;
    d.invResolution[0] = 1.0f / d.resolution[0];
    d.invResolution[1] = 1.0f / d.resolution[1];
    d.sdGuard = sd_guard_px / (int32_t)divisor;
    const uint32_t lw = divisor > 1 ? (fb_w + divisor - 1) / divisor : fb_w;
    const uint32_t lh = divisor > 1 ? (fb_h + divisor - 1) / divisor : fb_h;
    d.lowResolution[0] = (float)lw;
    d.lowResolution[1] = (float)lh;
    d.noiseScale[0] = d.resolution[0] / 4.0f;
    d.noiseScale[1] = d.resolution[1] / 4.0f;
    d.radius = radius;
    d.exponent = exponent;
    d.thickness = thickness;
    d.ssRadiusCutoff = 6.0f;   // VAOData.slang:43
    d.ssMaxRadius = 512.0f;    // VAOData.slang:44
    *out = d;
    if (sd_w) *sd_w = lw + 2u * (uint32_t)d.sdGuard;
    if (sd_h) *sd_h = lh + 2u * (uint32_t)d.sdGuard;
    return RSD_OK;
}
