// halo.hip -- device steps of the band split's sparse halo exchange (rsd/shard.py HaloFrame,
// DESIGN.md section 6; include/rsd.h rsd_halo_*).
//
// each rank owns contiguous screen bands; the SD texels its pass 1 touched inside another
// rank's band travel as (texel, rayMin, rayMax) triples and their N depths come back.  These kernels
// are the device side of those steps: the compaction of the touched texels (one ballot + one atomic per
// wave and region), the order-independent merge (atomicMin / atomicMax, the union SVAO.cpp:334-340's
// atomics would have produced on one GPU), and the SD-depth gather / scatter of the reply.  All are
// HBM-streaming: bytes per texel = 8 (read both words) + 12 per touched texel; per triple 12 + 2 atomics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "comm.h"
#include "rsd_internal.h"

namespace rsd {
namespace {

constexpr uint32_t kHaloBlock = 256;
constexpr uint32_t kFltMaxBits = 0x7f7fffffu;  // asuint(FLT_MAX): a cleared rayMin (SVAO.cpp:339)
constexpr uint32_t kMaxRegions = 64;

constexpr uint32_t kSdTile = 8;  // SD trace tile rows (sd_trace.hip kTile): the round-robin unit of the tiled split

struct HaloRegions {
    uint32_t n;
    uint32_t first[kMaxRegions + 1];  // first texel of each region (flattened grid of all regions' texels)
    uint32_t row0[kMaxRegions];
    uint32_t row1[kMaxRegions];
    uint32_t period[kMaxRegions];     // 1: contiguous rows; > 1: every period-th 8-row tile from row0
    uint32_t stride[kMaxRegions];
    int32_t* out[kMaxRegions];
    unsigned long long* count[kMaxRegions];
    uint32_t ilv;                     // 1: interleaved triples out[3k + c] (the band frame's), 0: rows of `stride`
    long long* row;                   // optional count row: row[0, rowN) zeroed, row[rowN] = extra
    uint32_t rowN;
    long long extra;
    uint32_t extraInCompact;          // 1: the counts are already zero; the compaction writes row[rowN] = extra
    long long* zeroRow;               // optional: a second row [0, rowN] cleared in the same launch (the next
                                      // frame's, double-buffered count rows of the band frame)
};

__global__ void halo_zero_kernel(HaloRegions R) {
    if (threadIdx.x < R.n) *R.count[threadIdx.x] = 0ull;
    if (R.row) {
        for (uint32_t i = threadIdx.x; i < R.rowN; i += blockDim.x) R.row[i] = 0;
        if (threadIdx.x == 0) R.row[R.rowN] = R.extra;
    }
    if (R.zeroRow)
        for (uint32_t i = threadIdx.x; i <= R.rowN; i += blockDim.x) R.zeroRow[i] = 0;
}

__global__ void __launch_bounds__(kHaloBlock) halo_compact_kernel(const uint32_t* __restrict__ rmin,
                                                                   const uint32_t* __restrict__ rmax, uint32_t sdW,
                                                                   HaloRegions R) {
    const uint32_t g = blockIdx.x * kHaloBlock + threadIdx.x;
    if (R.extraInCompact && g == 0u) R.row[R.rowN] = R.extra;
    if (R.zeroRow && g <= R.rowN) R.zeroRow[g] = 0;
    bool in = g < R.first[R.n];
    uint32_t r = 0;
    while (in && g >= R.first[r + 1]) ++r;
    uint32_t t = 0u;
    if (in) {
        const uint32_t e = g - R.first[r];
        uint32_t row;
        if (R.period[r] <= 1u) {
            row = R.row0[r] + e / sdW;
        } else {  // tile j of the region: SD tile row0 / 8 + j period (whole tiles; rows past row1 skipped)
            const uint32_t per = kSdTile * sdW, j = e / per;
            row = R.row0[r] + j * R.period[r] * kSdTile + (e % per) / sdW;
        }
        in = row < R.row1[r];
        t = row * sdW + e % sdW;
    }
    const uint32_t lo = in ? rmin[t] : kFltMaxBits, hi = in ? rmax[t] : 0u;
    const bool touched = lo != kFltMaxBits || hi != 0u;
    // one atomic per (wave, region) the wave's touched texels fall in
    const uint32_t lane = __lane_id();
    uint64_t pending = __ballot(touched);
    while (pending != 0ull) {
        const int leader = __ffsll((long long)pending) - 1;
        const uint32_t rl = (uint32_t)__shfl((int)r, leader);
        const uint64_t grp = __ballot(touched && r == rl);
        unsigned long long base = 0ull;
        if (lane == (uint32_t)leader) base = atomicAdd(R.count[rl], (unsigned long long)__popcll(grp));
        base = __shfl(base, leader);
        if (touched && r == rl) {
            const uint32_t k = (uint32_t)base + (uint32_t)__popcll(grp & ((1ull << lane) - 1ull));
            int32_t* o = R.out[rl];
            if (R.ilv) {
                o[3u * k] = (int32_t)t;
                o[3u * k + 1u] = (int32_t)lo;
                o[3u * k + 2u] = (int32_t)hi;
            } else {
                const uint32_t st = R.stride[rl];
                o[k] = (int32_t)t;
                o[st + k] = (int32_t)lo;
                o[2u * st + k] = (int32_t)hi;
            }
        }
        pending &= ~grp;
    }
}

// flattened work of up to kMaxRegions lists: list l covers items [first[l], first[l + 1])
struct HaloLists {
    uint32_t n;
    uint32_t first[kMaxRegions + 1];
    const int32_t* idx[kMaxRegions];  // merge: the triples; SD: the texel indices
    float* buf[kMaxRegions];          // SD: the packed depths
    uint32_t stride[kMaxRegions];     // merge: the triples' row stride
    uint32_t ilv;                     // 1: interleaved triples {texel, rayMin, rayMax} (merge; SD: index stride 3)
};

__device__ __forceinline__ uint32_t list_of(const HaloLists& H, uint32_t g) {
    uint32_t l = 0;
    while (g >= H.first[l + 1]) ++l;
    return l;
}

__global__ void __launch_bounds__(kHaloBlock) halo_merge_kernel(uint32_t* __restrict__ rmin, uint32_t* __restrict__ rmax,
                                                                 HaloLists H, uint32_t total, uint32_t interval) {
    const uint32_t g = blockIdx.x * kHaloBlock + threadIdx.x;
    if (g >= H.first[H.n]) return;
    const uint32_t l = list_of(H, g), k = g - H.first[l];
    const int32_t* tr = H.idx[l];
    const uint32_t i0 = H.ilv ? 3u * k : k, st = H.ilv ? 1u : H.stride[l];
    const uint32_t t = (uint32_t)tr[i0];
    if (t >= total) return;  // never: the sender's indices lie in the map
    if (interval) atomicMin(&rmin[t], (uint32_t)tr[i0 + st]);
    atomicMax(&rmax[t], (uint32_t)tr[i0 + 2u * st]);
}

// one lane per (list item, layer, channel): item-major within a list, so a list's lanes read its
// index once per layer and channel (the L x n x ch packed layout is written / read in order per layer)
template <bool GATHER>
__global__ void __launch_bounds__(kHaloBlock) halo_sd_kernel(float* __restrict__ sd, HaloLists H, uint32_t layers,
                                                              uint32_t texels, uint32_t ch) {
    const uint32_t g = blockIdx.x * kHaloBlock + threadIdx.x;  // over sum_l layers * n_l * ch
    if (g >= H.first[H.n]) return;
    const uint32_t l = list_of(H, g), e = g - H.first[l];
    const uint32_t n = (H.first[l + 1] - H.first[l]) / (layers * ch);
    const uint32_t per = n * ch, L = e / per, rem = e % per, k = rem / ch, c = rem % ch;
    const uint32_t t = (uint32_t)H.idx[l][H.ilv ? 3u * k : k];
    if (t >= texels) return;
    const size_t so = ((size_t)L * texels + t) * ch + c;
    if (GATHER) H.buf[l][e] = sd[so];
    else sd[so] = H.buf[l][e];
}

rsd_status launch_check(const char* what) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSD_OK : hip_fail(e, what);
}

// a batch of byte copies (the band frame's AO band packing / unpacking, the in-process communicator):
// 16-B lanes where a segment's source, destination and size are 16-B aligned, bytes otherwise
struct CopySegs {
    uint32_t n;
    uint64_t first[kMaxCopySegs + 1];  // first work item of each segment
    const uint8_t* src[kMaxCopySegs];
    uint8_t* dst[kMaxCopySegs];
    uint64_t bytes[kMaxCopySegs];
    uint32_t vec[kMaxCopySegs];        // 1: 16-B items
    unsigned long long* zero;          // optional: zero[0, zeroN) set to 0 by the first lanes (a side job)
    uint32_t zeroN;
};

__global__ void __launch_bounds__(kHaloBlock) copy_segments_kernel(CopySegs S) {
    if (S.zero && blockIdx.x == 0 && threadIdx.x < S.zeroN) S.zero[threadIdx.x] = 0ull;
    const uint64_t total = S.first[S.n];
    for (uint64_t g = (uint64_t)blockIdx.x * kHaloBlock + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * kHaloBlock) {
        uint32_t l = 0;
        while (g >= S.first[l + 1]) ++l;
        const uint64_t e = g - S.first[l];
        if (S.vec[l]) reinterpret_cast<uint4*>(S.dst[l])[e] = reinterpret_cast<const uint4*>(S.src[l])[e];
        else S.dst[l][e] = S.src[l][e];
    }
}

// The band frame's count matrix to the host without a copy engine or an event: one wave writes the n values
// to host-visible (pinned, fine-grained) memory after the sequence word's slot, each lane's stores released
// at system scope, then the sequence number with a system-scope release store -- the host polls that word.
__global__ void __launch_bounds__(64) publish_kernel(const long long* __restrict__ src, long long* dst, uint32_t n,
                                                      long long seq) {
    for (uint32_t i = threadIdx.x; i < n; i += 64u) dst[1u + i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&dst[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

rsd_status publish_counts(const int64_t* d_src, int64_t* dst_host_dev, uint32_t n, int64_t seq, hipStream_t s) {
    hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(64), 0, s, reinterpret_cast<const long long*>(d_src),
                       reinterpret_cast<long long*>(dst_host_dev), n, (long long)seq);
    return launch_check("publish_kernel launch");
}

rsd_status copy_segments(const CopySeg* segs, uint32_t n, hipStream_t s, uint64_t* zero, uint32_t zero_n) {
    if (n > kMaxCopySegs || zero_n > kHaloBlock) {
        set_error("copy_segments: more than 16 segments or 256 words to zero");
        return RSD_ERR_INVALID_ARG;
    }
    CopySegs S{};
    S.zero = reinterpret_cast<unsigned long long*>(zero);
    S.zeroN = zero ? zero_n : 0u;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(segs[i].src) | reinterpret_cast<uintptr_t>(segs[i].dst) |
                            (uintptr_t)segs[i].bytes;
        S.vec[S.n] = (a & 15u) == 0u ? 1u : 0u;
        S.src[S.n] = static_cast<const uint8_t*>(segs[i].src);
        S.dst[S.n] = static_cast<uint8_t*>(segs[i].dst);
        S.bytes[S.n] = segs[i].bytes;
        S.first[S.n] = total;
        total += S.vec[S.n] ? segs[i].bytes / 16u : segs[i].bytes;
        if (segs[i].bytes) ++S.n;
    }
    S.first[S.n] = total;
    if (total == 0 && S.zeroN == 0) return RSD_OK;
    const uint64_t blocks = std::max<uint64_t>(1u, std::min<uint64_t>((total + kHaloBlock - 1) / kHaloBlock, 4096u));
    hipLaunchKernelGGL(copy_segments_kernel, dim3((uint32_t)blocks), dim3(kHaloBlock), 0, s, S);
    return launch_check("copy_segments_kernel launch");
}

// The compaction of rsd_halo_compact; ilv = 1 writes interleaved triples (the band frame's layout: a
// peer's prefix is one contiguous transfer); row (optional): a count row whose [0, rowN) is zeroed and
// row[rowN] = extra in the same launch that zeroes the counts (the counts may point into it).
rsd_status halo_compact_impl(const uint32_t* d_ray_min, const uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h,
                             const rsd_halo_region* regions, uint32_t n_regions, bool ilv, int64_t* row,
                             uint32_t row_n, int64_t extra, hipStream_t s, bool zeroed, int64_t* zero_row) {
    if (!d_ray_min || !d_ray_max || (n_regions && !regions) || n_regions > kMaxRegions || row_n > 64u) {
        set_error("rsd_halo_compact: null buffer or more than 64 regions");
        return RSD_ERR_INVALID_ARG;
    }
    HaloRegions R{};
    R.n = n_regions;
    R.ilv = ilv ? 1u : 0u;
    R.row = reinterpret_cast<long long*>(row);
    R.rowN = row_n;
    R.extra = (long long)extra;
    R.zeroRow = reinterpret_cast<long long*>(zero_row);
    uint32_t total = 0;
    for (uint32_t r = 0; r < n_regions; ++r) {
        const rsd_halo_region& g = regions[r];
        const uint32_t period = g.period > 1u ? g.period : 1u;
        // the flattened texels of the region: its rows, or its whole tiles (rows past row1 masked)
        const uint64_t tiles = period > 1u && g.row1 > g.row0
                                   ? ((g.row1 - g.row0 + kSdTile - 1) / kSdTile + period - 1) / period : 0u;
        const uint64_t texels = period > 1u ? tiles * kSdTile * sd_w : (uint64_t)(g.row1 - g.row0) * sd_w;
        if (g.row0 > g.row1 || g.row1 > sd_h || !g.out || !g.count || g.stride < texels ||
            (period > 1u && g.row0 % kSdTile != 0u) || (uint64_t)total + texels > 0xffffffffull) {
            set_error("rsd_halo_compact: region rows outside the map, null output, stride below its texel count, "
                      "or a tiled region not starting on an 8-row tile");
            return RSD_ERR_INVALID_ARG;
        }
        R.first[r] = total;
        R.row0[r] = g.row0;
        R.row1[r] = g.row1;
        R.period[r] = period;
        R.stride[r] = g.stride;
        R.out[r] = g.out;
        R.count[r] = reinterpret_cast<unsigned long long*>(g.count);
        total += (uint32_t)texels;
    }
    R.first[n_regions] = total;
    if (n_regions == 0 && !row) return RSD_OK;
    if (zeroed && row && total > 0) {  // the caller zeroed the counts: the compaction alone, writing row[row_n]
        R.extraInCompact = 1u;
        hipLaunchKernelGGL(halo_compact_kernel, dim3((total + kHaloBlock - 1) / kHaloBlock), dim3(kHaloBlock), 0, s,
                           d_ray_min, d_ray_max, sd_w, R);
        return launch_check("halo_compact_kernel launch");
    }
    // the counts (and the count row) start at zero (one launch for all regions), then one compaction launch
    hipLaunchKernelGGL(halo_zero_kernel, dim3(1), dim3(64), 0, s, R);
    if (total == 0) return launch_check("halo_zero_kernel launch");
    hipLaunchKernelGGL(halo_compact_kernel, dim3((total + kHaloBlock - 1) / kHaloBlock), dim3(kHaloBlock), 0, s,
                       d_ray_min, d_ray_max, sd_w, R);
    return launch_check("halo_compact_kernel launch");
}

rsd_status halo_merge_impl(uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h,
                           const rsd_halo_list* lists, uint32_t n_lists, uint32_t ray_interval, bool ilv,
                           hipStream_t s) {
    if (!d_ray_min || !d_ray_max || (n_lists && !lists) || n_lists > kMaxRegions) {
        set_error("rsd_halo_merge: null buffer or more than 64 lists");
        return RSD_ERR_INVALID_ARG;
    }
    HaloLists H{};
    H.n = n_lists;
    H.ilv = ilv ? 1u : 0u;
    uint32_t total = 0;
    for (uint32_t l = 0; l < n_lists; ++l) {
        if ((lists[l].n && !lists[l].triples) || (!ilv && lists[l].stride < lists[l].n)) {
            set_error("rsd_halo_merge: null triples or stride below n");
            return RSD_ERR_INVALID_ARG;
        }
        H.first[l] = total;
        H.idx[l] = lists[l].triples;
        H.stride[l] = lists[l].stride;
        total += lists[l].n;
    }
    H.first[n_lists] = total;
    if (total == 0) return RSD_OK;
    hipLaunchKernelGGL(halo_merge_kernel, dim3((total + kHaloBlock - 1) / kHaloBlock), dim3(kHaloBlock), 0, s,
                       d_ray_min, d_ray_max, H, sd_w * sd_h, ray_interval ? 1u : 0u);
    return launch_check("halo_merge_kernel launch");
}

rsd_status halo_sd_impl(bool gather, float* sd, uint32_t layers, uint32_t sd_w, uint32_t sd_h, uint32_t ch,
                        const rsd_halo_sd_list* lists, uint32_t n_lists, bool ilv, hipStream_t s, const char* who) {
    if (!sd || (n_lists && !lists) || n_lists > kMaxRegions || !layers || !ch || ch > 4) {
        set_error(std::string(who) + ": null buffer, more than 64 lists, or layers / channels out of range");
        return RSD_ERR_INVALID_ARG;
    }
    HaloLists H{};
    H.n = n_lists;
    H.ilv = ilv ? 1u : 0u;
    uint64_t total = 0;
    for (uint32_t l = 0; l < n_lists; ++l) {
        if (lists[l].n && (!lists[l].idx || !lists[l].buf)) {
            set_error(std::string(who) + ": null index list or buffer");
            return RSD_ERR_INVALID_ARG;
        }
        H.first[l] = (uint32_t)total;
        H.idx[l] = lists[l].idx;
        H.buf[l] = lists[l].buf;
        total += (uint64_t)lists[l].n * layers * ch;
        if (total > 0xffffffffull) {
            set_error(std::string(who) + ": more than 2^32 values");
            return RSD_ERR_INVALID_ARG;
        }
    }
    H.first[n_lists] = (uint32_t)total;
    if (total == 0) return RSD_OK;
    const dim3 grid((uint32_t)((total + kHaloBlock - 1) / kHaloBlock));
    if (gather)
        hipLaunchKernelGGL(halo_sd_kernel<true>, grid, dim3(kHaloBlock), 0, s, sd, H, layers, sd_w * sd_h, ch);
    else
        hipLaunchKernelGGL(halo_sd_kernel<false>, grid, dim3(kHaloBlock), 0, s, sd, H, layers, sd_w * sd_h, ch);
    return launch_check(who);
}

}  // namespace rsd

using namespace rsd;

extern "C" rsd_status rsd_halo_compact(const uint32_t* d_ray_min, const uint32_t* d_ray_max, uint32_t sd_w,
                                       uint32_t sd_h, const rsd_halo_region* regions, uint32_t n_regions,
                                       rsd_stream stream) {
    return halo_compact_impl(d_ray_min, d_ray_max, sd_w, sd_h, regions, n_regions, false, nullptr, 0u, 0,
                             (hipStream_t)stream, false, nullptr);
}

extern "C" rsd_status rsd_halo_merge(uint32_t* d_ray_min, uint32_t* d_ray_max, uint32_t sd_w, uint32_t sd_h,
                                     const rsd_halo_list* lists, uint32_t n_lists, uint32_t ray_interval,
                                     rsd_stream stream) {
    return halo_merge_impl(d_ray_min, d_ray_max, sd_w, sd_h, lists, n_lists, ray_interval, false, (hipStream_t)stream);
}

extern "C" rsd_status rsd_halo_sd_gather(const float* d_sd, uint32_t layers, uint32_t sd_w, uint32_t sd_h, uint32_t ch,
                                         const rsd_halo_sd_list* lists, uint32_t n_lists, rsd_stream stream) {
    return halo_sd_impl(true, const_cast<float*>(d_sd), layers, sd_w, sd_h, ch, lists, n_lists, false,
                        (hipStream_t)stream, "rsd_halo_sd_gather");
}

extern "C" rsd_status rsd_halo_sd_scatter(float* d_sd, uint32_t layers, uint32_t sd_w, uint32_t sd_h, uint32_t ch,
                                          const rsd_halo_sd_list* lists, uint32_t n_lists, rsd_stream stream) {
    return halo_sd_impl(false, d_sd, layers, sd_w, sd_h, ch, lists, n_lists, false, (hipStream_t)stream,
                        "rsd_halo_sd_scatter");
}
