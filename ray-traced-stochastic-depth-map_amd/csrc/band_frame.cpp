// band_frame.cpp -- rsd_band_frame: one rank's share of a screen-band SVAO frame, issued from C++
// (include/rsd.h).
//
// The native form of the band split of SURVEY 8(e) (rsd/shard.py HaloFrame is its Python rehearsal):
// rank r of B owns the visible rows of its 32-row groups [g_r, g_{r+1}) for "AO 1" / "AO 2"
// (SVAORaster.ps.slang:29-122, SVAORaster2.ps.slang:48-65) and an SD share (round-robin 8-row tiles, or
// the SD rows under its band) for the trace (StochasticDepthMapRT.rt.slang:39-105).  Pass 1's interval
// atomics of a rank land only within the projected ssMaxRadius reach of its band (VAOData.slang:44,
// SVAO.cpp:700-723) -- on exactly the SD texels its pass 2 will read (Common.slang:164-168) -- so only
// those texels travel: (texel, rayMin, rayMax) triples to the texel's owner, and the owner's N depths of
// exactly those texels back.  The AO bands are all-gathered at the end (north_star).  Every exchange is
// stream-ordered through a Comm (RCCL or in-process, comm.h); the host waits only for the count matrix
// of a frame, which it reads in back() -- with frames in flight, long after it completed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>
#include <string>
#include <vector>

#include "comm.h"
#include "rsd_internal.h"

namespace rsd {
namespace {

int64_t floordiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
int64_t pymod(int64_t a, int64_t b) { const int64_t m = a % b; return m < 0 ? m + b : m; }

// Vertical reach (frame-buffer pixels) of an SVAO sample from its pixel: the AO disk (world radius R with
// R f / z <= ssMaxRadius, VAOData.slang:44; Common.slang:285-300) lies in the plane perpendicular to the
// view ray, so off-axis it projects larger than ssMaxRadius; evaluated over the frame border for the
// pinhole camera (Camera.cpp:99-185, preserveHeight), plus 4 px of slack (rsd/shard.py halo_px).
uint32_t halo_reach_px(uint32_t W, uint32_t H, double focal_length, double frame_height, double max_radius_px) {
    const double f = focal_length / frame_height * H;
    double worst = 0.0;
    auto cross = [](const double* u, const double* v, double* o) {
        o[0] = u[1] * v[2] - u[2] * v[1];
        o[1] = u[2] * v[0] - u[0] * v[2];
        o[2] = u[0] * v[1] - u[1] * v[0];
    };
    auto norm = [](const double* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); };
    for (int side = 0; side < 4; ++side)
        for (int i = 0; i <= 256; ++i) {
            const double t = i / 256.0;
            double x, y;
            switch (side) {
                case 0: x = (t - 0.5) * W; y = -0.5 * H; break;
                case 1: x = -0.5 * W; y = (t - 0.5) * H; break;
                case 2: x = 0.5 * W; y = (t - 0.5) * H; break;
                default: x = (t - 0.5) * W; y = 0.5 * H; break;
            }
            double d[3] = {x, y, f};
            const double dl = norm(d);
            for (double& c : d) c /= dl;
            const double P[3] = {d[0] / d[2], d[1] / d[2], 1.0};
            const double R = max_radius_px / f;
            const double ey[3] = {0.0, 1.0, 0.0}, ex[3] = {1.0, 0.0, 0.0};
            double a[3], b[3];
            cross(d, std::fabs(d[1]) < 0.99 ? ey : ex, a);
            const double al = norm(a);
            for (double& c : a) c /= al;
            cross(d, a, b);
            for (int k = 0; k < 64; ++k) {
                const double ang = k * (2.0 * M_PI / 64.0);
                const double c = std::cos(ang), s = std::sin(ang);
                const double S1 = P[1] + R * (c * a[1] + s * b[1]), S2 = P[2] + R * (c * a[2] + s * b[2]);
                worst = std::max(worst, std::fabs(f * S1 / S2 - y));
            }
        }
    return (uint32_t)std::ceil(worst) + 4u;
}

// a grow-only device buffer (grown rarely: a larger count than ever before, a re-split's larger regions)
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    rsd_status ensure(size_t bytes, hipStream_t s, uint64_t* grew) {
        if (bytes <= cap) return RSD_OK;
        if (p) {
            // a previous frame's transfer (RCCL on this stream; a local peer's copy, which this stream
            // waited for) may still read the old buffer
            RSD_HIP(hipStreamSynchronize(s));
            (void)hipFree(p);
            p = nullptr;
            cap = 0;
            if (grew) ++*grew;
        }
        const size_t n = bytes + bytes / 2 + 256;
        RSD_HIP(hipMalloc(&p, n));
        cap = n;
        return RSD_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct Region {
    bool valid = false;
    uint32_t lo = 0, hi = 0;  // SD rows
    uint32_t period = 1;      // > 1: every period-th 8-row tile from lo
    uint64_t texels = 0;      // the region's candidate texels (the compaction's capacity)
    uint64_t rows = 0;        // SD rows in the region
};

}  // namespace

class BandFrame {
public:
    ~BandFrame() {
        for (DevBuf* b : {&cand_all_, &row_, &mdev_}) b->release();
        for (auto* v : {&recv_tr_, &sd_send_, &sd_recv_})
            for (DevBuf& b : *v) b.release();
        if (mhost_) (void)hipHostFree(mhost_);
        for (auto& set : ev_)
            for (hipEvent_t& e : set)
                if (e) (void)hipEventDestroy(e);
    }

    rsd_status init(const rsd_svao_frame_desc& f, const rsd_band_params& bp, Comm* comm);
    rsd_status set_split(const uint32_t* split, uint32_t n);
    rsd_status front(const rsd_camera* cam, hipStream_t s);
    rsd_status back(void* const* events, hipStream_t s);
    void stats(rsd_band_stats& o) const;
    hipStream_t last_stream() const { return last_; }

private:
    rsd_status plan(hipStream_t s);
    std::vector<uint32_t> rebalanced(const std::vector<double>& costs) const;
    rsd_status mark(hipStream_t s);
    int64_t prev_cost_us() const;

    // the frame description (structs copied; buffers used in place)
    rsd_svao_frame_desc f_{};
    rsd_camera cam_{};
    rsd_vao_data vao_{};
    rsd_svao_params svp_{};
    rsd_sd_params sdp_{};
    rsd_band_params bp_{};
    Comm* comm_ = nullptr;
    uint32_t me_ = 0, world_ = 1;
    uint32_t guard_ = 0, div_ = 1, sdg_ = 0, V_ = 0, G_ = 0, L_ = 1, ch_ = 1, split_ = RSD_SD_SPLIT_ROWS;
    uint32_t halo_px_ = 0;
    bool consume_ = false, rebalance_ = false;
    bool intervals_clear_ = false;
    std::vector<uint32_t> gb_, next_gb_;
    // the partition implied by gb_
    std::vector<std::pair<uint32_t, uint32_t>> px_rows_, sd_rows_, window_, ao_rows_;
    std::vector<Region> iv_send_, iv_recv_;  // per peer: my touched texels in its share / its in mine
    uint32_t ao_max_ = 0;
    size_t ao_row_bytes_ = 0;
    // device state
    DevBuf cand_all_;                            // every peer's send triples (3 int32 per candidate texel)
    std::vector<size_t> cand_off_;               // per peer: int32 offset into cand_all_
    std::vector<rsd_halo_region> regions_;       // compaction regions (peers with a candidate region)
    std::vector<uint32_t> region_peer_;
    std::vector<DevBuf> recv_tr_, sd_send_, sd_recv_;
    DevBuf row_, mdev_;         // two count rows (frames alternate), the all-gathered matrix
    int64_t* mhost_ = nullptr;  // pinned: [0] sequence number, then the matrix (publish_counts)
    int64_t* mhost_dev_ = nullptr;
    int64_t seq_ = 0;
    hipEvent_t ev_[2][6] = {};
    uint32_t evn_ = 0;
    bool prev_valid_ = false;
    uint32_t prev_set_ = 0;
    // Re-split cadence (every fourth frame of this object): frame 4j + 1 records the six timing events (timed_;
    // 1.5 event records per frame on average); the back() of frame 4j + 2 reads their time once its count matrix
    // has arrived -- this object's frames run on one stream, so frame 4j + 1 has completed by then (cost_ready_,
    // -1 if not); front() of frame 4j + 3 puts it in the count row, the back() of frame 4j + 3 decides from every
    // rank's time (all ranks see the same matrix: all skip or all re-split) and front() of frame 4j + 4 applies it
    bool timed_ = false;
    int64_t cost_ready_ = -1;
    hipStream_t timed_stream_ = nullptr;
    bool next_forced_ = false;  // next_gb_ came from rsd_band_frame_set_split
    // the camera terms halo_px_ was computed from (a zoom changes the sample reach: re-plan)
    float halo_focal_ = 0.0f, halo_frame_h_ = 0.0f;
    bool open_ = false;
    hipStream_t last_ = nullptr;
    // statistics
    uint64_t frames_ = 0, blocked_ = 0, resplits_ = 0, b_iv_ = 0, b_sd_ = 0, b_ao_ = 0, growth_ = 0;
    uint64_t ns_front_ = 0, ns_back_ = 0, ns_wait_ = 0;

public:
    static uint64_t now_ns() {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    void add_front_ns(uint64_t ns) { ns_front_ += ns; }
    void add_back_ns(uint64_t ns) { ns_back_ += ns; }
};

rsd_status BandFrame::init(const rsd_svao_frame_desc& f, const rsd_band_params& bp, Comm* comm) {
    if (!f.cam || !f.vao || !f.svao || !f.sd || !f.scene || !f.d_depth || !f.d_normals || !f.d_ao || !f.d_stencil ||
        !f.d_ray_min || !f.d_ray_max || !f.d_sd || !f.sd_w || !f.sd_h) {
        set_error("rsd_band_frame_create: the frame description lacks a buffer or struct");
        return RSD_ERR_INVALID_ARG;
    }
    if (f.svao->secondary_depth_mode != 2u || !f.svao->ray_interval || !f.sd->ray_interval || f.sd->use_16bit) {
        set_error("rsd_band_frame_create: the band frame serves the StochasticDepth mode with RayInterval (32-bit SD "
                  "maps)");
        return RSD_ERR_UNSUPPORTED;
    }
    if (bp.divisor == 0 || bp.sd_split > RSD_SD_SPLIT_ROWS) {
        set_error("rsd_band_frame_create: divisor must be >= 1 and sd_split one of RSD_SD_SPLIT_*");
        return RSD_ERR_INVALID_ARG;
    }
    cam_ = *f.cam;
    vao_ = *f.vao;
    svp_ = *f.svao;
    sdp_ = *f.sd;
    bp_ = bp;
    f_ = f;
    f_.cam = &cam_;
    f_.vao = &vao_;
    f_.svao = &svp_;
    f_.sd = &sdp_;
    comm_ = comm;
    me_ = comm->rank();
    world_ = comm->world();
    if (world_ > 64) {
        set_error("rsd_band_frame_create: at most 64 ranks");
        return RSD_ERR_UNSUPPORTED;
    }
    guard_ = svp_.guard_band;
    div_ = bp.divisor;
    sdg_ = (uint32_t)std::max(0, vao_.sdGuard);
    if (2 * guard_ >= f.height || 2 * guard_ >= f.width) {
        set_error("rsd_band_frame_create: the guard band leaves no visible rows");
        return RSD_ERR_INVALID_ARG;
    }
    V_ = f.height - 2 * guard_;
    G_ = (V_ + 31) / 32;
    const uint32_t N = sdp_.sample_count;
    L_ = (N + 3) / 4;
    ch_ = std::min(N, 4u);
    split_ = bp.sd_split == RSD_SD_SPLIT_AUTO ? (div_ > 1 ? RSD_SD_SPLIT_TILES : RSD_SD_SPLIT_ROWS) : bp.sd_split;
    if (world_ == 1) split_ = RSD_SD_SPLIT_ROWS;
    consume_ = true;  // RayInterval: the trace resets the interval maps it read
    rebalance_ = bp.rebalance && world_ > 1;
    halo_px_ = halo_reach_px(f.width, f.height, cam_.focalLength, cam_.frameHeight, vao_.ssMaxRadius);
    halo_focal_ = cam_.focalLength;
    halo_frame_h_ = cam_.frameHeight;
    gb_.resize(world_ + 1);
    for (uint32_t r = 0; r <= world_; ++r) gb_[r] = (uint32_t)((uint64_t)G_ * r / world_);
    ao_row_bytes_ = (size_t)f.width * (svp_.dual_ao ? 2u : 1u);
    for (auto& set : ev_)
        for (hipEvent_t& e : set) RSD_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    RSD_HIP(hipHostMalloc((void**)&mhost_, sizeof(int64_t) * (1 + world_ * (world_ + 1)), hipHostMallocDefault));
    std::memset(mhost_, 0, sizeof(int64_t) * (1 + world_ * (world_ + 1)));
    RSD_HIP(hipHostGetDevicePointer((void**)&mhost_dev_, mhost_, 0));
    recv_tr_.resize(world_);
    sd_send_.resize(world_);
    sd_recv_.resize(world_);
    RSD_HIP(hipMalloc(&row_.p, 2 * sizeof(int64_t) * (world_ + 1)));
    row_.cap = 2 * sizeof(int64_t) * (world_ + 1);
    RSD_HIP(hipMalloc(&mdev_.p, sizeof(int64_t) * world_ * (world_ + 1)));
    mdev_.cap = sizeof(int64_t) * world_ * (world_ + 1);
    RSD_HIP(hipMemset(row_.p, 0, row_.cap));
    RSD_HIP(hipMemset(mdev_.p, 0, mdev_.cap));
    return plan(nullptr);
}

// rsd/shard.py HaloFrame._plan: pass bands, SD shares, windows, exchange regions, AO bands
rsd_status BandFrame::plan(hipStream_t s) {
    // a new split changes which SD texels this rank's traces write: its clean-tile stamps are void
    if (sdp_.d_tile_state) {
        const size_t b = (size_t)rsd_sd_tile_state_count(f_.sd_w, f_.sd_h) * sizeof(uint32_t);
        const hipError_t e = s ? hipMemsetAsync(sdp_.d_tile_state, 0, b, s) : hipMemset(sdp_.d_tile_state, 0, b);
        if (e != hipSuccess) return hip_fail(e, "rsd_band_frame (tile state)");
    }
    const uint32_t sdh = f_.sd_h, sdw = f_.sd_w, g = guard_, fbh = f_.height;
    px_rows_.assign(world_, {0, 0});
    for (uint32_t r = 0; r < world_; ++r) px_rows_[r] = {32 * gb_[r], 32 * gb_[r + 1]};
    // SD rows under each band: SD row of frame-buffer row y = y / div + sdGuard (SVAO.cpp:700-716)
    std::vector<uint32_t> S(world_ + 1);
    S[0] = 0;
    for (uint32_t r = 1; r < world_; ++r) S[r] = std::min(sdh, ((g + 32 * gb_[r]) / div_ + sdg_) / 8 * 8);
    S[world_] = sdh;
    for (uint32_t r = 1; r <= world_; ++r) S[r] = std::max(S[r], S[r - 1]);
    sd_rows_.assign(world_, {0, 0});
    window_.assign(world_, {0, 0});
    for (uint32_t r = 0; r < world_; ++r) {
        sd_rows_[r] = {S[r], S[r + 1]};
        const int64_t a_px = (int64_t)g + px_rows_[r].first - halo_px_;
        const int64_t b_px = (int64_t)g + std::min(px_rows_[r].second, V_) + halo_px_;
        const int64_t lo = std::max<int64_t>(0, floordiv(a_px, div_) + sdg_ - 1);
        const int64_t hi = std::min<int64_t>(sdh, floordiv(b_px, div_) + sdg_ + 2);
        window_[r] = {(uint32_t)lo, (uint32_t)std::max(lo, hi)};
    }
    const bool tiles = split_ == RSD_SD_SPLIT_TILES;
    const uint32_t period = tiles ? world_ : 1u;
    auto make = [&](uint32_t lo, uint32_t hi) {
        Region R;
        if (lo >= hi) return R;
        R.valid = true;
        R.lo = lo;
        R.hi = hi;
        R.period = period;
        if (period > 1) {
            const uint64_t nt = ((hi - lo + 7) / 8 + period - 1) / period;
            R.texels = nt * 8 * sdw;
            for (uint32_t t0 = lo; t0 < hi; t0 += 8 * period) R.rows += std::min(8u, hi - t0);
        } else {
            R.texels = (uint64_t)(hi - lo) * sdw;
            R.rows = hi - lo;
        }
        return R;
    };
    // tiles: the tiles of rank k inside window win (from the first tile of k at or after the window's first
    // tile, every world-th tile, rows below the window's end); rows: the overlap of the window and k's rows
    auto share = [&](uint32_t k, const std::pair<uint32_t, uint32_t>& win) {
        if (tiles) {
            int64_t t = win.first / 8;
            t += pymod((int64_t)k - t, world_);
            return make((uint32_t)std::min<int64_t>(8 * t, win.second), win.second);
        }
        return make(std::max(win.first, sd_rows_[k].first), std::min(win.second, sd_rows_[k].second));
    };
    iv_send_.assign(world_, Region{});
    iv_recv_.assign(world_, Region{});
    for (uint32_t k = 0; k < world_; ++k) {
        if (k == me_) continue;
        iv_send_[k] = share(k, window_[me_]);
        iv_recv_[k] = share(me_, window_[k]);
    }
    // AO bands (frame-buffer rows), padded to the largest for one all-gather; pass 1 dispatches roundup32 of
    // the visible rows (SVAO.cpp:347-349), so the last band also writes up to 31 guard-band rows
    ao_rows_.assign(world_, {0, 0});
    ao_max_ = 0;
    for (uint32_t r = 0; r < world_; ++r) {
        ao_rows_[r] = {g + px_rows_[r].first, std::min(fbh, g + px_rows_[r].second)};
        ao_max_ = std::max(ao_max_, ao_rows_[r].second - ao_rows_[r].first);
    }
    // the compaction's output: one allocation, each peer's candidate capacity in interleaved triples
    cand_off_.assign(world_, 0);
    size_t total = 0;
    for (uint32_t k = 0; k < world_; ++k) {
        cand_off_[k] = total;
        if (iv_send_[k].valid) total += 3 * iv_send_[k].texels;
    }
    rsd_status st = cand_all_.ensure(std::max<size_t>(total, 1) * sizeof(int32_t), s, &growth_);
    if (st != RSD_OK) return st;
    regions_.clear();
    region_peer_.clear();
    int32_t* cand = static_cast<int32_t*>(cand_all_.p);
    for (uint32_t k = 0; k < world_; ++k) {
        const Region& R = iv_send_[k];
        if (!R.valid) continue;
        rsd_halo_region h{};
        h.row0 = R.lo;
        h.row1 = R.hi;
        h.out = cand + cand_off_[k];
        h.stride = (uint32_t)R.texels;
        h.period = R.period;
        h.count = static_cast<int64_t*>(row_.p) + k;
        regions_.push_back(h);
        region_peer_.push_back(k);
    }
    return RSD_OK;
}

rsd_status BandFrame::mark(hipStream_t s) {
    if (!timed_) return RSD_OK;
    const uint32_t set = (evn_ / 6) % 2, i = evn_ % 6;
    ++evn_;
    RSD_HIP(hipEventRecord(ev_[set][i], s));
    return RSD_OK;
}

// this object's previous frame's compute time (us): -1 while its events are incomplete (never waits;
// every rank then sees the -1 and nobody re-balances this frame)
int64_t BandFrame::prev_cost_us() const {
    if (!rebalance_ || !prev_valid_) return -1;
    const hipEvent_t* e = ev_[prev_set_];
    if (hipEventQuery(e[5]) != hipSuccess) return -1;  // the last of the six (one stream: the others came first)
    double us = 0.0;
    for (int i = 0; i < 6; i += 2) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, e[i], e[i + 1]) != hipSuccess) return -1;
        us += (double)ms * 1e3;
    }
    return (int64_t)us;
}

// rsd/shard.py HaloFrame._rebalanced: cost spread uniformly over each band's groups, boundaries where the
// cumulative cost crosses k / world of the total, moved half-way from the current split (damping), at least
// one group per rank; kept unless the slowest band is predicted >= 3 % faster
std::vector<uint32_t> BandFrame::rebalanced(const std::vector<double>& costs) const {
    const uint32_t G = G_, W = world_;
    std::vector<double> cum(G + 1, 0.0);
    {
        uint32_t i = 0;
        for (uint32_t r = 0; r < W; ++r) {
            const uint32_t n = gb_[r + 1] - gb_[r];
            const double d = std::max(costs[r], 1e-3) / std::max<uint32_t>(n, 1);
            for (uint32_t j = 0; j < n; ++j, ++i) cum[i + 1] = cum[i] + d;
        }
    }
    const double total = cum[G];
    std::vector<uint32_t> nw(W + 1, 0);
    for (uint32_t k = 1; k < W; ++k) {
        const double target = total * k / W;
        // first i >= 1 with cum[i] >= target
        uint32_t j = (uint32_t)(std::lower_bound(cum.begin() + 1, cum.end(), target) - cum.begin());
        j = std::min(j, G);
        if (j > 0 && target - cum[j - 1] < cum[j] - target) --j;
        nw[k] = (uint32_t)std::nearbyint(0.5 * gb_[k] + 0.5 * j);  // ties to even, like Python's round
    }
    nw[W] = G;
    if (G >= W)
        for (uint32_t k = 1; k < W; ++k) nw[k] = std::min(std::max(nw[k], nw[k - 1] + 1), G - (W - k));
    double pred = 0.0, cur = 0.0;
    for (uint32_t k = 0; k < W; ++k) {
        pred = std::max(pred, cum[nw[k + 1]] - cum[nw[k]]);
        cur = std::max(cur, cum[gb_[k + 1]] - cum[gb_[k]]);
    }
    if (pred > 0.97 * cur) return gb_;
    return nw;
}

// a split chosen by the caller (every rank the same), applied by the next front(): a skewed start for tests of the
// re-balancing, or a split carried over from an earlier run
rsd_status BandFrame::set_split(const uint32_t* split, uint32_t n) {
    if (!split || n != world_ + 1 || split[0] != 0 || split[world_] != G_) {
        set_error("rsd_band_frame_set_split: need world + 1 group boundaries from 0 to the group count");
        return RSD_ERR_INVALID_ARG;
    }
    for (uint32_t k = 0; k < world_; ++k)
        if (split[k + 1] < split[k] || (G_ >= world_ && split[k + 1] == split[k])) {
            set_error("rsd_band_frame_set_split: boundaries must increase (one group per rank at least)");
            return RSD_ERR_INVALID_ARG;
        }
    next_gb_.assign(split, split + n);
    next_forced_ = true;
    return RSD_OK;
}

rsd_status BandFrame::front(const rsd_camera* cam, hipStream_t s) {
    if (open_) {
        set_error("rsd_band_frame_front: front() twice without back()");
        return RSD_ERR_INVALID_ARG;
    }
    last_ = s;
    if (cam) cam_ = *cam;
    // a zoom (focal length) or a new sensor height changes how far a sample reaches (ssMaxRadius projected,
    // VAOData.slang:44): the windows and exchange regions follow it -- every rank gets the same camera
    bool replan = false;
    if (cam_.focalLength != halo_focal_ || cam_.frameHeight != halo_frame_h_) {
        halo_px_ = halo_reach_px(f_.width, f_.height, cam_.focalLength, cam_.frameHeight, vao_.ssMaxRadius);
        halo_focal_ = cam_.focalLength;
        halo_frame_h_ = cam_.frameHeight;
        replan = true;
    }
    if (!next_gb_.empty() && next_gb_ != gb_) {
        gb_ = next_gb_;
        if (!next_forced_) ++resplits_;
        replan = true;
    }
    next_gb_.clear();
    next_forced_ = false;
    if (replan) {
        rsd_status st = plan(s);
        if (st != RSD_OK) return st;
    }
    rsd_status st = RSD_OK;
    if (!(consume_ && intervals_clear_)) {
        st = rsd_svao_clear_intervals(f_.d_ray_min, f_.d_ray_max, f_.sd_w * f_.sd_h, s);
        if (st != RSD_OK) return st;
    }
    // the cost entry of the count row: this object's frame 4j + 1, read by the back() of frame 4j + 2
    const int64_t prev_us = frames_ % 4 == 3 ? cost_ready_ : -1;
    if (frames_ % 4 == 3) cost_ready_ = -1;
    timed_ = rebalance_ && frames_ % 4 == 1;
    if (timed_) timed_stream_ = s;
    if ((st = mark(s)) != RSD_OK) return st;
    st = rsd_svao_pass1_rows(&cam_, &vao_, &svp_, f_.d_depth, f_.d_normals, f_.width, f_.height, f_.d_ao, f_.d_stencil,
                             f_.d_ray_min, f_.d_ray_max, f_.sd_w, f_.sd_h, px_rows_[me_].first, px_rows_[me_].second, s);
    if (st != RSD_OK) return st;
    if ((st = mark(s)) != RSD_OK) return st;
    // every peer's touched texels as interleaved triples, their counts in this frame's count row (row[me]
    // stays 0; the previous frame's compaction zeroed it) and this object's last compute time in row[world],
    // one launch, which also zeroes the other row for the next frame
    int64_t* rows = static_cast<int64_t*>(row_.p);
    int64_t* row = rows + (frames_ % 2) * (world_ + 1);
    int64_t* other = rows + ((frames_ + 1) % 2) * (world_ + 1);
    for (size_t i = 0; i < regions_.size(); ++i) regions_[i].count = row + region_peer_[i];
    st = halo_compact_impl(f_.d_ray_min, f_.d_ray_max, f_.sd_w, f_.sd_h, regions_.data(), (uint32_t)regions_.size(),
                           true, row, world_, prev_us, s, true, other);
    if (st != RSD_OK) return st;
    st = comm_->all_gather(row, mdev_.p, sizeof(int64_t) * (world_ + 1), s);
    if (st != RSD_OK) return st;
    // the matrix to the host, with a sequence number the host polls in back() (no copy engine, no event)
    st = publish_counts(static_cast<const int64_t*>(mdev_.p), mhost_dev_, world_ * (world_ + 1), ++seq_, s);
    if (st != RSD_OK) return st;
    open_ = true;
    return RSD_OK;
}

rsd_status BandFrame::back(void* const* events, hipStream_t s) {
    if (!open_) {
        set_error("rsd_band_frame_back: back() without front()");
        return RSD_ERR_INVALID_ARG;
    }
    open_ = false;
    last_ = s;
    const uint32_t W = world_, me = me_;
    // the counts of THIS frame on the host (with frames in flight: long complete)
    volatile const int64_t* pub = mhost_;
    if (pub[0] != seq_) {
        ++blocked_;
        const uint64_t w0 = now_ns();
        for (uint64_t spin = 0; pub[0] != seq_; ++spin) {
            if (spin > 64) std::this_thread::yield();
            if ((spin & 1023u) == 1023u && now_ns() - w0 > 60000000000ull) {
                set_error("rsd_band_frame_back: the count matrix did not arrive within 60 s (a failed kernel or "
                          "collective on this stream?)");
                return RSD_ERR_HIP;
            }
        }
        ns_wait_ += now_ns() - w0;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    std::vector<int64_t> M((size_t)W * (W + 1));
    for (size_t i = 0; i < M.size(); ++i) M[i] = pub[1 + i];
    auto cnt = [&](uint32_t from, uint32_t to) { return (uint64_t)std::max<int64_t>(0, M[(size_t)from * (W + 1) + to]); };
    // frame 4j + 2: the timed frame 4j + 1 ran before this frame's counts on this stream -- its time is final
    if (rebalance_ && frames_ % 4 == 2) cost_ready_ = s == timed_stream_ ? prev_cost_us() : -1;
    // re-split every fourth frame (every rank sees the same counts: all skip or all re-split)
    if (rebalance_ && frames_ % 4 == 3) {
        std::vector<double> costs(W);
        bool ok = true;
        for (uint32_t k = 0; k < W; ++k) {
            const int64_t c = M[(size_t)k * (W + 1) + W];
            ok = ok && c >= 0;
            costs[k] = (double)c;
        }
        if (ok) next_gb_ = rebalanced(costs);
    }
    rsd_status st = RSD_OK;
    // interval halo: my triples to each texel's owner, theirs into my share
    std::vector<Xfer> sends, recvs;
    std::vector<rsd_halo_list> merge;
    int32_t* cand = static_cast<int32_t*>(cand_all_.p);
    for (uint32_t k = 0; k < W; ++k) {
        if (k == me) continue;
        const uint64_t ns = iv_send_[k].valid ? cnt(me, k) : 0, nr = cnt(k, me);
        if (ns) {
            sends.push_back({cand + cand_off_[k], 12 * ns, k});
            b_iv_ += 12 * ns;
        }
        if (nr) {
            if ((st = recv_tr_[k].ensure(12 * nr, s, &growth_)) != RSD_OK) return st;
            recvs.push_back({recv_tr_[k].p, 12 * nr, k});
            merge.push_back({static_cast<const int32_t*>(recv_tr_[k].p), (uint32_t)nr, 0u});
        }
    }
    if (!sends.empty() || !recvs.empty()) {
        if ((st = comm_->exchange(sends.data(), (uint32_t)sends.size(), recvs.data(), (uint32_t)recvs.size(), s)) != RSD_OK)
            return st;
    }
    if (!merge.empty()) {
        st = halo_merge_impl(f_.d_ray_min, f_.d_ray_max, f_.sd_w, f_.sd_h, merge.data(), (uint32_t)merge.size(), 1u,
                             true, s);
        if (st != RSD_OK) return st;
    }
    // the SD trace of this rank's share (consuming resets the WHOLE interval map for the next frame)
    if (events && events[0]) RSD_HIP(hipEventRecord((hipEvent_t)events[0], s));
    if ((st = mark(s)) != RSD_OK) return st;
    const uint32_t tf = (consume_ ? RSD_SD_CONSUME_INTERVALS : 0u) | (bp_.throughput ? RSD_SD_THROUGHPUT : 0u);
    if (split_ == RSD_SD_SPLIT_TILES)
        st = rsd_sd_trace_band_ex(f_.scene, &cam_, &sdp_, f_.d_depth, f_.width, f_.height, f_.d_ray_min, f_.d_ray_max,
                                  f_.d_sd, f_.sd_w, f_.sd_h, me, W, tf, nullptr, s);
    else
        st = rsd_sd_trace_rows(f_.scene, &cam_, &sdp_, f_.d_depth, f_.width, f_.height, f_.d_ray_min, f_.d_ray_max,
                               f_.d_sd, f_.sd_w, f_.sd_h, sd_rows_[me].first, sd_rows_[me].second, tf, nullptr, s);
    if (st != RSD_OK) return st;
    intervals_clear_ = consume_;
    if ((st = mark(s)) != RSD_OK) return st;
    if (events && events[1]) RSD_HIP(hipEventRecord((hipEvent_t)events[1], s));
    // SD halo: the depths of exactly the texels each peer sent me go back to it
    const size_t per = sizeof(float) * L_ * ch_;
    std::vector<rsd_halo_sd_list> gat, sca;
    sends.clear();
    recvs.clear();
    for (uint32_t k = 0; k < W; ++k) {
        if (k == me) continue;
        const uint64_t nr = cnt(k, me), ns = iv_send_[k].valid ? cnt(me, k) : 0;
        if (nr) {  // reply to k: my depths at k's indices
            if ((st = sd_send_[k].ensure(per * nr, s, &growth_)) != RSD_OK) return st;
            gat.push_back({static_cast<const int32_t*>(recv_tr_[k].p), static_cast<float*>(sd_send_[k].p), (uint32_t)nr, 0u});
            sends.push_back({sd_send_[k].p, per * nr, k});
            b_sd_ += per * nr;
        }
        if (ns) {  // k's depths at my indices
            if ((st = sd_recv_[k].ensure(per * ns, s, &growth_)) != RSD_OK) return st;
            sca.push_back({cand + cand_off_[k], static_cast<float*>(sd_recv_[k].p), (uint32_t)ns, 0u});
            recvs.push_back({sd_recv_[k].p, per * ns, k});
        }
    }
    if (!gat.empty()) {
        st = halo_sd_impl(true, f_.d_sd, L_, f_.sd_w, f_.sd_h, ch_, gat.data(), (uint32_t)gat.size(), true, s,
                          "rsd_band_frame_back: SD gather");
        if (st != RSD_OK) return st;
    }
    if (!sends.empty() || !recvs.empty()) {
        if ((st = comm_->exchange(sends.data(), (uint32_t)sends.size(), recvs.data(), (uint32_t)recvs.size(), s)) != RSD_OK)
            return st;
    }
    if (!sca.empty()) {
        st = halo_sd_impl(false, f_.d_sd, L_, f_.sd_w, f_.sd_h, ch_, sca.data(), (uint32_t)sca.size(), true, s,
                          "rsd_band_frame_back: SD scatter");
        if (st != RSD_OK) return st;
    }
    if ((st = mark(s)) != RSD_OK) return st;
    st = rsd_svao_pass2_rows(&cam_, &vao_, &svp_, f_.d_depth, f_.d_normals, f_.width, f_.height, f_.d_stencil, f_.d_sd,
                             f_.sd_w, f_.sd_h, f_.d_ao, px_rows_[me].first, px_rows_[me].second, s);
    if (st != RSD_OK) return st;
    if ((st = mark(s)) != RSD_OK) return st;
    if (timed_) {
        prev_set_ = ((evn_ - 1) / 6) % 2;
        prev_valid_ = true;
    }
    // AO bands: every rank's rows straight from its image into every other rank's image (point-to-point:
    // each xGMI link carries one band; no gather buffer, no unpack launch)
    uint8_t* ao = f_.d_ao;
    const auto mine = ao_rows_[me];
    const uint64_t mineBytes = (uint64_t)(mine.second - mine.first) * ao_row_bytes_;
    sends.clear();
    recvs.clear();
    for (uint32_t k = 0; k < W; ++k) {
        if (k == me) continue;
        if (mineBytes) sends.push_back({ao + (size_t)mine.first * ao_row_bytes_, mineBytes, k});
        const uint64_t kb = (uint64_t)(ao_rows_[k].second - ao_rows_[k].first) * ao_row_bytes_;
        if (kb) recvs.push_back({ao + (size_t)ao_rows_[k].first * ao_row_bytes_, kb, k});
    }
    if (!sends.empty() || !recvs.empty()) {
        if ((st = comm_->exchange(sends.data(), (uint32_t)sends.size(), recvs.data(), (uint32_t)recvs.size(), s)) != RSD_OK)
            return st;
    }
    b_ao_ += mineBytes * (W - 1);
    ++frames_;
    return RSD_OK;
}

void BandFrame::stats(rsd_band_stats& o) const {
    o = rsd_band_stats{};
    o.rank = me_;
    o.world = world_;
    o.sd_split = split_;
    o.groups = G_;
    for (uint32_t k = 0; k <= world_ && k < 65; ++k) o.split[k] = gb_[k];
    o.sd_row0 = sd_rows_[me_].first;
    o.sd_row1 = sd_rows_[me_].second;
    o.halo_px = halo_px_;
    o.frames = frames_;
    o.blocked_waits = blocked_;
    o.resplits = resplits_;
    o.bytes_intervals = b_iv_;
    o.bytes_sd = b_sd_;
    o.bytes_ao = b_ao_;
    const uint64_t sd_row = (uint64_t)L_ * f_.sd_w * ch_ * sizeof(float);
    for (uint32_t k = 0; k < world_; ++k) {
        if (iv_send_[k].valid) o.dense_intervals += 2 * 4 * iv_send_[k].rows * f_.sd_w;
        if (iv_recv_[k].valid) o.dense_sd += iv_recv_[k].rows * sd_row;
    }
    o.growth_syncs = growth_;
    o.host_front_ns = ns_front_;
    o.host_back_ns = ns_back_;
    o.host_wait_ns = ns_wait_;
}

}  // namespace rsd

struct rsd_band_frame {
    rsd::BandFrame* impl = nullptr;
};

using namespace rsd;

extern "C" rsd_status rsd_band_frame_create(const rsd_svao_frame_desc* frame, const rsd_band_params* params,
                                            rsd_comm* comm, rsd_band_frame** out) {
    if (!frame || !params || !comm || !comm->impl || !out) {
        set_error("rsd_band_frame_create: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    BandFrame* bf = new BandFrame();
    rsd_status st = bf->init(*frame, *params, comm->impl);
    if (st != RSD_OK) {
        delete bf;
        return st;
    }
    *out = new rsd_band_frame{bf};
    return RSD_OK;
}

extern "C" rsd_status rsd_band_frame_set_split(rsd_band_frame* bf, const uint32_t* split, uint32_t n) {
    if (!bf || !bf->impl) {
        set_error("rsd_band_frame_set_split: null frame");
        return RSD_ERR_INVALID_ARG;
    }
    return bf->impl->set_split(split, n);
}

extern "C" rsd_status rsd_band_frame_front(rsd_band_frame* bf, const rsd_camera* cam, rsd_stream stream) {
    if (!bf || !bf->impl) {
        set_error("rsd_band_frame_front: null frame");
        return RSD_ERR_INVALID_ARG;
    }
    const uint64_t t0 = BandFrame::now_ns();
    const rsd_status st = bf->impl->front(cam, (hipStream_t)stream);
    bf->impl->add_front_ns(BandFrame::now_ns() - t0);
    return st;
}

extern "C" rsd_status rsd_band_frame_back(rsd_band_frame* bf, void* const* events, rsd_stream stream) {
    if (!bf || !bf->impl) {
        set_error("rsd_band_frame_back: null frame");
        return RSD_ERR_INVALID_ARG;
    }
    const uint64_t t0 = BandFrame::now_ns();
    const rsd_status st = bf->impl->back(events, (hipStream_t)stream);
    bf->impl->add_back_ns(BandFrame::now_ns() - t0);
    return st;
}

extern "C" rsd_status rsd_band_frame_stats(const rsd_band_frame* bf, rsd_band_stats* out) {
    if (!bf || !bf->impl || !out) {
        set_error("rsd_band_frame_stats: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    bf->impl->stats(*out);
    return RSD_OK;
}

extern "C" void rsd_band_frame_release(rsd_band_frame* bf) {
    if (!bf) return;
    if (bf->impl) {
        (void)hipStreamSynchronize(bf->impl->last_stream());  // its transfers may still read the buffers
        delete bf->impl;
    }
    delete bf;
}
