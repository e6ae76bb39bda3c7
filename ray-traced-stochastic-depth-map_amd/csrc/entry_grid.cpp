// entry_grid.cpp -- host build of the segment entry grid (entry_grid.h).
#include "entry_grid.h"

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>

namespace rsd {

namespace {

constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kLeaf = 0x80000000u;  // bvh_traverse.h kLeafBit
constexpr double kLoose = 0.5 + 1.0 / 16.0;  // loose-cell growth per side, in cells

struct Item {
    uint32_t code;  // traversal encoding: 8 * node index, or leaf bit | (count - 1) << 29 | record offset
    int32_t node;   // wide node index (inner), -1 for a leaf
    float lo[3], hi[3];
    float area;
};

struct Cell {
    int64_t i, j, k;
    uint8_t n;
    uint32_t f[kEntryCap];  // item indices
};

uint32_t fbits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

struct Builder {
    std::vector<Item> items;  // [0] = root, 1 + 4 n + j = child slot j of wide node n

    bool overlaps(uint32_t it, const double lo[3], const double hi[3]) const {
        const Item& x = items[it];
        for (int a = 0; a < 3; ++a)
            if ((double)x.lo[a] > hi[a] || (double)x.hi[a] < lo[a]) return false;
        return true;
    }

    // children of item `it` (inner) overlapping the box
    int children(uint32_t it, const double lo[3], const double hi[3], uint32_t out[4]) const {
        int n = 0;
        const int32_t nd = items[it].node;
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t c = 1u + 4u * (uint32_t)nd + j;
            if (items[c].code != kNone && overlaps(c, lo, hi)) out[n++] = c;
        }
        return n;
    }

    // frontier of the box from a covering list (every triangle overlapping the box is under `in`)
    int refine(const uint32_t* in, int nin, const double lo[3], const double hi[3], uint32_t out[kEntryCap]) const {
        int n = 0;
        for (int q = 0; q < nin; ++q)
            if (overlaps(in[q], lo, hi)) out[n++] = in[q];
        while (true) {
            int best = -1;
            float bestArea = -1.0f;
            uint32_t bc[4];
            int bn = 0;
            for (int q = 0; q < n; ++q) {
                if (items[out[q]].node < 0 || items[out[q]].area <= bestArea) continue;
                uint32_t c[4];
                const int m = children(out[q], lo, hi, c);
                if (n - 1 + m > (int)kEntryCap) continue;
                best = q;
                bestArea = items[out[q]].area;
                bn = m;
                std::copy(c, c + m, bc);
            }
            if (best < 0) break;
            // replace out[best] by its overlapping children (keeps the list order stable)
            uint32_t tmp[kEntryCap + 4];
            int t = 0;
            for (int q = 0; q < n; ++q) {
                if (q == best) for (int c = 0; c < bn; ++c) tmp[t++] = bc[c];
                else tmp[t++] = out[q];
            }
            n = t;
            std::copy(tmp, tmp + t, out);
        }
        return n;
    }
};

}  // namespace

EntryGrid build_entry_grid(const std::vector<float>& nodes, uint32_t triOff, uint64_t max_cells, unsigned threads) {
    const auto t0 = std::chrono::steady_clock::now();
    EntryGrid g;
    const uint32_t nn = (uint32_t)(nodes.size() / 32);
    if (nn == 0) return g;
    Builder b;
    b.items.resize(1 + 4 * (size_t)nn);
    for (uint32_t n = 0; n < nn; ++n) {
        const float* nd = &nodes[32 * (size_t)n];
        for (uint32_t j = 0; j < 4; ++j) {
            Item& it = b.items[1 + 4 * (size_t)n + j];
            const uint32_t ref = fbits(nd[24 + j]), cnt = fbits(nd[28 + j]);
            if (ref == kNone) { it.code = kNone; it.node = -1; continue; }
            it.code = cnt ? (kLeaf | ((cnt - 1u) << 29) | (triOff + 3u * ref)) : 8u * ref;
            it.node = cnt ? -1 : (int32_t)ref;
            for (int a = 0; a < 3; ++a) { it.lo[a] = nd[8 * a + j]; it.hi[a] = nd[8 * a + 4 + j]; }
            const float dx = it.hi[0] - it.lo[0], dy = it.hi[1] - it.lo[1], dz = it.hi[2] - it.lo[2];
            it.area = dx * dy + dy * dz + dz * dx;
        }
    }
    Item& root = b.items[0];
    root.code = 0u;
    root.node = 0;
    bool any = false;
    for (int a = 0; a < 3; ++a) { root.lo[a] = INFINITY; root.hi[a] = -INFINITY; }
    for (uint32_t j = 0; j < 4; ++j) {
        const Item& c = b.items[1 + j];
        if (c.code == kNone) continue;
        any = true;
        for (int a = 0; a < 3; ++a) { root.lo[a] = std::min(root.lo[a], c.lo[a]); root.hi[a] = std::max(root.hi[a], c.hi[a]); }
    }
    if (!any) return g;
    root.area = INFINITY;
    double ext = 0.0, mag = 0.0;
    for (int a = 0; a < 3; ++a) {
        ext = std::max(ext, (double)root.hi[a] - (double)root.lo[a]);
        mag = std::max({mag, std::fabs((double)root.lo[a]), std::fabs((double)root.hi[a])});
        g.origin[a] = root.lo[a];
    }
    // a power-of-two-friendly edge a little above the bounds' (every coordinate strictly inside)
    g.extent = (float)std::max(ext * (1.0 + 1.0 / 1024.0), 1e-6 * std::max(mag, 1.0));
    const double E = g.extent;
    // finest level whose 1/16-cell margin still dwarfs the device's float rounding of a cell index
    // (a few ulp of the coordinate magnitude)
    const double ulpMag = std::ldexp(std::max(mag + E, 1e-30), -23);
    uint32_t rlimit = 0;
    while (rlimit < kEntryMaxLevel && std::ldexp(E, -(int)(rlimit + 1)) / 16.0 > 64.0 * ulpMag) ++rlimit;

    auto loose = [&](uint32_t r, int64_t i, int64_t j, int64_t k, double lo[3], double hi[3]) {
        const double s = std::ldexp(E, -(int)r);
        const int64_t ix[3] = {i, j, k};
        for (int a = 0; a < 3; ++a) {
            lo[a] = (double)g.origin[a] + ((double)ix[a] - kLoose) * s;
            hi[a] = (double)g.origin[a] + ((double)ix[a] + 1.0 + kLoose) * s;
        }
    };
    std::vector<std::vector<Cell>> levels;
    {
        std::vector<Cell> l0;
        const uint32_t rootList[1] = {0u};
        for (int64_t i = -1; i <= 1; ++i)
            for (int64_t j = -1; j <= 1; ++j)
                for (int64_t k = -1; k <= 1; ++k) {
                    double lo[3], hi[3];
                    loose(0, i, j, k, lo, hi);
                    Cell c{i, j, k, 0, {}};
                    c.n = (uint8_t)b.refine(rootList, 1, lo, hi, c.f);
                    if (c.n) l0.push_back(c);
                }
        levels.push_back(std::move(l0));
    }
    uint64_t total = levels[0].size();
    threads = std::max(1u, std::min(threads, 64u));
    for (uint32_t r = 0; r < rlimit; ++r) {
        const std::vector<Cell>& par = levels.back();
        const int64_t hiIdx = (int64_t)1 << (r + 1);
        std::vector<std::vector<Cell>> part(threads);
        auto work = [&](unsigned t) {
            const size_t n0 = par.size() * t / threads, n1 = par.size() * (t + 1) / threads;
            for (size_t p = n0; p < n1; ++p) {
                const Cell& pc = par[p];
                for (int ch = 0; ch < 8; ++ch) {
                    const int64_t i = 2 * pc.i + (ch & 1), j = 2 * pc.j + (ch >> 1 & 1), k = 2 * pc.k + (ch >> 2);
                    if (i < -1 || j < -1 || k < -1 || i > hiIdx || j > hiIdx || k > hiIdx) continue;
                    double lo[3], hi[3];
                    loose(r + 1, i, j, k, lo, hi);
                    Cell c{i, j, k, 0, {}};
                    c.n = (uint8_t)b.refine(pc.f, pc.n, lo, hi, c.f);
                    if (c.n) part[t].push_back(c);
                }
            }
        };
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < threads; ++t) pool.emplace_back(work, t);
        work(0);
        for (auto& th : pool) th.join();
        size_t cnt = 0;
        for (auto& v : part) cnt += v.size();
        if (total + cnt > max_cells) break;
        std::vector<Cell> next;
        next.reserve(cnt);
        for (auto& v : part) next.insert(next.end(), v.begin(), v.end());
        total += cnt;
        levels.push_back(std::move(next));
    }
    g.rmax = (uint32_t)levels.size() - 1;
    g.cells = (uint32_t)total;
    uint32_t bits = 4;
    while ((1ull << bits) < 2 * total) ++bits;
    const uint32_t cap = 1u << bits, mask = cap - 1u;
    g.slots.assign(4 * (size_t)cap, 0u);
    for (uint32_t r = 0; r < levels.size(); ++r)
        for (const Cell& c : levels[r]) {
            const uint64_t key = entry_key(r, c.i, c.j, c.k);
            uint32_t h = entry_hash(key, bits), probe = 0;
            while (g.slots[4 * (size_t)h] != 0u || g.slots[4 * (size_t)h + 1] != 0u) { h = (h + 1u) & mask; ++probe; }
            g.max_probe = std::max(g.max_probe, probe);
            uint32_t* s = &g.slots[4 * (size_t)h];
            s[0] = (uint32_t)key;
            s[1] = (uint32_t)(key >> 32);
            s[2] = ((uint32_t)(g.items.size() / 8) << 4) | c.n;
            for (int q = 0; q < c.n; ++q) {
                const Item& it = b.items[c.f[q]];
                float code;
                std::memcpy(&code, &it.code, 4);
                g.items.insert(g.items.end(), {code, it.lo[0], it.lo[1], it.lo[2], it.hi[0], it.hi[1], it.hi[2], 0.0f});
            }
        }
    g.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return g;
}

}  // namespace rsd
