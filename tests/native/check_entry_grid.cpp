// check_entry_grid.cpp -- host check of the segment entry grid's coverage property (csrc/entry_grid.h).
//
// A random triangle scene is built with librsd's own host BVH builder and entry-grid builder.  For
// random ray segments (short and long, inside and outside the scene), the SD setup kernel's lookup
// (sd_trace.hip entry_lookup, restated here with the same float operations) picks a cell; every
// triangle the segment clearly crosses (double precision, margins away from edges and interval
// ends) must lie under one of that cell's frontier items, and a cell reported absent must have no
// such triangle.  With a spatial-split budget (4th argument, bvh_build.h BvhOptions) the BVH holds
// several references of a triangle, each in a leaf whose box covers part of it: then the leaf under
// the frontier must hold a reference of the crossed triangle whose box contains the crossing point
// (the split boxes cover the triangle).  Prints "violations N" (0 expected).
#include <map>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <set>
#include <vector>

#include "bvh_build.h"
#include "entry_grid.h"

using namespace rsd;

namespace {
constexpr uint32_t kLeaf = 0x80000000u, kOff = 0x1fffffffu, kNone = 0xffffffffu;

uint32_t fbits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

struct V3 { float x, y, z; };

struct Box { float lo[3], hi[3]; };

// the primitives under an item (traversal encoding), each with the boxes of the leaves holding it
void collect(const FlatBvh& b, uint32_t triOff, uint32_t item, const Box& box, std::map<uint32_t, std::vector<Box>>& out) {
    if (item & kLeaf) {
        const uint32_t cnt = ((item >> 29) & 3u) + 1u, first = ((item & kOff) - triOff) / 3u;
        for (uint32_t k = 0; k < cnt; ++k) out[fbits(b.tris[12 * (size_t)(first + k) + 3])].push_back(box);
        return;
    }
    const float* nd = &b.nodes[(size_t)(item / 8u) * 32];
    for (int j = 0; j < 4; ++j) {
        const uint32_t ref = fbits(nd[24 + j]), cnt = fbits(nd[28 + j]);
        if (ref == kNone) continue;
        const Box c{{nd[0 + j], nd[8 + j], nd[16 + j]}, {nd[4 + j], nd[12 + j], nd[20 + j]}};
        collect(b, triOff, cnt ? (kLeaf | ((cnt - 1u) << 29) | (triOff + 3u * ref)) : 8u * ref, c, out);
    }
}

// sd_trace.hip entry_lookup, same float operations; returns -1 dead, 0 root, else slot value
int64_t lookup(const EntryGrid& g, V3 o, V3 d, float TMin, float TMax) {
    const float pad = 0x1p-14f * (std::fabs(o.x) + std::fabs(o.y) + std::fabs(o.z) + TMax) + 1e-30f;
    const V3 p0{o.x + d.x * TMin, o.y + d.y * TMin, o.z + d.z * TMin};
    const V3 p1{o.x + d.x * TMax, o.y + d.y * TMax, o.z + d.z * TMax};
    const float lx = std::fmin(p0.x, p1.x) - pad, hx = std::fmax(p0.x, p1.x) + pad;
    const float ly = std::fmin(p0.y, p1.y) - pad, hy = std::fmax(p0.y, p1.y) + pad;
    const float lz = std::fmin(p0.z, p1.z) - pad, hz = std::fmax(p0.z, p1.z) + pad;
    const float m = std::fmax(std::fmax(hx - lx, hy - ly), hz - lz);
    const float E = g.extent;
    if (!(m <= E)) return 0;
    int R = std::min((int)g.rmax, std::ilogb(E / m));
    while (R > 0 && m > std::ldexp(E, -R)) --R;
    const float sc = std::ldexp(1.0f, R) / E;
    const int i = (int)std::floor((0.5f * (lx + hx) - g.origin[0]) * sc);
    const int j = (int)std::floor((0.5f * (ly + hy) - g.origin[1]) * sc);
    const int k = (int)std::floor((0.5f * (lz + hz) - g.origin[2]) * sc);
    const int hi = 1 << R;
    if (i < -1 || j < -1 || k < -1 || i > hi || j > hi || k > hi) return -1;
    const uint64_t key = entry_key((uint32_t)R, i, j, k);
    uint32_t bits = 0;
    while ((4ull << bits) < g.slots.size()) ++bits;
    uint32_t h = entry_hash(key, bits);
    for (uint32_t n = 0; n <= g.max_probe; ++n, h = (h + 1u) & ((1u << bits) - 1u)) {
        const uint32_t* s = &g.slots[4 * (size_t)h];
        if (s[0] == (uint32_t)key && s[1] == (uint32_t)(key >> 32)) return s[2];
        if (s[0] == 0u && s[1] == 0u) break;
    }
    return -1;
}

// does the segment clearly cross the triangle (double, margins)?  th: the crossing's t
bool clear_hit(const double o[3], const double d[3], double t0, double t1, const float* v, double& th) {
    const double e1[3] = {v[4] - v[0], v[5] - v[1], v[6] - v[2]}, e2[3] = {v[8] - v[0], v[9] - v[1], v[10] - v[2]};
    const double p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
    const double det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    if (std::fabs(det) < 1e-12) return false;
    const double s[3] = {o[0] - v[0], o[1] - v[1], o[2] - v[2]};
    const double u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) / det;
    const double q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const double w = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) / det;
    const double t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) / det;
    const double eps = 1e-4;
    th = t;
    return u > eps && w > eps && u + w < 1.0 - eps && t > t0 + 1e-4 * (1.0 + t0) && t < t1 - 1e-4 * (1.0 + t1);
}
}  // namespace

int main(int argc, char** argv) {
    const uint32_t nTris = argc > 1 ? (uint32_t)atoi(argv[1]) : 20000, nRays = argc > 2 ? (uint32_t)atoi(argv[2]) : 20000;
    const float off = argc > 3 ? (float)atof(argv[3]) : 0.0f;  // scene and rays translated (coordinate magnitude)
    BvhOptions opt;
    opt.split_budget = argc > 4 ? atof(argv[4]) : 0.0;
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    std::vector<float> pos;
    std::vector<uint32_t> idx;
    for (uint32_t t = 0; t < nTris; ++t) {
        const float cx = off + 40.0f * U(rng) - 20.0f, cy = off + 12.0f * U(rng), cz = off + 40.0f * U(rng) - 20.0f;
        const float s = t % 97 == 0 ? 8.0f : 0.05f + 0.5f * U(rng);  // a few large triangles
        for (int k = 0; k < 3; ++k) {
            pos.push_back(cx + s * (U(rng) - 0.5f));
            pos.push_back(cy + s * (U(rng) - 0.5f));
            pos.push_back(cz + s * (U(rng) - 0.5f));
            idx.push_back(3 * t + k);
        }
    }
    const FlatBvh b = build_bvh(pos.data(), 3 * nTris, idx.data(), nTris, nullptr, 4, opt);
    const uint32_t triOff = (uint32_t)(b.nodes.size() / 4);
    const EntryGrid g = build_entry_grid(b.nodes, triOff, 1u << 18, 4);
    std::printf("cells %u levels %u probe %u references %u spatial_splits %u\n", g.cells, g.rmax + 1, g.max_probe,
                b.stats.references, b.stats.spatial_splits);
    const uint32_t nRec = (uint32_t)(b.tris.size() / 12);
    uint64_t violations = 0, checkedHits = 0, rootRays = 0, deadRays = 0;
    for (uint32_t r = 0; r < nRays; ++r) {
        const V3 o{off + 60.0f * U(rng) - 30.0f, off + 20.0f * U(rng) - 4.0f, off + 60.0f * U(rng) - 30.0f};
        V3 d{U(rng) - 0.5f, U(rng) - 0.5f, U(rng) - 0.5f};
        float TMin = 40.0f * U(rng);
        if (r % 5 != 0) {
            // aimed at a point of a random triangle: the segment brackets that hit
            const float* tv = &b.tris[12 * (size_t)(rng() % nRec)];
            float a = U(rng), c = U(rng);
            if (a + c > 1.0f) { a = 1.0f - a; c = 1.0f - c; }
            const V3 p{tv[0] + a * (tv[4] - tv[0]) + c * (tv[8] - tv[0]), tv[1] + a * (tv[5] - tv[1]) + c * (tv[9] - tv[1]),
                       tv[2] + a * (tv[6] - tv[2]) + c * (tv[10] - tv[2])};
            d = {p.x - o.x, p.y - o.y, p.z - o.z};
        }
        const float l = std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
        d = {d.x / l, d.y / l, d.z / l};
        const float len = r % 10 == 0 ? 20.0f * U(rng) : 1.5f * U(rng) * U(rng);  // mostly short, some long
        if (r % 5 != 0) TMin = std::fmax(0.0f, l - len * U(rng));
        const float TMax = TMin + len;
        const int64_t v = lookup(g, o, d, TMin, TMax);
        std::map<uint32_t, std::vector<Box>> under;
        if (v == 0) { ++rootRays; continue; }
        if (v > 0) {
            const uint32_t first = (uint32_t)v >> 4, n = (uint32_t)v & 15u;
            for (uint32_t e = 0; e < n; ++e) {
                const float* it = &g.items[8 * (size_t)(first + e)];
                collect(b, triOff, fbits(it[0]), Box{{it[1], it[2], it[3]}, {it[4], it[5], it[6]}}, under);
            }
        } else {
            ++deadRays;
        }
        const double od[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
        for (uint32_t t = 0; t < nTris; ++t) {
            float tv[12];
            for (int j = 0; j < 3; ++j)
                for (int k = 0; k < 3; ++k) tv[4 * j + k] = pos[3 * (size_t)idx[3 * (size_t)t + j] + k];
            double th;
            if (!clear_hit(od, dd, TMin, TMax, tv, th)) continue;
            ++checkedHits;
            const double ph[3] = {od[0] + dd[0] * th, od[1] + dd[1] * th, od[2] + dd[2] * th};
            bool covered = false;
            auto f = under.find(t);
            if (f != under.end())
                for (const Box& bx : f->second) {
                    bool in = true;
                    for (int k = 0; k < 3; ++k) in = in && ph[k] >= bx.lo[k] && ph[k] <= bx.hi[k];
                    covered = covered || in;
                }
            if (!covered) ++violations;
        }
    }
    std::printf("rays %u root %llu dead %llu hits %llu violations %llu\n", nRays, (unsigned long long)rootRays,
                (unsigned long long)deadRays, (unsigned long long)checkedHits, (unsigned long long)violations);
    return violations ? 1 : 0;
}
