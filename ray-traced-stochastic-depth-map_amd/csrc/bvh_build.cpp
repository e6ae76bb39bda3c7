// bvh_build.cpp -- binned-SAH BVH2 builder (host, multithreaded).  See bvh_build.h.
#include "bvh_build.h"

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <thread>

namespace rsd {
namespace {

struct Aabb {
    float lo[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                   std::numeric_limits<float>::infinity()};
    float hi[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                   -std::numeric_limits<float>::infinity()};
    void grow(const Aabb& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    void grow(const float* p) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    bool empty() const { return !(lo[0] <= hi[0]); }
    double area() const {
        if (empty()) return 0.0;
        double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct TNode {             // temporary binary-tree node
    Aabb box;
    int32_t left = -1, right = -1;
    uint32_t first = 0, count = 0;  // leaf range in `order`
};

constexpr int kBins = 32;
constexpr double kTraversalCostDefault = 1.0;  // relative to one triangle test
// RSD_BVH_TCOST overrides the SAH traversal cost (build-quality experiments; results do not depend
// on the tree for canonical traces)
const double kTraversalCost = [] {
    const char* e = std::getenv("RSD_BVH_TCOST");
    return e && std::atof(e) > 0.0 ? std::atof(e) : kTraversalCostDefault;
}();

struct Builder {
    const std::vector<Aabb>& tb;       // triangle boxes
    const std::vector<float>& cent;    // centroids, 3 per triangle
    std::vector<uint32_t>& order;
    std::vector<TNode>& nodes;
    std::atomic<uint32_t> next{0};
    std::atomic<uint32_t> maxDepth{0};

    Builder(const std::vector<Aabb>& b, const std::vector<float>& c, std::vector<uint32_t>& o, std::vector<TNode>& n)
        : tb(b), cent(c), order(o), nodes(n) {}

    uint32_t alloc() { return next.fetch_add(1); }

    void make_leaf(uint32_t id, uint32_t first, uint32_t count, uint32_t depth) {
        nodes[id].first = first;
        nodes[id].count = count;
        nodes[id].left = nodes[id].right = -1;
        uint32_t d = maxDepth.load();
        while (depth > d && !maxDepth.compare_exchange_weak(d, depth)) {}
    }

    // Partition [first, first+count) at the centroid median of `axis`.
    uint32_t median_split(uint32_t first, uint32_t count, int axis) {
        uint32_t half = count / 2;
        std::nth_element(order.begin() + first, order.begin() + first + half, order.begin() + first + count,
                         [&](uint32_t a, uint32_t b) { return cent[3 * a + axis] < cent[3 * b + axis]; });
        return half;
    }

    void build(uint32_t id, uint32_t first, uint32_t count, uint32_t depth, int spawn) {
        Aabb box, cb;
        for (uint32_t i = first; i < first + count; ++i) {
            box.grow(tb[order[i]]);
            cb.grow(&cent[3 * order[i]]);
        }
        nodes[id].box = box;
        if (count <= 1) { make_leaf(id, first, count, depth); return; }

        uint32_t nleft = 0;
        // remaining budget: after this depth, median splits need ceil(log2(count)) more levels
        uint32_t need = 0;
        while ((1u << need) < (count + kBvhMaxLeaf - 1) / kBvhMaxLeaf) ++need;
        const bool forceMedian = depth + need + 1 >= kBvhMaxDepth;

        int bestAxis = -1;
        int bestBin = -1;
        double bestCost = std::numeric_limits<double>::infinity();
        if (!forceMedian) {
            for (int axis = 0; axis < 3; ++axis) {
                float ext = cb.hi[axis] - cb.lo[axis];
                if (!(ext > 0.0f)) continue;
                Aabb bb[kBins];
                uint32_t bc[kBins] = {0};
                const float scale = (float)kBins / ext;
                for (uint32_t i = first; i < first + count; ++i) {
                    uint32_t t = order[i];
                    int b = std::min(kBins - 1, (int)((cent[3 * t + axis] - cb.lo[axis]) * scale));
                    bb[b].grow(tb[t]);
                    bc[b]++;
                }
                double rightArea[kBins];
                uint32_t rightCount[kBins];
                Aabb acc;
                uint32_t n = 0;
                for (int b = kBins - 1; b > 0; --b) {
                    acc.grow(bb[b]);
                    n += bc[b];
                    rightArea[b] = acc.area();
                    rightCount[b] = n;
                }
                acc = Aabb();
                n = 0;
                for (int b = 0; b < kBins - 1; ++b) {
                    acc.grow(bb[b]);
                    n += bc[b];
                    if (n == 0 || rightCount[b + 1] == 0) continue;
                    double cost = acc.area() * n + rightArea[b + 1] * rightCount[b + 1];
                    if (cost < bestCost) { bestCost = cost; bestAxis = axis; bestBin = b; }
                }
            }
        }
        const double pa = std::max(box.area(), 1e-30);
        if (bestAxis >= 0) {
            double splitCost = kTraversalCost + bestCost / pa;
            if (count <= kBvhMaxLeaf && splitCost >= (double)count) { make_leaf(id, first, count, depth); return; }
            const float ext = cb.hi[bestAxis] - cb.lo[bestAxis];
            const float scale = (float)kBins / ext;
            auto mid = std::partition(order.begin() + first, order.begin() + first + count, [&](uint32_t t) {
                int b = std::min(kBins - 1, (int)((cent[3 * t + bestAxis] - cb.lo[bestAxis]) * scale));
                return b <= bestBin;
            });
            nleft = (uint32_t)(mid - (order.begin() + first));
        }
        if (nleft == 0 || nleft == count) {
            if (count <= kBvhMaxLeaf) { make_leaf(id, first, count, depth); return; }
            int axis = 0;
            float e0 = cb.hi[0] - cb.lo[0], e1 = cb.hi[1] - cb.lo[1], e2 = cb.hi[2] - cb.lo[2];
            if (e1 > e0 && e1 >= e2) axis = 1;
            else if (e2 > e0 && e2 > e1) axis = 2;
            nleft = median_split(first, count, axis);
        }
        uint32_t l = alloc(), r = alloc();
        nodes[id].left = (int32_t)l;
        nodes[id].right = (int32_t)r;
        nodes[id].count = 0;
        if (spawn > 0 && count > 50000) {
            std::thread th([&, l, first, nleft, depth, spawn] { build(l, first, nleft, depth + 1, spawn - 1); });
            build(r, first + nleft, count - nleft, depth + 1, spawn - 1);
            th.join();
        } else {
            build(l, first, nleft, depth + 1, 0);
            build(r, first + nleft, count - nleft, depth + 1, 0);
        }
    }
};

inline float bits_as_float(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

}  // namespace

FlatBvh build_bvh(const float* pos, uint32_t nv, const uint32_t* ind, uint32_t nt, const uint32_t* flags,
                  unsigned threads) {
    (void)nv;
    auto t0 = std::chrono::steady_clock::now();
    FlatBvh out;
    std::vector<Aabb> tb(nt);
    std::vector<float> cent(3 * (size_t)nt);
    for (uint32_t i = 0; i < nt; ++i) {
        for (int j = 0; j < 3; ++j) tb[i].grow(pos + 3 * (size_t)ind[3 * (size_t)i + j]);
        for (int k = 0; k < 3; ++k) cent[3 * (size_t)i + k] = 0.5f * (tb[i].lo[k] + tb[i].hi[k]);
    }
    std::vector<uint32_t> order(nt);
    for (uint32_t i = 0; i < nt; ++i) order[i] = i;
    std::vector<TNode> nodes(2 * (size_t)std::max<uint32_t>(nt, 1) + 1);
    Builder b(tb, cent, order, nodes);
    uint32_t root = b.alloc();
    int spawn = 0;
    for (unsigned t = std::max(1u, threads); t > 1; t >>= 1) ++spawn;
    if (nt > 0) b.build(root, 0, nt, 0, spawn);
    else nodes[root].count = 0;
    const uint32_t ntmp = b.next.load();

    // ---- collapse the binary tree into 4-wide nodes and flatten (DFS order keeps a node
    // and its nearest subtree close in memory).  Each wide node stores all child boxes.
    out.tris.reserve(12 * (size_t)nt);
    auto emit_tris = [&](const TNode& leaf) -> uint32_t {
        uint32_t first = (uint32_t)(out.tris.size() / 12);
        for (uint32_t k = 0; k < leaf.count; ++k) {
            uint32_t t = order[leaf.first + k];
            for (int j = 0; j < 3; ++j) {
                const float* p = pos + 3 * (size_t)ind[3 * (size_t)t + j];
                out.tris.push_back(p[0]);
                out.tris.push_back(p[1]);
                out.tris.push_back(p[2]);
                uint32_t w = j == 0 ? t : (j == 1 ? (flags ? flags[t] : 0u) : 0u);
                out.tris.push_back(bits_as_float(w));
            }
        }
        return first;
    };
    auto down = [](float v) { return std::nextafter(std::nextafter(v, -INFINITY), -INFINITY); };
    auto up = [](float v) { return std::nextafter(std::nextafter(v, INFINITY), INFINITY); };
    uint32_t nwide = 0;
    // recursive: returns the wide-node index of binary node `n` (an inner node, or the root)
    uint32_t wideDepth = 0;
    std::function<uint32_t(uint32_t, uint32_t)> build_wide = [&](uint32_t n, uint32_t level) -> uint32_t {
        const uint32_t me = nwide++;
        wideDepth = std::max(wideDepth, level);
        out.nodes.resize(32 * (size_t)nwide, 0.0f);
        uint32_t ch[kBvhWidth];
        int nc = 0;
        if (nodes[n].left < 0) {
            if (nodes[n].count) ch[nc++] = n;  // a leaf root: one leaf child
        } else {
            ch[nc++] = (uint32_t)nodes[n].left;
            ch[nc++] = (uint32_t)nodes[n].right;
            while (nc < (int)kBvhWidth) {  // open the largest inner child
                int best = -1;
                double ba = -1.0;
                for (int i = 0; i < nc; ++i)
                    if (nodes[ch[i]].left >= 0 && nodes[ch[i]].box.area() > ba) { ba = nodes[ch[i]].box.area(); best = i; }
                if (best < 0) break;
                const uint32_t c = ch[best];
                ch[best] = (uint32_t)nodes[c].left;
                ch[nc++] = (uint32_t)nodes[c].right;
            }
        }
        uint32_t ref[kBvhWidth], cnt[kBvhWidth];
        float lo[kBvhWidth][3], hi[kBvhWidth][3];
        for (uint32_t i = 0; i < kBvhWidth; ++i) {
            ref[i] = 0xffffffffu;
            cnt[i] = 0;
            for (int k = 0; k < 3; ++k) lo[i][k] = hi[i][k] = 0.0f;
        }
        for (int i = 0; i < nc; ++i) {
            const TNode& c = nodes[ch[i]];
            for (int k = 0; k < 3; ++k) { lo[i][k] = down(c.box.lo[k]); hi[i][k] = up(c.box.hi[k]); }
            if (c.left >= 0) { ref[i] = build_wide(ch[i], level + 1); cnt[i] = 0; }
            else { ref[i] = emit_tris(c); cnt[i] = c.count; }
        }
        float* nd = &out.nodes[32 * (size_t)me];
        for (uint32_t i = 0; i < kBvhWidth; ++i) {
            nd[0 + i] = lo[i][0];  nd[4 + i] = hi[i][0];
            nd[8 + i] = lo[i][1];  nd[12 + i] = hi[i][1];
            nd[16 + i] = lo[i][2]; nd[20 + i] = hi[i][2];
            nd[24 + i] = bits_as_float(ref[i]);
            nd[28 + i] = bits_as_float(cnt[i]);
        }
        return me;
    };
    build_wide(root, 1);
    const uint32_t ninner = nwide;

    // statistics
    double rootArea = std::max(nodes[root].box.area(), 1e-30), sah = 0.0;
    uint32_t leaves = 0;
    for (uint32_t i = 0; i < ntmp; ++i) {
        const TNode& n = nodes[i];
        double a = n.box.area() / rootArea;
        if (n.left >= 0) sah += kTraversalCost * a;
        else if (n.count) { sah += a * n.count; ++leaves; }
    }
    out.stats.inner_nodes = ninner;
    out.stats.leaves = leaves;
    out.stats.max_depth = b.maxDepth.load();
    out.stats.wide_depth = wideDepth;
    out.stats.sah_cost = sah;
    out.stats.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return out;
}

}  // namespace rsd
