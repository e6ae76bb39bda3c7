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

// ---- spatial-split builder (SBVH, bvh_build.h BvhOptions) ----------------------------------------
struct Ref {
    Aabb box;      // bounds of the part of `tri` this reference covers (clipped, outward, padded)
    uint32_t tri;
};

constexpr int kSplitBins = 32;

struct SplitBuilder {
    const float* pos;
    const uint32_t* ind;
    std::vector<TNode>& nodes;
    std::vector<uint32_t>& leafTris;
    std::atomic<uint32_t> next{0}, leafNext{0}, maxDepth{0}, splits{0};
    std::atomic<int64_t> budget;
    double minOverlap;
    float pad;

    SplitBuilder(const float* p, const uint32_t* i, std::vector<TNode>& n, std::vector<uint32_t>& lt, int64_t b,
                 double mo, float pd)
        : pos(p), ind(i), nodes(n), leafTris(lt), budget(b), minOverlap(mo), pad(pd) {}

    // bounds of triangle t clipped to lo <= x[axis] <= hi (double), rounded outward to float, padded,
    // and intersected with `within`; empty if the triangle does not reach the slab
    Aabb clip(uint32_t t, int axis, double lo, double hi, const Aabb& within) const {
        double poly[9][3], tmp[9][3];
        int n = 3;
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) poly[j][k] = pos[3 * (size_t)ind[3 * (size_t)t + j] + k];
        for (int side = 0; side < 2 && n > 0; ++side) {
            const double c = side == 0 ? lo : hi;
            auto inside = [&](const double* v) { return side == 0 ? v[axis] >= c : v[axis] <= c; };
            int m = 0;
            for (int j = 0; j < n; ++j) {
                const double* a = poly[j];
                const double* b = poly[(j + 1) % n];
                const bool ia = inside(a), ib = inside(b);
                if (ia) { for (int k = 0; k < 3; ++k) tmp[m][k] = a[k]; ++m; }
                if (ia != ib) {
                    const double s = (c - a[axis]) / (b[axis] - a[axis]);
                    for (int k = 0; k < 3; ++k) tmp[m][k] = a[k] + s * (b[k] - a[k]);
                    tmp[m][axis] = c;
                    ++m;
                }
            }
            n = m;
            for (int j = 0; j < n; ++j)
                for (int k = 0; k < 3; ++k) poly[j][k] = tmp[j][k];
        }
        Aabb r;
        if (n == 0) return r;
        for (int k = 0; k < 3; ++k) {
            double l = poly[0][k], h = poly[0][k];
            for (int j = 1; j < n; ++j) { l = std::min(l, poly[j][k]); h = std::max(h, poly[j][k]); }
            float fl = (float)l, fh = (float)h;
            if ((double)fl > l) fl = std::nextafter(fl, -INFINITY);
            if ((double)fh < h) fh = std::nextafter(fh, INFINITY);
            r.lo[k] = std::max(fl - pad, within.lo[k]);
            r.hi[k] = std::min(fh + pad, within.hi[k]);
            if (!(r.lo[k] <= r.hi[k])) return Aabb();
        }
        return r;
    }

    void make_leaf(uint32_t id, const std::vector<Ref>& refs, uint32_t depth) {
        const uint32_t first = leafNext.fetch_add((uint32_t)refs.size());
        for (size_t i = 0; i < refs.size(); ++i) leafTris[first + i] = refs[i].tri;
        nodes[id].first = first;
        nodes[id].count = (uint32_t)refs.size();
        nodes[id].left = nodes[id].right = -1;
        uint32_t d = maxDepth.load();
        while (depth > d && !maxDepth.compare_exchange_weak(d, depth)) {}
    }

    static float centroid(const Ref& r, int axis) { return 0.5f * (r.box.lo[axis] + r.box.hi[axis]); }

    void build(uint32_t id, std::vector<Ref>& refs, uint32_t depth, int spawn) {
        Aabb box, cb;
        for (const Ref& r : refs) {
            box.grow(r.box);
            float c[3] = {centroid(r, 0), centroid(r, 1), centroid(r, 2)};
            cb.grow(c);
        }
        nodes[id].box = box;
        const uint32_t count = (uint32_t)refs.size();
        if (count <= 1) { make_leaf(id, refs, depth); return; }
        uint32_t need = 0;
        while ((1u << need) < (count + kBvhMaxLeaf - 1) / kBvhMaxLeaf) ++need;
        const bool forceMedian = depth + need + 1 >= kBvhMaxDepth - 4;

        // object split: binned SAH over the references' centroids
        int oAxis = -1, oBin = -1;
        double oCost = std::numeric_limits<double>::infinity();
        Aabb oLeft, oRight;
        if (!forceMedian) {
            for (int axis = 0; axis < 3; ++axis) {
                const float ext = cb.hi[axis] - cb.lo[axis];
                if (!(ext > 0.0f)) continue;
                Aabb bb[kBins];
                uint32_t bc[kBins] = {0};
                const float scale = (float)kBins / ext;
                for (const Ref& r : refs) {
                    const int b = std::min(kBins - 1, (int)((centroid(r, axis) - cb.lo[axis]) * scale));
                    bb[b].grow(r.box);
                    bc[b]++;
                }
                Aabb rightBox[kBins];
                uint32_t rightCount[kBins];
                Aabb acc;
                uint32_t n = 0;
                for (int b = kBins - 1; b > 0; --b) {
                    acc.grow(bb[b]);
                    n += bc[b];
                    rightBox[b] = acc;
                    rightCount[b] = n;
                }
                acc = Aabb();
                n = 0;
                for (int b = 0; b < kBins - 1; ++b) {
                    acc.grow(bb[b]);
                    n += bc[b];
                    if (n == 0 || rightCount[b + 1] == 0) continue;
                    const double cost = acc.area() * n + rightBox[b + 1].area() * rightCount[b + 1];
                    if (cost < oCost) {
                        oCost = cost; oAxis = axis; oBin = b; oLeft = acc; oRight = rightBox[b + 1];
                    }
                }
            }
        }
        // spatial split: chopped binning of the references over the node's box
        int sAxis = -1;
        double sCost = std::numeric_limits<double>::infinity(), sPlane = 0.0;
        if (oAxis >= 0 && budget.load() > 0) {
            Aabb ov;
            for (int k = 0; k < 3; ++k) { ov.lo[k] = std::max(oLeft.lo[k], oRight.lo[k]); ov.hi[k] = std::min(oLeft.hi[k], oRight.hi[k]); }
            const bool overlaps = ov.lo[0] <= ov.hi[0] && ov.lo[1] <= ov.hi[1] && ov.lo[2] <= ov.hi[2];
            if (overlaps && ov.area() > minOverlap) {
                for (int axis = 0; axis < 3; ++axis) {
                    const double lo = box.lo[axis], ext = (double)box.hi[axis] - lo;
                    if (!(ext > 4.0 * pad)) continue;
                    const double w = ext / kSplitBins;
                    Aabb bb[kSplitBins];
                    uint32_t enter[kSplitBins] = {0}, exit[kSplitBins] = {0};
                    for (const Ref& r : refs) {
                        int b0 = (int)((r.box.lo[axis] - lo) / w), b1 = (int)((r.box.hi[axis] - lo) / w);
                        b0 = std::clamp(b0, 0, kSplitBins - 1);
                        b1 = std::clamp(b1, b0, kSplitBins - 1);
                        if (b0 == b1) { bb[b0].grow(r.box); }
                        else {
                            for (int b = b0; b <= b1; ++b) {
                                const double sl = b == b0 ? -INFINITY : lo + b * w;
                                const double sh = b == b1 ? INFINITY : lo + (b + 1) * w;
                                const Aabb c = clip(r.tri, axis, sl, sh, r.box);
                                if (!c.empty()) bb[b].grow(c);
                            }
                        }
                        enter[b0]++;
                        exit[b1]++;
                    }
                    Aabb rightBox[kSplitBins];
                    uint32_t rightCount[kSplitBins];
                    Aabb acc;
                    uint32_t n = 0;
                    for (int b = kSplitBins - 1; b > 0; --b) {
                        acc.grow(bb[b]);
                        n += exit[b];
                        rightBox[b] = acc;
                        rightCount[b] = n;
                    }
                    acc = Aabb();
                    n = 0;
                    for (int b = 0; b < kSplitBins - 1; ++b) {
                        acc.grow(bb[b]);
                        n += enter[b];
                        if (n == 0 || rightCount[b + 1] == 0) continue;
                        const double cost = acc.area() * n + rightBox[b + 1].area() * rightCount[b + 1];
                        if (cost < sCost) { sCost = cost; sAxis = axis; sPlane = lo + (b + 1) * w; }
                    }
                }
            }
        }
        const double pa = std::max(box.area(), 1e-30);
        const double bestCost = std::min(oCost, sCost);
        if (count <= kBvhMaxLeaf && (oAxis < 0 || kTraversalCost + bestCost / pa >= (double)count)) {
            make_leaf(id, refs, depth);
            return;
        }
        std::vector<Ref> left, right;
        bool done = false;
        if (sAxis >= 0 && sCost < oCost) {
            // partition with reference unsplitting (Stich et al. 2009, 4.4)
            const int a = sAxis;
            Aabb lb, rb;
            std::vector<uint32_t> straddle;
            for (uint32_t i = 0; i < count; ++i) {
                const Ref& r = refs[i];
                if (r.box.hi[a] <= sPlane) { left.push_back(r); lb.grow(r.box); }
                else if (r.box.lo[a] >= sPlane) { right.push_back(r); rb.grow(r.box); }
                else straddle.push_back(i);
            }
            int64_t dup = 0;
            std::vector<Ref> sl, sr;
            for (uint32_t i : straddle) {
                const Ref& r = refs[i];
                const Aabb cl = clip(r.tri, a, -INFINITY, sPlane, r.box), cr = clip(r.tri, a, sPlane, INFINITY, r.box);
                if (cl.empty()) { right.push_back(r); rb.grow(r.box); continue; }
                if (cr.empty()) { left.push_back(r); lb.grow(r.box); continue; }
                const double nl = (double)left.size() + sl.size(), nr = (double)right.size() + sr.size();
                Aabb lbS = lb, rbS = rb, lbU = lb, rbU = rb;
                lbS.grow(cl); rbS.grow(cr); lbU.grow(r.box); rbU.grow(r.box);
                const double cSplit = lbS.area() * (nl + 1) + rbS.area() * (nr + 1);
                const double cLeft = lbU.area() * (nl + 1) + rb.area() * nr;
                const double cRight = lb.area() * nl + rbU.area() * (nr + 1);
                if (cLeft <= cSplit && cLeft <= cRight) { left.push_back(r); lb = lbU; }
                else if (cRight <= cSplit) { right.push_back(r); rb = rbU; }
                else {
                    sl.push_back(Ref{cl, r.tri});
                    sr.push_back(Ref{cr, r.tri});
                    lb = lbS;
                    rb = rbS;
                    ++dup;
                }
            }
            if ((left.size() + sl.size()) > 0 && (right.size() + sr.size()) > 0 &&
                (left.size() + sl.size()) < count + dup && (right.size() + sr.size()) < count + dup &&
                budget.fetch_sub(dup) >= dup) {
                left.insert(left.end(), sl.begin(), sl.end());
                right.insert(right.end(), sr.begin(), sr.end());
                if (dup) splits.fetch_add(1);
                done = true;
            } else {
                if (dup) budget.fetch_add(dup);
                left.clear();
                right.clear();
            }
        }
        if (!done && oAxis >= 0) {
            const float ext = cb.hi[oAxis] - cb.lo[oAxis];
            const float scale = (float)kBins / ext;
            for (const Ref& r : refs) {
                const int b = std::min(kBins - 1, (int)((centroid(r, oAxis) - cb.lo[oAxis]) * scale));
                (b <= oBin ? left : right).push_back(r);
            }
            done = !left.empty() && !right.empty();
            if (!done) { left.clear(); right.clear(); }
        }
        if (!done) {
            if (count <= kBvhMaxLeaf) { make_leaf(id, refs, depth); return; }
            int axis = 0;
            const float e0 = cb.hi[0] - cb.lo[0], e1 = cb.hi[1] - cb.lo[1], e2 = cb.hi[2] - cb.lo[2];
            if (e1 > e0 && e1 >= e2) axis = 1;
            else if (e2 > e0 && e2 > e1) axis = 2;
            const uint32_t half = count / 2;
            std::nth_element(refs.begin(), refs.begin() + half, refs.end(),
                             [&](const Ref& x, const Ref& y) { return centroid(x, axis) < centroid(y, axis); });
            left.assign(refs.begin(), refs.begin() + half);
            right.assign(refs.begin() + half, refs.end());
        }
        std::vector<Ref>().swap(refs);
        const uint32_t l = next.fetch_add(2), r = l + 1;
        nodes[id].left = (int32_t)l;
        nodes[id].right = (int32_t)r;
        nodes[id].count = 0;
        if (spawn > 0 && count > 50000) {
            std::thread th([&, l, depth, spawn] { build(l, left, depth + 1, spawn - 1); });
            build(r, right, depth + 1, spawn - 1);
            th.join();
        } else {
            build(l, left, depth + 1, 0);
            build(r, right, depth + 1, 0);
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
                  unsigned threads, const BvhOptions& opt) {
    (void)nv;
    auto t0 = std::chrono::steady_clock::now();
    FlatBvh out;
    std::vector<Aabb> tb(nt);
    std::vector<float> cent(3 * (size_t)nt);
    for (uint32_t i = 0; i < nt; ++i) {
        for (int j = 0; j < 3; ++j) tb[i].grow(pos + 3 * (size_t)ind[3 * (size_t)i + j]);
        for (int k = 0; k < 3; ++k) cent[3 * (size_t)i + k] = 0.5f * (tb[i].lo[k] + tb[i].hi[k]);
    }
    int spawn = 0;
    for (unsigned t = std::max(1u, threads); t > 1; t >>= 1) ++spawn;
    std::vector<uint32_t> order;     // leaf triangle ids: TNode first / count index it
    std::vector<TNode> nodes;
    uint32_t root = 0, ntmp = 0;
    const int64_t extra = opt.split_budget > 0.0 ? (int64_t)(opt.split_budget * nt) : 0;
    if (extra > 0 && nt > 0) {
        Aabb all;
        for (uint32_t i = 0; i < nt; ++i) all.grow(tb[i]);
        float mag = 0.0f;
        for (int k = 0; k < 3; ++k) mag = std::max({mag, std::fabs(all.lo[k]), std::fabs(all.hi[k])});
        order.assign((size_t)nt + (size_t)extra, 0u);
        nodes.resize(2 * ((size_t)nt + (size_t)extra) + 1);
        SplitBuilder sb(pos, ind, nodes, order, extra, opt.split_alpha * all.area(), (float)(opt.split_pad * mag));
        std::vector<Ref> refs(nt);
        for (uint32_t i = 0; i < nt; ++i) refs[i] = Ref{tb[i], i};
        root = sb.next.fetch_add(1);
        sb.build(root, refs, 0, spawn);
        ntmp = sb.next.load();
        out.stats.max_depth = sb.maxDepth.load();
        out.stats.references = sb.leafNext.load();
        out.stats.spatial_splits = sb.splits.load();
    } else {
        order.resize(nt);
        for (uint32_t i = 0; i < nt; ++i) order[i] = i;
        nodes.resize(2 * (size_t)std::max<uint32_t>(nt, 1) + 1);
        Builder b(tb, cent, order, nodes);
        root = b.alloc();
        if (nt > 0) b.build(root, 0, nt, 0, spawn);
        else nodes[root].count = 0;
        ntmp = b.next.load();
        out.stats.max_depth = b.maxDepth.load();
        out.stats.references = nt;
    }

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
    out.stats.wide_depth = wideDepth;
    out.stats.sah_cost = sah;
    out.stats.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return out;
}

}  // namespace rsd
