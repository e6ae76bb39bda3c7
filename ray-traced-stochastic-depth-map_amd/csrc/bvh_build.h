// bvh_build.h -- host BVH2 builder for librsd.
//
// Replaces the driver-built DXR BLAS/TLAS (Scene.cpp:3091 buildBlas, :3628 buildTlas):
// a binned-SAH binary BVH over the world-space triangle soup, flattened into the
// layout the HIP traversal kernels read from HBM:
//
//   4-wide node (128 B) = 8 x 16 B, structure-of-arrays over the 4 children:
//       {lo.x[4]} {hi.x[4]} {lo.y[4]} {hi.y[4]} {lo.z[4]} {hi.z[4]} {ref[4]} {cnt[4]}
//     cnt > 0: leaf child, ref = first triangle record, cnt (<= 4) triangles
//     cnt = 0: inner child, ref = node index;  ref = 0xffffffff: empty slot
//   triangle record (48 B) = {v0.xyz, prim id}, {v1.xyz, flags}, {v2.xyz, 0}
//
// The binary SAH tree is collapsed into 4-wide nodes (open the largest inner child
// until 4 children): one 128-B fetch tests 4 children, halving the dependent-load
// chain of a traversal -- the SD trace is latency-bound.
#pragma once
#include <cstdint>
#include <vector>

namespace rsd {

struct BvhStats {
    uint32_t inner_nodes = 0;
    uint32_t leaves = 0;
    uint32_t max_depth = 0;   // binary SAH tree
    uint32_t wide_depth = 0;  // inner 4-wide nodes on the longest root-to-leaf path (the root counts 1)
    uint32_t references = 0;  // triangle records (> triangle count with spatial splits)
    uint32_t spatial_splits = 0;
    double sah_cost = 0.0;
    double build_ms = 0.0;
};

struct FlatBvh {
    std::vector<float> nodes;   // 32 floats per wide node (the last 8 are uint32 bits)
    std::vector<float> tris;    // 12 floats per triangle record
    BvhStats stats;
};

constexpr uint32_t kBvhMaxDepth = 60;   // traversal stack is 64 entries
constexpr uint32_t kBvhMaxLeaf = 4;
constexpr uint32_t kBvhWidth = 4;

// Spatial splits (SBVH, Stich et al. 2009): where the two boxes of the best object split overlap
// by more than `split_alpha` of the root's area, a split of the node's box at a bin plane that
// clips straddling triangles into both children is also priced; the cheaper one is taken.  A
// triangle then has several references (leaves whose clipped boxes cover parts of it), each
// with its own triangle record: the canonical any-hit stream is unchanged (a walk keeps each
// (t, prim) key once), traversal-order streams need a tree without splits.  `split_budget`
// bounds the extra references (fraction of the triangle count; 0 = no spatial split).
// Clipped boxes are computed in double, rounded outward and padded by `split_pad` x the
// scene's largest coordinate magnitude, so that a hit within the slab test's rounding of a
// split plane lies in both children.
struct BvhOptions {
    double split_budget = 0.0;
    double split_alpha = 1e-5;
    double split_pad = 1.0 / 65536.0;
};

// positions: float3[nv]; indices: uint32[3*nt]; flags: uint32[nt] or nullptr
FlatBvh build_bvh(const float* positions, uint32_t nv, const uint32_t* indices, uint32_t nt,
                  const uint32_t* flags, unsigned threads, const BvhOptions& opt = BvhOptions());

}  // namespace rsd
