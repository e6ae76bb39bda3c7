// bvh_build.h -- host BVH2 builder for librsd.
//
// Replaces the driver-built DXR BLAS/TLAS (Scene.cpp:3091 buildBlas, :3628 buildTlas):
// a binned-SAH binary BVH over the world-space triangle soup, flattened into the
// layout the HIP traversal kernels read from HBM:
//
//   node (64 B) = 4 x 16 B:  {c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y}
//                            {c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y}
//                            {c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z}
//                            {c0.ref,  c1.ref,  c0.cnt,  c1.cnt }   (uint32)
//     cnt > 0: leaf child, ref = first triangle record, cnt triangles
//     cnt = 0: inner child, ref = node index (0xffffffff + empty box: no child)
//   triangle record (48 B) = {v0.xyz, prim id}, {v1.xyz, flags}, {v2.xyz, 0}
//
// Both child boxes live in the parent, so one 64-B fetch tests two children.
#pragma once
#include <cstdint>
#include <vector>

namespace rsd {

struct BvhStats {
    uint32_t inner_nodes = 0;
    uint32_t leaves = 0;
    uint32_t max_depth = 0;
    double sah_cost = 0.0;
    double build_ms = 0.0;
};

struct FlatBvh {
    std::vector<float> nodes;   // 16 floats per inner node (the last 4 are uint32 bits)
    std::vector<float> tris;    // 12 floats per triangle record
    BvhStats stats;
};

constexpr uint32_t kBvhMaxDepth = 60;   // traversal stack is 64 entries
constexpr uint32_t kBvhMaxLeaf = 4;

// positions: float3[nv]; indices: uint32[3*nt]; flags: uint32[nt] or nullptr
FlatBvh build_bvh(const float* positions, uint32_t nv, const uint32_t* indices, uint32_t nt,
                  const uint32_t* flags, unsigned threads);

}  // namespace rsd
