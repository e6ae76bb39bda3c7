// entry_grid.h -- segment entry grid: where a short SD ray segment may start its BVH walk.
//
// Every live SD ray of an SVAO frame is a short segment [TMin, TMax] around the visible surface
// (SVAO's ray interval, SVAO.cpp:334-340 / SVAORaster.ps.slang:85-97).  Walked from the root, such
// a segment spends most of its dependent steps descending the top of the tree.  The
// canonical any-hit stream depends only on the SET of triangles the segment hits (rsd.h
// RSD_HIT_ORDER_CANONICAL), so the walk may start anywhere that provably covers that set.
//
// The grid: a cube over the scene's bounds, levels R = 0..rmax with cells of edge s_R = extent / 2^R.
// The LOOSE cell (R, i, j, k) is the cell grown by half a cell (plus a 1/16 margin) on every side.
// For each loose cell that any BVH box overlaps, the host stores its FRONTIER: at most kEntryCap
// BVH items (4-wide nodes or leaves) such that every triangle whose box overlaps the loose cell
// lies under one of them -- found by expanding the root while the list fits, keeping only the
// children whose boxes overlap the cell.  A segment whose (padded) AABB has extent m <= s_R and
// whose centre lies in cell i of level R is inside that loose cell, so its hits are all under the
// frontier.  The setup kernel tests the frontier items' boxes against the ray (the test the walk
// applies to every child it pushes) and the walk starts from the items that pass instead of the
// root, with the same box and triangle tests below them (same hit set, same bits).  A cell absent
// from the table overlaps no BVH box, and a frontier none of whose boxes the ray passes holds no
// hit: either way the texel keeps DEFAULT_DEPTH without a walk.
#pragma once
#include <cstdint>
#include <vector>

#include "bvh_build.h"

namespace rsd {

constexpr uint32_t kEntryCap = 8;         // frontier items per cell (one row-walk step)
constexpr uint32_t kEntryMaxLevel = 14;   // level + 1 fits the key's 4 bits, cell indices + 1 its 20
static_assert(kEntryMaxLevel + 1 < 16, "entry_key stores level + 1 in 4 bits (bits 60-63)");
static_assert((1u << kEntryMaxLevel) + 1 < (1u << 20), "entry_key stores cell index + 1 in 20 bits");

struct EntryGrid {
    float origin[3] = {0.0f, 0.0f, 0.0f};  // the cube's low corner (the root box's)
    float extent = 1.0f;                   // the cube's edge
    uint32_t rmax = 0;                     // finest level stored (every cell of it overlapping a box)
    uint32_t max_probe = 0;                // longest linear-probe run of the hash table
    uint32_t cells = 0;                    // stored cells (all levels)
    double build_ms = 0.0;
    // open-addressing table (capacity a power of two, key 0 = empty): {key_lo, key_hi, val, 0},
    // val = first item << 4 | item count (1..kEntryCap)
    std::vector<uint32_t> slots;
    // entries, 8 floats each: {item code bits, box lo.xyz, box hi.xyz, 0} -- the BVH item (the
    // traversal's encoding) and its box, which the setup kernel tests against the ray
    std::vector<float> items;
};

// key of loose cell (r, i, j, k), i, j, k >= -1
inline uint64_t entry_key(uint32_t r, int64_t i, int64_t j, int64_t k) {
    return ((uint64_t)(r + 1) << 60) | ((uint64_t)(i + 1) << 40) | ((uint64_t)(j + 1) << 20) | (uint64_t)(k + 1);
}
inline uint32_t entry_hash(uint64_t key, uint32_t bits) {
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

// nodes / triOff: the flattened BVH (FlatBvh::nodes, tri_offset in float4 units).  max_cells bounds
// the table (levels are added while the total fits).
EntryGrid build_entry_grid(const std::vector<float>& nodes, uint32_t triOff, uint64_t max_cells, unsigned threads);

}  // namespace rsd
