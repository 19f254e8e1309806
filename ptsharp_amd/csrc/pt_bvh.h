// pt_bvh.h — host-side binned-SAH BVH2 over primitive AABBs.
//
// Replaces the reference's k-d tree (Tree.NewTree / Node.Split, Tree.cs:22-29,
// 201-265) as the acceleration structure.  The k-d tree returns the exact
// nearest hit (leaves test every shape with no t-clipping, Tree.cs:115-128), so
// any correct acceleration structure yields the same hit; this one is shaped
// for the GPU: 32-B nodes, children stored as adjacent pairs on 64-B lines,
// depth bounded by kMaxDepth so the traversal stack fits a fixed LDS budget.
#pragma once
#include <stdint.h>
#include <vector>

namespace pt {

constexpr int kMaxDepth = 32;     // = LDS traversal stack entries per lane
constexpr int kMaxLeafSize = 4;

// 32-byte node; nodes[0] is the root, nodes[1] is padding, every child pair
// (left = 2k, right = 2k+1) starts on a 64-byte boundary.
struct BvhNode {
    float bmin[3];
    uint32_t a;      // inner: index of the left child (even); leaf: first primitive
    float bmax[3];
    uint32_t b;      // inner: 0; leaf: primitive count (>= 1)
};
static_assert(sizeof(BvhNode) == 32, "BvhNode must be 32 bytes");

struct BvhResult {
    std::vector<BvhNode> nodes;
    std::vector<uint32_t> order;  // order[i] = input primitive stored at position i
    int max_depth = 0;
    int leaves = 0;
};

// prim_min/prim_max: [n][3] AABBs.  Builds with up to `threads` host threads.
void build_bvh(const float* prim_min, const float* prim_max, int64_t n, int threads, BvhResult& out);

}  // namespace pt
