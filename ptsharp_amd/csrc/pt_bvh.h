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
#include <cstddef>
#include <vector>

namespace pt {

constexpr int kMaxDepth = 32;     // BVH2 depth bound
// Traversal stack entries per lane: the BVH4 collapse keeps every root-to-leaf path's pushes
// within it (the traversal kernels hold the first kLdsStack in LDS and the rest in a
// per-thread global column; the megakernel all in LDS).  A larger budget lets the collapse
// fill more nodes to four children (fewer, wider steps per ray).
// The BVH4 collapses keep every path within kStack4Budget pushes (48 or 64 measured: the BVH 1 % smaller, no
// faster); the 8-wide triangle BVH pushes up to 7 per node and is collapsed within kStackMax.
constexpr int kStack4Budget = 32;
constexpr int kStackMax = 64;
static_assert(kStack4Budget >= kMaxDepth, "the collapse needs at least the BVH2 depth");
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

// prim_min/prim_max: [n][3] AABBs.  Builds with up to `threads` host threads; leaves hold
// at most max_leaf (1..kMaxLeafSize) primitives.
// fill_leaves: a node of at most max_leaf primitives is always a leaf.  The triangle BVH's leaves
// are 128-B chunks that one traversal step reads whole (7 loads for 1, 2 or 3 triangles), so a
// leaf of three costs about what a leaf of one does, and SAH's per-primitive cost (which splits
// most 3-triangle nodes) only adds steps.
// bins: SAH bins per axis (2..256).
void build_bvh(const float* prim_min, const float* prim_max, int64_t n, int threads, BvhResult& out,
               int max_leaf = kMaxLeafSize, bool fill_leaves = false, int bins = 32);

// 4-wide BVH collapsed from the BVH2: one 128-byte node (one cache line) per
// step of the traversal instead of a 64-byte child pair, so a ray makes about
// half as many dependent loads.  Node = 32 words, children as SoA:
//   [0..3] lo.x  [4..7] hi.x  [8..11] lo.y  [12..15] hi.y  [16..19] lo.z  [20..23] hi.z
//   [24..27] child ref  [28..31] 0
// ref: bit31 = 0 → inner node index; bit31 = 1 → leaf, bits 29..30 = count-1,
// bits 0..28 = first primitive; kEmpty4 = unused slot.  Node 0 is the root.
constexpr uint32_t kEmpty4 = 0x7FFFFFFFu;
constexpr int kNode4Words = 32;

struct Bvh4Result {
    std::vector<uint32_t> words;   // kNode4Words per node
    int stack_need = 0;            // worst-case traversal stack entries (<= budget)
    int depth = 0;
    int64_t children = 0;          // used child slots (fill = children / (4 * nodes))
    size_t nodes() const { return words.size() / kNode4Words; }
};

// A traversal pushes up to (children - 1) entries per node, so collapsing is
// limited on the tallest paths to keep every root-to-leaf path's pushes within
// `stack_budget` (the LDS stack depth) — the guarantee the BVH2 had by depth.
void collapse_bvh4(const BvhResult& bvh2, int stack_budget, Bvh4Result& out);

// The SAH-optimal collapse (pt_bvh.cpp SahCollapser): children chosen by a dynamic program over the
// BVH2 that minimises the expected traversal cost, c_step per step (inner node or leaf chunk) and
// c_tri per triangle test, weighted by surface area; BVH2 subtrees of at most max_leaf triangles may
// merge into one leaf chunk.  Subtrees whose DP choice would break stack_budget on some path are
// collapsed greedily (collapse_bvh4), so the bound holds.
void collapse_bvh4_sah(const BvhResult& bvh2, int stack_budget, Bvh4Result& out, double c_step = 1.0,
                       double c_tri = 0.5, int max_leaf = 3);

// 8-wide BVH with quantized child boxes: one 128-byte line per node, as a BVH4 node, for about a quarter
// fewer steps per ray (tools/bvh_quality.cpp's wide-node model on the C4 ray mix: closest hit 7.97 → 6.08
// steps, shadow 11.34 → 8.24).  Node = 32 words:
//   [0..2]  origin x, y, z (fp32: the union of the child boxes' lower corner)
//   [3]     bits 0-23: exponents ex, ey, ez (biased by 127: step 2^(e-127)), bits 24-27: inner children
//           n_in, bits 28-31: children n (1..8)
//   [4]     the first inner child's node index (inner children are consecutive, slots 0 .. n_in-1)
//   [5]     0x80000000 + the first leaf chunk's index - n_in (leaf slots n_in .. n-1 are consecutive chunks; slot
//           k's ref is [5] + k: bit 31 and the chunk index; the chunk's word 0 holds its triangle count)
//   [6]     2 bits per slot: a leaf slot's triangle count - 1 (host checks)
//   [7]     0
//   [8..31] the child bounds as binary16 integers q (0..kQMax = 2047, exact in binary16; pt_bvh.cpp), SoA: lo.x[8] hi.x[8]
//           lo.y[8] hi.y[8] lo.z[8] hi.z[8]; bound = origin + q·step, a superset of the child's box;
//           an empty slot has lo = +inf, hi = -inf.
// A traversal computes a slab distance as fma(q, step/d, (origin - o)/d).
constexpr int kNode8Words = 32;
struct Bvh8Result {
    std::vector<uint32_t> words;         // kNode8Words per node; node 0 is the root
    std::vector<uint32_t> chunk_first;   // per leaf chunk: its first primitive (position in BvhResult::order)
    std::vector<uint8_t> chunk_count;    // per leaf chunk: its primitives (1 .. max_leaf)
    int stack_need = 0;                  // worst-case traversal stack entries (<= budget)
    int depth = 0;
    int64_t children = 0;
    size_t nodes() const { return words.size() / kNode8Words; }
};
// The SAH-optimal 8-wide collapse (collapse_bvh4_sah's dynamic program with 8 slots; subtrees whose choice
// would break stack_budget are collapsed greedily, 8-wide) and the quantization.  Leaves: BVH2 subtrees of at
// most max_leaf primitives, one chunk each.
void collapse_bvh8q(const BvhResult& bvh2, int stack_budget, Bvh8Result& out, double c_step = 1.0, double c_tri = 0.5,
                    int max_leaf = 3);
// The box a slot's quantized bounds describe, in exact arithmetic rounded outward to fp32 (host checks).
void bvh8_child_box(const uint32_t* node, int slot, float lo[3], float hi[3]);

}  // namespace pt
