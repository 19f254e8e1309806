// pt_bvh.cpp — parallel binned-SAH BVH2 builder (host, C++17 threads).
#include "pt_bvh.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <mutex>
#include <thread>

namespace pt {
namespace {

struct Aabb {
    float lo[3], hi[3];
    void reset() { for (int k = 0; k < 3; k++) { lo[k] = INFINITY; hi[k] = -INFINITY; } }
    void grow(const Aabb& o) { for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], o.lo[k]); hi[k] = std::max(hi[k], o.hi[k]); } }
    void grow_pt(const float* p) { for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); } }
    float area() const {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.f;
        // clamp huge boxes (planes are never in a BVH, but keep the cost finite)
        return 2.f * (std::min(dx, 1e18f) * std::min(dy, 1e18f) + std::min(dy, 1e18f) * std::min(dz, 1e18f) +
                      std::min(dz, 1e18f) * std::min(dx, 1e18f));
    }
};

constexpr int kBins = 32;
constexpr int64_t kParallelCutoff = 16384;

struct Builder {
    const float* pmin;
    const float* pmax;
    std::vector<float> cent;      // [n][3]
    std::vector<uint32_t> idx;    // permutation being partitioned
    std::vector<BvhNode>& nodes;
    std::atomic<uint32_t> next_pair{2};
    std::atomic<int> max_depth{0};
    std::atomic<int> leaves{0};
    std::atomic<int> live_threads{1};
    int max_threads;
    int max_leaf;
    bool fill_leaves;

    Builder(const float* a, const float* b, int64_t n, std::vector<BvhNode>& out, int threads, int leaf, bool fill)
        : pmin(a), pmax(b), cent((size_t)n * 3), idx((size_t)n), nodes(out), max_threads(threads), max_leaf(leaf),
          fill_leaves(fill) {
        for (int64_t i = 0; i < n; i++) {
            idx[(size_t)i] = (uint32_t)i;
            for (int k = 0; k < 3; k++) cent[(size_t)i * 3 + k] = 0.5f * (pmin[i * 3 + k] + pmax[i * 3 + k]);
        }
    }

    Aabb prim_box(uint32_t p) const {
        Aabb b;
        for (int k = 0; k < 3; k++) { b.lo[k] = pmin[(size_t)p * 3 + k]; b.hi[k] = pmax[(size_t)p * 3 + k]; }
        return b;
    }

    void make_leaf(uint32_t ni, int64_t begin, int64_t end, int depth) {
        nodes[ni].a = (uint32_t)begin;
        nodes[ni].b = (uint32_t)(end - begin);
        leaves++;
        int md = max_depth.load();
        while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {}
    }

    void build(uint32_t ni, int64_t begin, int64_t end, int depth) {
        Aabb bounds, cb;
        bounds.reset(); cb.reset();
        for (int64_t i = begin; i < end; i++) {
            uint32_t p = idx[(size_t)i];
            bounds.grow(prim_box(p));
            cb.grow_pt(&cent[(size_t)p * 3]);
        }
        for (int k = 0; k < 3; k++) { nodes[ni].bmin[k] = bounds.lo[k]; nodes[ni].bmax[k] = bounds.hi[k]; }
        int64_t n = end - begin;
        if (n <= 1 || depth >= kMaxDepth || (fill_leaves && n <= max_leaf)) { make_leaf(ni, begin, end, depth); return; }

        int axis = 0;
        float ext[3];
        for (int k = 0; k < 3; k++) ext[k] = cb.hi[k] - cb.lo[k];
        if (ext[1] > ext[axis]) axis = 1;
        if (ext[2] > ext[axis]) axis = 2;
        int64_t mid = -1;
        // Depth budget: with n > 2^(kMaxDepth-depth-1) only an object-median split keeps
        // every leaf within kMaxDepth (children <= ceil(n/2)).
        bool force_median = (kMaxDepth - depth - 1) < 62 && n > ((int64_t)1 << (kMaxDepth - depth - 1));
        if (ext[axis] <= 0.f) {
            // all centroids coincide: split by count (or leaf if small)
            if (n <= max_leaf) { make_leaf(ni, begin, end, depth); return; }
            mid = begin + n / 2;
        } else if (force_median) {
            mid = begin + n / 2;
            std::nth_element(idx.begin() + begin, idx.begin() + mid, idx.begin() + end, [&](uint32_t a, uint32_t b) {
                return cent[(size_t)a * 3 + axis] < cent[(size_t)b * 3 + axis];
            });
        } else {
            // binned SAH over all three axes
            float best_cost = INFINITY; int best_axis = -1, best_split = -1;
            for (int ax = 0; ax < 3; ax++) {
                if (ext[ax] <= 0.f) continue;
                Aabb bb[kBins]; int cnt[kBins] = {0};
                for (int b = 0; b < kBins; b++) bb[b].reset();
                float scale = (float)kBins / ext[ax];
                for (int64_t i = begin; i < end; i++) {
                    uint32_t p = idx[(size_t)i];
                    int b = (int)((cent[(size_t)p * 3 + ax] - cb.lo[ax]) * scale);
                    b = std::min(std::max(b, 0), kBins - 1);
                    cnt[b]++;
                    bb[b].grow(prim_box(p));
                }
                float rarea[kBins]; int rcnt[kBins];
                Aabb acc; acc.reset(); int c = 0;
                for (int b = kBins - 1; b > 0; b--) { acc.grow(bb[b]); c += cnt[b]; rarea[b] = acc.area(); rcnt[b] = c; }
                acc.reset(); c = 0;
                for (int b = 0; b < kBins - 1; b++) {
                    acc.grow(bb[b]); c += cnt[b];
                    if (c == 0 || rcnt[b + 1] == 0) continue;
                    float cost = acc.area() * (float)c + rarea[b + 1] * (float)rcnt[b + 1];
                    if (cost < best_cost) { best_cost = cost; best_axis = ax; best_split = b; }
                }
            }
            float leaf_cost = bounds.area() * (float)n;
            // traversal step ~ 1 box pair, intersection ~ 1: split cost = 1*area + sum(area*count)
            if (best_axis < 0 || (n <= max_leaf && best_cost + bounds.area() >= leaf_cost)) {
                if (n <= max_leaf) { make_leaf(ni, begin, end, depth); return; }
                mid = begin + n / 2;
                std::nth_element(idx.begin() + begin, idx.begin() + mid, idx.begin() + end, [&](uint32_t a, uint32_t b) {
                    return cent[(size_t)a * 3 + axis] < cent[(size_t)b * 3 + axis];
                });
            } else {
                float scale = (float)kBins / ext[best_axis];
                float lo = cb.lo[best_axis];
                auto it = std::partition(idx.begin() + begin, idx.begin() + end, [&](uint32_t p) {
                    int b = (int)((cent[(size_t)p * 3 + best_axis] - lo) * scale);
                    b = std::min(std::max(b, 0), kBins - 1);
                    return b <= best_split;
                });
                mid = it - idx.begin();
                if (mid == begin || mid == end) mid = begin + n / 2;
            }
        }
        uint32_t pair = next_pair.fetch_add(2);
        nodes[ni].a = pair;
        nodes[ni].b = 0;
        bool spawn = (n >= kParallelCutoff) && live_threads.load() < max_threads;
        if (spawn) {
            live_threads++;
            std::thread th([&, pair, begin, mid, depth] { build(pair, begin, mid, depth + 1); live_threads--; });
            build(pair + 1, mid, end, depth + 1);
            th.join();
        } else {
            build(pair, begin, mid, depth + 1);
            build(pair + 1, mid, end, depth + 1);
        }
    }
};

}  // namespace

void build_bvh(const float* prim_min, const float* prim_max, int64_t n, int threads, BvhResult& out, int max_leaf,
               bool fill_leaves) {
    out.nodes.clear();
    out.order.clear();
    out.max_depth = 0;
    out.leaves = 0;
    if (n <= 0) return;
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    out.nodes.assign((size_t)(2 * n + 2), BvhNode{});
    Builder b(prim_min, prim_max, n, out.nodes, threads, std::min(std::max(max_leaf, 1), kMaxLeafSize), fill_leaves);
    b.build(0, 0, n, 0);
    out.nodes.resize(b.next_pair.load());
    // padding node 1: an empty leaf
    std::memset(&out.nodes[1], 0, sizeof(BvhNode));
    out.order = std::move(b.idx);
    out.max_depth = b.max_depth.load();
    out.leaves = b.leaves.load();
}

namespace {

struct Collapser {
    const std::vector<BvhNode>& n2;
    Bvh4Result& out;
    int budget;
    std::vector<int> height;  // BVH2 stack need below a node (leaf: 0)

    bool is_leaf(uint32_t i) const { return n2[i].b != 0; }
    float area(uint32_t i) const {
        const BvhNode& n = n2[i];
        float dx = n.bmax[0] - n.bmin[0], dy = n.bmax[1] - n.bmin[1], dz = n.bmax[2] - n.bmin[2];
        return dx * dy + dy * dz + dz * dx;
    }
    int fill_height(uint32_t i) {
        if (is_leaf(i)) return height[i] = 0;
        int l = fill_height(n2[i].a), r = fill_height(n2[i].a + 1);
        return height[i] = 1 + std::max(l, r);
    }
    uint32_t ref_of(uint32_t i, uint32_t node4_of_inner) const {
        if (is_leaf(i)) return 0x80000000u | ((n2[i].b - 1u) << 29) | (n2[i].a & 0x1FFFFFFFu);
        return node4_of_inner;
    }
    uint32_t alloc() {
        out.words.resize(out.words.size() + kNode4Words, 0u);
        return (uint32_t)(out.nodes() - 1);
    }
    // children set of BVH4 node `at` built from BVH2 subtree `C` (initial set), ancestors pushed A
    void emit(uint32_t at, std::vector<uint32_t> C, int A, int depth) {
        out.depth = std::max(out.depth, depth);
        for (;;) {
            if (C.size() >= 4) break;
            // expand the largest inner child whose expansion keeps the stack budget
            int pick = -1;
            float best = -1.f;
            for (size_t k = 0; k < C.size(); k++) {
                if (is_leaf(C[k])) continue;
                int maxh = 0;
                for (size_t j = 0; j < C.size(); j++)
                    if (j != k) maxh = std::max(maxh, height[C[j]]);
                maxh = std::max(maxh, std::max(height[n2[C[k]].a], height[n2[C[k]].a + 1]));
                if (A + (int)C.size() + maxh > budget) continue;   // |C'| - 1 = |C|
                float a = area(C[k]);
                if (a > best) { best = a; pick = (int)k; }
            }
            if (pick < 0) break;
            uint32_t e = C[(size_t)pick];
            C[(size_t)pick] = n2[e].a;
            C.push_back(n2[e].a + 1);
        }
        const int pushed = A + (int)C.size() - 1;
        out.stack_need = std::max(out.stack_need, pushed);
        out.children += (int64_t)C.size();
        uint32_t refs[4] = {kEmpty4, kEmpty4, kEmpty4, kEmpty4};
        std::vector<std::pair<uint32_t, uint32_t>> inner;  // (bvh2 node, bvh4 node)
        for (size_t k = 0; k < C.size(); k++) {
            uint32_t node4 = 0;
            if (!is_leaf(C[k])) { node4 = alloc(); inner.emplace_back(C[k], node4); }
            refs[k] = ref_of(C[k], node4);
        }
        uint32_t* w = &out.words[(size_t)at * kNode4Words];
        for (size_t k = 0; k < 4; k++) {
            float lo[3] = {0.f, 0.f, 0.f}, hi[3] = {0.f, 0.f, 0.f};
            if (k < C.size())
                for (int ax = 0; ax < 3; ax++) { lo[ax] = n2[C[k]].bmin[ax]; hi[ax] = n2[C[k]].bmax[ax]; }
            for (int ax = 0; ax < 3; ax++) {
                std::memcpy(&w[8 * ax + k], &lo[ax], 4);
                std::memcpy(&w[8 * ax + 4 + k], &hi[ax], 4);
            }
            w[24 + k] = refs[k];
        }
        for (auto& pr : inner) emit(pr.second, {n2[pr.first].a, n2[pr.first].a + 1}, pushed, depth + 1);
    }
};

}  // namespace

void collapse_bvh4(const BvhResult& bvh2, int stack_budget, Bvh4Result& out) {
    out.words.clear();
    out.stack_need = 0;
    out.depth = 0;
    out.children = 0;
    if (bvh2.nodes.empty()) return;
    Collapser c{bvh2.nodes, out, stack_budget, std::vector<int>(bvh2.nodes.size(), 0)};
    c.fill_height(0);
    const uint32_t root = c.alloc();
    if (c.is_leaf(0)) c.emit(root, {0u}, 0, 0);
    else c.emit(root, {bvh2.nodes[0].a, bvh2.nodes[0].a + 1}, 0, 0);
}

}  // namespace pt
