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

constexpr int kMaxBins = 256;
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
    int bins;

    Builder(const float* a, const float* b, int64_t n, std::vector<BvhNode>& out, int threads, int leaf, bool fill, int nbins)
        : pmin(a), pmax(b), cent((size_t)n * 3), idx((size_t)n), nodes(out), max_threads(threads), max_leaf(leaf),
          fill_leaves(fill), bins(std::min(std::max(nbins, 2), kMaxBins)) {
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
                const int kBins = bins;
                Aabb bb[kMaxBins]; int cnt[kMaxBins] = {0};
                for (int b = 0; b < kBins; b++) bb[b].reset();
                float scale = (float)kBins / ext[ax];
                for (int64_t i = begin; i < end; i++) {
                    uint32_t p = idx[(size_t)i];
                    int b = (int)((cent[(size_t)p * 3 + ax] - cb.lo[ax]) * scale);
                    b = std::min(std::max(b, 0), kBins - 1);
                    cnt[b]++;
                    bb[b].grow(prim_box(p));
                }
                float rarea[kMaxBins]; int rcnt[kMaxBins];
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
                const int kBins = bins;
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
               bool fill_leaves, int bins) {
    out.nodes.clear();
    out.order.clear();
    out.max_depth = 0;
    out.leaves = 0;
    if (n <= 0) return;
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    out.nodes.assign((size_t)(2 * n + 2), BvhNode{});
    Builder b(prim_min, prim_max, n, out.nodes, threads, std::min(std::max(max_leaf, 1), kMaxLeafSize), fill_leaves, bins);
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

// SAH-optimal 4-wide collapse (the dynamic program of Ylitie, Karras and Laine 2017, "Efficient
// incoherent ray traversal on GPUs through compressed wide BVHs", §4.1, for 4 slots).  cost(n, i) is
// the least expected cost of BVH2 subtree n when it may take up to i child slots of the wide node
// above it: one slot holds it as a leaf chunk (at most kChunkTris triangles, contiguous in `order`,
// so any BVH2 subtree that small can become one) or as an inner node of its own; more slots let its
// children (or their children) be lifted into the parent.  A step (an inner node or a leaf chunk:
// one 128-B line) costs c_step, a triangle test c_tri, each weighted by its box's surface area.
struct SahCollapser {
    const std::vector<BvhNode>& n2;
    Bvh4Result& out;
    double c_step, c_tri;
    int max_leaf;
    Collapser* greedy;             // budget-keeping fallback for subtrees on the tallest paths (heights filled)
    int budget;
    std::vector<double> cost;      // [node][4]: cost(n, i + 1)
    std::vector<int8_t> choice;    // [node][4]: 0 = one slot (leaf or inner), -1 = as with one slot fewer, k > 0: k slots to the left child
    std::vector<uint8_t> as_leaf;  // one slot: a leaf chunk rather than an inner node
    std::vector<uint32_t> prims, first;

    bool is_leaf(uint32_t i) const { return n2[i].b != 0; }
    double area(uint32_t i) const {
        const BvhNode& n = n2[i];
        double dx = (double)n.bmax[0] - n.bmin[0], dy = (double)n.bmax[1] - n.bmin[1], dz = (double)n.bmax[2] - n.bmin[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
        return dx * dy + dy * dz + dz * dx;
    }
    void solve(uint32_t n) {
        double* C = &cost[(size_t)n * 4];
        int8_t* ch = &choice[(size_t)n * 4];
        const double a = area(n);
        if (is_leaf(n)) {
            prims[n] = n2[n].b;
            first[n] = n2[n].a;
            for (int i = 0; i < 4; i++) { C[i] = a * (c_step + c_tri * (double)prims[n]); ch[i] = 0; }
            as_leaf[n] = 1;
            return;
        }
        const uint32_t l = n2[n].a, r = l + 1;
        solve(l);
        solve(r);
        prims[n] = prims[l] + prims[r];
        first[n] = first[l];
        const double* CL = &cost[(size_t)l * 4];
        const double* CR = &cost[(size_t)r * 4];
        auto dist = [&](int j, int& kbest) {   // j slots between the two children
            double best = INFINITY;
            kbest = -1;
            for (int k = 1; k < j; k++) {
                const double c = CL[k - 1] + CR[j - k - 1];
                if (c < best) { best = c; kbest = k; }
            }
            return best;
        };
        int k4;
        const double inner = a * c_step + dist(4, k4);
        const double leaf = (int)prims[n] <= max_leaf ? a * (c_step + c_tri * (double)prims[n]) : INFINITY;
        as_leaf[n] = leaf <= inner;
        C[0] = std::min(leaf, inner);
        ch[0] = 0;
        for (int i = 2; i <= 4; i++) {
            int k;
            const double d = dist(i, k);
            if (d < C[i - 2]) { C[i - 1] = d; ch[i - 1] = (int8_t)k; }
            else { C[i - 1] = C[i - 2]; ch[i - 1] = -1; }
        }
    }
    // the BVH2 nodes that fill the slots of subtree n given i slots
    void slots(uint32_t n, int i, std::vector<uint32_t>& outs) const {
        const int8_t c = choice[(size_t)n * 4 + (size_t)(i - 1)];
        if (c == 0) { outs.push_back(n); return; }
        if (c < 0) { slots(n, i - 1, outs); return; }
        slots(n2[n].a, c, outs);
        slots(n2[n].a + 1, i - c, outs);
    }
    uint32_t alloc() {
        out.words.resize(out.words.size() + kNode4Words, 0u);
        return (uint32_t)(out.nodes() - 1);
    }
    // wide node `at` for BVH2 inner node n (its 4 slots), A entries pushed by the ancestors
    void emit(uint32_t at, uint32_t n, int A, int depth) {
        out.depth = std::max(out.depth, depth);
        std::vector<uint32_t> C;
        slots(n2[n].a, choice_split(n), C);
        slots(n2[n].a + 1, 4 - choice_split(n), C);
        const int pushed = A + (int)C.size() - 1;
        // The stack bound: below a child c the greedy collapse can always finish within
        // pushed + height(c) entries (its BVH2 pushes); where the DP's choice would leave a path
        // without that room, this subtree is collapsed greedily instead (it keeps the bound by
        // construction, as long as A + height(n) <= budget, which holds from the root down).
        int maxh = 0;
        for (uint32_t c : C) maxh = std::max(maxh, as_leaf[c] ? 0 : greedy->height[c]);
        if (pushed + maxh > budget) {
            greedy->emit(at, {n2[n].a, n2[n].a + 1}, A, depth);
            return;
        }
        out.stack_need = std::max(out.stack_need, pushed);
        out.children += (int64_t)C.size();
        uint32_t refs[4] = {kEmpty4, kEmpty4, kEmpty4, kEmpty4};
        std::vector<std::pair<uint32_t, uint32_t>> inner;
        for (size_t k = 0; k < C.size(); k++) {
            const uint32_t c = C[k];
            if (as_leaf[c]) {
                refs[k] = 0x80000000u | ((prims[c] - 1u) << 29) | (first[c] & 0x1FFFFFFFu);
            } else {
                const uint32_t node4 = alloc();
                inner.emplace_back(c, node4);
                refs[k] = node4;
            }
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
        for (auto& pr : inner) emit(pr.second, pr.first, pushed, depth + 1);
    }
    int choice_split(uint32_t n) const {   // the left child's share of an inner node's 4 slots
        const double* CL = &cost[(size_t)n2[n].a * 4];
        const double* CR = &cost[(size_t)(n2[n].a + 1) * 4];
        int kbest = 1;
        double best = INFINITY;
        for (int k = 1; k < 4; k++) {
            const double c = CL[k - 1] + CR[4 - k - 1];
            if (c < best) { best = c; kbest = k; }
        }
        return kbest;
    }
};

}  // namespace

void collapse_bvh4_sah(const BvhResult& bvh2, int stack_budget, Bvh4Result& out, double c_step, double c_tri, int max_leaf) {
    out.words.clear();
    out.stack_need = 0;
    out.depth = 0;
    out.children = 0;
    if (bvh2.nodes.empty()) return;
    const size_t nn = bvh2.nodes.size();
    Collapser g{bvh2.nodes, out, stack_budget, std::vector<int>(nn, 0)};
    g.fill_height(0);
    SahCollapser c{bvh2.nodes, out, c_step, c_tri, max_leaf, &g, stack_budget, std::vector<double>(nn * 4, 0.0),
                   std::vector<int8_t>(nn * 4, 0), std::vector<uint8_t>(nn, 0), std::vector<uint32_t>(nn, 0),
                   std::vector<uint32_t>(nn, 0)};
    c.solve(0);
    const uint32_t root = c.alloc();
    if (c.is_leaf(0)) {   // a lone leaf: the root node holds it in slot 0
        uint32_t* w = &out.words[0];
        for (int k = 0; k < 4; k++) w[24 + k] = kEmpty4;
        for (int ax = 0; ax < 3; ax++) {
            std::memcpy(&w[8 * ax], &bvh2.nodes[0].bmin[ax], 4);
            std::memcpy(&w[8 * ax + 4], &bvh2.nodes[0].bmax[ax], 4);
        }
        w[24] = 0x80000000u | ((bvh2.nodes[0].b - 1u) << 29) | (bvh2.nodes[0].a & 0x1FFFFFFFu);
        out.children = 1;
        return;
    }
    c.emit(root, 0, 0, 0);
}

namespace {

// ---- 8-wide quantized collapse (pt_bvh.h collapse_bvh8q)
constexpr int kW8 = 8;
constexpr uint32_t kQMax = 2047;   // child bounds as binary16 integers: 0..2047 are exact

uint16_t half_of_int(uint32_t q) {   // an integer 0..2047 as binary16 bits (exact)
    if (q == 0) return 0;
    int e = 31 - __builtin_clz(q);   // 2^e <= q < 2^(e+1), e <= 10
    return (uint16_t)(((uint32_t)(e + 15) << 10) | ((q - (1u << e)) << (10 - e)));
}
uint32_t int_of_half(uint16_t h) {   // the inverse, for the integers half_of_int makes
    if (h == 0) return 0;
    const int e = (int)(h >> 10) - 15;
    return (1u << e) + ((uint32_t)(h & 0x3FFu) >> (10 - e));
}

struct Wide8 {
    const std::vector<BvhNode>& n2;
    Bvh8Result& out;
    double c_step, c_tri;
    int max_leaf, budget;
    std::vector<int> height;       // BVH2 stack need below a node (greedy bound)
    std::vector<double> cost;      // [node][8]: cost(n, i + 1)
    std::vector<int8_t> choice;    // [node][8]: 0 one slot, -1 as with one slot fewer, k > 0: k slots to the left child
    std::vector<uint8_t> as_leaf;  // one slot: a leaf chunk rather than an inner node
    std::vector<uint32_t> prims, first;

    bool is_leaf(uint32_t i) const { return n2[i].b != 0; }
    double area(uint32_t i) const {
        const BvhNode& n = n2[i];
        double dx = (double)n.bmax[0] - n.bmin[0], dy = (double)n.bmax[1] - n.bmin[1], dz = (double)n.bmax[2] - n.bmin[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
        return dx * dy + dy * dz + dz * dx;
    }
    int fill_height(uint32_t i) {
        if (is_leaf(i)) return height[i] = 0;
        const int l = fill_height(n2[i].a), r = fill_height(n2[i].a + 1);
        return height[i] = 1 + std::max(l, r);
    }
    double dist(uint32_t n, int j, int& kbest) const {
        const double* CL = &cost[(size_t)n2[n].a * kW8];
        const double* CR = &cost[(size_t)(n2[n].a + 1) * kW8];
        double best = INFINITY;
        kbest = -1;
        for (int k = 1; k < j; k++) {
            const double c = CL[k - 1] + CR[j - k - 1];
            if (c < best) { best = c; kbest = k; }
        }
        return best;
    }
    void solve(uint32_t n) {
        double* C = &cost[(size_t)n * kW8];
        int8_t* ch = &choice[(size_t)n * kW8];
        const double a = area(n);
        if (is_leaf(n)) {
            prims[n] = n2[n].b;
            first[n] = n2[n].a;
            for (int i = 0; i < kW8; i++) { C[i] = a * (c_step + c_tri * (double)prims[n]); ch[i] = 0; }
            as_leaf[n] = 1;
            return;
        }
        const uint32_t l = n2[n].a, r = l + 1;
        solve(l);
        solve(r);
        prims[n] = prims[l] + prims[r];
        first[n] = first[l];
        int kw;
        const double inner = a * c_step + dist(n, kW8, kw);
        const double leaf = (int)prims[n] <= max_leaf ? a * (c_step + c_tri * (double)prims[n]) : INFINITY;
        as_leaf[n] = leaf <= inner;
        C[0] = std::min(leaf, inner);
        ch[0] = 0;
        for (int i = 2; i <= kW8; i++) {
            int k;
            const double d = dist(n, i, k);
            if (d < C[i - 2]) { C[i - 1] = d; ch[i - 1] = (int8_t)k; }
            else { C[i - 1] = C[i - 2]; ch[i - 1] = -1; }
        }
    }
    void slots(uint32_t n, int i, std::vector<uint32_t>& outs) const {
        const int8_t c = choice[(size_t)n * kW8 + (size_t)(i - 1)];
        if (c == 0) { outs.push_back(n); return; }
        if (c < 0) { slots(n, i - 1, outs); return; }
        slots(n2[n].a, c, outs);
        slots(n2[n].a + 1, i - c, outs);
    }
    // greedy children of subtree root set C within the budget (collapse_bvh4's rule, 8 slots)
    void greedy(std::vector<uint32_t>& C, int A) const {
        while (C.size() < (size_t)kW8) {
            int pick = -1;
            double best = -1.0;
            for (size_t k = 0; k < C.size(); k++) {
                if (is_leaf(C[k])) continue;
                int maxh = 0;
                for (size_t j = 0; j < C.size(); j++)
                    if (j != k) maxh = std::max(maxh, height[C[j]]);
                maxh = std::max(maxh, std::max(height[n2[C[k]].a], height[n2[C[k]].a + 1]));
                if (A + (int)C.size() + maxh > budget) continue;
                const double a = area(C[k]);
                if (a > best) { best = a; pick = (int)k; }
            }
            if (pick < 0) break;
            const uint32_t e = C[(size_t)pick];
            C[(size_t)pick] = n2[e].a;
            C.push_back(n2[e].a + 1);
        }
    }
    std::vector<int> need_memo;    // [node]: stack entries the DP collapse of subtree n pushes on its worst path
    void dp_children(uint32_t n, std::vector<uint32_t>& C) const {
        int k;
        (void)dist(n, kW8, k);
        slots(n2[n].a, k, C);
        slots(n2[n].a + 1, kW8 - k, C);
    }
    int need(uint32_t n) {
        int& r = need_memo[n];
        if (r >= 0) return r;
        std::vector<uint32_t> C;
        dp_children(n, C);
        int m = 0;
        for (uint32_t c : C)
            if (!as_leaf[c]) m = std::max(m, need(c));
        return r = (int)C.size() - 1 + m;
    }
    uint32_t alloc(int k) {
        const uint32_t at = (uint32_t)out.nodes();
        out.words.resize(out.words.size() + (size_t)k * kNode8Words, 0u);
        return at;
    }
    // node `at` for BVH2 inner node n, A entries pushed by the ancestors.  The DP's children when its whole
    // collapse below keeps the stack within the budget (need), else the greedy children, which keep it by
    // construction (A + height(n) <= budget holds from the root down, the BVH2 depth being bounded).
    void emit(uint32_t at, uint32_t n, int A, int depth) {
        out.depth = std::max(out.depth, depth);
        std::vector<uint32_t> C;
        bool leafy[kW8] = {false};
        const bool dp = A + need(n) <= budget;
        if (dp) {
            dp_children(n, C);
        } else {
            C = {n2[n].a, n2[n].a + 1};
            greedy(C, A);
        }
        for (size_t k = 0; k < C.size(); k++) leafy[k] = dp ? as_leaf[C[k]] != 0 : is_leaf(C[k]);
        // inner children first, then leaves (pt_bvh.h layout)
        std::vector<uint32_t> inner, leaves;
        for (size_t k = 0; k < C.size(); k++) (leafy[k] ? leaves : inner).push_back(C[k]);
        C = inner;
        C.insert(C.end(), leaves.begin(), leaves.end());
        const int nc = (int)C.size(), nin = (int)inner.size();
        const int pushed = A + nc - 1;
        out.stack_need = std::max(out.stack_need, pushed);
        out.children += nc;
        const uint32_t base_in = nin ? alloc(nin) : 0u;
        const uint32_t base_chunk = (uint32_t)out.chunk_first.size();
        uint32_t cnt_bits = 0;
        for (int k = nin; k < nc; k++) {
            const uint32_t c = C[(size_t)k];
            const uint32_t np = dp ? prims[c] : n2[c].b, fp = dp ? first[c] : n2[c].a;
            out.chunk_first.push_back(fp);
            out.chunk_count.push_back((uint8_t)np);
            cnt_bits |= (np - 1u) << (2 * k);
        }
        uint32_t* w = &out.words[(size_t)at * kNode8Words];
        // quantization, per axis: origin = the children's lowest bound, step 2^e the least power of two with
        // every bound within kQMax steps; q rounded outward (exact arithmetic in double)
        uint32_t ebits = 0;
        uint16_t qb[6][kW8];
        for (int ax = 0; ax < 3; ax++) {
            float o = INFINITY, top = -INFINITY;
            for (uint32_t c : C) { o = std::min(o, n2[c].bmin[ax]); top = std::max(top, n2[c].bmax[ax]); }
            const double ext = (double)top - (double)o;
            int e = -126;
            while (e < 127 && std::ldexp((double)kQMax, e) < ext) e++;
            for (;;) {   // the outward rounding can need one more step
                bool ok = true;
                for (int k = 0; k < nc && ok; k++) {
                    const double hi = std::ceil(((double)n2[C[(size_t)k]].bmax[ax] - (double)o) / std::ldexp(1.0, e));
                    ok = hi <= (double)kQMax;
                }
                if (ok || e >= 127) break;
                e++;
            }
            std::memcpy(&w[ax], &o, 4);
            ebits |= (uint32_t)(e + 127) << (8 * ax);
            for (int k = 0; k < kW8; k++) {
                if (k >= nc) { qb[2 * ax][k] = 0x7C00; qb[2 * ax + 1][k] = 0xFC00; continue; }   // +inf / -inf
                const double step = std::ldexp(1.0, e);
                const double lo = std::floor(((double)n2[C[(size_t)k]].bmin[ax] - (double)o) / step);
                const double hi = std::ceil(((double)n2[C[(size_t)k]].bmax[ax] - (double)o) / step);
                qb[2 * ax][k] = half_of_int((uint32_t)std::max(0.0, lo));
                qb[2 * ax + 1][k] = half_of_int((uint32_t)std::min((double)kQMax, std::max(0.0, hi)));
            }
        }
        w[3] = ebits | ((uint32_t)nin << 24) | ((uint32_t)nc << 28);
        w[4] = base_in;
        w[5] = 0x80000000u + base_chunk - (uint32_t)nin;   // leaf slot k's ref (0x80000000 | chunk) is w[5] + k
        w[6] = cnt_bits;
        w[7] = 0;
        for (int r = 0; r < 6; r++)
            for (int k = 0; k < kW8; k += 2) w[8 + 4 * r + k / 2] = (uint32_t)qb[r][k] | ((uint32_t)qb[r][k + 1] << 16);
        for (int k = 0; k < nin; k++) emit(base_in + (uint32_t)k, C[(size_t)k], pushed, depth + 1);
    }
};

}  // namespace

void bvh8_child_box(const uint32_t* w, int slot, float lo[3], float hi[3]) {
    for (int ax = 0; ax < 3; ax++) {
        float o;
        std::memcpy(&o, &w[ax], 4);
        const int e = (int)((w[3] >> (8 * ax)) & 0xFFu) - 127;
        const uint16_t hl = (uint16_t)(w[8 + 8 * ax + slot / 2] >> (16 * (slot & 1)));
        const uint16_t hh = (uint16_t)(w[12 + 8 * ax + slot / 2] >> (16 * (slot & 1)));
        if (hl == 0x7C00) { lo[ax] = INFINITY; hi[ax] = -INFINITY; continue; }
        const double l = (double)o + std::ldexp((double)int_of_half(hl), e), h = (double)o + std::ldexp((double)int_of_half(hh), e);
        float fl = (float)l, fh = (float)h;
        if ((double)fl > l) fl = std::nextafter(fl, -INFINITY);
        if ((double)fh < h) fh = std::nextafter(fh, INFINITY);
        lo[ax] = fl;
        hi[ax] = fh;
    }
}

void collapse_bvh8q(const BvhResult& bvh2, int stack_budget, Bvh8Result& out, double c_step, double c_tri, int max_leaf) {
    out = Bvh8Result{};
    if (bvh2.nodes.empty()) return;
    const size_t nn = bvh2.nodes.size();
    Wide8 c{bvh2.nodes, out, c_step, c_tri, max_leaf, stack_budget, std::vector<int>(nn, 0), std::vector<double>(nn * kW8, 0.0),
            std::vector<int8_t>(nn * kW8, 0), std::vector<uint8_t>(nn, 0), std::vector<uint32_t>(nn, 0),
            std::vector<uint32_t>(nn, 0), std::vector<int>(nn, -1)};
    c.fill_height(0);
    c.solve(0);
    const uint32_t root = c.alloc(1);
    if (c.is_leaf(0)) {   // a lone leaf: the root node holds it in slot 0
        uint32_t* w = &out.words[0];
        for (int ax = 0; ax < 3; ax++) std::memcpy(&w[ax], &bvh2.nodes[0].bmin[ax], 4);
        uint32_t ebits = 0;
        for (int ax = 0; ax < 3; ax++) {
            const double ext = (double)bvh2.nodes[0].bmax[ax] - (double)bvh2.nodes[0].bmin[ax];
            int e = -126;
            while (e < 127 && std::ldexp((double)kQMax, e) < ext) e++;
            ebits |= (uint32_t)(e + 127) << (8 * ax);
            const double hi = std::ceil(ext / std::ldexp(1.0, e));
            for (int k = 0; k < kW8; k += 2) {
                const uint32_t lo0 = 0, hi0 = half_of_int((uint32_t)std::min((double)kQMax, hi));
                w[8 + 8 * ax + k / 2] = k == 0 ? (lo0 | (0x7C00u << 16)) : (0x7C00u | (0x7C00u << 16));
                w[12 + 8 * ax + k / 2] = k == 0 ? (hi0 | (0xFC00u << 16)) : (0xFC00u | (0xFC00u << 16));
            }
        }
        w[3] = ebits | (0u << 24) | (1u << 28);
        w[4] = 0;
        w[5] = 0x80000000u;   // the ref of chunk 0 - n_in (0)
        w[6] = (bvh2.nodes[0].b - 1u);
        out.chunk_first.push_back(bvh2.nodes[0].a);
        out.chunk_count.push_back((uint8_t)bvh2.nodes[0].b);
        out.children = 1;
        return;
    }
    c.emit(root, 0, 0, 0);
}

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
