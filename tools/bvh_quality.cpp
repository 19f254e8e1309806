// bvh_quality — host-side measure of triangle-BVH4 quality on the C4 frame's ray mix.
//
// The closest-hit and shadow kernels are bound by their traversal steps (a step = one 128-B line:
// an inner BVH4 node or a leaf chunk), so a tree is judged by the steps an actual ray mix takes
// through it.  This tool builds the BVH the library builds (pt_bvh.cpp: binned-SAH BVH2, leaves of
// <= 3 triangles, 4-wide collapse within the 32-entry stack) in its variants, then traces on the CPU:
//   depth 0  camera rays of a strided pixel grid (Camera.CastRay without the jitter),
//   depth 1+ cosine bounces from every hit (mesh triangles, or the floor y = 0), no origin offset,
//            as the reference's Ray.Bounce starts at the hit point,
//   shadow   from every hit to the two light spheres' centres (any-hit),
// and reports steps, node steps, leaf steps and triangle tests per ray, by depth, plus the tree's
// SAH cost.  Input: tools/dump_c4_mesh.py's file (triangles after FitInside, camera basis).
//   usage: bvh_quality MESH.bin [stride] [variant ...]   variant: greedy | sah
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "../ptsharp_amd/csrc/pt_bvh.h"
#include "../ptsharp_amd/csrc/pt_math.h"

using namespace pt;

struct Mesh {
    int n = 0;
    std::vector<float> v1, v2, v3;
    float cam_p[3], cam_u[3], cam_v[3], cam_w[3], cam_m;
};

static bool load(const char* path, Mesh& m) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    int32_t n = 0;
    bool ok = std::fread(&n, 4, 1, f) == 1;
    m.n = n;
    m.v1.resize((size_t)n * 3); m.v2.resize((size_t)n * 3); m.v3.resize((size_t)n * 3);
    ok = ok && std::fread(m.v1.data(), 4, (size_t)n * 3, f) == (size_t)n * 3;
    ok = ok && std::fread(m.v2.data(), 4, (size_t)n * 3, f) == (size_t)n * 3;
    ok = ok && std::fread(m.v3.data(), 4, (size_t)n * 3, f) == (size_t)n * 3;
    ok = ok && std::fread(m.cam_p, 4, 3, f) == 3 && std::fread(m.cam_u, 4, 3, f) == 3 && std::fread(m.cam_v, 4, 3, f) == 3 &&
         std::fread(m.cam_w, 4, 3, f) == 3 && std::fread(&m.cam_m, 4, 1, f) == 1;
    std::fclose(f);
    return ok;
}

struct Tree {
    std::vector<uint32_t> words;   // BVH4 nodes, pt_bvh.h layout
    std::vector<uint32_t> order;   // leaf position -> triangle
    int stack_need = 0;
    size_t nodes = 0, leaves = 0;
    double fill = 0;
};

struct Count {
    double rays = 0, nodes = 0, leaves = 0, tris = 0, inside = 0;   // inside: steps whose box holds the origin
    void add(const Count& o) { rays += o.rays; nodes += o.nodes; leaves += o.leaves; tris += o.tris; inside += o.inside; }
};

struct Tracer {
    const Mesh& m;
    const Tree& T;
    v3 tv1(uint32_t p) const { uint32_t s = T.order[p]; return v3{m.v1[3 * s], m.v1[3 * s + 1], m.v1[3 * s + 2]}; }
    v3 tv2(uint32_t p) const { uint32_t s = T.order[p]; return v3{m.v2[3 * s], m.v2[3 * s + 1], m.v2[3 * s + 2]}; }
    v3 tv3(uint32_t p) const { uint32_t s = T.order[p]; return v3{m.v3[3 * s], m.v3[3 * s + 1], m.v3[3 * s + 2]}; }

    // closest hit (any = false) or any hit before tlim (any = true); ordered BVH4 traversal, near child first
    std::vector<uint32_t>* lines = nullptr;   // (cache study) the 128-B lines a traversal touches, in order
    double trace(v3 o, v3 d, bool any, double tlim, Count& c, int32_t& prim) const {
        c.rays++;
        const v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        double best = any ? tlim : kHitInf;
        prim = -1;
        float tmax = (float)best;
        uint32_t stack[64];
        int sp = 0;
        uint32_t ref = 0;
        for (;;) {
            if (lines) lines->push_back(ref & 0x80000000u ? (uint32_t)T.nodes + (ref & 0x1FFFFFFFu) : ref);
            if (!(ref & 0x80000000u)) {
                c.nodes++;
                const float* w = reinterpret_cast<const float*>(&T.words[(size_t)ref * kNode4Words]);
                const uint32_t* refs = &T.words[(size_t)ref * kNode4Words + 24];
                float key[4];
                uint32_t ch[4];
                int nh = 0;
                for (int k = 0; k < 4; k++) {
                    if (refs[k] == kEmpty4) continue;
                    const float tx0 = (w[k] - o.x) * invd.x, tx1 = (w[4 + k] - o.x) * invd.x;
                    const float ty0 = (w[8 + k] - o.y) * invd.y, ty1 = (w[12 + k] - o.y) * invd.y;
                    const float tz0 = (w[16 + k] - o.z) * invd.z, tz1 = (w[20 + k] - o.z) * invd.z;
                    const float tn = std::fmax(std::fmax(std::fmin(tx0, tx1), std::fmin(ty0, ty1)), std::fmax(std::fmin(tz0, tz1), 0.f));
                    const float tf = std::fmin(std::fmin(std::fmax(tx0, tx1), std::fmax(ty0, ty1)), std::fmin(std::fmax(tz0, tz1), tmax));
                    if (tn <= tf) {
                        key[nh] = tn; ch[nh] = refs[k]; nh++;
                        if (o.x >= w[k] && o.x <= w[4 + k] && o.y >= w[8 + k] && o.y <= w[12 + k] && o.z >= w[16 + k] &&
                            o.z <= w[20 + k])
                            c.inside++;
                    }
                }
                for (int a = 1; a < nh; a++)   // sort by entry distance
                    for (int b = a; b > 0 && key[b] < key[b - 1]; b--) { std::swap(key[b], key[b - 1]); std::swap(ch[b], ch[b - 1]); }
                if (nh > 0) {
                    for (int k = nh - 1; k >= 1; k--) stack[sp++] = ch[k];
                    ref = ch[0];
                    continue;
                }
            } else {
                c.leaves++;
                const uint32_t first = ref & 0x1FFFFFFFu, cnt = ((ref >> 29) & 3u) + 1u;
                for (uint32_t k = 0; k < cnt; k++) {
                    c.tris++;
                    const v3 a = tv1(first + k);
                    const double t = isect_tri(a, sub(tv2(first + k), a), sub(tv3(first + k), a), o, d);
                    if (t < best) {
                        best = t;
                        prim = (int32_t)(first + k);
                        tmax = (float)t * 1.0000002f;
                        if (any) return best;
                    }
                }
            }
            if (sp == 0) break;
            ref = stack[--sp];
        }
        return best;
    }
};

// ---------------------------------------------------------------- wide-node model
// A W-wide tree collapsed from the same BVH2 by the SAH dynamic program (Ylitie et al. 2017 §4.1, W
// slots), child boxes optionally quantized to Q bits per bound relative to the node's own box (an fp32
// origin and a power-of-two step per axis, decoded as origin + q·step in fp32 and widened until they
// hold the exact box: the compressed wide BVH's format), leaves of <= 3 triangles as today's 128-B
// chunks.  A node line: W = 8 with Q = 8 is 80 B (origin 12, exponents 3, mask 1, child and triangle
// bases 8, per-child meta 8, bounds 48), W = 8 with Q = 16 is 128 B, W = 4 in fp32 is today's 128 B.
// Every node and every leaf chunk is one 128-B line, so steps = distinct lines a ray reads.
struct WChild {
    float lo[3], hi[3];
    uint32_t ref;   // inner node index, or 0x80000000 | (count-1) << 29 | first
};
struct WNode {
    std::vector<WChild> c;
};
struct WideTree {
    int W = 4, Q = 0;
    std::vector<WNode> nodes;
    size_t leaves = 0;
    double fill = 0;
    int depth = 0;
};
struct WideCollapser {
    const std::vector<BvhNode>& n2;
    int W;
    double c_step = 1.0, c_tri = 0.5;
    int max_leaf = 3;
    std::vector<double> cost;    // [node][W]
    std::vector<int8_t> choice;  // [node][W]
    std::vector<uint8_t> as_leaf;
    std::vector<uint32_t> prims, first;
    bool is_leaf(uint32_t i) const { return n2[i].b != 0; }
    double area(uint32_t i) const {
        const BvhNode& n = n2[i];
        double dx = (double)n.bmax[0] - n.bmin[0], dy = (double)n.bmax[1] - n.bmin[1], dz = (double)n.bmax[2] - n.bmin[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
        return dx * dy + dy * dz + dz * dx;
    }
    double dist(uint32_t n, int j, int& kbest) const {
        const double* CL = &cost[(size_t)n2[n].a * W];
        const double* CR = &cost[(size_t)(n2[n].a + 1) * W];
        double best = INFINITY;
        kbest = -1;
        for (int k = 1; k < j; k++) {
            const double c = CL[k - 1] + CR[j - k - 1];
            if (c < best) { best = c; kbest = k; }
        }
        return best;
    }
    void solve(uint32_t n) {
        {
            double* C = &cost[(size_t)n * W];
            int8_t* ch = &choice[(size_t)n * W];
            const double a = area(n);
            if (is_leaf(n)) {
                prims[n] = n2[n].b; first[n] = n2[n].a;
                for (int i = 0; i < W; i++) { C[i] = a * (c_step + c_tri * (double)prims[n]); ch[i] = 0; }
                as_leaf[n] = 1;
                return;
            }
            const uint32_t l = n2[n].a, r = l + 1;
            solve(l);
            solve(r);
            prims[n] = prims[l] + prims[r];
            first[n] = std::min(first[l], first[r]);
            int kw;
            const double inner = a * c_step + dist(n, W, kw);
            const double leaf = (int)prims[n] <= max_leaf ? a * (c_step + c_tri * (double)prims[n]) : INFINITY;
            as_leaf[n] = leaf <= inner;
            C[0] = std::min(leaf, inner);
            ch[0] = 0;
            for (int i = 2; i <= W; i++) {
                int k;
                const double d = dist(n, i, k);
                if (d < C[i - 2]) { C[i - 1] = d; ch[i - 1] = (int8_t)k; }
                else { C[i - 1] = C[i - 2]; ch[i - 1] = -1; }
            }
        }
    }
    void slots(uint32_t n, int i, std::vector<uint32_t>& outs) const {
        const int8_t c = choice[(size_t)n * W + (size_t)(i - 1)];
        if (c == 0) { outs.push_back(n); return; }
        if (c < 0) { slots(n, i - 1, outs); return; }
        slots(n2[n].a, c, outs);
        slots(n2[n].a + 1, i - c, outs);
    }
    void emit(WideTree& T, uint32_t at, uint32_t n, int depth) {
        T.depth = std::max(T.depth, depth);
        int k;
        (void)dist(n, W, k);
        std::vector<uint32_t> C;
        slots(n2[n].a, k, C);
        slots(n2[n].a + 1, W - k, C);
        std::vector<std::pair<uint32_t, uint32_t>> inner;
        for (uint32_t c : C) {
            WChild w;
            for (int ax = 0; ax < 3; ax++) { w.lo[ax] = n2[c].bmin[ax]; w.hi[ax] = n2[c].bmax[ax]; }
            if (as_leaf[c]) {
                w.ref = 0x80000000u | ((prims[c] - 1u) << 29) | (first[c] & 0x1FFFFFFFu);
                T.leaves++;
            } else {
                w.ref = (uint32_t)T.nodes.size();
                T.nodes.emplace_back();
                inner.emplace_back(c, w.ref);
            }
            T.nodes[at].c.push_back(w);
        }
        for (auto& pr : inner) emit(T, pr.second, pr.first, depth + 1);
    }
};
// Q-bit child bounds relative to the node's box: the decoded box holds the exact one.
static void quantize(WideTree& T) {
    if (T.Q <= 0) return;
    const float qmax = (float)((1 << T.Q) - 1);
    for (WNode& nd : T.nodes) {
        for (int ax = 0; ax < 3; ax++) {
            float o = INFINITY, e = -INFINITY;
            for (const WChild& c : nd.c) { o = std::fmin(o, c.lo[ax]); e = std::fmax(e, c.hi[ax]); }
            int ex = 0;
            const double ext = (double)e - (double)o;
            (void)std::frexp(ext / qmax, &ex);   // 2^ex > ext / qmax
            for (;;) {
                const float step = std::ldexp(1.0f, ex);
                bool ok = true;
                std::vector<WChild> qc = nd.c;
                for (WChild& c : qc) {
                    float ql = std::floor((float)(((double)c.lo[ax] - o) / step)), qh = std::ceil((float)(((double)c.hi[ax] - o) / step));
                    while (ql > 0 && o + ql * step > c.lo[ax]) ql -= 1.f;
                    while (o + qh * step < c.hi[ax]) qh += 1.f;
                    if (ql < 0 || qh > qmax) { ok = false; break; }
                    c.lo[ax] = o + ql * step;
                    c.hi[ax] = o + qh * step;
                    if (c.lo[ax] > nd.c[&c - &qc[0]].lo[ax]) { ok = false; break; }
                }
                if (ok) { nd.c = qc; break; }
                ex++;
            }
        }
    }
}
static void build_wide(const Mesh& m, int W, int Q, WideTree& T, std::vector<uint32_t>& order, double& build_s) {
    const size_t n = (size_t)m.n;
    std::vector<float> lo(n * 3), hi(n * 3);
    for (size_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            const float a = m.v1[3 * i + k], b = m.v2[3 * i + k], c = m.v3[3 * i + k];
            float l = std::fmin(std::fmin(a, b), c), h = std::fmax(std::fmax(a, b), c);
            const float e = std::fmax(std::fabs(l), std::fabs(h)) * 2.0e-6f + 1e-30f;
            lo[3 * i + k] = l - e; hi[3 * i + k] = h + e;
        }
    const auto t0 = std::chrono::steady_clock::now();
    BvhResult b2;
    build_bvh(lo.data(), hi.data(), (int64_t)n, 0, b2, 3, false, std::getenv("BINS") ? std::atoi(std::getenv("BINS")) : 32);
    WideCollapser wc{b2.nodes, W};
    const size_t nn = b2.nodes.size();
    wc.cost.assign(nn * W, 0.0);
    wc.choice.assign(nn * W, 0);
    wc.as_leaf.assign(nn, 0);
    wc.prims.assign(nn, 0);
    wc.first.assign(nn, 0);
    wc.solve(0);
    T.W = W;
    T.Q = Q;
    T.nodes.emplace_back();
    wc.emit(T, 0, 0, 0);
    quantize(T);
    build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    order = b2.order;
    size_t used = 0;
    for (const WNode& nd : T.nodes) used += nd.c.size();
    T.fill = (double)used / ((double)W * (double)T.nodes.size());
}
struct WideTracer {
    const Mesh& m;
    const WideTree& T;
    const std::vector<uint32_t>& order;
    v3 tv(const std::vector<float>& a, uint32_t p) const { uint32_t s = order[p]; return v3{a[3 * s], a[3 * s + 1], a[3 * s + 2]}; }
    double trace(v3 o, v3 d, bool any, double tlim, Count& c, int32_t& prim, double& tests, int& max_stack) const {
        c.rays++;
        const v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        double best = any ? tlim : kHitInf;
        prim = -1;
        float tmax = (float)best;
        std::vector<uint32_t> stack;
        uint32_t ref = 0;
        for (;;) {
            if (!(ref & 0x80000000u)) {
                c.nodes++;
                const WNode& nd = T.nodes[ref];
                float key[16];
                uint32_t ch[16];
                int nh = 0;
                for (const WChild& w : nd.c) {
                    tests++;
                    const float tx0 = (w.lo[0] - o.x) * invd.x, tx1 = (w.hi[0] - o.x) * invd.x;
                    const float ty0 = (w.lo[1] - o.y) * invd.y, ty1 = (w.hi[1] - o.y) * invd.y;
                    const float tz0 = (w.lo[2] - o.z) * invd.z, tz1 = (w.hi[2] - o.z) * invd.z;
                    const float tn = std::fmax(std::fmax(std::fmin(tx0, tx1), std::fmin(ty0, ty1)), std::fmax(std::fmin(tz0, tz1), 0.f));
                    const float tf = std::fmin(std::fmin(std::fmax(tx0, tx1), std::fmax(ty0, ty1)), std::fmin(std::fmax(tz0, tz1), tmax));
                    if (tn <= tf) {
                        key[nh] = tn; ch[nh] = w.ref; nh++;
                        if (o.x >= w.lo[0] && o.x <= w.hi[0] && o.y >= w.lo[1] && o.y <= w.hi[1] && o.z >= w.lo[2] && o.z <= w.hi[2])
                            c.inside++;
                    }
                }
                static const int order_mode = std::getenv("PUSH_ORDER") ? std::atoi(std::getenv("PUSH_ORDER")) : 0;
                if (order_mode == 0) {   // nearest first, the rest far-to-near (sorted)
                    for (int a = 1; a < nh; a++)
                        for (int b = a; b > 0 && key[b] < key[b - 1]; b--) { std::swap(key[b], key[b - 1]); std::swap(ch[b], ch[b - 1]); }
                } else if (nh > 1) {     // nearest first, the rest in slot order (popped lowest slot first)
                    int mi = 0;
                    for (int a = 1; a < nh; a++) if (key[a] < key[mi]) mi = a;
                    std::swap(key[0], key[mi]); std::swap(ch[0], ch[mi]);
                    // keep slots 1..nh-1 in their original relative order
                    uint32_t c2[16];
                    int m = 0;
                    for (int a = 1; a < nh; a++) c2[m++] = ch[a];
                    for (int a = 0; a < m; a++) ch[1 + a] = c2[a];
                }
                if (nh > 0) {
                    for (int k = nh - 1; k >= 1; k--) stack.push_back(ch[k]);
                    max_stack = std::max(max_stack, (int)stack.size());
                    ref = ch[0];
                    continue;
                }
            } else {
                c.leaves++;
                const uint32_t first = ref & 0x1FFFFFFFu, cnt = ((ref >> 29) & 3u) + 1u;
                for (uint32_t k = 0; k < cnt; k++) {
                    c.tris++;
                    const v3 a = tv(m.v1, first + k);
                    const double t = isect_tri(a, sub(tv(m.v2, first + k), a), sub(tv(m.v3, first + k), a), o, d);
                    if (t < best) {
                        best = t;
                        prim = (int32_t)(first + k);
                        tmax = (float)t * 1.0000002f;
                        if (any) return best;
                    }
                }
            }
            if (stack.empty()) break;
            ref = stack.back();
            stack.pop_back();
        }
        return best;
    }
};

static double tree_sah(const Tree& T, double c_tri) {
    // expected steps per ray through the root box: Σ P(node)·1 + Σ P(leaf)·(1 + n·c_tri), P = area ratio
    auto area = [](const float* lo, const float* hi) {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return (double)(dx * dy + dy * dz + dz * dx);
    };
    const float* w0 = reinterpret_cast<const float*>(T.words.data());
    float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 4; k++) {
        if (T.words[24 + k] == kEmpty4) continue;
        for (int ax = 0; ax < 3; ax++) { rlo[ax] = std::fmin(rlo[ax], w0[8 * ax + k]); rhi[ax] = std::fmax(rhi[ax], w0[8 * ax + 4 + k]); }
    }
    const double ar = area(rlo, rhi);
    double cost = 1.0;   // the root step
    for (size_t n = 0; n < T.nodes; n++) {
        const float* w = reinterpret_cast<const float*>(&T.words[n * kNode4Words]);
        const uint32_t* refs = &T.words[n * kNode4Words + 24];
        for (int k = 0; k < 4; k++) {
            if (refs[k] == kEmpty4) continue;
            float lo[3] = {w[k], w[8 + k], w[16 + k]}, hi[3] = {w[4 + k], w[12 + k], w[20 + k]};
            const double p = area(lo, hi) / ar;
            cost += (refs[k] & 0x80000000u) ? p * (1.0 + c_tri * (double)(((refs[k] >> 29) & 3u) + 1u)) : p;
        }
    }
    return cost;
}

static void build(const Mesh& m, const std::string& variant, Tree& T, double& build_s) {
    const size_t n = (size_t)m.n;
    std::vector<float> lo(n * 3), hi(n * 3);
    for (size_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            const float a = m.v1[3 * i + k], b = m.v2[3 * i + k], c = m.v3[3 * i + k];
            float l = std::fmin(std::fmin(a, b), c), h = std::fmax(std::fmax(a, b), c);
            const float e = std::fmax(std::fabs(l), std::fabs(h)) * 2.0e-6f + 1e-30f;   // pt_api.hip pad_box
            lo[3 * i + k] = l - e; hi[3 * i + k] = h + e;
        }
    const auto t0 = std::chrono::steady_clock::now();
    BvhResult b2;
    build_bvh(lo.data(), hi.data(), (int64_t)n, 0, b2, 3, false, std::getenv("BINS") ? std::atoi(std::getenv("BINS")) : 32);
    Bvh4Result b4;
    if (variant == "sah") collapse_bvh4_sah(b2, kStack4Budget, b4);
    else if (variant == "sah_nb") collapse_bvh4_sah(b2, 1000, b4);
    else if (variant == "greedy_nb") collapse_bvh4(b2, 1000, b4);
    else collapse_bvh4(b2, kStack4Budget, b4);
    build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    T.words = b4.words;
    T.order = b2.order;
    T.stack_need = b4.stack_need;
    T.nodes = b4.nodes();
    T.fill = (double)b4.children / (4.0 * (double)T.nodes);
    T.leaves = 0;
    for (size_t i = 0; i < T.nodes; i++)
        for (int k = 0; k < 4; k++) {
            const uint32_t r = T.words[i * kNode4Words + 24 + k];
            if (r != kEmpty4 && (r & 0x80000000u)) T.leaves++;
        }
}

// L2 study: rays leaving random points of the mesh (cosine bounces about the outward face normal,
// the deep rays of the C4 frame), their traversal lines fed through 8 LRU caches of 4 MB (32768
// 128-B lines, one per XCD), with the rays dealt to the caches round-robin (the kernels today) or by
// the region of the mesh their origin lies in (the origin triangle's position in BVH order, in 8
// contiguous ranges).  Reports the hit rate of each deal.
struct Lru {
    size_t cap;
    std::vector<uint32_t> key;                 // slot -> line
    std::vector<int> prev, next;
    std::unordered_map<uint32_t, int> where;
    int head = -1, tail = -1, used = 0;
    explicit Lru(size_t c) : cap(c), key(c), prev(c, -1), next(c, -1) { where.reserve(c * 2); }
    void unlink(int s) {
        if (prev[s] >= 0) next[prev[s]] = next[s]; else head = next[s];
        if (next[s] >= 0) prev[next[s]] = prev[s]; else tail = prev[s];
    }
    void front(int s) { prev[s] = -1; next[s] = head; if (head >= 0) prev[head] = s; head = s; if (tail < 0) tail = s; }
    bool access(uint32_t line) {
        auto it = where.find(line);
        if (it != where.end()) { unlink(it->second); front(it->second); return true; }
        int s;
        if ((size_t)used < cap) s = used++;
        else { s = tail; unlink(s); where.erase(key[s]); }
        key[s] = line; where[line] = s; front(s);
        return false;
    }
};
static void cache_study(const Mesh& m, const Tree& T, long nrays) {
    // Round 6: also the work of each origin region (lines per ray summed by region, 64 fine
    // ranges of BVH order), the imbalance of the 8-way deal by equal ray counts and by equal work (8 contiguous
    // runs of the fine ranges cut at equal cumulative lines), and the L2 hit rate of the work-balanced deal.
    Tracer tr{m, T};
    std::vector<uint32_t> pos_of(m.n);
    for (size_t p = 0; p < T.order.size(); p++) pos_of[T.order[p]] = (uint32_t)p;
    double cx = 0, cy = 0, cz = 0;
    for (int i = 0; i < m.n; i++) { cx += m.v1[3 * i]; cy += m.v1[3 * i + 1]; cz += m.v1[3 * i + 2]; }
    cx /= m.n; cy /= m.n; cz /= m.n;
    std::mt19937_64 rng(777);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    constexpr int kFine = 64;
    Count c;
    std::vector<uint32_t> lines;
    std::vector<std::vector<uint32_t>> ray_lines(nrays);
    std::vector<int> ray_fine(nrays);
    double fine_lines[kFine] = {0}, fine_rays[kFine] = {0};
    for (long r = 0; r < nrays; r++) {
        const int tri = (int)(U(rng) * m.n) % m.n;
        const v3 a{m.v1[3 * tri], m.v1[3 * tri + 1], m.v1[3 * tri + 2]}, b{m.v2[3 * tri], m.v2[3 * tri + 1], m.v2[3 * tri + 2]};
        const v3 cc{m.v3[3 * tri], m.v3[3 * tri + 1], m.v3[3 * tri + 2]};
        double u = U(rng), v = U(rng);
        if (u + v > 1) { u = 1 - u; v = 1 - v; }
        const v3 p = add(add(a, muls(sub(b, a), u)), muls(sub(cc, a), v));
        v3 nrm = normalize(cross(sub(b, a), sub(cc, a)));
        if ((p.x - cx) * nrm.x + (p.y - cy) * nrm.y + (p.z - cz) * nrm.z < 0) nrm = neg(nrm);
        const double r1 = U(rng) * 2 * kPi, r2 = U(rng), r2s = std::sqrt(r2);
        const v3 ax = std::fabs(nrm.x) > 0.1f ? v3{0.f, 1.f, 0.f} : v3{1.f, 0.f, 0.f};
        const v3 e1 = normalize(cross(ax, nrm)), e2 = cross(nrm, e1);
        const v3 d = normalize(add(add(muls(e1, std::cos(r1) * r2s), muls(e2, std::sin(r1) * r2s)), muls(nrm, std::sqrt(1 - r2))));
        lines.clear();
        tr.lines = &lines;
        int32_t prim;
        tr.trace(p, d, false, 0, c, prim);
        ray_lines[r] = lines;
        const int f = (int)((uint64_t)pos_of[tri] * kFine / (uint64_t)m.n);
        ray_fine[r] = f;
        fine_lines[f] += (double)lines.size();
        fine_rays[f] += 1.0;
    }
    // deals: 0 round-robin, 1 equal-count regions (8 ranges of BVH order), 2 equal-work regions
    int cut[9];
    {
        double total = 0, accw = 0;
        for (int f = 0; f < kFine; f++) total += fine_lines[f];
        int g = 1;
        cut[0] = 0;
        for (int f = 0; f < kFine && g < 8; f++) {
            accw += fine_lines[f];
            if (accw >= total * g / 8.0) cut[g++] = f + 1;
        }
        while (g < 8) { cut[g] = cut[g - 1]; g++; }
        cut[8] = kFine;
    }
    auto region_of = [&](int deal, long r) {
        if (deal == 0) return (int)(r % 8);
        if (deal == 1) return ray_fine[r] * 8 / kFine;
        int g = 0;
        while (g < 7 && ray_fine[r] >= cut[g + 1]) g++;
        return g;
    };
    const char* names[3] = {"round-robin", "equal-count regions", "equal-work regions"};
    std::printf("equal-work cuts (of %d fine ranges):", kFine);
    for (int g = 0; g <= 8; g++) std::printf(" %d", cut[g]);
    std::printf("\n");
    for (int deal = 0; deal < 3; deal++) {
        std::vector<Lru> l2;
        for (int k = 0; k < 8; k++) l2.emplace_back(32768);
        double work[8] = {0}, rays[8] = {0};
        long acc = 0, hit = 0;
        for (long r = 0; r < nrays; r++) {
            const int g = region_of(deal, r);
            work[g] += (double)ray_lines[r].size();
            rays[g] += 1;
            for (uint32_t l : ray_lines[r]) { acc++; hit += l2[g].access(l); }
        }
        double mx = 0, mean = 0;
        for (int g = 0; g < 8; g++) { mx = std::max(mx, work[g]); mean += work[g] / 8; }
        std::printf("cache study, %s: L2 (8 x 4 MB LRU) hit rate %.3f, lines per XCD max/mean %.3f, rays per XCD:", names[deal],
                    (double)hit / acc, mx / mean);
        for (int g = 0; g < 8; g++) std::printf(" %.0f", rays[g]);
        std::printf(", lines per XCD:");
        for (int g = 0; g < 8; g++) std::printf(" %.0f", work[g]);
        std::printf("\n");
    }
    // Concurrency (INFLIGHT rays per XCD stepping together, one line per ray per round, a finished ray replaced
    // by the XCD's next): the GPU keeps ~49k rays in flight per XCD (32 CUs x 24 waves x 64 lanes), so a line is
    // reused only while the rays near it are in flight.  Deals: round-robin; 8 equal-count regions; 64 fine
    // regions, XCD g taking regions g, g + 8, ... one after another (its in-flight rays share one fine region).
    if (const char* inf_env = std::getenv("INFLIGHT")) {
        const size_t K = (size_t)std::atol(inf_env);
        for (int deal = 0; deal < 3; deal++) {
            std::vector<std::vector<long>> order(8);
            if (deal == 2) {
                for (int g = 0; g < 8; g++)
                    for (int f = g; f < kFine; f += 8)
                        for (long r = 0; r < nrays; r++) if (ray_fine[r] == f) order[g].push_back(r);
            } else {
                for (long r = 0; r < nrays; r++) order[deal == 0 ? (int)(r % 8) : ray_fine[r] * 8 / kFine].push_back(r);
            }
            long acc = 0, hit = 0;
            double rounds_max = 0;
            for (int g = 0; g < 8; g++) {
                Lru l2(32768);
                std::vector<long> slot_ray(K, -1);
                std::vector<size_t> slot_pos(K, 0);
                size_t next = 0, active = 0;
                for (size_t k = 0; k < K && next < order[g].size(); k++) { slot_ray[k] = order[g][next++]; active++; }
                double rounds = 0;
                while (active) {
                    rounds++;
                    for (size_t k = 0; k < K; k++) {
                        if (slot_ray[k] < 0) continue;
                        const std::vector<uint32_t>& L = ray_lines[slot_ray[k]];
                        if (slot_pos[k] < L.size()) { acc++; hit += l2.access(L[slot_pos[k]++]); }
                        if (slot_pos[k] >= L.size()) {
                            slot_pos[k] = 0;
                            if (next < order[g].size()) slot_ray[k] = order[g][next++];
                            else { slot_ray[k] = -1; active--; }
                        }
                    }
                }
                rounds_max = std::max(rounds_max, rounds);
            }
            std::printf("cache study, %zu rays in flight per XCD, %s: L2 hit rate %.3f, rounds of the slowest XCD %.0f\n", K,
                        deal == 0 ? "round-robin" : deal == 1 ? "8 equal-count regions" : "64 regions, 8 per XCD in turn",
                        (double)hit / acc, rounds_max);
        }
    }
    std::printf("cache study: %ld surface rays, %.2f lines/ray; lines per ray by fine region (64 ranges of BVH order):", nrays,
                (double)c.nodes / std::max(c.rays, 1.0) + (double)c.leaves / std::max(c.rays, 1.0));
    for (int f = 0; f < kFine; f++) std::printf(" %.1f", fine_rays[f] ? fine_lines[f] / fine_rays[f] : 0.0);
    std::printf("\n");
}

// The library's 8-wide quantized tree (pt_bvh.cpp collapse_bvh8q) as a WideTree, decoded boxes.
static void build_p8(const Mesh& m, WideTree& T, std::vector<uint32_t>& order, double& build_s, int& stack_need) {
    const size_t n = (size_t)m.n;
    std::vector<float> lo(n * 3), hi(n * 3);
    for (size_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            const float a = m.v1[3 * i + k], b = m.v2[3 * i + k], c = m.v3[3 * i + k];
            float l = std::fmin(std::fmin(a, b), c), h = std::fmax(std::fmax(a, b), c);
            const float e = std::fmax(std::fabs(l), std::fabs(h)) * 2.0e-6f + 1e-30f;
            lo[3 * i + k] = l - e; hi[3 * i + k] = h + e;
        }
    const auto t0 = std::chrono::steady_clock::now();
    BvhResult b2;
    build_bvh(lo.data(), hi.data(), (int64_t)n, 0, b2, 3, false, std::getenv("BINS") ? std::atoi(std::getenv("BINS")) : 32);
    Bvh8Result b8;
    collapse_bvh8q(b2, std::getenv("BUDGET8") ? std::atoi(std::getenv("BUDGET8")) : 64, b8, 1.0,
                   std::getenv("C_TRI") ? std::atof(std::getenv("C_TRI")) : 0.5);
    build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    stack_need = b8.stack_need;
    T.W = 8;
    T.Q = 11;
    T.nodes.assign(b8.nodes(), WNode{});
    size_t bad = 0, prims = 0;
    for (size_t i = 0; i < b8.nodes(); i++) {
        const uint32_t* w = &b8.words[i * kNode8Words];
        const int nc = (int)(w[3] >> 28), nin = (int)((w[3] >> 24) & 15u);
        for (int k = 0; k < nc; k++) {
            WChild c;
            bvh8_child_box(w, k, c.lo, c.hi);
            if (k < nin) c.ref = w[4] + (uint32_t)k;
            else {
                const uint32_t ch = (w[5] + (uint32_t)k) & 0x7FFFFFFFu;
                c.ref = 0x80000000u | ((uint32_t)(b8.chunk_count[ch] - 1) << 29) | b8.chunk_first[ch];
                prims += b8.chunk_count[ch];
                T.leaves++;
            }
            T.nodes[i].c.push_back(c);
        }
    }
    // containment: every leaf chunk's triangles inside the decoded boxes on its path is what the traversal
    // needs; checked here on the leaves' own boxes
    for (size_t i = 0; i < b8.nodes(); i++)
        for (const WChild& c : T.nodes[i].c)
            if (c.ref & 0x80000000u) {
                const uint32_t f = c.ref & 0x1FFFFFFFu, cnt = ((c.ref >> 29) & 3u) + 1u;
                for (uint32_t t = f; t < f + cnt; t++)
                    for (int k = 0; k < 3; k++)
                        if (lo[3 * b2.order[t] + k] < c.lo[k] || hi[3 * b2.order[t] + k] > c.hi[k]) bad++;
            }
    order = b2.order;
    size_t used = 0;
    for (const WNode& nd : T.nodes) used += nd.c.size();
    T.fill = (double)used / (8.0 * (double)T.nodes.size());
    std::printf("p8: %zu nodes, %zu chunks, %zu primitives in chunks (of %zu), %zu bounds outside their box, stack %d\n",
                b8.nodes(), b8.chunk_first.size(), prims, n, bad, stack_need);
}

// The C4 ray mix (main's loop) through a wide tree: steps (lines) per ray by depth and for shadow rays.
static void run_wide(const Mesh& m, int W, int Q, int stride) {
    WideTree T;
    std::vector<uint32_t> order;
    double bs = 0;
    int sneed = 0;
    if (W == 0) build_p8(m, T, order, bs, sneed);
    else build_wide(m, W, Q, T, order, bs);
    WideTracer tr{m, T, order};
    const int Wd = 1920, H = 1080, kDepth = 4;
    const v3 lights[2] = {v3{0.f, 5.f, 0.f}, v3{4.f, 5.f, 4.f}};
    Count cd[kDepth + 1], csh;
    double tests_c = 0, tests_s = 0;
    int max_stack = 0;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const v3 cp{m.cam_p[0], m.cam_p[1], m.cam_p[2]}, cu{m.cam_u[0], m.cam_u[1], m.cam_u[2]};
    const v3 cv{m.cam_v[0], m.cam_v[1], m.cam_v[2]}, cw{m.cam_w[0], m.cam_w[1], m.cam_w[2]};
    for (int y = stride / 2; y < H; y += stride)
        for (int x = stride / 2; x < Wd; x += stride) {
            const double aspect = Wd / (double)H;
            const double px = ((x + 0.5 - 0.5) / (Wd - 1.0)) * 2 - 1, py = ((y + 0.5 - 0.5) / (H - 1.0)) * 2 - 1;
            v3 d = normalize(add(add(muls(cu, -px * aspect), muls(cv, -py)), muls(cw, m.cam_m)));
            v3 o = cp;
            for (int depth = 0; depth <= kDepth; depth++) {
                int32_t prim;
                double t = tr.trace(o, d, false, 0, cd[depth], prim, tests_c, max_stack);
                v3 nrm;
                if (d.y < 0) {
                    const double tf = -(double)o.y / (double)d.y;
                    if (tf > kEps && tf < t) { t = tf; prim = -2; }
                }
                if (prim == -1) break;
                const v3 p = add(o, muls(d, t));
                if (prim == -2) nrm = v3{0.f, 1.f, 0.f};
                else {
                    const v3 a = tr.tv(m.v1, (uint32_t)prim);
                    nrm = normalize(cross(sub(tr.tv(m.v2, (uint32_t)prim), a), sub(tr.tv(m.v3, (uint32_t)prim), a)));
                    if (dotf(nrm, d) > 0) nrm = neg(nrm);
                }
                for (const v3& L : lights) {
                    const v3 ld = normalize(sub(L, p));
                    const double tl = (double)lengthf(sub(L, p)) - 1.0;
                    int32_t sprim;
                    tr.trace(p, ld, true, tl, csh, sprim, tests_s, max_stack);
                }
                const double r1 = U(rng) * 2 * kPi, r2 = U(rng), r2s = std::sqrt(r2);
                const v3 ax = std::fabs(nrm.x) > 0.1f ? v3{0.f, 1.f, 0.f} : v3{1.f, 0.f, 0.f};
                const v3 u = normalize(cross(ax, nrm)), vv = cross(nrm, u);
                d = normalize(add(add(muls(u, std::cos(r1) * r2s), muls(vv, std::sin(r1) * r2s)), muls(nrm, std::sqrt(1 - r2))));
                o = p;
            }
        }
    Count all;
    for (auto& c : cd) all.add(c);
    std::printf("wide W=%d Q=%d nodes %zu leaves %zu fill %.3f depth %d max stack %d build %.2fs\n", W, Q, T.nodes.size(),
                T.leaves, T.fill, T.depth, max_stack, bs);
    auto row = [](const char* name, const Count& c, double tests) {
        if (c.rays == 0) return;
        std::printf("  %-9s rays %9.0f  steps/ray %6.3f  nodes/ray %6.3f  leaves/ray %6.3f  tris/ray %6.3f  origin-box %6.3f  box tests/ray %6.2f\n",
                    name, c.rays, (c.nodes + c.leaves) / c.rays, c.nodes / c.rays, c.leaves / c.rays, c.tris / c.rays,
                    c.inside / c.rays, tests / c.rays);
    };
    row("closest", all, tests_c);
    for (int k = 0; k <= kDepth; k++) {
        char nm[16];
        std::snprintf(nm, sizeof nm, "depth %d", k);
        row(nm, cd[k], NAN);
    }
    row("shadow", csh, tests_s);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: %s MESH.bin [stride] [variant ...]\n", argv[0]); return 2; }
    Mesh m;
    if (!load(argv[1], m)) { std::fprintf(stderr, "cannot read %s\n", argv[1]); return 2; }
    const int stride = argc > 2 ? std::atoi(argv[2]) : 16;
    std::vector<std::string> variants;
    for (int i = 3; i < argc; i++) variants.push_back(argv[i]);
    if (variants.empty()) variants = {"greedy", "sah"};
    const int W = 1920, H = 1080, kDepth = 4;
    const v3 lights[2] = {v3{0.f, 5.f, 0.f}, v3{4.f, 5.f, 4.f}};
    for (const auto& var : variants) {
        int wide = 0, qbits = 0;   // (not W: the image width below)
        if (var == "p8" || std::sscanf(var.c_str(), "w%dq%d", &wide, &qbits) == 2) {   // wide-node model: w8q8, w8q16, w4q0 ...; p8: the library's
            if (var == "p8") wide = 0;
            run_wide(m, wide, qbits, stride);
            continue;
        }
        Tree T;
        double bs = 0;
        build(m, var, T, bs);
        if (const char* cs = std::getenv("CACHE_RAYS")) { cache_study(m, T, std::atol(cs)); continue; }
        Tracer tr{m, T};
        Count cd[kDepth + 1], csh;
        std::vector<uint32_t> pos_of(m.n);
        for (size_t q = 0; q < T.order.size(); q++) pos_of[T.order[q]] = (uint32_t)q;
        long region[kDepth + 1][8] = {{0}};   // mesh hits per origin region (8 ranges of BVH order), by depth
        std::mt19937_64 rng(12345);
        std::uniform_real_distribution<double> U(0.0, 1.0);
        const v3 cp{m.cam_p[0], m.cam_p[1], m.cam_p[2]}, cu{m.cam_u[0], m.cam_u[1], m.cam_u[2]};
        const v3 cv{m.cam_v[0], m.cam_v[1], m.cam_v[2]}, cw{m.cam_w[0], m.cam_w[1], m.cam_w[2]};
        const auto t0 = std::chrono::steady_clock::now();
        for (int y = stride / 2; y < H; y += stride)
            for (int x = stride / 2; x < W; x += stride) {
                const double aspect = W / (double)H;
                const double px = ((x + 0.5 - 0.5) / (W - 1.0)) * 2 - 1, py = ((y + 0.5 - 0.5) / (H - 1.0)) * 2 - 1;
                v3 d = normalize(add(add(muls(cu, -px * aspect), muls(cv, -py)), muls(cw, m.cam_m)));
                v3 o = cp;
                for (int depth = 0; depth <= kDepth; depth++) {
                    int32_t prim;
                    double t = tr.trace(o, d, false, 0, cd[depth], prim);
                    v3 nrm;
                    if (d.y < 0) {   // the floor (the cube's top face, y = 0), tested beside the BVH as the kernels do
                        const double tf = -(double)o.y / (double)d.y;
                        if (tf > kEps && tf < t) { t = tf; prim = -2; }
                    }
                    if (prim == -1) break;
                    const v3 p = add(o, muls(d, t));
                    if (prim == -2) nrm = v3{0.f, 1.f, 0.f};
                    else {
                        region[depth][(uint64_t)prim * 8 / (uint64_t)m.n]++;
                        const v3 a = tr.tv1((uint32_t)prim);
                        nrm = normalize(cross(sub(tr.tv2((uint32_t)prim), a), sub(tr.tv3((uint32_t)prim), a)));
                        if (dotf(nrm, d) > 0) nrm = neg(nrm);
                    }
                    for (const v3& L : lights) {   // shadow rays (hard, to the centre), any-hit before the light
                        const v3 ld = normalize(sub(L, p));
                        const double tl = (double)lengthf(sub(L, p)) - 1.0;
                        int32_t sprim;
                        tr.trace(p, ld, true, tl, csh, sprim);
                    }
                    // cosine bounce
                    const double r1 = U(rng) * 2 * kPi, r2 = U(rng), r2s = std::sqrt(r2);
                    const v3 ax = std::fabs(nrm.x) > 0.1f ? v3{0.f, 1.f, 0.f} : v3{1.f, 0.f, 0.f};
                    const v3 u = normalize(cross(ax, nrm)), vv = cross(nrm, u);
                    d = normalize(add(add(muls(u, std::cos(r1) * r2s), muls(vv, std::sin(r1) * r2s)), muls(nrm, std::sqrt(1 - r2))));
                    o = p;
                }
            }
        const double ts = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        Count all;
        for (auto& c : cd) all.add(c);
        std::printf("variant %-8s nodes %zu leaves %zu fill %.3f stack %d build %.2fs sah(ctri=0.5) %.3f trace %.1fs\n", var.c_str(),
                    T.nodes, T.leaves, T.fill, T.stack_need, bs, tree_sah(T, 0.5), ts);
        auto row = [](const char* name, const Count& c) {
            if (c.rays == 0) return;
            std::printf("  %-9s rays %9.0f  steps/ray %6.3f  nodes/ray %6.3f  leaves/ray %6.3f  tris/ray %6.3f  origin-box steps/ray %6.3f\n",
                        name, c.rays, (c.nodes + c.leaves) / c.rays, c.nodes / c.rays, c.leaves / c.rays, c.tris / c.rays,
                        c.inside / c.rays);
        };
        row("closest", all);
        for (int k = 0; k <= kDepth; k++) {
            char nm[16];
            std::snprintf(nm, sizeof nm, "depth %d", k);
            row(nm, cd[k]);
        }
        row("shadow", csh);
        for (int k = 0; k <= kDepth; k++) {
            long t = 0;
            for (int g = 0; g < 8; g++) t += region[k][g];
            std::printf("  mesh hits of depth %d by region:", k);
            for (int g = 0; g < 8; g++) std::printf(" %.3f", t ? (double)region[k][g] / t : 0.0);
            std::printf("\n");
        }
        std::fflush(stdout);
    }
    return 0;
}
