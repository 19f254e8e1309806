// bvh8_check — the 8-wide quantized triangle BVH (ptsharp_amd/csrc/pt_bvh.cpp collapse_bvh8q) on the host:
//   * structure: every primitive in exactly one leaf chunk of 1..3, node children 1..8 with the inner ones
//     first, child indices in range, every node reached once from the root, the stack bound (the pushes
//     Σ (children - 1) on every root-to-leaf path) within kStackMax and equal to the reported need;
//   * boxes: every slot box on a primitive's path (bvh8_child_box, exact decode) holds the primitive's padded
//     box (pt_api.hip pad_box); empty slots are +inf / -inf;
//   * the device's slab arithmetic (pt_device.h node8_step: fma(q, step/d, (origin - o)/d) in fp32, near /
//     far by direction sign, the far distance widened by 2^-21 relative) restated here: a ray whose exact
//     fp64 slab test enters a primitive's box before tmax also enters every quantized box on that
//     primitive's path — the quantized tree never culls a box the exact one keeps.
// usage: bvh8_check [rays_per_case]      exit 0 = every check held
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../ptsharp_amd/csrc/pt_bvh.h"

static long failures = 0;
#define CHECK(c)                                                                       \
    do {                                                                               \
        if (!(c)) {                                                                    \
            if (failures < 20) std::fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
            failures++;                                                                \
        }                                                                              \
    } while (0)

static float half_to_float(uint16_t h) {   // binary16 -> fp32 (the integers and +-inf the builder stores)
    if ((h & 0x7FFFu) == 0x7C00u) return (h & 0x8000u) ? -INFINITY : INFINITY;
    if (h == 0) return 0.f;
    const int e = (int)((h >> 10) & 31) - 15;
    return std::ldexp(1.f + (float)(h & 0x3FFu) / 1024.f, e);
}
static float q_of(const uint32_t* w, int word0, int slot) {
    return half_to_float((uint16_t)(w[word0 + slot / 2] >> (16 * (slot & 1))));
}

struct Box { float lo[3], hi[3]; };

// node8_step's slab test of slot k (fp32, fma), on the host
static bool slab8(const uint32_t* w, int k, const float o[3], const float invd[3], float tmax) {
    float tn = 0.f, tf = tmax;
    float tns[3], tfs[3];
    for (int ax = 0; ax < 3; ax++) {
        float org;
        std::memcpy(&org, &w[ax], 4);
        const uint32_t eb = (w[3] >> (8 * ax)) & 0xFFu;
        uint32_t sb = eb << 23;
        float s;
        std::memcpy(&s, &sb, 4);
        const float a = (org - o[ax]) * invd[ax], b = s * invd[ax];
        const bool flip = invd[ax] < 0.f;
        const float qn = q_of(w, flip ? 12 + 8 * ax : 8 + 8 * ax, k), qf = q_of(w, flip ? 8 + 8 * ax : 12 + 8 * ax, k);
        tns[ax] = std::fmaf(qn, b, a);
        tfs[ax] = std::fmaf(qf, b, a);
    }
    tn = std::fmax(std::fmax(tns[0], tns[1]), std::fmax(tns[2], 0.f));
    tf = std::fmin(std::fmin(tfs[0], tfs[1]), std::fmin(tfs[2], tmax));
    return tn <= tf * 1.0000005f;   // (node8_step tests every slot: an empty one must miss by its bounds)
}
// exact slab test of a box (fp64), entry before tmax
static bool slab_exact(const Box& b, const float o[3], const float d[3], double tmax) {
    double tn = 0.0, tf = tmax;
    for (int ax = 0; ax < 3; ax++) {
        if (d[ax] == 0.f) {
            if (o[ax] < b.lo[ax] || o[ax] > b.hi[ax]) return false;
            continue;
        }
        double t0 = ((double)b.lo[ax] - o[ax]) / d[ax], t1 = ((double)b.hi[ax] - o[ax]) / d[ax];
        if (t0 > t1) std::swap(t0, t1);
        tn = std::max(tn, t0);
        tf = std::min(tf, t1);
    }
    return tn <= tf;
}

static void run_case(const char* name, std::vector<float>& lo, std::vector<float>& hi, int rays, unsigned seed) {
    const int64_t n = (int64_t)lo.size() / 3;
    // the tree is built on the boxes padded as pt_api.hip pad_box pads them (the fp32 slab tests' margin);
    // the rays below test the exact, unpadded boxes
    std::vector<float> plo = lo, phi = hi;
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            const float m = std::max(std::fabs(lo[3 * i + k]), std::fabs(hi[3 * i + k]));
            const float e = m * 2.0e-6f + 1e-30f;
            plo[3 * i + k] -= e;
            phi[3 * i + k] += e;
        }
    pt::BvhResult b2;
    pt::build_bvh(plo.data(), phi.data(), n, 8, b2, 3, false, 128);
    pt::Bvh8Result b8;
    pt::collapse_bvh8q(b2, pt::kStackMax, b8);
    const size_t nn = b8.nodes();
    CHECK(nn > 0);
    CHECK(b8.stack_need <= pt::kStackMax);
    // structure
    std::vector<int> seen((size_t)n, 0), reached(nn, 0), chunk_seen(b8.chunk_first.size(), 0);
    std::vector<std::pair<uint32_t, int>> todo{{0u, 0}};
    int need = 0;
    std::vector<Box> prim((size_t)n);
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) { prim[(size_t)i].lo[k] = lo[3 * i + k]; prim[(size_t)i].hi[k] = hi[3 * i + k]; }
    // per chunk / node: the path of (node, slot) above it, for the ray check
    std::vector<std::vector<std::pair<uint32_t, int>>> chunk_path(b8.chunk_first.size());
    std::vector<std::vector<std::pair<uint32_t, int>>> node_path(nn);
    while (!todo.empty()) {
        const auto [nd, pushed] = todo.back();
        todo.pop_back();
        CHECK(nd < nn);
        if (nd >= nn) continue;
        reached[nd]++;
        const uint32_t* w = &b8.words[(size_t)nd * pt::kNode8Words];
        const int nc = (int)(w[3] >> 28), nin = (int)((w[3] >> 24) & 15u);
        CHECK(nc >= 1 && nc <= 8 && nin <= nc);
        const int p = pushed + nc - 1;
        need = std::max(need, p);
        for (int k = nc; k < 8; k++)
            for (int ax = 0; ax < 3; ax++) {
                CHECK(std::isinf(q_of(w, 8 + 8 * ax, k)) && q_of(w, 8 + 8 * ax, k) > 0);
                CHECK(std::isinf(q_of(w, 12 + 8 * ax, k)) && q_of(w, 12 + 8 * ax, k) < 0);
            }
        for (int k = 0; k < nc; k++) {
            Box sb;
            pt::bvh8_child_box(w, k, sb.lo, sb.hi);
            if (k < nin) {
                const uint32_t c = w[4] + (uint32_t)k;
                CHECK(c < nn);
                if (c >= nn) continue;
                node_path[c] = node_path[nd];
                node_path[c].push_back({nd, k});
                todo.push_back({c, p});
            } else {
                CHECK(((w[5] + (uint32_t)k) & 0x80000000u) != 0);   // a leaf ref
                const uint32_t ch = (w[5] + (uint32_t)k) & 0x7FFFFFFFu;
                CHECK(ch < b8.chunk_first.size());
                if (ch >= b8.chunk_first.size()) continue;
                chunk_seen[ch]++;
                const uint32_t cnt = ((w[6] >> (2 * k)) & 3u) + 1u;
                CHECK(cnt == b8.chunk_count[ch] && cnt >= 1 && cnt <= 3);
                chunk_path[ch] = node_path[nd];
                chunk_path[ch].push_back({nd, k});
                for (uint32_t t = b8.chunk_first[ch]; t < b8.chunk_first[ch] + cnt; t++) {
                    CHECK(t < (uint32_t)n);
                    if (t >= (uint32_t)n) continue;
                    const uint32_t pi = b2.order[t];
                    seen[pi]++;
                    for (int ax = 0; ax < 3; ax++) CHECK(plo[3 * (size_t)pi + ax] >= sb.lo[ax] && phi[3 * (size_t)pi + ax] <= sb.hi[ax]);
                }
            }
        }
    }
    long outside = 0;   // every primitive's (padded) box inside every slot box on its path
    for (size_t c = 0; c < chunk_path.size(); c++)
        for (const auto& [nd, k] : chunk_path[c]) {
            Box sb;
            pt::bvh8_child_box(&b8.words[(size_t)nd * pt::kNode8Words], k, sb.lo, sb.hi);
            for (uint32_t t = b8.chunk_first[c]; t < b8.chunk_first[c] + b8.chunk_count[c]; t++)
                for (int ax = 0; ax < 3; ax++)
                    if (plo[3 * (size_t)b2.order[t] + ax] < sb.lo[ax] || phi[3 * (size_t)b2.order[t] + ax] > sb.hi[ax]) outside++;
        }
    CHECK(outside == 0);
    for (int64_t i = 0; i < n; i++) CHECK(seen[(size_t)i] == 1);
    for (size_t i = 0; i < nn; i++) CHECK(reached[i] == 1);
    for (size_t i = 0; i < chunk_seen.size(); i++) CHECK(chunk_seen[i] == 1);
    CHECK(need == b8.stack_need);
    // rays: every primitive box the exact test enters lies under quantized boxes the fp32 test enters
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    float glo[3] = {INFINITY, INFINITY, INFINITY}, ghi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) { glo[k] = std::min(glo[k], lo[3 * i + k]); ghi[k] = std::max(ghi[k], hi[3 * i + k]); }
    std::vector<uint32_t> chunk_of((size_t)n);
    for (size_t c = 0; c < b8.chunk_first.size(); c++)
        for (uint32_t t = b8.chunk_first[c]; t < b8.chunk_first[c] + b8.chunk_count[c]; t++) chunk_of[b2.order[t]] = (uint32_t)c;
    long tested = 0, entered = 0, culled = 0, empty_hits = 0;
    for (int r = 0; r < rays; r++) {
        float o[3], d[3], invd[3];
        const uint32_t target = (uint32_t)(U(rng) * (float)n) % (uint32_t)n;
        for (int k = 0; k < 3; k++) {
            const float ext = ghi[k] - glo[k];
            o[k] = (r % 3 == 0) ? glo[k] - ext + 3.f * ext * U(rng)                       // anywhere around
                              : prim[target].lo[k] + (prim[target].hi[k] - prim[target].lo[k]) * U(rng);   // on a box
            d[k] = U(rng) * 2.f - 1.f;
        }
        if (r % 7 == 0) d[r % 3] = 0.f;   // a zero direction component
        const float len = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        if (len == 0.f) continue;
        for (int k = 0; k < 3; k++) { d[k] /= len; invd[k] = 1.f / d[k]; }
        const float tmax = (r % 2) ? INFINITY : (float)(0.1 + 3.0 * U(rng));
        // a sample of primitives: the target and 64 random ones
        for (int j = 0; j < 65; j++) {
            const uint32_t p = j == 0 ? target : (uint32_t)(U(rng) * (float)n) % (uint32_t)n;
            tested++;
            if (!slab_exact(prim[p], o, d, (double)tmax)) continue;
            entered++;
            for (const auto& [nd, k] : chunk_path[chunk_of[p]]) {
                const uint32_t* w = &b8.words[(size_t)nd * pt::kNode8Words];
                if (!slab8(w, k, o, invd, tmax)) { culled++; break; }
                for (int e = (int)(w[3] >> 28); e < 8; e++) if (slab8(w, e, o, invd, tmax)) empty_hits++;
            }
        }
    }
    CHECK(culled == 0);
    CHECK(empty_hits == 0);
    std::printf("%s: %lld primitives, %zu nodes, %zu chunks, stack %d; rays: %ld primitive boxes tested, %ld entered, %ld "
                "culled by the quantized tree, %ld empty slots hit\n", name, (long long)n, nn, b8.chunk_first.size(), b8.stack_need, tested, entered,
                culled, empty_hits);
}

int main(int argc, char** argv) {
    const int rays = argc > 1 ? std::atoi(argv[1]) : 2000;
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(-10.f, 10.f), S(0.001f, 0.3f);
    for (int64_t n : {1, 2, 3, 4, 9, 100, 5000, 200000}) {   // random boxes, a cluster of coincident ones
        std::vector<float> lo((size_t)n * 3), hi((size_t)n * 3);
        for (int64_t i = 0; i < n; i++)
            for (int k = 0; k < 3; k++) {
                const float c = (i % 97 == 0) ? 1.f : U(rng);
                lo[(size_t)i * 3 + k] = c - S(rng);
                hi[(size_t)i * 3 + k] = c + S(rng);
            }
        char nm[64];
        std::snprintf(nm, sizeof nm, "random %lld", (long long)n);
        run_case(nm, lo, hi, rays, 11u + (unsigned)n);
    }
    {   // a triangulated sphere far from the origin, large coordinates, flat boxes on axis-aligned faces
        std::vector<float> lo, hi;
        const int G = 180;
        for (int a = 0; a < G; a++)
            for (int b = 0; b < G; b++) {
                const double th = M_PI * (a + 0.5) / G, ph = 2 * M_PI * (b + 0.5) / G;
                const float x = (float)(1000.0 + std::sin(th) * std::cos(ph)), y = (float)(-500.0 + std::sin(th) * std::sin(ph));
                const float z = (b % 9 == 0) ? 3.f : (float)std::cos(th);   // some flat in z
                const float e = 0.02f;
                lo.insert(lo.end(), {x - e, y - e, z - (b % 9 == 0 ? 0.f : e)});
                hi.insert(hi.end(), {x + e, y + e, z + (b % 9 == 0 ? 0.f : e)});
            }
        run_case("far sphere", lo, hi, rays, 99u);
    }
    std::printf("bvh8_check: %ld failures\n", failures);
    return failures == 0 ? 0 : 1;
}
