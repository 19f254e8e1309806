// sanitize_host.cpp — the host C++ of this repo under AddressSanitizer + UndefinedBehaviorSanitizer
// or ThreadSanitizer (tests/native/Makefile: `make asan`, `make tsan`; SURVEY.md §5 "race detection").
//
// Sanitizer runtimes must be the first thing a process loads, so a Python test run cannot carry
// them without preloading the runtime into the interpreter; this driver is a plain executable that
// links the sanitised objects directly and exercises the same paths the CPU suite does:
//   * pt_bvh.cpp  — the threaded binned-SAH build (8 threads) and the BVH4 collapse, with the
//                   structural invariants checked (every primitive once, boxes nested);
//   * pt_obj.cpp  — pt_obj_load on well-formed files (v, v/vt, v/vt/vn, v//vn, CRLF, tabs, a
//                   line longer than the read block), on malformed ones (every error path), and
//                   pt_mesh_smooth_normals on the result;
//   * the oracle  — or_scene_create (k-d trees, Tree.cs) and threaded or_render_pass (8 threads,
//                   the RenderParallel restatement), main + adaptive + firefly passes, plus the
//                   serial Render twin; the reference's own latent races (Buffer.cs:33-44 AddSample,
//                   Box.cs:96-114 Partition) are the kind of bug TSan would report here.
// Exit status 0 and no sanitizer report = clean.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/ptsharp_hip.h"
#include "../../oracle/oracle.h"
#include "../../ptsharp_amd/csrc/pt_bvh.h"

static int failures = 0;
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
            failures++;                                                           \
        }                                                                         \
    } while (0)

static void bvh_case(int64_t n, int threads, unsigned seed) {
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> U(-10.f, 10.f), S(0.001f, 0.3f);
    std::vector<float> lo((size_t)n * 3), hi((size_t)n * 3);
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            const float c = (i % 97 == 0) ? 1.f : U(rng);   // a cluster of coincident boxes too
            lo[(size_t)i * 3 + k] = c - S(rng);
            hi[(size_t)i * 3 + k] = c + S(rng);
        }
    pt::BvhResult b2;
    pt::build_bvh(lo.data(), hi.data(), n, threads, b2);
    std::vector<int> seen((size_t)n, 0);
    for (uint32_t p : b2.order) { CHECK(p < (uint32_t)n); if (p < (uint32_t)n) seen[p]++; }
    for (int64_t i = 0; i < n; i++) CHECK(seen[(size_t)i] == 1);
    CHECK(b2.max_depth <= pt::kMaxDepth);
    // inner nodes contain their children
    for (size_t i = 0; i < b2.nodes.size(); i++) {
        const pt::BvhNode& nd = b2.nodes[i];
        if (i == 1 || nd.b != 0) continue;   // padding slot, leaves
        for (uint32_t c = nd.a; c < nd.a + 2 && c < b2.nodes.size(); c++)
            for (int k = 0; k < 3; k++) {
                CHECK(b2.nodes[c].bmin[k] >= nd.bmin[k]);
                CHECK(b2.nodes[c].bmax[k] <= nd.bmax[k]);
            }
    }
    pt::Bvh4Result b4;
    pt::collapse_bvh4(b2, pt::kStack4Budget, b4);
    CHECK(b4.stack_need <= pt::kStack4Budget);
    CHECK(b4.nodes() > 0);
    std::printf("bvh: %lld prims, %d threads: %zu BVH2 nodes (depth %d), %zu BVH4 nodes (stack %d)\n", (long long)n,
                threads, b2.nodes.size(), b2.max_depth, b4.nodes(), b4.stack_need);
}

static std::string write_file(const char* name, const std::string& body) {
    std::string p = std::string("/tmp/pt_sanitize_") + name;
    FILE* f = std::fopen(p.c_str(), "wb");
    std::fwrite(body.data(), 1, body.size(), f);
    std::fclose(f);
    return p;
}

static void obj_cases() {
    // well-formed: a displaced grid as v/vt/vn, v//vn, v/vt and plain v faces, CRLF and CR line ends,
    // upper case, a tab-separated (unknown) line, and one line longer than the 1-MB read block
    std::string s = "# grid\r\nMTLLIB none.mtl\nusemtl x\n";
    const int G = 40;
    for (int y = 0; y <= G; y++)
        for (int x = 0; x <= G; x++) {
            char b[128];
            std::snprintf(b, sizeof b, "v %.9g %.9g %.9g\n", x * 0.1, std::sin(x * 0.3) * std::cos(y * 0.2), y * 0.1);
            s += b;
            std::snprintf(b, sizeof b, "VT %.9g %.9g\r", x / (double)G, y / (double)G);
            s += b;
            s += "vn 0 1 0\n";
        }
    s += "v\t1 2 3\n";
    s += "# " + std::string((1u << 20) + 17, 'x') + "\n";
    auto id = [&](int x, int y) { return y * (G + 1) + x + 1; };
    for (int y = 0; y < G; y++)
        for (int x = 0; x < G; x++) {
            const int a = id(x, y), b = id(x + 1, y), c = id(x + 1, y + 1), d = id(x, y + 1);
            char f[160];
            switch ((x + y) % 4) {
                case 0: std::snprintf(f, sizeof f, "f %d/%d/%d %d/%d/%d %d/%d/%d %d/%d/%d\n", a, a, a, b, b, b, c, c, c, d, d, d); break;
                case 1: std::snprintf(f, sizeof f, "f %d//%d %d//%d %d//%d\nf %d//%d %d//%d %d//%d\n", a, a, b, b, c, c, a, a, c, c, d, d); break;
                case 2: std::snprintf(f, sizeof f, "F %d/%d %d/%d %d/%d %d/%d\r\n", a, a, b, b, c, c, d, d); break;
                default: std::snprintf(f, sizeof f, "f %d %d %d\nf %d %d %d", a, b, c, a, c, d); s += f; s += "\n"; continue;
            }
            s += f;
        }
    pt_mesh_data m;
    CHECK(pt_obj_load(write_file("grid.obj", s).c_str(), &m) == PT_OK);
    std::printf("obj: grid %d triangles\n", m.num_triangles);
    CHECK(m.num_triangles > 2 * G * G - 10);
    CHECK(pt_mesh_smooth_normals(m.num_triangles, m.v1, m.v2, m.v3, m.n1, m.n2, m.n3) == PT_OK);
    for (int i = 0; i < m.num_triangles * 3; i++) CHECK(std::isfinite(m.n1[i]));
    pt_mesh_free(&m);
    pt_mesh_free(&m);   // idempotent
    // no trailing newline, a lone "\r" at the very end
    CHECK(pt_obj_load(write_file("tail.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\r").c_str(), &m) == PT_OK);
    CHECK(m.num_triangles == 1);
    pt_mesh_free(&m);
    // every error path
    const char* bad[] = {"v 1 2\n", "v 1 x 3\n", "vt 1\n", "v 0 0 0\nf 1 2 3\n", "v 0 0 0\nf 1/x 1 1\n",
                         "v 0 0 0\nv 1 0 0\nv 0 1 0\nvt 0 0\nf 1/1/9 2/1/1 3/1/1\n", "v 0 0 0\nvt 0 0\nf 1/5 1/1 1/1\n",
                         "v 0 0 0\nf -1 1 1\n", "vn 1e99999 0 0\n"};
    int k = 0;
    for (const char* b : bad) {
        char name[32];
        std::snprintf(name, sizeof name, "bad%d.obj", k++);
        const int rc = pt_obj_load(write_file(name, b).c_str(), &m);
        if (rc == PT_OK) pt_mesh_free(&m);
        CHECK(rc != PT_OK || !std::strcmp(b, "vn 1e99999 0 0\n"));   // strtof overflow reads inf, as float.Parse
    }
    CHECK(pt_obj_load("/tmp/pt_sanitize_does_not_exist.obj", &m) == PT_ERR_INVALID_ARG);
    CHECK(std::strlen(pt_obj_last_error()) > 0);
    CHECK(pt_obj_load(nullptr, &m) != PT_OK);
}

// gopher3 (Example.cs:1542-1564, two spheres for the OBJ) plus a 2-triangle quad and a small mesh
static void oracle_cases(int threads) {
    std::vector<or_material> mats(4);
    std::memset(mats.data(), 0, mats.size() * sizeof(or_material));
    auto mat = [&](int i, double r, double g, double b, double e, double idx, double gloss) {
        mats[i].color[0] = r; mats[i].color[1] = g; mats[i].color[2] = b;
        mats[i].emittance = e; mats[i].index = idx; mats[i].gloss = gloss; mats[i].reflectivity = -1;
    };
    mat(0, 0.988, 0.98, 0.882, 0, 1.5, 10 * M_PI / 180);   // wall
    mat(1, 1, 1, 1, 80, 1, 0);                            // light
    mat(2, 0, 0, 0, 0, 1.2, 30 * M_PI / 180);
    mat(3, 0.2, 0.3, 0.36, 0, 2, 0);
    const float sc[] = {4, 10, 1, 0, 1, 0, 0, 0.5f, 1.5f};
    const double sr[] = {1, 1, 0.5};
    const int32_t sm[] = {1, 2, 3};
    const float cmin[] = {-10, -1, -10, -10, -1, -10}, cmax[] = {-2, 10, 10, 10, 0, 10};
    const int32_t cm[] = {0, 0};
    // a small mesh: a fan of 32 triangles around (1, 0.5, -1)
    const int T = 32;
    std::vector<float> v1(T * 3), v2(T * 3), v3(T * 3), n(T * 3, 0.f), t(T * 3, 0.f);
    std::vector<int32_t> tm(T, 3);
    for (int i = 0; i < T; i++) {
        const double a0 = 2 * M_PI * i / T, a1 = 2 * M_PI * (i + 1) / T;
        const float c[3] = {1.f, 0.5f, -1.f};
        for (int k = 0; k < 3; k++) v1[i * 3 + k] = c[k];
        v2[i * 3 + 0] = c[0] + 0.4f * (float)std::cos(a0); v2[i * 3 + 1] = c[1] + 0.2f; v2[i * 3 + 2] = c[2] + 0.4f * (float)std::sin(a0);
        v3[i * 3 + 0] = c[0] + 0.4f * (float)std::cos(a1); v3[i * 3 + 1] = c[1] + 0.2f; v3[i * 3 + 2] = c[2] + 0.4f * (float)std::sin(a1);
        n[i * 3 + 1] = 1.f;
    }
    const int32_t kinds[] = {1, 1, 0, 0, 0, 4};   // cubes, spheres, the mesh (shape kinds as in the ABI)
    const int32_t idx[] = {0, 1, 0, 1, 2, 0};
    const int32_t mfirst[] = {0}, mcount[] = {T};
    or_scene_desc d;
    std::memset(&d, 0, sizeof d);
    d.num_materials = 4; d.materials = mats.data();
    d.num_shapes = 6; d.shape_kind = kinds; d.shape_index = idx;
    d.num_spheres = 3; d.sphere_center = sc; d.sphere_radius = sr; d.sphere_material = sm;
    d.num_cubes = 2; d.cube_min = cmin; d.cube_max = cmax; d.cube_material = cm;
    d.num_triangles = T; d.tri_v1 = v1.data(); d.tri_v2 = v2.data(); d.tri_v3 = v3.data();
    d.tri_n1 = n.data(); d.tri_n2 = n.data(); d.tri_n3 = n.data(); d.tri_material = tm.data();
    d.tri_t1 = t.data(); d.tri_t2 = t.data(); d.tri_t3 = t.data();
    d.num_meshes = 1; d.mesh_first = mfirst; d.mesh_count = mcount;
    void* sc_ = or_scene_create(&d);
    CHECK(sc_ != nullptr);
    if (!sc_) return;
    or_camera cam;
    std::memset(&cam, 0, sizeof cam);
    // LookAt((4,1,0), (0,0.9,0), up, 40) (Camera.cs:23-35), precomputed
    const float w[3] = {-0.999688f, -0.0249922f, 0.f};
    const float u[3] = {0.f, 0.f, -1.f};
    const float v[3] = {-0.0249922f, 0.999688f, 0.f};
    std::memcpy(cam.w, w, sizeof w); std::memcpy(cam.u, u, sizeof u); std::memcpy(cam.v, v, sizeof v);
    cam.p[0] = 4; cam.p[1] = 1; cam.p[2] = 0;
    cam.m = 1.0 / std::tan(20 * M_PI / 180);
    or_sampler smp{4, 4, 1, 1, 0, 1};
    const int W = 48, H = 32;
    std::vector<double> M((size_t)W * H * 3, 0.0), V((size_t)W * H * 3, 0.0);
    std::vector<int32_t> N((size_t)W * H, 0);
    int64_t rays = 0;
    for (int pass = 0; pass < 3; pass++) {
        or_pass_params pp;
        std::memset(&pp, 0, sizeof pp);
        pp.spp = 2; pp.seed = 99; pp.pass_index = (uint32_t)pass + 1;
        pp.adaptive_samples = pass == 1 ? 2 : 0;
        pp.firefly_samples = pass == 2 ? 3 : 0;
        rays += or_render_pass(sc_, W, H, &cam, &smp, &pp, M.data(), V.data(), N.data(), threads, 0);
    }
    or_pass_params sp;
    std::memset(&sp, 0, sizeof sp);
    sp.spp = 1; sp.seed = 5; sp.pass_index = 4; sp.flags = OR_PASS_SERIAL; sp.adaptive_samples = 2; sp.firefly_samples = 2;
    rays += or_render_pass(sc_, W, H, &cam, &smp, &sp, M.data(), V.data(), N.data(), threads, 0);
    int64_t lit = 0;
    for (double x : M) lit += x > 0;
    for (int32_t x : N) CHECK(x >= 4);
    std::printf("oracle: %d threads, %lld rays, %lld lit channels, %lld k-d nodes\n", threads, (long long)rays,
                (long long)lit, (long long)or_scene_tree_nodes(sc_));
    CHECK(rays > 0 && lit > 0);
    or_scene_destroy(sc_);
}

int main() {
    bvh_case(20000, 8, 1);
    bvh_case(200000, 8, 2);
    bvh_case(37, 8, 3);
    bvh_case(1, 1, 4);
    obj_cases();
    oracle_cases(8);
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("sanitize_host: all checks passed\n");
    return 0;
}
