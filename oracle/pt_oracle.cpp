// pt_oracle.cpp — CPU restatement of PTSharp's per-pixel render hot path.
//
// TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity against the C# reference is
// UNPINNED (no runnable reference, no reference fixtures); this
// file restates the reference line by line and is pinned by analytic KATs.
//
// Numeric model: PTSharp's Vector stores a
// System.Numerics.Vector3 (fp32) behind double accessors (Vector.cs:201-234),
// so every Add/Sub/Mul/Div re-rounds to fp32 (equivalent to an fp32 op),
// MulScalar(double) is float(double(x)*s) (Vector.cs:435), Dot/Length/Cross/
// Normalize are fp32 Vector3 ops (Vector.cs:356,372,384,391); scalars (t, det,
// Fresnel, trig) are fp64; Colour is fp64 (Colour.cs:10-12).  Build with
// -ffp-contract=off so no FMA contraction changes the rounding sequence.
//
// Only deliberate deviation: Random.Shared is replaced by the counter-based
// stream below (keys documented in DESIGN.md §RNG); the GPU kernels use the
// identical stream, so GPU-vs-oracle is a same-seed comparison.
#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------- constants
const double EPS = 1e-9;            // Util.EPS  (Util.cs:11)
const double HIT_INF = (double)1e9f;  // Hit.INF = 1e9F (Hit.cs:6)
const double PI = 3.14159265358979323846;  // Math.PI

// ---------------------------------------------------------------- RNG
inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}
inline uint64_t camera_key(uint64_t seed, uint32_t pass, uint64_t pixel, uint32_t sample) {
    uint64_t k = mix64(seed + 0x243F6A8885A308D3ull);
    k = mix64(k ^ ((uint64_t)pass + 0x13198A2E03707344ull));
    k = mix64(k ^ (pixel + 0xA4093822299F31D0ull));
    return mix64(k ^ ((uint64_t)sample + 0x082EFA98EC4E6C89ull));
}
inline uint64_t child_key(uint64_t k, uint32_t c) { return mix64(k ^ ((uint64_t)c + 0x452821E638D01377ull)); }
inline uint64_t light_key(uint64_t k, uint32_t i) { return mix64(k ^ ((uint64_t)i + 0xBE5466CF34E90C6Cull)); }
// Random.Shared.NextDouble(): 53 random bits in [0,1).
inline double draw(uint64_t k, uint32_t dim) {
    return (double)(mix64(k + (uint64_t)(dim + 1) * 0x9E3779B97F4A7C15ull) >> 11) * (1.0 / 9007199254740992.0);
}
// Draw slots per child edge.
enum { D_STRATUM_U = 0, D_STRATUM_V = 1, D_REFLECT = 2, D_RUV_Z = 3, D_RUV_A = 4,
       D_LIGHT = 5, D_SS_RUV_Z = 6, D_SS_RUV_A = 7, D_SS_XY = 8 };
// Camera-key slots.
enum { D_JX = 0, D_JY = 1, D_LENS_ANGLE = 2, D_LENS_RADIUS = 3 };

// ---------------------------------------------------------------- .NET Math.Min/Max (double)
inline double net_max(double a, double b) {
    if (a != b) { if (!std::isnan(a)) return b < a ? a : b; return a; }
    return std::signbit(b) ? a : b;
}
inline double net_min(double a, double b) {
    if (a != b) { if (!std::isnan(a)) return a < b ? a : b; return a; }
    return std::signbit(a) ? a : b;
}

// ---------------------------------------------------------------- Vector (Vector.cs:193-543)
struct V { float x, y, z; };
inline V vmk(double x, double y, double z) { return V{(float)x, (float)y, (float)z}; }
inline V vadd(V a, V b) { return V{a.x + b.x, a.y + b.y, a.z + b.z}; }   // Vector.Add  :408
inline V vsub(V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z}; }   // Vector.Sub  :411
inline V vmul(V a, V b) { return V{a.x * b.x, a.y * b.y, a.z * b.z}; }   // Vector.Mul  :414
inline V vdiv(V a, V b) { return V{a.x / b.x, a.y / b.y, a.z / b.z}; }   // Vector.Div  :417
inline V vmuls(V a, double s) {                                          // MulScalar   :435
    return V{(float)((double)a.x * s), (float)((double)a.y * s), (float)((double)a.z * s)};
}
inline float dotf(V a, V b) {                                            // Vector3.Dot
    float xx = a.x * b.x, yy = a.y * b.y, zz = a.z * b.z;
    float s = xx + yy;
    return s + zz;
}
inline double vdot(V a, V b) { return (double)dotf(a, b); }              // Vector.Dot  :370
inline V vcross(V a, V b) {                                              // Vector3.Cross
    float x1 = a.y * b.z, x2 = a.z * b.y;
    float y1 = a.z * b.x, y2 = a.x * b.z;
    float z1 = a.x * b.y, z2 = a.y * b.x;
    return V{x1 - x2, y1 - y2, z1 - z2};
}
inline float lenf(V a) { return std::sqrt(dotf(a, a)); }                 // Vector3.Length
inline double vlen(V a) { return (double)lenf(a); }
inline V vnorm(V a) { float l = lenf(a); return V{a.x / l, a.y / l, a.z / l}; }  // Vector3.Normalize
inline V vneg(V a) { return V{-a.x, -a.y, -a.z}; }                       // Negate :396
inline V vmin(V a, V b) { return vmk(net_min(a.x, b.x), net_min(a.y, b.y), net_min(a.z, b.z)); }
inline V vmax(V a, V b) { return vmk(net_max(a.x, b.x), net_max(a.y, b.y), net_max(a.z, b.z)); }
inline V vzero() { return V{0.f, 0.f, 0.f}; }
inline V vload(const float* p) { return V{p[0], p[1], p[2]}; }

// Vector.RandomUnitVector (Vector.cs:339-347)
inline V random_unit_vector(uint64_t key, uint32_t dz, uint32_t da) {
    double z = draw(key, dz) * 2.0 - 1.0;
    double a = draw(key, da) * 2.0 * PI;
    double r = std::sqrt(1.0 - z * z);
    double x = std::sin(a);
    double y = std::cos(a);
    return vmk(r * x, r * y, z);
}
// Vector.Reflect (Vector.cs:497): this = normal
inline V vreflect(V n, V i) { return vsub(i, vmuls(n, 2 * vdot(n, i))); }
// Vector.Refract (Vector.cs:500-514)
inline V vrefract(V n, V i, double n1, double n2) {
    double nr = n1 / n2;
    double cosI = -vdot(n, i);
    double sinT2 = nr * nr * (1 - cosI * cosI);
    if (sinT2 > 1) return vzero();
    double cosT = std::sqrt(1 - sinT2);
    return vadd(vmuls(i, nr), vmuls(n, nr * cosI - cosT));
}
// Vector.Reflectance (Vector.cs:517-536)
inline double vreflectance(V n, V i, double n1, double n2) {
    double nr2 = (n1 * n1) / (n2 * n2);
    double cosI = -vdot(n, i);
    double sinT2 = nr2 * (1 - cosI * cosI);
    if (sinT2 > 1) return 1;
    double cosT = std::sqrt(1 - sinT2);
    double cosI_n1 = n1 * cosI;
    double cosT_n2 = n2 * cosT;
    double rOrth = (cosI_n1 - cosT_n2) / (cosI_n1 + cosT_n2);
    double rPar = (cosT_n2 - cosI_n1) / (cosT_n2 + cosI_n1);
    return (rOrth * rOrth + rPar * rPar) / 2;
}

// ---------------------------------------------------------------- Colour (fp64)
struct C { double r, g, b; };
inline C cadd(C a, C b) { return C{a.r + b.r, a.g + b.g, a.b + b.b}; }
inline C csub(C a, C b) { return C{a.r - b.r, a.g - b.g, a.b - b.b}; }
inline C cmul(C a, C b) { return C{a.r * b.r, a.g * b.g, a.b * b.b}; }
inline C cmuls(C a, double s) { return C{a.r * s, a.g * s, a.b * s}; }
inline C cdivs(C a, double s) { return C{a.r / s, a.g / s, a.b / s}; }
inline C cmix(C a, C b, double pct) { return cadd(cmuls(a, 1 - pct), cmuls(b, pct)); }  // Colour.Mix :219
const C BLACK{0, 0, 0};

// ---------------------------------------------------------------- Ray / Box
struct Ray { V o, d; };
inline V ray_position(const Ray& r, double t) { return vadd(r.o, vmuls(r.d, t)); }  // Ray.Position :19

struct Box { V min, max; };
// Box.Intersect (Box.cs:72-94)
inline void box_intersect(const Box& b, const Ray& r, double& tmin, double& tmax) {
    double x1 = ((double)b.min.x - (double)r.o.x) / (double)r.d.x;
    double y1 = ((double)b.min.y - (double)r.o.y) / (double)r.d.y;
    double z1 = ((double)b.min.z - (double)r.o.z) / (double)r.d.z;
    double x2 = ((double)b.max.x - (double)r.o.x) / (double)r.d.x;
    double y2 = ((double)b.max.y - (double)r.o.y) / (double)r.d.y;
    double z2 = ((double)b.max.z - (double)r.o.z) / (double)r.d.z;
    if (x1 > x2) std::swap(x1, x2);
    if (y1 > y2) std::swap(y1, y2);
    if (z1 > z2) std::swap(z1, z2);
    tmin = net_max(net_max(x1, y1), z1);
    tmax = net_min(net_min(x2, y2), z2);
}
inline Box box_extend(const Box& a, const Box& b) { return Box{vmin(a.min, b.min), vmax(a.max, b.max)}; }
inline V box_center(const Box& b) { return vadd(b.min, vmul(vsub(b.max, b.min), vmk(0.5, 0.5, 0.5))); }  // Box.Center :318
inline double box_outer_radius(const Box& b) { return vlen(vsub(b.min, box_center(b))); }              // :320

// ---------------------------------------------------------------- scene
enum Kind { K_SPHERE = 0, K_CUBE = 1, K_PLANE = 2, K_TRI = 3, K_MESH = 4, K_SDF = 5, K_VOLUME = 6, K_XFORM = 7 };
enum SdfOp { S_SPHERE = 0, S_CUBE, S_CYLINDER, S_CAPSULE, S_TORUS, S_TRANSFORM, S_SCALE, S_UNION, S_DIFFERENCE,
             S_INTERSECTION, S_REPEAT };

struct Material {
    C color; double emittance, index, gloss, tint, reflectivity; bool transparent;
    int tex, ntex, btex, gtex;  // texture slots, 0-based (-1 = null)
    double bump_multiplier;
};
// ColorTexture (Texture.cs:96-252): Width x Height fp64 Colour texels, row-major.
struct Tex {
    int w, h;
    std::vector<double> d;
    C at(size_t i) const { return C{d[3 * i], d[3 * i + 1], d[3 * i + 2]}; }
};
struct Sphere { V center; double radius; int mat; Box box; };
struct Cube { V min, max; int mat; };
struct Plane { V point, normal; int mat; };
struct Tri { V v1, v2, v3, n1, n2, n3; int mat; V t1, t2, t3; };
struct ShapeRef { int kind; int idx; };
struct SdfNode { int op; std::vector<int> kids; double p[8]; double M[16], Inv[16]; };
struct SdfShape { int root; int mat; Box box; };
struct VolWindow { double lo, hi; int mat; };
struct Volume { int w, h, d; double zscale; std::vector<double> data; std::vector<VolWindow> windows; Box box; };
struct Xform { int kind, idx; double M[16], Inv[16]; Box box; };

struct Hit { double t; int kind; int idx; };  // kind: K_* of the primitive hit (mesh hits report K_TRI)
const Hit NOHIT{HIT_INF, -1, -1};

struct KdNode {
    int axis;  // 0 none (leaf), 1 x, 2 y, 3 z  (Axis.cs)
    double point;
    int left, right;
    std::vector<ShapeRef> shapes;
};
struct KdTree {
    Box box;
    std::vector<KdNode> nodes;  // nodes[0] = root
};

struct Scene {
    std::vector<Material> mats;
    std::vector<Sphere> spheres;
    std::vector<Cube> cubes;
    std::vector<Plane> planes;
    std::vector<Tri> tris;
    std::vector<int> mesh_first, mesh_count;
    std::vector<KdTree> mesh_trees;
    std::vector<ShapeRef> shapes;
    std::vector<ShapeRef> lights;  // Scene.Lights (Scene.cs:33-37)
    KdTree tree;
    C env;
    std::vector<Tex> texs;
    int env_tex = -1;        // Scene.Texture (-1 = null)
    double env_angle = 0;    // Scene.TextureAngle
    std::vector<SdfNode> sdf;
    std::vector<SdfShape> sdf_shapes;
    std::vector<Volume> volumes;
    std::vector<Xform> xforms;
    int default_mat = 0;     // `new Material()` (all zero): Volume.MaterialAt when no window is near
};

// ---------------------------------------------------------------- primitives
// Sphere.Intersect (Sphere.cs:40-60)
inline double sphere_t(V center, double radius, const Ray& r) {
    V to = vsub(r.o, center);
    double b = vdot(to, r.d);
    double c = vdot(to, to) - radius * radius;
    double d = b * b - c;
    if (d > 0) {
        d = std::sqrt(d);
        double t1 = -b - d;
        if (t1 > EPS) return t1;
        double t2 = -b + d;
        if (t2 > EPS) return t2;
    }
    return HIT_INF;
}
// Cube.Intersect (Cube.cs:35-47)
inline double cube_t(V mn, V mx, const Ray& r) {
    V n = vdiv(vsub(mn, r.o), r.d);
    V f = vdiv(vsub(mx, r.o), r.d);
    V n2 = vmin(n, f), f2 = vmax(n, f);
    double t0 = net_max(net_max(n2.x, n2.y), n2.z);
    double t1 = net_min(net_min(f2.x, f2.y), f2.z);
    if (t0 > 0 && t0 < t1) return t0;
    return HIT_INF;
}
// Plane.Intersect (Plane.cs:36-50)
inline double plane_t(V point, V normal, const Ray& r) {
    double d = vdot(normal, r.d);
    if (std::fabs(d) < EPS) return HIT_INF;
    V a = vsub(point, r.o);
    double t = vdot(a, normal) / d;
    if (t < EPS) return HIT_INF;
    return t;
}
// Triangle.Intersect, Möller–Trumbore (Triangle.cs:95-124)
inline double tri_t(V v1, V v2, V v3, const Ray& r) {
    V e1 = vsub(v2, v1);
    V e2 = vsub(v3, v1);
    V h = vcross(r.d, e2);
    double det = vdot(e1, h);
    if (det > -EPS && det < EPS) return HIT_INF;
    double invDet = 1.0 / det;
    V s = vsub(r.o, v1);
    double u = vdot(s, h) * invDet;
    if (u < 0 || u > 1) return HIT_INF;
    V q = vcross(s, e1);
    double v = vdot(r.d, q) * invDet;
    if (v < 0 || (u + v) > 1) return HIT_INF;
    double t = vdot(e2, q) * invDet;
    if (t < EPS) return HIT_INF;
    return t;
}
// Cube.NormalAt (Cube.cs:57-69), including the EPS face-match quirk.
inline V cube_normal(V mn, V mx, V p) {
    if (std::fabs((double)p.x - (double)mn.x) < EPS) return vmk(-1, 0, 0);
    if (std::fabs((double)p.x - (double)mx.x) < EPS) return vmk(1, 0, 0);
    if (std::fabs((double)p.y - (double)mn.y) < EPS) return vmk(0, -1, 0);
    if (std::fabs((double)p.y - (double)mx.y) < EPS) return vmk(0, 1, 0);
    if (std::fabs((double)p.z - (double)mn.z) < EPS) return vmk(0, 0, -1);
    if (std::fabs((double)p.z - (double)mx.z) < EPS) return vmk(0, 0, 1);
    return vmk(0, 1, 0);
}
// Triangle.Barycentric (Triangle.cs:208-223)
inline void barycentric(const Tri& t, V p, double& bu, double& bv, double& bw) {
    V v0 = vsub(t.v2, t.v1);
    V v1 = vsub(t.v3, t.v1);
    V v2 = vsub(p, t.v1);
    double d00 = vdot(v0, v0);
    double d01 = vdot(v0, v1);
    double d11 = vdot(v1, v1);
    double d20 = vdot(v2, v0);
    double d21 = vdot(v2, v1);
    double d = d00 * d11 - d01 * d01;
    bv = (d11 * d20 - d01 * d21) / d;
    bw = (d00 * d21 - d01 * d20) / d;
    bu = 1 - bv - bw;
}
// Triangle.NormalAt without maps (Triangle.cs:142-145, 186-188).
inline V tri_normal(const Tri& t, V p) {
    double bu, bv, bw;
    barycentric(t, p, bu, bv, bw);
    V n = vadd(vadd(vmuls(t.n1, bu), vmuls(t.n2, bv)), vmuls(t.n3, bw));
    return vnorm(n);
}

// ---------------------------------------------------------------- textures (Texture.cs:96-252)
// Util.Modf / ColorTexture.Fract (Util.cs:108-113, Texture.cs:218-222): the fractional part, sign kept.
inline double fract(double x) { return x - std::trunc(x); }
// Texel coordinates are Convert.ToInt32(Math.Truncate(.)) / (int) casts, which throw
// OverflowException in the reference for non-finite inputs (CheckForOverflowUnderflow);
// such a lookup returns black here (and on the GPU).
// ColorTexture.BilinearSample (Texture.cs:188-216)
C bilinear(const Tex& t, double u, double v) {
    if (u == 1) u -= EPS;
    if (v == 1) v -= EPS;
    double w = (double)t.w - 1;
    double h = (double)t.h - 1;
    double uw = u * w, vh = v * h;
    if (!std::isfinite(uw) || !std::isfinite(vh)) return BLACK;
    double X = std::trunc(uw), x = uw - X;
    double Y = std::trunc(vh), y = vh - Y;
    int x0 = (int)X, y0 = (int)Y, x1 = x0 + 1, y1 = y0 + 1;
    C c00 = t.at((size_t)y0 * t.w + x0);
    C c01 = t.at((size_t)y1 * t.w + x0);
    C c10 = t.at((size_t)y0 * t.w + x1);
    C c11 = t.at((size_t)y1 * t.w + x1);
    C c = BLACK;
    c = cadd(c, cmuls(c00, (1 - x) * (1 - y)));
    c = cadd(c, cmuls(c10, x * (1 - y)));
    c = cadd(c, cmuls(c01, (1 - x) * y));
    c = cadd(c, cmuls(c11, x * y));
    return c;
}
// ITexture.Sample (Texture.cs:224-229)
C tex_sample(const Tex& t, double u, double v) {
    u = fract(fract(u) + 1);
    v = fract(fract(v) + 1);
    return bilinear(t, u, 1 - v);
}
// ITexture.NormalSample (Texture.cs:231-237)
V tex_normal_sample(const Tex& t, double u, double v) {
    u = fract(fract(u) + 1);
    v = fract(fract(v) + 1);
    C c = bilinear(t, u, 1 - v);
    return vnorm(vmk(c.r * 2 - 1, c.g * 2 - 1, c.b * 2 - 1));
}
// ITexture.BumpSample (Texture.cs:239-251).  At v == 0 the reference reads row Height
// (y = (int)(1 * Height)) and throws IndexOutOfRangeException; the row is clamped here.
V tex_bump_sample(const Tex& t, double u, double v) {
    u = fract(fract(u) + 1);
    v = fract(fract(v) + 1);
    v = 1 - v;
    double fx = u * t.w, fy = v * t.h;
    if (!std::isfinite(fx) || !std::isfinite(fy)) return vzero();
    int x = std::min((int)fx, t.w - 1), y = std::min((int)fy, t.h - 1);
    auto clampi = [](int a, int lo, int hi) { return a < lo ? lo : (a > hi ? hi : a); };  // Util.ClampInt
    int x1 = clampi(x - 1, 0, t.w - 1), x2 = clampi(x + 1, 0, t.w - 1);
    int y1 = clampi(y - 1, 0, t.h - 1), y2 = clampi(y + 1, 0, t.h - 1);
    C cx = csub(t.at((size_t)y * t.w + x1), t.at((size_t)y * t.w + x2));
    C cy = csub(t.at((size_t)y1 * t.w + x), t.at((size_t)y2 * t.w + x));
    return vmk(cx.r, cy.r, 0);
}
inline bool vnonzero(V a) { return !(a.x == 0 && a.y == 0 && a.z == 0); }  // Vector != Vector.Zero (Vector.cs:446-454)

// Triangle.NormalAt with NormalTexture / BumpTexture (Triangle.cs:142-189).
V tri_normal_mapped(const Tri& t, V p, const Tex* ntex, const Tex* btex, double bump_multiplier) {
    double u, v, w;
    barycentric(t, p, u, v, w);
    V n = vadd(vadd(vmuls(t.n1, u), vmuls(t.n2, v)), vmuls(t.n3, w));
    if (ntex) {
        V b = vadd(vadd(vmuls(t.t1, u), vmuls(t.t2, v)), vmuls(t.t3, w));
        V ns = tex_normal_sample(*ntex, b.x, b.y);
        if (vnonzero(ns)) {
            V dv1 = vsub(t.v2, t.v1), dv2 = vsub(t.v3, t.v1);
            V dt1 = vsub(t.t2, t.t1), dt2 = vsub(t.t3, t.t1);
            V T = vnorm(vsub(vmuls(dv1, dt2.y), vmuls(dv2, dt1.y)));
            V B = vnorm(vsub(vmuls(dv2, dt1.x), vmuls(dv1, dt2.x)));
            V N = vcross(T, B);
            // Matrix(T.X, B.X, N.X, 0, ...).MulDirection(ns) (Matrix.cs:144-150): fp64 rows, then Normalize
            double x = (double)T.x * ns.x + (double)B.x * ns.y + (double)N.x * ns.z;
            double y = (double)T.y * ns.x + (double)B.y * ns.y + (double)N.y * ns.z;
            double z = (double)T.z * ns.x + (double)B.z * ns.y + (double)N.z * ns.z;
            n = vnorm(vmk(x, y, z));
        }
    }
    if (btex) {
        V b = vadd(vadd(vmuls(t.t1, u), vmuls(t.t2, v)), vmuls(t.t3, w));
        V bump = tex_bump_sample(*btex, b.x, b.y);
        if (vnonzero(bump)) {
            V dv1 = vsub(t.v2, t.v1), dv2 = vsub(t.v3, t.v1);
            V dt1 = vsub(t.t2, t.t1), dt2 = vsub(t.t3, t.t1);
            V tangent = vnorm(vsub(vmuls(dv1, dt2.y), vmuls(dv2, dt1.y)));
            V bitangent = vnorm(vsub(vmuls(dv2, dt1.x), vmuls(dv1, dt2.x)));
            n = vadd(n, vmuls(tangent, (double)bump.x * bump_multiplier));
            n = vadd(n, vmuls(bitangent, (double)bump.y * bump_multiplier));
        }
    }
    return vnorm(n);
}

inline Box tri_box(const Tri& t) { return Box{vmin(vmin(t.v1, t.v2), t.v3), vmax(vmax(t.v1, t.v2), t.v3)}; }

// ---------------------------------------------------------------- Matrix (Matrix.cs), row-major M11..M44
// MulPosition (Matrix.cs:134-141): fp64 rows, then a Vector (fp32).
inline V mat_position(const double* m, V b) {
    double x = m[0] * b.x + m[1] * b.y + m[2] * b.z + m[3];
    double y = m[4] * b.x + m[5] * b.y + m[6] * b.z + m[7];
    double z = m[8] * b.x + m[9] * b.y + m[10] * b.z + m[11];
    return vmk(x, y, z);
}
// MulDirection (Matrix.cs:144-150), normalised
inline V mat_direction(const double* m, V b) {
    double x = m[0] * b.x + m[1] * b.y + m[2] * b.z;
    double y = m[4] * b.x + m[5] * b.y + m[6] * b.z;
    double z = m[8] * b.x + m[9] * b.y + m[10] * b.z;
    return vnorm(vmk(x, y, z));
}
// Transpose().MulDirection (Matrix.cs:176, 144-150)
inline V mat_direction_transposed(const double* m, V b) {
    double x = m[0] * b.x + m[4] * b.y + m[8] * b.z;
    double y = m[1] * b.x + m[5] * b.y + m[9] * b.z;
    double z = m[2] * b.x + m[6] * b.y + m[10] * b.z;
    return vnorm(vmk(x, y, z));
}
// MulBox (Matrix.cs:156-173)
inline Box mat_box(const double* m, const Box& box) {
    V r = vmk(m[0], m[4], m[8]), u = vmk(m[1], m[5], m[9]), b = vmk(m[2], m[6], m[10]), t = vmk(m[3], m[7], m[11]);
    V xa = vmuls(r, box.min.x), xb = vmuls(r, box.max.x);
    V ya = vmuls(u, box.min.y), yb = vmuls(u, box.max.y);
    V za = vmuls(b, box.min.z), zb = vmuls(b, box.max.z);
    V xlo = vmin(xa, xb), xhi = vmax(xa, xb), ylo = vmin(ya, yb), yhi = vmax(ya, yb), zlo = vmin(za, zb), zhi = vmax(za, zb);
    return Box{vadd(vadd(vadd(xlo, ylo), zlo), t), vadd(vadd(vadd(xhi, yhi), zhi), t)};
}

// ---------------------------------------------------------------- SDF (SDF.cs)
// Vector.LengthN (Vector.cs:359-367)
inline double length_n(V a, double n) {
    if (n == 2) return vlen(a);
    V b = V{std::fabs(a.x), std::fabs(a.y), std::fabs(a.z)};  // Abs (Vector.cs:402-405)
    return std::pow(std::pow((double)b.x, n) + std::pow((double)b.y, n) + std::pow((double)b.z, n), 1 / n);
}
// SDF.Evaluate per node kind (SDF.cs:131-548)
double sdf_eval(const Scene& s, int ni, V p) {
    const SdfNode& n = s.sdf[(size_t)ni];
    switch (n.op) {
        case S_SPHERE: return length_n(p, n.p[1]) - n.p[0];
        case S_CUBE: {
            double x = p.x, y = p.y, z = p.z;
            if (x < 0) x = -x;
            if (y < 0) y = -y;
            if (z < 0) z = -z;
            x -= (double)(float)n.p[0] / 2;
            y -= (double)(float)n.p[1] / 2;
            z -= (double)(float)n.p[2] / 2;
            double a = x;
            if (y > a) a = y;
            if (z > a) a = z;
            if (a > 0) a = 0;
            if (x < 0) x = 0;
            if (y < 0) y = 0;
            if (z < 0) z = 0;
            double b = std::sqrt(x * x + y * y + z * z);
            return a + b;
        }
        case S_CYLINDER: {
            double x = std::sqrt((double)p.x * p.x + (double)p.z * p.z);
            double y = p.y;
            if (x < 0) x = -x;
            if (y < 0) y = -y;
            x -= n.p[0];
            y -= n.p[1] / 2;
            double a = x;
            if (y > a) a = y;
            if (a > 0) a = 0;
            if (x < 0) x = 0;
            if (y < 0) y = 0;
            double b = std::sqrt(x * x + y * y);
            return a + b;
        }
        case S_CAPSULE: {
            V A = vmk(n.p[0], n.p[1], n.p[2]), B = vmk(n.p[3], n.p[4], n.p[5]);
            V pa = vsub(p, A), ba = vsub(B, A);
            double h = net_max(0, net_min(1, vdot(pa, ba) / vdot(ba, ba)));
            return length_n(vsub(pa, vmuls(ba, h)), n.p[7]) - n.p[6];
        }
        case S_TORUS: {
            V q = vmk(length_n(V{p.x, p.y, 0.f}, n.p[2]) - n.p[0], p.z, 0);
            return length_n(q, n.p[3]) - n.p[1];
        }
        case S_TRANSFORM: return sdf_eval(s, n.kids[0], mat_position(n.Inv, p));
        case S_SCALE: return sdf_eval(s, n.kids[0], vmk((double)p.x / n.p[0], (double)p.y / n.p[0], (double)p.z / n.p[0])) * n.p[0];
        case S_UNION: {
            double result = 0;
            for (size_t i = 0; i < n.kids.size(); i++) {
                double d = sdf_eval(s, n.kids[i], p);
                if (i == 0 || d < result) result = d;
            }
            return result;
        }
        case S_DIFFERENCE: {
            double result = 0;
            for (size_t i = 0; i < n.kids.size(); i++) {
                double d = sdf_eval(s, n.kids[i], p);
                if (i == 0) result = d;
                else if (-d > result) result = -d;
            }
            return result;
        }
        case S_INTERSECTION: {
            double result = 0;
            for (size_t i = 0; i < n.kids.size(); i++) {
                double d = sdf_eval(s, n.kids[i], p);
                if (i == 0 || d > result) result = d;
            }
            return result;
        }
        default: {  // S_REPEAT: p.Mod(Step).Sub(Step.DivScalar(2)) (Vector.cs:420-426)
            V st = vmk(n.p[0], n.p[1], n.p[2]);
            V m = vmk((double)p.x - (double)st.x * std::floor((double)p.x / st.x),
                      (double)p.y - (double)st.y * std::floor((double)p.y / st.y),
                      (double)p.z - (double)st.z * std::floor((double)p.z / st.z));
            V half = vmk((double)st.x / 2, (double)st.y / 2, (double)st.z / 2);
            return sdf_eval(s, n.kids[0], vsub(m, half));
        }
    }
}
// SDF.BoundingBox per node kind
Box sdf_box(const Scene& s, int ni) {
    const SdfNode& n = s.sdf[(size_t)ni];
    switch (n.op) {
        case S_SPHERE: { double r = n.p[0]; return Box{vmk(-r, -r, -r), vmk(r, r, r)}; }
        case S_CUBE: {
            double x = (double)(float)n.p[0] / 2, y = (double)(float)n.p[1] / 2, z = (double)(float)n.p[2] / 2;
            return Box{vmk(-x, -y, -z), vmk(x, y, z)};
        }
        case S_CYLINDER: { double r = n.p[0], h = n.p[1] / 2; return Box{vmk(-r, -h, -r), vmk(r, h, r)}; }
        case S_CAPSULE: {
            V A = vmk(n.p[0], n.p[1], n.p[2]), B = vmk(n.p[3], n.p[4], n.p[5]);
            V a = vmin(A, B), b = vmax(A, B);
            double r = n.p[6];
            return Box{vmk(a.x - r, a.y - r, a.z - r), vmk(b.x + r, b.y + r, b.z + r)};  // SubScalar / AddScalar
        }
        case S_TORUS: { double a = n.p[1], b = n.p[1] + n.p[0]; return Box{vmk(-b, -b, a), vmk(b, b, a)}; }
        case S_TRANSFORM: return mat_box(n.M, sdf_box(s, n.kids[0]));
        case S_SCALE: {
            double f = (double)(float)n.p[0];   // new Matrix().Scale(new Vector(f, f, f))
            double m[16] = {f, 0, 0, 0, 0, f, 0, 0, 0, 0, f, 0, 0, 0, 0, 1};
            return mat_box(m, sdf_box(s, n.kids[0]));
        }
        case S_UNION:
        case S_INTERSECTION: {
            Box r{vzero(), vzero()};
            for (size_t i = 0; i < n.kids.size(); i++) r = i == 0 ? sdf_box(s, n.kids[i]) : box_extend(r, sdf_box(s, n.kids[i]));
            return r;
        }
        case S_DIFFERENCE: return sdf_box(s, n.kids[0]);
        default: return Box{vzero(), vzero()};   // RepeatSDF: new Box()
    }
}
// SDFShape.Intersect (SDF.cs:32-76): sphere tracing inside the box.
double sdf_t(const Scene& s, const SdfShape& sh, const Ray& ray) {
    const double epsilon = (double)0.00001f, start = (double)0.0001f, jump_size = (double)0.001f;
    double t1, t2;
    box_intersect(sh.box, ray, t1, t2);
    if (t2 < t1 || t2 < 0) return HIT_INF;
    double t = net_max(start, t1);
    bool jump = true;
    for (int i = 0; i < 1000; i++) {
        double d = sdf_eval(s, sh.root, ray_position(ray, t));
        if (jump && d < 0) {
            t -= jump_size;
            jump = false;
            continue;
        }
        if (d < epsilon) return t;
        if (jump && d < jump_size) d = jump_size;
        t += d;
        if (t > t2) return HIT_INF;
    }
    return HIT_INF;
}
// SDFShape.NormalAt (SDF.cs:83-92)
V sdf_normal(const Scene& s, const SdfShape& sh, V p) {
    const double e = 0.0001;
    double x = p.x, y = p.y, z = p.z;
    auto ev = [&](double a, double b, double c) { return sdf_eval(s, sh.root, vmk(a, b, c)); };
    return vnorm(vmk(ev(x - e, y, z) - ev(x + e, y, z), ev(x, y - e, z) - ev(x, y + e, z), ev(x, y, z - e) - ev(x, y, z + e)));
}

// ---------------------------------------------------------------- Volume (Volume.cs)
inline double vol_get(const Volume& v, int x, int y, int z) {  // Volume.Get (Volume.cs:40-46)
    if (x < 0 || y < 0 || z < 0 || x >= v.w || y >= v.h || z >= v.d) return 0;
    return v.data[(size_t)x + (size_t)y * v.w + (size_t)z * v.w * v.h];
}
// Volume.Sample (Volume.cs:73-105), including its y-from-z slip (:77).  Non-finite or
// out-of-int-range coordinates (an OverflowException in the reference) sample 0.
double vol_sample(const Volume& v, double x, double y, double z) {
    (void)y;
    z /= v.zscale;
    x = ((x + 1) / 2) * (double)v.w;
    y = ((z + 1) / 2) * (double)v.h;
    z = ((z + 2) / 2) * (double)v.d;
    const double lim = 2147483647.0;
    if (!(std::fabs(x) < lim && std::fabs(y) < lim && std::fabs(z) < lim)) return 0;
    int x0 = (int)std::floor(x), y0 = (int)std::floor(y), z0 = (int)std::floor(z);
    int x1 = x0 + 1, y1 = y0 + 1, z1 = z0 + 1;
    double v000 = vol_get(v, x0, y0, z0), v001 = vol_get(v, x0, y0, z1), v010 = vol_get(v, x0, y1, z0);
    double v011 = vol_get(v, x0, y1, z1), v100 = vol_get(v, x1, y0, z0), v101 = vol_get(v, x1, y0, z1);
    double v110 = vol_get(v, x1, y1, z0), v111 = vol_get(v, x1, y1, z1);
    x -= (double)x0;
    y -= (double)y0;
    z -= (double)z0;
    double c00 = v000 * (1 - x) + v100 * x;
    double c01 = v001 * (1 - x) + v101 * x;
    double c10 = v010 * (1 - x) + v110 * x;
    double c11 = v011 * (1 - x) + v111 * x;
    double c0 = c00 * (1 - y) + c10 * y;
    double c1 = c01 * (1 - y) + c11 * y;
    return c0 * (1 - z) + c1 * z;
}
// Volume.Sign (Volume.cs:114-131): `i` is never incremented, so below a window is 1.
int vol_sign(const Volume& v, V a) {
    double s = vol_sample(v, a.x, a.y, a.z);
    for (const VolWindow& w : v.windows) {
        if (s < w.lo) return 1;
        if (s > w.hi) continue;
        return 0;
    }
    return (int)v.windows.size() + 1;
}
// Volume.NormalAt (Volume.cs:138-145)
V vol_normal(const Volume& v, V p) {
    const double eps = (double)0.001f;
    return vnorm(vmk(vol_sample(v, p.x - eps, p.y, p.z) - vol_sample(v, p.x + eps, p.y, p.z),
                     vol_sample(v, p.x, p.y - eps, p.z) - vol_sample(v, p.x, p.y + eps, p.z),
                     vol_sample(v, p.x, p.y, p.z - eps) - vol_sample(v, p.x, p.y, p.z + eps)));
}
// Volume.MaterialAt (Volume.cs:148-166): the window holding the sample, else the nearest.
int vol_material(const Scene& s, const Volume& v, V p) {
    double be = (double)1e9f;
    int bm = s.default_mat;
    double smp = vol_sample(v, p.x, p.y, p.z);
    for (const VolWindow& w : v.windows) {
        if (smp >= w.lo && smp <= w.hi) return w.mat;
        double e = net_min(std::fabs(smp - w.lo), std::fabs(smp - w.hi));
        if (e < be) { be = e; bm = w.mat; }
    }
    return bm;
}
// Volume.Intersect (Volume.cs:168-197).  The reference has no iteration bound; 2^24
// steps stand in for it (a ray that needs more never ends in the reference).
double vol_t(const Volume& v, const Ray& ray) {
    double tmin, tmax;
    box_intersect(v.box, ray, tmin, tmax);
    double step = (double)(1.0f / 512.0f);
    double start = net_max(step, tmin);
    int sign = -1;
    int64_t iters = 0;
    for (double t = start; t <= tmax && iters < (1 << 24); t += step, iters++) {
        int sg = vol_sign(v, ray_position(ray, t));
        if (sg == 0 || (sign >= 0 && sg != sign)) {
            t -= step;
            step /= 64;
            t += step;
            for (int i = 0; i < 64; i++) {
                if (vol_sign(v, ray_position(ray, t)) == 0) return t - step;
                t += step;
            }
        }
        sign = sg;
    }
    return HIT_INF;
}

// IShape.UVector (Sphere.cs:62-69 with its p.Y-for-p.Z slip, Cube.cs:49-53, Plane.cs:52-55,
// Triangle.cs:127-136).  Returns (u, v, 0) as the Vector the reference builds.
V shape_uv(const Scene& s, int kind, int idx, V p) {
    switch (kind) {
        case K_SPHERE: {
            V q = vsub(p, s.spheres[idx].center);
            double u = std::atan2((double)q.z, (double)q.x);
            double v = std::atan2((double)q.y, vlen(V{q.x, 0.f, q.y}));
            u = 1 - (u + PI) / (2 * PI);
            v = (v + PI / 2) / PI;
            return vmk(u, v, 0);
        }
        case K_CUBE: {
            V q = vdiv(vsub(p, s.cubes[idx].min), vsub(s.cubes[idx].max, s.cubes[idx].min));
            return V{q.x, q.z, 0.f};
        }
        case K_TRI: {
            const Tri& t = s.tris[idx];
            double u, v, w;
            barycentric(t, p, u, v, w);
            V n = vadd(vadd(vadd(vzero(), vmuls(t.t1, u)), vmuls(t.t2, v)), vmuls(t.t3, w));
            return V{n.x, n.y, 0.f};
        }
        case K_XFORM: return shape_uv(s, s.xforms[(size_t)idx].kind, s.xforms[(size_t)idx].idx, p);  // Shape.UVector(uv)
        default: return vzero();  // Plane, Mesh, SDFShape, Volume .UVector
    }
}
// Material.MaterialAt (Material.cs:124-138): the colour / gloss a shading point sees.
struct Surf { C color; double gloss; };
Surf material_at(const Scene& s, int kind, int idx, int mat, V p) {
    const Material& m = s.mats[mat];
    Surf r{m.color, m.gloss};
    if (m.tex < 0 && m.gtex < 0) return r;
    V uv = shape_uv(s, kind, idx, p);
    if (m.tex >= 0) r.color = tex_sample(s.texs[m.tex], uv.x, uv.y);
    if (m.gtex >= 0) {
        C c = tex_sample(s.texs[m.gtex], uv.x, uv.y);
        r.gloss = (c.r + c.g + c.b) / 3;
    }
    return r;
}

Box shape_box(const Scene& s, ShapeRef r) {
    switch (r.kind) {
        case K_SDF: return s.sdf_shapes[(size_t)r.idx].box;
        case K_VOLUME: return s.volumes[(size_t)r.idx].box;
        case K_XFORM: return s.xforms[(size_t)r.idx].box;
        case K_SPHERE: return s.spheres[r.idx].box;
        case K_CUBE: return Box{s.cubes[r.idx].min, s.cubes[r.idx].max};
        case K_PLANE: return Box{vmk(-1e9, -1e9, -1e9), vmk(1e9, 1e9, 1e9)};  // Plane.cs:31-34 (Util.INF)
        case K_TRI: return tri_box(s.tris[r.idx]);
        case K_MESH: {  // Mesh.BoundingBox (Mesh.cs:88-120)
            int f = s.mesh_first[r.idx], n = s.mesh_count[r.idx];
            V mn = s.tris[f].v1, mx = s.tris[f].v1;
            for (int i = f; i < f + n; i++) {
                const Tri& t = s.tris[i];
                mn = vmin(vmin(vmin(mn, t.v1), t.v2), t.v3);
                mx = vmax(vmax(vmax(mx, t.v1), t.v2), t.v3);
            }
            return Box{mn, mx};
        }
    }
    return Box{vzero(), vzero()};
}

// ---------------------------------------------------------------- k-d tree build (Tree.cs:22-29,130-265)
struct TreeBuilder {
    const Scene& s;
    KdTree& tree;
    std::vector<Box> boxcache;  // by position in `all`
    TreeBuilder(const Scene& s_, KdTree& t) : s(s_), tree(t) {}

    // Box.Partition (Box.cs:96-114)
    static void partition(const Box& b, int axis, double point, bool& l, bool& r) {
        switch (axis) {
            case 1: l = b.min.x <= point; r = b.max.x >= point; break;
            case 2: l = b.min.y <= point; r = b.max.y >= point; break;
            default: l = b.min.z <= point; r = b.max.z >= point; break;
        }
    }
    static int partition_score(const std::vector<Box>& boxes, int axis, double point) {
        int left = 0, right = 0;
        for (const Box& b : boxes) {
            bool l, r; partition(b, axis, point, l, r);
            if (l) left++;
            if (r) right++;
        }
        return left >= right ? left : right;
    }
    // Node.Median over a ConcurrentBag filled in insertion order L = [min0,max0,min1,...]:
    // enumeration is LIFO, the count is always even (2 per shape), so the
    // "median" is (L[n-1] + L[n]) / 2 with n = #shapes (Tree.cs:130-148, 208-226).
    static double median(const std::vector<double>& L) {
        if (L.empty()) return 0;
        size_t cnt = L.size();
        std::vector<double> R(L.rbegin(), L.rend());
        size_t mid = cnt / 2;
        if (cnt % 2 == 1) return R[mid];
        return (R[cnt / 2 - 1] + R[cnt / 2]) / 2;
    }
    int new_node(std::vector<ShapeRef>&& shapes) {
        KdNode n; n.axis = 0; n.point = 0; n.left = n.right = -1; n.shapes = std::move(shapes);
        tree.nodes.push_back(std::move(n));
        return (int)tree.nodes.size() - 1;
    }
    void split(int node, int depth) {  // Node.Split (Tree.cs:201-265)
        std::vector<ShapeRef> shapes = tree.nodes[node].shapes;
        if (shapes.size() < 8) return;
        std::vector<Box> boxes(shapes.size());
        std::vector<double> xs, ys, zs;
        xs.reserve(2 * shapes.size()); ys.reserve(2 * shapes.size()); zs.reserve(2 * shapes.size());
        for (size_t i = 0; i < shapes.size(); i++) {
            boxes[i] = shape_box(s, shapes[i]);
            xs.push_back(boxes[i].min.x); xs.push_back(boxes[i].max.x);
            ys.push_back(boxes[i].min.y); ys.push_back(boxes[i].max.y);
            zs.push_back(boxes[i].min.z); zs.push_back(boxes[i].max.z);
        }
        double mx = median(xs), my = median(ys), mz = median(zs);
        int best = (int)(shapes.size() * 0.85);
        int bestAxis = 0; double bestPoint = 0.0;
        int sx = partition_score(boxes, 1, mx);
        if (sx < best) { best = sx; bestAxis = 1; bestPoint = mx; }
        int sy = partition_score(boxes, 2, my);
        if (sy < best) { best = sy; bestAxis = 2; bestPoint = my; }
        int sz = partition_score(boxes, 3, mz);
        if (sz < best) { best = sz; bestAxis = 3; bestPoint = mz; }
        if (bestAxis == 0) return;
        // Partition into ConcurrentBags; ToArray() yields LIFO (reverse insertion) order.
        std::vector<ShapeRef> l, r;
        for (size_t i = 0; i < shapes.size(); i++) {
            bool bl, br; partition(boxes[i], bestAxis, bestPoint, bl, br);
            if (bl) l.push_back(shapes[i]);
            if (br) r.push_back(shapes[i]);
        }
        std::reverse(l.begin(), l.end());
        std::reverse(r.begin(), r.end());
        tree.nodes[node].axis = bestAxis;
        tree.nodes[node].point = bestPoint;
        int li = new_node(std::move(l));
        int ri = new_node(std::move(r));
        tree.nodes[node].left = li;
        tree.nodes[node].right = ri;
        split(li, depth + 1);
        split(ri, depth + 1);
        tree.nodes[node].shapes.clear();
        tree.nodes[node].shapes.shrink_to_fit();
    }
    void build(const std::vector<ShapeRef>& shapes) {  // Tree.NewTree (Tree.cs:22-29)
        tree.nodes.clear();
        if (!shapes.empty()) {
            Box b = shape_box(s, shapes[0]);
            for (const ShapeRef& r : shapes) b = box_extend(b, shape_box(s, r));
            tree.box = b;
        } else {
            tree.box = Box{vzero(), vzero()};
        }
        int root = new_node(std::vector<ShapeRef>(shapes));
        split(root, 0);
    }
};

// Intersect of a shape that can sit inside a TransformedShape (Sphere, Cube, Plane, SDFShape, Volume).
double inner_t(const Scene& s, int kind, int idx, const Ray& ray) {
    switch (kind) {
        case K_SPHERE: return sphere_t(s.spheres[(size_t)idx].center, s.spheres[(size_t)idx].radius, ray);
        case K_CUBE: return cube_t(s.cubes[(size_t)idx].min, s.cubes[(size_t)idx].max, ray);
        case K_PLANE: return plane_t(s.planes[(size_t)idx].point, s.planes[(size_t)idx].normal, ray);
        case K_SDF: return sdf_t(s, s.sdf_shapes[(size_t)idx], ray);
        case K_VOLUME: return vol_t(s.volumes[(size_t)idx], ray);
    }
    return HIT_INF;
}
Hit mesh_hit(const Scene& s, int mesh, const Ray& ray);   // Mesh.Intersect through its own tree (below)
// The inner shape's Hit (a mesh reports the Triangle it hit, as Mesh.Intersect does).
Hit inner_hit(const Scene& s, int kind, int idx, const Ray& ray) {
    if (kind == K_MESH) return mesh_hit(s, idx, ray);
    double t = inner_t(s, kind, idx, ray);
    return t < HIT_INF ? Hit{t, kind, idx} : NOHIT;
}
// TransformedShape.Intersect (TransformedShape.cs:43-73) up to hit.T: the inner shape's hit
// mapped back to world space, T = |position - origin| (fp32 Length).
inline Ray xform_shape_ray(const Xform& x, const Ray& r) {  // Matrix.Inverse().MulRay(r)
    return Ray{mat_position(x.Inv, r.o), mat_direction(x.Inv, r.d)};
}
double xform_t(const Scene& s, const Xform& x, const Ray& r) {
    Ray sr = xform_shape_ray(x, r);
    Hit h = inner_hit(s, x.kind, x.idx, sr);
    if (!(h.t < HIT_INF)) return HIT_INF;
    V position = mat_position(x.M, ray_position(sr, h.t));
    return vlen(vsub(position, r.o));
}

// ---------------------------------------------------------------- tracing
struct Tracer {
    const Scene& s;
    bool brute;
    uint64_t rays = 0;
    Tracer(const Scene& s_, bool b) : s(s_), brute(b) {}

    Hit shape_intersect(ShapeRef r, const Ray& ray) const {
        double t = HIT_INF;
        switch (r.kind) {
            case K_SPHERE: t = sphere_t(s.spheres[r.idx].center, s.spheres[r.idx].radius, ray); break;
            case K_CUBE: t = cube_t(s.cubes[r.idx].min, s.cubes[r.idx].max, ray); break;
            case K_PLANE: t = plane_t(s.planes[r.idx].point, s.planes[r.idx].normal, ray); break;
            case K_TRI: { const Tri& tr = s.tris[r.idx]; t = tri_t(tr.v1, tr.v2, tr.v3, ray); break; }
            case K_SDF: t = sdf_t(s, s.sdf_shapes[(size_t)r.idx], ray); break;
            case K_VOLUME: t = vol_t(s.volumes[(size_t)r.idx], ray); break;
            case K_XFORM: t = xform_t(s, s.xforms[(size_t)r.idx], ray); break;
            case K_MESH:
                if (brute) {
                    Hit h = NOHIT;
                    int f = s.mesh_first[r.idx], n = s.mesh_count[r.idx];
                    for (int i = f; i < f + n; i++) {
                        const Tri& tr = s.tris[i];
                        double tt = tri_t(tr.v1, tr.v2, tr.v3, ray);
                        if (tt < h.t) h = Hit{tt, K_TRI, i};
                    }
                    return h;
                }
                return tree_intersect(s.mesh_trees[r.idx], ray);  // Mesh.Intersect (Mesh.cs:83-86)
        }
        if (t < HIT_INF) return Hit{t, r.kind, r.idx};
        return NOHIT;
    }
    // Node.IntersectShapes (Tree.cs:115-128): strict '<', first shape wins ties.
    Hit intersect_shapes(const std::vector<ShapeRef>& shapes, const Ray& ray) const {
        Hit hit = NOHIT;
        for (const ShapeRef& r : shapes) {
            Hit h = shape_intersect(r, ray);
            if (h.t < hit.t) hit = h;
        }
        return hit;
    }
    // Node.Intersect (Tree.cs:67-113)
    Hit node_intersect(const KdTree& tr, int ni, const Ray& r, double tmin, double tmax) const {
        const KdNode& n = tr.nodes[ni];
        double tsplit; bool leftFirst;
        switch (n.axis) {
            case 0: return intersect_shapes(n.shapes, r);
            case 1: tsplit = (n.point - (double)r.o.x) / (double)r.d.x;
                    leftFirst = ((double)r.o.x < n.point) || ((double)r.o.x == n.point && r.d.x <= 0); break;
            case 2: tsplit = (n.point - (double)r.o.y) / (double)r.d.y;
                    leftFirst = ((double)r.o.y < n.point) || ((double)r.o.y == n.point && r.d.y <= 0); break;
            default: tsplit = (n.point - (double)r.o.z) / (double)r.d.z;
                    leftFirst = ((double)r.o.z < n.point) || ((double)r.o.z == n.point && r.d.z <= 0); break;
        }
        int first = leftFirst ? n.left : n.right;
        int second = leftFirst ? n.right : n.left;
        if (tsplit > tmax || tsplit <= 0) return node_intersect(tr, first, r, tmin, tmax);
        if (tsplit < tmin) return node_intersect(tr, second, r, tmin, tmax);
        Hit h1 = node_intersect(tr, first, r, tmin, tsplit);
        if (h1.t <= tsplit) return h1;
        Hit h2 = node_intersect(tr, second, r, tsplit, net_min(tmax, h1.t));
        return h1.t <= h2.t ? h1 : h2;
    }
    // Tree.Intersect (Tree.cs:31-42)
    Hit tree_intersect(const KdTree& tr, const Ray& r) const {
        if (tr.nodes.empty()) return NOHIT;
        double tmin, tmax;
        box_intersect(tr.box, r, tmin, tmax);
        if (tmax < tmin || tmax <= 0) return NOHIT;
        return node_intersect(tr, 0, r, tmin, tmax);
    }
    // Scene.Intersect (Scene.cs:75-79): counts every call.
    Hit intersect(const Ray& r) {
        rays++;
        if (brute) return intersect_shapes(s.shapes, r);
        return tree_intersect(s.tree, r);
    }
};

Hit mesh_hit(const Scene& s, int mesh, const Ray& ray) { return Tracer(s, false).tree_intersect(s.mesh_trees[(size_t)mesh], ray); }

struct HitInfo { V position, normal; Ray ray; int mat; bool inside; C color; double gloss; };

V shape_normal(const Scene& s, const Hit& h, V p) {
    switch (h.kind) {
        case K_SPHERE: return vnorm(vsub(p, s.spheres[h.idx].center));  // Sphere.NormalAt :78-81
        case K_CUBE: return cube_normal(s.cubes[h.idx].min, s.cubes[h.idx].max, p);
        case K_PLANE: return s.planes[h.idx].normal;                      // Plane.NormalAt :61-64
        case K_SDF: return sdf_normal(s, s.sdf_shapes[(size_t)h.idx], p);
        case K_VOLUME: return vol_normal(s.volumes[(size_t)h.idx], p);
        default: {
            const Tri& t = s.tris[h.idx];
            const Material& m = s.mats[t.mat];
            if (m.ntex < 0 && m.btex < 0) return tri_normal(t, p);
            return tri_normal_mapped(t, p, m.ntex >= 0 ? &s.texs[m.ntex] : nullptr,
                                     m.btex >= 0 ? &s.texs[m.btex] : nullptr, m.bump_multiplier);
        }
    }
}
// IShape.MaterialAt(p): the material index a shape reports at p.
int material_index_at(const Scene& s, int kind, int idx, V p) {
    switch (kind) {
        case K_SPHERE: return s.spheres[(size_t)idx].mat;
        case K_CUBE: return s.cubes[(size_t)idx].mat;
        case K_PLANE: return s.planes[(size_t)idx].mat;
        case K_TRI: return s.tris[(size_t)idx].mat;
        case K_SDF: return s.sdf_shapes[(size_t)idx].mat;
        case K_VOLUME: return vol_material(s, s.volumes[(size_t)idx], p);
        case K_XFORM: return material_index_at(s, s.xforms[(size_t)idx].kind, s.xforms[(size_t)idx].idx, p);
        default: return s.default_mat;   // Mesh.MaterialAt: `new Material()`
    }
}
// Hit.Info (Hit.cs:26-55); SDFShape / Volume keep inside = false (Hit.cs:42-49).
HitInfo hit_info(const Scene& s, const Hit& h, const Ray& r) {
    HitInfo info;
    if (h.kind == K_XFORM) {  // the HitInfo TransformedShape.Intersect builds (TransformedShape.cs:52-70)
        const Xform& x = s.xforms[(size_t)h.idx];
        Ray sr = xform_shape_ray(x, r);
        Hit ih = inner_hit(s, x.kind, x.idx, sr);   // hit.Shape: the inner shape (a mesh's Triangle)
        V sp = ray_position(sr, ih.t);
        V sn = shape_normal(s, ih, sp);
        info.position = mat_position(x.M, sp);
        V normal = mat_direction_transposed(x.Inv, sn);   // Matrix.Inverse().Transpose().MulDirection
        info.mat = material_index_at(s, ih.kind, ih.idx, sp);
        Surf sf = material_at(s, ih.kind, ih.idx, info.mat, sp);
        info.color = sf.color;
        info.gloss = sf.gloss;
        info.inside = false;
        if (vdot(sn, sr.d) > 0) { normal = vneg(normal); info.inside = true; }
        info.normal = normal;
        info.ray = Ray{info.position, normal};
        return info;
    }
    info.position = ray_position(r, h.t);
    V normal = shape_normal(s, h, info.position);
    info.mat = material_index_at(s, h.kind, h.idx, info.position);
    Surf sf = material_at(s, h.kind, h.idx, info.mat, info.position);
    info.color = sf.color;
    info.gloss = sf.gloss;
    info.inside = false;
    if (vdot(normal, r.d) > 0) {
        normal = vneg(normal);
        info.inside = h.kind != K_SDF && h.kind != K_VOLUME;
    }
    info.normal = normal;
    info.ray = Ray{info.position, normal};
    return info;
}

// ---------------------------------------------------------------- sampler (Sampler.cs)
struct Sampler {
    int fh, mb; bool dl, ss; int light_mode, spec_mode;
};

struct Integrator {
    const Scene& s;
    const Sampler& smp;
    Tracer& tr;
    Integrator(const Scene& s_, const Sampler& m, Tracer& t) : s(s_), smp(m), tr(t) {}

    // Util.Cone (Util.cs:17-32)
    V cone(V direction, double theta, double u, double v, uint64_t key) {
        if (theta < EPS) return direction;
        theta = theta * (1 - (2 * std::acos(u) / PI));
        double m1 = std::sin(theta);
        double m2 = std::cos(theta);
        double a = v * 2 * PI;
        V q = random_unit_vector(key, D_RUV_Z, D_RUV_A);
        V sv = vcross(direction, q);
        V tv = vcross(direction, sv);
        V d = vadd(vadd(vadd(vzero(), vmuls(sv, m1 * std::cos(a))), vmuls(tv, m1 * std::sin(a))), vmuls(direction, m2));
        return vnorm(d);
    }
    // Ray.WeightedBounce (Ray.cs:28-35), on the normal ray n
    Ray weighted_bounce(const Ray& n, double u, double v, uint64_t key) {
        double radius = std::sqrt(u);
        double theta = 2 * PI * v;
        V sv = vnorm(vcross(n.d, random_unit_vector(key, D_RUV_Z, D_RUV_A)));
        V tv = vcross(n.d, sv);
        V d = vadd(vadd(vadd(vzero(), vmuls(sv, radius * std::cos(theta))), vmuls(tv, radius * std::sin(theta))),
                   vmuls(n.d, std::sqrt(1 - u)));
        return Ray{n.o, d};
    }
    // Ray.Bounce (Ray.cs:44-85); bounce type 0 Any, 1 Diffuse, 2 Specular (BounceType.cs)
    Ray bounce(const Ray& in, const HitInfo& info, double u, double v, int btype, uint64_t key,
               bool& reflected, double& p) {
        const Material& m = s.mats[info.mat];
        const Ray& n = info.ray;
        double n1 = 1.0, n2 = m.index;
        if (info.inside) std::swap(n1, n2);
        p = m.reflectivity >= 0 ? m.reflectivity : vreflectance(n.d, in.d, n1, n2);
        bool reflect;
        switch (btype) {
            case 0: reflect = draw(key, D_REFLECT) < p; break;
            case 1: reflect = false; break;
            default: reflect = true; break;
        }
        if (reflect) {
            Ray r{n.o, vreflect(n.d, in.d)};
            reflected = true;
            return Ray{r.o, cone(r.d, info.gloss, u, v, key)};
        } else if (m.transparent) {
            Ray r{n.o, vrefract(n.d, in.d, n1, n2)};
            r.o = vadd(r.o, vmuls(r.d, 1e-4));
            reflected = true;
            p = 1 - p;
            return Ray{r.o, cone(r.d, info.gloss, u, v, key)};
        }
        reflected = false;
        p = 1 - p;
        return weighted_bounce(n, u, v, key);
    }
    bool light_identity(ShapeRef light, const Hit& h) const {
        // hit.Shape != light is a reference compare (Sampler.cs:264): class shapes
        // compare equal to themselves; a struct Triangle is re-boxed per Hit, never equal.
        if (light.kind == K_TRI || light.kind == K_MESH || light.kind == K_XFORM) return false;
        return h.kind == light.kind && h.idx == light.idx;
    }
    // Sampler.sampleLight (Sampler.cs:212-296)
    C sample_light(const Ray& n, ShapeRef light, uint64_t key) {
        V center; double radius;
        if (light.kind == K_SPHERE) {
            radius = s.spheres[light.idx].radius;
            center = s.spheres[light.idx].center;
        } else {
            Box b = shape_box(s, light);
            radius = box_outer_radius(b);
            center = box_center(b);
        }
        V point = center;
        if (smp.ss) {
            for (uint32_t k = 0; k < 256; k++) {
                double x = draw(key, D_SS_XY + 2 * k) * 2 - 1;
                double y = draw(key, D_SS_XY + 2 * k + 1) * 2 - 1;
                if (x * x + y * y <= 1) {
                    V l = vnorm(vsub(center, n.o));
                    V u = vnorm(vcross(l, random_unit_vector(key, D_SS_RUV_Z, D_SS_RUV_A)));
                    V v = vcross(l, u);
                    point = vadd(vadd(center, vmuls(u, x * radius)), vmuls(v, y * radius));
                    break;
                }
            }
        }
        V rayDirection = vnorm(vsub(point, n.o));
        double diffuse = vdot(rayDirection, n.d);
        if (diffuse <= 0) return BLACK;
        Ray ray{n.o, rayDirection};
        Hit hit = tr.intersect(ray);
        if (!(hit.t < HIT_INF) || !light_identity(light, hit)) return BLACK;
        double hyp = vlen(vsub(center, n.o));
        double theta = std::asin(radius / hyp);
        double adj = radius / std::tan(theta);
        double d = std::cos(theta) * adj;
        double r = std::sin(theta) * adj;
        double coverage = (r * r) / (d * d);
        if (hyp < radius) coverage = 1;
        coverage = net_min(coverage, 1);
        int mi = material_index_at(s, light.kind, light.idx, point);
        // Material.MaterialAt(light, point) (Sampler.cs:292): the colour at the sampled point
        Surf sf = material_at(s, light.kind, light.idx, mi, point);
        double mm = s.mats[mi].emittance * diffuse * coverage;
        return cmuls(sf.color, mm);
    }
    // Sampler.sampleLights (Sampler.cs:191-210)
    C sample_lights(const Ray& n, uint64_t key) {
        int nLights = (int)s.lights.size();
        if (nLights == 0) return BLACK;
        if (smp.light_mode == 1) {
            C result{0, 0, 0};
            for (int i = 0; i < nLights; i++) result = cadd(result, sample_light(n, s.lights[i], light_key(key, (uint32_t)i)));
            return cdivs(result, nLights);
        }
        int idx = (int)(draw(key, D_LIGHT) * nLights);
        if (idx >= nLights) idx = nLights - 1;
        return cmuls(sample_light(n, s.lights[idx], key), (double)nLights);
    }
    // DefaultSampler.sample (Sampler.cs:55-145); Russian roulette is never enabled.
    // sampleEnvironment (Sampler.cs:177-189)
    C sample_environment(const Ray& r) const {
        if (s.env_tex < 0) return s.env;
        V d = r.d;
        double u = std::atan2((double)d.z, (double)d.x) + s.env_angle;
        double v = std::atan2((double)d.y, vlen(V{d.x, 0.f, d.z}));
        u = (u + PI) / (2 * PI);
        v = (v + PI / 2) / PI;
        return tex_sample(s.texs[s.env_tex], u, v);
    }
    C sample(const Ray& ray, bool emission, int samples, int depth, uint64_t node) {
        if (depth > smp.mb) return BLACK;
        Hit hit = tr.intersect(ray);
        if (!(hit.t < HIT_INF)) return sample_environment(ray);
        HitInfo info = hit_info(s, hit, ray);
        const Material& material = s.mats[info.mat];
        C result{0, 0, 0};
        if (material.emittance > 0) {
            if (smp.dl && !emission) return BLACK;
            result = cadd(result, cmuls(info.color, material.emittance * samples));
        }
        int n = (int)std::sqrt((double)samples);
        int ma, mb;
        if (smp.spec_mode == 2 || (depth == 0 && smp.spec_mode == 1)) { ma = 1; mb = 2; }
        else { ma = 0; mb = 0; }
        int nm = mb - ma + 1;
        for (int u = 0; u < n; u++) {
            for (int v = 0; v < n; v++) {
                for (int mode = ma; mode <= mb; mode++) {
                    uint32_t c = (uint32_t)((u * n + v) * nm + (mode - ma));
                    uint64_t E = child_key(node, c);
                    double fu = ((double)u + draw(E, D_STRATUM_U)) / (double)n;
                    double fv = ((double)(float)v + draw(E, D_STRATUM_V)) / (double)n;
                    bool reflected; double p;
                    Ray newRay = bounce(ray, info, fu, fv, mode, E, reflected, p);
                    if (mode == 0) p = 1;
                    if (p > 0 && reflected) {
                        C indirect = sample(newRay, reflected, 1, depth + 1, E);
                        C tinted = cmix(indirect, cmul(info.color, indirect), material.tint);
                        result = cadd(result, cmuls(tinted, p));
                    }
                    if (p > 0 && !reflected) {
                        C indirect = sample(newRay, reflected, 1, depth + 1, E);
                        C direct = BLACK;
                        if (smp.dl) direct = sample_lights(info.ray, E);
                        result = cadd(result, cmuls(cmul(info.color, cadd(direct, indirect)), p));
                    }
                }
            }
        }
        return cdivs(result, (double)(n * n));
    }
};

// Camera.CastRay (Camera.cs:98-119)
Ray cast_ray(const or_camera& cam, int x, int y, int w, int h, double u, double v, uint64_t key) {
    double aspect = w / (double)h;
    double px = ((x + u - 0.5) / (w - 1.0)) * 2 - 1;
    double py = ((y + v - 0.5) / (h - 1.0)) * 2 - 1;
    V cu = vload(cam.u), cv = vload(cam.v), cw = vload(cam.w), cp = vload(cam.p);
    V d = vnorm(vadd(vadd(vadd(vzero(), vmuls(cu, -px * aspect)), vmuls(cv, -py)), vmuls(cw, cam.m)));
    V p = cp;
    if (cam.aperture_radius > 0) {
        V focalPoint = vadd(cp, vmuls(d, cam.focal_distance));
        double angle = draw(key, D_LENS_ANGLE) * 2 * PI;
        double radius = draw(key, D_LENS_RADIUS) * cam.aperture_radius;
        p = vadd(p, vmuls(cu, std::cos(angle) * radius));
        p = vadd(p, vmuls(cv, std::sin(angle) * radius));
        d = vnorm(vsub(focalPoint, p));
    }
    return Ray{p, d};
}

// Pixel.AddSample (Buffer.cs:33-44)
inline void welford(double* m, double* v, int32_t* n, C s) {
    (*n)++;
    if (*n == 1) { m[0] = s.r; m[1] = s.g; m[2] = s.b; return; }
    C M{m[0], m[1], m[2]}, Vv{v[0], v[1], v[2]};
    C mo = M;
    M = cadd(M, cdivs(csub(s, M), (double)*n));
    Vv = cadd(Vv, cmul(csub(s, mo), csub(s, M)));
    m[0] = M.r; m[1] = M.g; m[2] = M.b;
    v[0] = Vv.r; v[1] = Vv.g; v[2] = Vv.b;
}

Sampler make_sampler(const or_sampler* s) {
    return Sampler{s->first_hit_samples, s->max_bounces, s->direct_lighting != 0, s->soft_shadows != 0,
                   s->light_mode, s->specular_mode};
}

// One pixel of RenderParallel (Renderer.cs:287-310) or of the stratified path (:233-253).
void render_pixel(Integrator& in, const or_camera& cam, int x, int y, int w, int h, const or_pass_params& pp,
                  double* M, double* Vv, int32_t* N) {
    uint64_t pix = (uint64_t)y * (uint64_t)w + (uint64_t)x;
    size_t i = (size_t)pix;
    if (pp.stratified) {
        int sppRoot = (int)std::sqrt((double)pp.spp);
        for (int u = 0; u < sppRoot; u++)
            for (int v = 0; v < sppRoot; v++) {
                uint64_t K = camera_key(pp.seed, pp.pass_index, pix, (uint32_t)(u * sppRoot + v));
                double fu = ((double)u + 0.5) / (double)sppRoot;
                double fv = ((double)v + 0.5) / (double)sppRoot;
                Ray ray = cast_ray(cam, x, y, w, h, fu, fv, K);
                C smp = in.sample(ray, true, in.smp.fh, 0, K);
                welford(M + 3 * i, Vv + 3 * i, N + i, smp);
            }
        return;
    }
    C c{0, 0, 0};
    for (int p = 0; p < pp.spp; p++) {
        uint64_t K = camera_key(pp.seed, pp.pass_index, pix, (uint32_t)p);
        double xOffset = draw(K, D_JX);
        double yOffset = draw(K, D_JY);
        double fu = (x + xOffset) / w;  // the jitter bug: CastRay adds x again
        double fv = (y + yOffset) / h;
        Ray ray = cast_ray(cam, x, y, w, h, fu, fv, K);
        c = cadd(c, in.sample(ray, true, in.smp.fh, 0, K));
    }
    c = cdivs(c, (double)pp.spp);
    welford(M + 3 * i, Vv + 3 * i, N + i, c);
}

// Sample-index domains of the per-pass extra phases: the main
// loop uses 0..spp-1.
constexpr uint32_t kAdaptiveBase = 0x40000000u, kFireflyBase = 0x80000000u;

// One sample of the adaptive / firefly loops: CastRay(x, y, w, h, NextDouble(),
// NextDouble()) — these loops pass the jitter directly (Renderer.cs:357-361, 432).
C extra_sample(Integrator& in, const or_camera& cam, int x, int y, int w, int h, const or_pass_params& pp,
               uint32_t sample) {
    uint64_t pix = (uint64_t)y * (uint64_t)w + (uint64_t)x;
    uint64_t K = camera_key(pp.seed, pp.pass_index, pix, sample);
    double fu = draw(K, D_JX), fv = draw(K, D_JY);
    Ray ray = cast_ray(cam, x, y, w, h, fu, fv, K);
    return in.sample(ray, true, in.smp.fh, 0, K);
}

// Renderer.Render's firefly loop (Renderer.cs:184-186): CastRay(x, y, w, h, fu, fv) with
// fu = (x + NextDouble()) * invWidth, invWidth = 1.0f / w evaluated in float (:98-99).
C serial_firefly_sample(Integrator& in, const or_camera& cam, int x, int y, int w, int h, const or_pass_params& pp,
                        uint32_t sample) {
    uint64_t pix = (uint64_t)y * (uint64_t)w + (uint64_t)x;
    uint64_t K = camera_key(pp.seed, pp.pass_index, pix, sample);
    const double inv_w = (double)(1.0f / (float)w), inv_h = (double)(1.0f / (float)h);
    double fu = ((double)x + draw(K, D_JX)) * inv_w, fv = ((double)y + draw(K, D_JY)) * inv_h;
    Ray ray = cast_ray(cam, x, y, w, h, fu, fv, K);
    return in.sample(ray, true, in.smp.fh, 0, K);
}

// Renderer.Render's adaptive branch (Renderer.cs:155-160): v = StandardDeviation().MaxComponent(),
// v = Math.Clamp(v / AdaptiveThreshold, 0, 1), v = Math.Pow(v, AdaptiveExponent), and
// AdaptiveSamples * (int)v samples.  Both knobs are 1 (Renderer.cs:45-46, private, never set
// elsewhere), so (int)v is 1 exactly when the deviation reaches 1; NaN gives (int)NaN, whose
// product with AdaptiveSamples is never positive.
bool adaptive_serial_candidate(const double* V, int32_t N) {
    if (N < 2) return false;
    double r = std::sqrt(V[0] / (double)(N - 1)), g = std::sqrt(V[1] / (double)(N - 1)),
           b = std::sqrt(V[2] / (double)(N - 1));
    double v = net_max(net_max(r, g), b) / 1.0;
    if (!(v >= 0.0)) return false;   // NaN
    v = std::pow(std::min(v, 1.0), 1.0);
    return (int)v == 1;
}

// buf.StandardDeviation(x, y).MaxComponent() > FireflyThreshold (= 1, Renderer.cs:48, 426):
// Variance() is black below 2 samples, else V / (N-1) (Buffer.cs:48-55); Pow(0.5) is the
// correctly rounded root, i.e. sqrt.
bool firefly_candidate(const double* V, int32_t N) {
    if (N < 2) return false;
    double r = std::sqrt(V[0] / (double)(N - 1)), g = std::sqrt(V[1] / (double)(N - 1)),
           b = std::sqrt(V[2] / (double)(N - 1));
    return net_max(net_max(r, g), b) > 1.0;
}

// IsFirefly + CalculateLocalDeviation (Renderer.cs:473-537), 3x3 window clipped to the
// image.  The reference reads the neighbours while other threads update them; here
// they come from `snap` (M at the start of the firefly phase) and the pixel's own M
// is live (`own`), which is what the pixel's own thread sees in the reference.
bool is_firefly(C s, int x, int y, int w, int h, const double* snap, const double* own) {
    double brightness = s.r * 0.2126 + s.g * 0.7152 + s.b * 0.0722;
    if (!(brightness > 0.9)) return false;
    int sx = std::max(0, x - 1), sy = std::max(0, y - 1);
    int ex = std::min(w - 1, x + 1), ey = std::min(h - 1, y + 1);
    double tr = 0, tg = 0, tb = 0;
    int count = 0;
    for (int j = sy; j <= ey; j++)
        for (int i = sx; i <= ex; i++) {
            const double* c = (i == x && j == y) ? own : snap + 3 * ((size_t)j * (size_t)w + (size_t)i);
            tr += c[0]; tg += c[1]; tb += c[2];
            count++;
        }
    double ar = tr / count, ag = tg / count, ab = tb / count;
    double dr = std::fabs(s.r - ar), dg = std::fabs(s.g - ag), db = std::fabs(s.b - ab);
    return std::sqrt(dr * dr + dg * dg + db * db) > 0.2;
}

template <class F>
void parallel_tasks(int64_t ntasks, int nthreads, F&& fn) {
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
    std::atomic<int64_t> next{0};
    auto worker = [&](int tid) {
        for (;;) {
            int64_t t = next.fetch_add(1);
            if (t >= ntasks) break;
            fn(t, tid);
        }
    };
    if (nthreads == 1) { worker(0); return; }
    std::vector<std::thread> th;
    for (int i = 0; i < nthreads; i++) th.emplace_back(worker, i);
    for (auto& t : th) t.join();
}

Scene* build_scene(const or_scene_desc* d) {
    Scene* s = new Scene();
    for (int i = 0; i < d->num_materials; i++) {
        const or_material& m = d->materials[i];
        s->mats.push_back(Material{C{m.color[0], m.color[1], m.color[2]}, m.emittance, m.index, m.gloss, m.tint,
                                   m.reflectivity, m.transparent != 0, m.texture - 1, m.normal_texture - 1,
                                   m.bump_texture - 1, m.gloss_texture - 1, m.bump_multiplier});
    }
    s->default_mat = (int)s->mats.size();   // `new Material()`: all zero
    s->mats.push_back(Material{C{0, 0, 0}, 0, 0, 0, 0, 0, false, -1, -1, -1, -1, 0});
    for (int i = 0; i < d->num_sdf_nodes; i++) {
        const or_sdf_node& n = d->sdf_nodes[i];
        SdfNode o;
        o.op = n.op;
        for (int k = 0; k < n.num_children; k++) o.kids.push_back(d->sdf_children[n.first_child + k]);
        std::memcpy(o.p, n.params, sizeof o.p);
        std::memcpy(o.M, n.matrix, sizeof o.M);
        std::memcpy(o.Inv, n.inverse, sizeof o.Inv);
        s->sdf.push_back(std::move(o));
    }
    for (int i = 0; i < d->num_sdf_shapes; i++)
        s->sdf_shapes.push_back(SdfShape{d->sdf_shapes[i].root, d->sdf_shapes[i].material, Box{vzero(), vzero()}});
    for (auto& sh : s->sdf_shapes) sh.box = sdf_box(*s, sh.root);   // SDFShape.BoundingBox = SDF.BoundingBox()
    for (int i = 0; i < d->num_volumes; i++) {
        const or_volume& v = d->volumes[i];
        Volume o;
        o.w = v.w; o.h = v.h; o.d = v.d; o.zscale = v.zscale;
        o.data.assign(v.data, v.data + (size_t)v.w * v.h * v.d);
        for (int k = 0; k < v.num_windows; k++)
            o.windows.push_back(VolWindow{v.windows[k].lo, v.windows[k].hi, v.windows[k].material});
        o.box = Box{vload(v.box_min), vload(v.box_max)};
        s->volumes.push_back(std::move(o));
    }
    for (int i = 0; i < d->num_textures; i++) {
        const or_texture& t = d->textures[i];
        s->texs.push_back(Tex{t.width, t.height, std::vector<double>(t.data, t.data + 3 * (size_t)t.width * t.height)});
    }
    s->env_tex = d->env_texture - 1;
    s->env_angle = d->env_texture_angle;
    for (int i = 0; i < d->num_spheres; i++) {
        V c = vload(d->sphere_center + 3 * i);
        double r = d->sphere_radius[i];
        // Sphere.NewSphere (Sphere.cs:27-33)
        Box b{vmk((double)c.x - r, (double)c.y - r, (double)c.z - r), vmk((double)c.x + r, (double)c.y + r, (double)c.z + r)};
        s->spheres.push_back(Sphere{c, r, d->sphere_material[i], b});
    }
    for (int i = 0; i < d->num_cubes; i++)
        s->cubes.push_back(Cube{vload(d->cube_min + 3 * i), vload(d->cube_max + 3 * i), d->cube_material[i]});
    for (int i = 0; i < d->num_planes; i++)
        s->planes.push_back(Plane{vload(d->plane_point + 3 * i), vload(d->plane_normal + 3 * i), d->plane_material[i]});
    for (int i = 0; i < d->num_triangles; i++) {
        V t1 = d->tri_t1 ? vload(d->tri_t1 + 3 * i) : vzero();
        V t2 = d->tri_t2 ? vload(d->tri_t2 + 3 * i) : vzero();
        V t3 = d->tri_t3 ? vload(d->tri_t3 + 3 * i) : vzero();
        s->tris.push_back(Tri{vload(d->tri_v1 + 3 * i), vload(d->tri_v2 + 3 * i), vload(d->tri_v3 + 3 * i),
                              vload(d->tri_n1 + 3 * i), vload(d->tri_n2 + 3 * i), vload(d->tri_n3 + 3 * i),
                              d->tri_material[i], t1, t2, t3});
    }
    for (int i = 0; i < d->num_meshes; i++) {
        s->mesh_first.push_back(d->mesh_first[i]);
        s->mesh_count.push_back(d->mesh_count[i]);
    }
    for (int i = 0; i < d->num_transformed; i++) {
        const or_transformed_shape& x = d->transformed[i];
        Xform o;
        o.kind = x.shape_kind; o.idx = x.shape_index;
        std::memcpy(o.M, x.matrix, sizeof o.M);
        std::memcpy(o.Inv, x.inverse, sizeof o.Inv);
        s->xforms.push_back(o);
    }
    for (auto& x : s->xforms) x.box = mat_box(x.M, shape_box(*s, ShapeRef{x.kind, x.idx}));  // TransformedShape.BoundingBox
    for (int i = 0; i < d->num_shapes; i++) {
        ShapeRef r{d->shape_kind[i], d->shape_index[i]};
        s->shapes.push_back(r);
        // Scene.Add (Scene.cs:29-38): MaterialAt(new Vector()).Emittance > 0; Mesh.MaterialAt is `default`.
        double em = s->mats[(size_t)material_index_at(*s, r.kind, r.idx, vzero())].emittance;
        if (em > 0) s->lights.push_back(r);
    }
    s->env = C{d->env_color[0], d->env_color[1], d->env_color[2]};
    // Scene.Compile: each Mesh builds its own tree over its triangles, then the top-level tree.
    s->mesh_trees.resize(s->mesh_first.size());
    std::vector<int> mesh_ids(s->mesh_first.size());
    for (size_t i = 0; i < mesh_ids.size(); i++) mesh_ids[i] = (int)i;
    parallel_tasks((int64_t)mesh_ids.size(), 0, [&](int64_t mi, int) {
        std::vector<ShapeRef> tri_refs;
        int f = s->mesh_first[mi], n = s->mesh_count[mi];
        for (int t = f; t < f + n; t++) tri_refs.push_back(ShapeRef{K_TRI, t});
        TreeBuilder(*s, s->mesh_trees[mi]).build(tri_refs);
    });
    TreeBuilder(*s, s->tree).build(s->shapes);
    return s;
}

}  // namespace

// ====================================================================== C API
extern "C" {

void* or_scene_create(const or_scene_desc* desc) {
    if (!desc) return nullptr;
    return build_scene(desc);
}
void or_scene_destroy(void* scene) { delete (Scene*)scene; }
int64_t or_scene_tree_nodes(void* scene) {
    Scene* s = (Scene*)scene;
    int64_t n = (int64_t)s->tree.nodes.size();
    for (auto& t : s->mesh_trees) n += (int64_t)t.nodes.size();
    return n;
}

int64_t or_render_pass(void* scene, int32_t width, int32_t height, const or_camera* cam, const or_sampler* smp,
                       const or_pass_params* pass, double* m, double* v, int32_t* n, int32_t num_threads,
                       int32_t brute_force) {
    const Scene& s = *(Scene*)scene;
    Sampler sm = make_sampler(smp);
    // RenderParallel (Renderer.cs:257-312): 256² tiles of 32² sub-tiles; here a task is one
    // 32² tile (tile id = ty*ceil(W/32)+tx), the same granularity as the reference's sub-tile task.
    int tx = (width + 31) / 32, ty = (height + 31) / 32;
    std::vector<int32_t> tiles;
    if (pass->num_tiles > 0) tiles.assign(pass->tiles, pass->tiles + pass->num_tiles);
    else { tiles.resize((size_t)tx * ty); for (int i = 0; i < tx * ty; i++) tiles[i] = i; }
    int nt = num_threads <= 0 ? (int)std::max(1u, std::thread::hardware_concurrency()) : num_threads;
    std::vector<uint64_t> rays((size_t)nt, 0);
    auto for_tiles = [&](auto&& per_pixel) {
        parallel_tasks((int64_t)tiles.size(), nt, [&](int64_t t, int tid) {
            int tile = tiles[(size_t)t];
            int x0 = (tile % tx) * 32, y0 = (tile / tx) * 32;
            Tracer tr(s, brute_force != 0);
            Integrator in(s, sm, tr);
            for (int y = y0; y < std::min(y0 + 32, (int)height); y++)
                for (int x = x0; x < std::min(x0 + 32, (int)width); x++) per_pixel(in, x, y);
            rays[(size_t)tid] += tr.rays;
        });
    };
    for_tiles([&](Integrator& in, int x, int y) { render_pixel(in, *cam, x, y, width, height, *pass, m, v, n); });
    if (pass->flags & OR_PASS_SERIAL) {
        // Renderer.Render (Renderer.cs:80-198): after a pixel's main samples, its adaptive samples
        // (:153-175) then its firefly samples (:177-191), each AddSample'd.  The decisions read the
        // pixel's own Buffer only, so this second sweep over the pixels is the same computation.
        for_tiles([&](Integrator& in, int x, int y) {
            size_t i = (size_t)y * (size_t)width + (size_t)x;
            if (pass->adaptive_samples > 0 && adaptive_serial_candidate(v + 3 * i, n[i]))
                for (int j = 0; j < pass->adaptive_samples; j++)
                    welford(m + 3 * i, v + 3 * i, n + i,
                            extra_sample(in, *cam, x, y, width, height, *pass, kAdaptiveBase + (uint32_t)j));
            if (pass->firefly_samples > 0 && firefly_candidate(v + 3 * i, n[i]))
                for (int j = 0; j < pass->firefly_samples; j++)
                    welford(m + 3 * i, v + 3 * i, n + i,
                            serial_firefly_sample(in, *cam, x, y, width, height, *pass, kFireflyBase + (uint32_t)j));
        });
    } else if (pass->adaptive_samples > 0) {
        // Adaptive phase (Renderer.cs:340-410): every pixel gets AdaptiveSamples
        // individual AddSample calls.  The second loop only feeds pixelVariances,
        // which nothing reads, so it is not traced.
        for_tiles([&](Integrator& in, int x, int y) {
            size_t i = (size_t)y * (size_t)width + (size_t)x;
            for (int j = 0; j < pass->adaptive_samples; j++)
                welford(m + 3 * i, v + 3 * i, n + i,
                        extra_sample(in, *cam, x, y, width, height, *pass, kAdaptiveBase + (uint32_t)j));
        });
    }
    if (!(pass->flags & OR_PASS_SERIAL) && pass->firefly_samples > 0) {
        // Firefly phase (Renderer.cs:412-470).  skippedPixels is created empty per call
        // and each pixel is visited once, so only its first branch is reachable.
        std::vector<double> snap(m, m + 3 * (size_t)width * (size_t)height);
        for_tiles([&](Integrator& in, int x, int y) {
            size_t i = (size_t)y * (size_t)width + (size_t)x;
            if (!firefly_candidate(v + 3 * i, n[i])) return;
            for (int j = 0; j < pass->firefly_samples; j++) {
                C smp = extra_sample(in, *cam, x, y, width, height, *pass, kFireflyBase + (uint32_t)j);
                if (is_firefly(smp, x, y, width, height, snap.data(), m + 3 * i)) break;
                welford(m + 3 * i, v + 3 * i, n + i, smp);
            }
        });
    }
    uint64_t total = 0;
    for (uint64_t r : rays) total += r;
    return (int64_t)total;
}

int64_t or_render_pixels(void* scene, int32_t width, int32_t height, const or_camera* cam, const or_sampler* smp,
                         const or_pass_params* pass, int64_t pix_begin, int64_t pix_end, int64_t pix_stride,
                         double* m, double* v, int32_t* n, int32_t num_threads) {
    const Scene& s = *(Scene*)scene;
    Sampler sm = make_sampler(smp);
    if (pix_stride <= 0) pix_stride = 1;
    int64_t count = (pix_end - pix_begin + pix_stride - 1) / pix_stride;
    const int64_t chunk = 64;
    int nt = num_threads <= 0 ? (int)std::max(1u, std::thread::hardware_concurrency()) : num_threads;
    std::vector<uint64_t> rays((size_t)nt, 0);
    parallel_tasks((count + chunk - 1) / chunk, nt, [&](int64_t t, int tid) {
        Tracer tr(s, false);
        Integrator in(s, sm, tr);
        for (int64_t k = t * chunk; k < std::min(count, (t + 1) * chunk); k++) {
            int64_t pix = pix_begin + k * pix_stride;
            render_pixel(in, *cam, (int)(pix % width), (int)(pix / width), width, height, *pass, m, v, n);
        }
        rays[(size_t)tid] += tr.rays;
    });
    uint64_t total = 0;
    for (uint64_t r : rays) total += r;
    return (int64_t)total;
}

double or_intersect(void* scene, const float origin[3], const float dir[3], int32_t brute_force, int32_t* out_kind,
                    int32_t* out_index) {
    const Scene& s = *(Scene*)scene;
    Tracer tr(s, brute_force != 0);
    Hit h = tr.intersect(Ray{vload(origin), vload(dir)});
    if (out_kind) *out_kind = h.kind;
    if (out_index) *out_index = h.idx;
    return h.t;
}

int32_t or_hit_info(void* scene, const float origin[3], const float dir[3], float out_pos[3], float out_normal[3],
                    int32_t* out_inside, int32_t* out_mat) {
    const Scene& s = *(Scene*)scene;
    Tracer tr(s, false);
    Ray r{vload(origin), vload(dir)};
    Hit h = tr.intersect(r);
    if (!(h.t < HIT_INF)) return 0;
    HitInfo info = hit_info(s, h, r);
    out_pos[0] = info.position.x; out_pos[1] = info.position.y; out_pos[2] = info.position.z;
    out_normal[0] = info.normal.x; out_normal[1] = info.normal.y; out_normal[2] = info.normal.z;
    *out_inside = info.inside ? 1 : 0;
    *out_mat = info.mat;
    return 1;
}

void or_cast_ray(const or_camera* cam, int32_t x, int32_t y, int32_t w, int32_t h, double u, double v, uint64_t key,
                 float out_origin[3], float out_dir[3]) {
    Ray r = cast_ray(*cam, x, y, w, h, u, v, key);
    out_origin[0] = r.o.x; out_origin[1] = r.o.y; out_origin[2] = r.o.z;
    out_dir[0] = r.d.x; out_dir[1] = r.d.y; out_dir[2] = r.d.z;
}

double or_prim_intersect(int32_t kind, const float* a, const float* b, const float* c, double radius,
                         const float origin[3], const float dir[3]) {
    Ray r{vload(origin), vload(dir)};
    switch (kind) {
        case K_SPHERE: return sphere_t(vload(a), radius, r);
        case K_CUBE: return cube_t(vload(a), vload(b), r);
        case K_PLANE: return plane_t(vload(a), vload(b), r);
        default: return tri_t(vload(a), vload(b), vload(c), r);
    }
}

void or_prim_normal(int32_t kind, const float* a, const float* b, const float* c, const float* n1, const float* n2,
                    const float* n3, const float pos[3], float out_normal[3]) {
    V p = vload(pos), n;
    switch (kind) {
        case K_SPHERE: n = vnorm(vsub(p, vload(a))); break;
        case K_CUBE: n = cube_normal(vload(a), vload(b), p); break;
        case K_PLANE: n = vload(b); break;
        default: {
            Tri t{vload(a), vload(b), vload(c), vload(n1), vload(n2), vload(n3), 0, vzero(), vzero(), vzero()};
            n = tri_normal(t, p);
        }
    }
    out_normal[0] = n.x; out_normal[1] = n.y; out_normal[2] = n.z;
}

int32_t or_bounce(void* scene, const float origin[3], const float dir[3], double u, double v, int32_t btype,
                  uint64_t key, float out_origin[3], float out_dir[3], int32_t* out_reflected, double* out_p) {
    const Scene& s = *(Scene*)scene;
    Tracer tr(s, false);
    Ray r{vload(origin), vload(dir)};
    Hit h = tr.intersect(r);
    if (!(h.t < HIT_INF)) return 0;
    HitInfo info = hit_info(s, h, r);
    Sampler smp{1, 0, true, true, 0, 0};
    Integrator in(s, smp, tr);
    bool reflected;
    double p;
    Ray o = in.bounce(r, info, u, v, btype, key, reflected, p);
    out_origin[0] = o.o.x; out_origin[1] = o.o.y; out_origin[2] = o.o.z;
    out_dir[0] = o.d.x; out_dir[1] = o.d.y; out_dir[2] = o.d.z;
    *out_reflected = reflected ? 1 : 0;
    *out_p = p;
    return 1;
}

void or_cone(const float dir[3], double theta, double u, double v, uint64_t key, float out[3]) {
    Scene s;
    Tracer tr(s, true);
    Sampler smp{1, 0, true, true, 0, 0};
    Integrator in(s, smp, tr);
    V d = in.cone(vload(dir), theta, u, v, key);
    out[0] = d.x; out[1] = d.y; out[2] = d.z;
}

int32_t or_lights(void* scene, int32_t* kinds, int32_t* indices, int32_t cap) {
    const Scene& s = *(Scene*)scene;
    for (int32_t i = 0; i < (int32_t)s.lights.size() && i < cap; i++) {
        kinds[i] = s.lights[(size_t)i].kind;
        indices[i] = s.lights[(size_t)i].idx;
    }
    return (int32_t)s.lights.size();
}

int64_t or_sample_light(void* scene, const float origin[3], const float normal[3], int32_t light, uint64_t key,
                        int32_t soft_shadows, double out[3]) {
    const Scene& s = *(Scene*)scene;
    Tracer tr(s, false);
    Sampler smp{1, 0, true, soft_shadows != 0, 0, 0};
    Integrator in(s, smp, tr);
    C c = in.sample_light(Ray{vload(origin), vload(normal)}, s.lights[(size_t)light], key);
    out[0] = c.r; out[1] = c.g; out[2] = c.b;
    return (int64_t)tr.rays;
}

int64_t or_sample_lights(void* scene, const float origin[3], const float normal[3], uint64_t key, int32_t light_mode,
                         int32_t soft_shadows, double out[3]) {
    const Scene& s = *(Scene*)scene;
    Tracer tr(s, false);
    Sampler smp{1, 0, true, soft_shadows != 0, light_mode, 0};
    Integrator in(s, smp, tr);
    C c = in.sample_lights(Ray{vload(origin), vload(normal)}, key);
    out[0] = c.r; out[1] = c.g; out[2] = c.b;
    return (int64_t)tr.rays;
}

int32_t or_any_nearer(void* scene, const float origin[3], const float dir[3], double t_light) {
    const Scene& s = *(Scene*)scene;
    Tracer tr(s, true);
    const Ray r{vload(origin), vload(dir)};
    for (const ShapeRef& sh : s.shapes)
        if (tr.shape_intersect(sh, r).t < t_light) return 1;
    return 0;
}

void or_texture_sample(void* scene, int32_t texture, int32_t kind, double u, double v, double out[3]) {
    const Scene& s = *(Scene*)scene;
    const Tex& t = s.texs[(size_t)(texture - 1)];
    if (kind == 0) {
        C c = tex_sample(t, u, v);
        out[0] = c.r; out[1] = c.g; out[2] = c.b;
        return;
    }
    V r = kind == 1 ? tex_normal_sample(t, u, v) : tex_bump_sample(t, u, v);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

void or_shape_uv(void* scene, int32_t kind, int32_t index, const float p[3], float out_uv[3]) {
    V r = shape_uv(*(Scene*)scene, kind, index, vload(p));
    out_uv[0] = r.x; out_uv[1] = r.y; out_uv[2] = r.z;
}

void or_environment(void* scene, const float dir[3], double out[3]) {
    const Scene& s = *(Scene*)scene;
    Tracer tr(s, false);
    Sampler sm{1, 0, false, false, 0, 0};
    Integrator in(s, sm, tr);
    C c = in.sample_environment(Ray{vzero(), vload(dir)});
    out[0] = c.r; out[1] = c.g; out[2] = c.b;
}

int32_t or_hit_surface(void* scene, const float origin[3], const float dir[3], double out_color[3], double* out_gloss) {
    const Scene& s = *(Scene*)scene;
    Tracer tr(s, false);
    Ray r{vload(origin), vload(dir)};
    Hit h = tr.intersect(r);
    if (!(h.t < HIT_INF)) return 0;
    HitInfo info = hit_info(s, h, r);
    out_color[0] = info.color.r; out_color[1] = info.color.g; out_color[2] = info.color.b;
    *out_gloss = info.gloss;
    return 1;
}

double or_sdf_evaluate(void* scene, int32_t node, const float p[3]) { return sdf_eval(*(Scene*)scene, node, vload(p)); }

double or_volume_sample(void* scene, int32_t volume, double x, double y, double z) {
    return vol_sample(((Scene*)scene)->volumes[(size_t)volume], x, y, z);
}

void or_shape_box(void* scene, int32_t kind, int32_t index, float out_min[3], float out_max[3]) {
    Box b = shape_box(*(Scene*)scene, ShapeRef{kind, index});
    out_min[0] = b.min.x; out_min[1] = b.min.y; out_min[2] = b.min.z;
    out_max[0] = b.max.x; out_max[1] = b.max.y; out_max[2] = b.max.z;
}

uint64_t or_camera_key(uint64_t seed, uint32_t pass, uint64_t pixel, uint32_t sample) {
    return camera_key(seed, pass, pixel, sample);
}
uint64_t or_child_key(uint64_t key, uint32_t child) { return child_key(key, child); }
uint64_t or_light_key(uint64_t key, uint32_t light) { return light_key(key, light); }
double or_draw(uint64_t key, uint32_t dim) { return draw(key, dim); }

}  // extern "C"
