// pt_math.h — numeric core of the render path, shared by the gfx950 kernels and
// the host-side scene preparation.
//
// PTSharp's Vector keeps a System.Numerics.Vector3 (fp32) behind double
// accessors (PTSharpCore/Vector.cs:201-234): Add/Sub/Mul/Div round to fp32 after
// every operation, MulScalar(double) is float(double(x)*s) (Vector.cs:435), and
// Dot/Cross/Length/Normalize are fp32 Vector3 operations (Vector.cs:356-393).
// Scalars that the reference keeps in double (ray t, det, Fresnel terms, trig)
// stay double here so hit positions and branch decisions reproduce the same
// rounding sequence.  Everything is compiled with -ffp-contract=off.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define PT_HD __host__ __device__ __forceinline__
#else
#define PT_HD inline
#endif
// A pointer into hipMalloc memory, as a global-segment pointer in device code: its loads are global_load,
// not the flat_load the compiler must use for a generic pointer (a flat load also waits on the LDS
// counter); the plain pointer elsewhere.
#if defined(__HIP_DEVICE_COMPILE__)
#define PT_GLOBAL(T) const __attribute__((address_space(1))) T*
#else
#define PT_GLOBAL(T) const T*
#endif

#pragma clang fp contract(off)

namespace pt {

constexpr double kEps = 1e-9;                 // Util.EPS (Util.cs:11)
constexpr double kHitInf = 1000000000.0;      // Hit.INF = 1e9F (Hit.cs:6)
constexpr double kPi = 3.14159265358979323846;

struct v3 { float x, y, z; };

PT_HD v3 mk(double x, double y, double z) { return v3{(float)x, (float)y, (float)z}; }
PT_HD v3 add(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PT_HD v3 sub(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PT_HD v3 mul(v3 a, v3 b) { return v3{a.x * b.x, a.y * b.y, a.z * b.z}; }
PT_HD v3 divv(v3 a, v3 b) { return v3{a.x / b.x, a.y / b.y, a.z / b.z}; }
PT_HD v3 muls(v3 a, double s) {
    return v3{(float)((double)a.x * s), (float)((double)a.y * s), (float)((double)a.z * s)};
}
PT_HD float dotf(v3 a, v3 b) {
    float xx = a.x * b.x;
    float yy = a.y * b.y;
    float zz = a.z * b.z;
    float s = xx + yy;
    return s + zz;
}
PT_HD double dot(v3 a, v3 b) { return (double)dotf(a, b); }
PT_HD v3 cross(v3 a, v3 b) {
    float x1 = a.y * b.z, x2 = a.z * b.y;
    float y1 = a.z * b.x, y2 = a.x * b.z;
    float z1 = a.x * b.y, z2 = a.y * b.x;
    return v3{x1 - x2, y1 - y2, z1 - z2};
}
PT_HD float lengthf(v3 a) { return sqrtf(dotf(a, a)); }
PT_HD v3 normalize(v3 a) {
    float l = lengthf(a);
    return v3{a.x / l, a.y / l, a.z / l};
}
PT_HD v3 neg(v3 a) { return v3{-a.x, -a.y, -a.z}; }
PT_HD v3 zero3() { return v3{0.f, 0.f, 0.f}; }

// .NET Math.Max / Math.Min on double (NaN-propagating, -0 < +0).
PT_HD double net_max(double a, double b) {
    if (a != b) { if (!(a != a)) return b < a ? a : b; return a; }
    return signbit(b) ? a : b;
}
PT_HD double net_min(double a, double b) {
    if (a != b) { if (!(a != a)) return a < b ? a : b; return a; }
    return signbit(a) ? a : b;
}
PT_HD v3 vmin(v3 a, v3 b) { return mk(net_min(a.x, b.x), net_min(a.y, b.y), net_min(a.z, b.z)); }
PT_HD v3 vmax(v3 a, v3 b) { return mk(net_max(a.x, b.x), net_max(a.y, b.y), net_max(a.z, b.z)); }

// ------------------------------------------------------------------ RNG
// Counter-based replacement for Random.Shared.  A draw is a
// pure function of (key, dim), so the GPU's iterative path order and the
// recursive CPU order consume identical numbers.
PT_HD uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}
PT_HD uint64_t camera_key(uint64_t seed, uint32_t pass, uint64_t pixel, uint32_t sample) {
    uint64_t k = mix64(seed + 0x243F6A8885A308D3ull);
    k = mix64(k ^ ((uint64_t)pass + 0x13198A2E03707344ull));
    k = mix64(k ^ (pixel + 0xA4093822299F31D0ull));
    return mix64(k ^ ((uint64_t)sample + 0x082EFA98EC4E6C89ull));
}
// Sample-index domains of camera_key: the main loop uses 0..spp-1, the adaptive
// and firefly phases (Renderer.cs:340-470) their own ranges.
constexpr uint32_t kAdaptiveSampleBase = 0x40000000u;
constexpr uint32_t kFireflySampleBase = 0x80000000u;
PT_HD uint64_t child_key(uint64_t k, uint32_t c) { return mix64(k ^ ((uint64_t)c + 0x452821E638D01377ull)); }
PT_HD uint64_t light_key(uint64_t k, uint32_t i) { return mix64(k ^ ((uint64_t)i + 0xBE5466CF34E90C6Cull)); }
PT_HD double draw(uint64_t k, uint32_t dim) {
    return (double)(mix64(k + (uint64_t)(dim + 1) * 0x9E3779B97F4A7C15ull) >> 11) * (1.0 / 9007199254740992.0);
}
// x / n for the sampler's stratum counts (n = FirstHitSamples' square root or its square, >= 1): when n
// is a power of two its reciprocal is exact, and x · (1/n) is the same correctly rounded value as x / n
// (fp64 division is a ~10-instruction sequence at the fp64 rate; C2's 16 children per camera hit
// take two each).  strata_recip gives 1/n, or 0 for other n (then div_strata divides).
PT_HD double strata_recip(int n) { return n > 0 && (n & (n - 1)) == 0 ? ldexp(1.0, -__builtin_ctz((unsigned)n)) : 0.0; }
PT_HD double div_strata(double x, int n, double rn) { return rn != 0.0 ? x * rn : x / (double)n; }
enum : uint32_t { D_STRATUM_U = 0, D_STRATUM_V = 1, D_REFLECT = 2, D_RUV_Z = 3, D_RUV_A = 4,
                  D_LIGHT = 5, D_SS_RUV_Z = 6, D_SS_RUV_A = 7, D_SS_XY = 8 };
enum : uint32_t { D_JX = 0, D_JY = 1, D_LENS_ANGLE = 2, D_LENS_RADIUS = 3 };

// PT_DEVICE_SINCOS: the device's reduction and kernels on the host too (tools/sincos_flip_rate.cpp
// compares them with glibc's sin and cos at the call sites).
#if defined(__HIP_DEVICE_COMPILE__) || defined(PT_DEVICE_SINCOS)
// fdlibm's __kernel_sin / __kernel_cos (k_sin.c, k_cos.c: degree-13 / -14 minimax on
// [-π/4, π/4]) on the reduced argument y0 + y1.
PT_HD void sincos_kernel(double x, double y, double& s, double& c) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x, w = z * z, v = z * x;
    const double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    s = x - ((z * (0.5 * y - v * r) - y) - v * S1);
    const double rc = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    const double hz = 0.5 * z, ww = 1.0 - hz;
    c = ww + (((1.0 - ww) - hz) + (z * rc - x * y));
}
#endif
// sin and cos of one fp64 argument.  Every caller's argument lies in [0, 2π] (2π·draw, or a
// cone angle below the material's gloss), so the device reduces by π/2 in double-double —
// k·(π/2)_hi with its exact fma error, r = x − k·hi exact by Sterbenz — and evaluates the
// fdlibm kernels: within 1 ulp of glibc's sin / cos, and the fp32 vectors the reference builds
// from them (r·sin, r·cos rounded to float) identical on 2·10^7 sampled arguments
// (tools/check_sincos.cpp, removed in 188afd0; its successor tools/sincos_flip_rate.cpp covers random
// radii and the call sites' float expressions, profiles/r03_sincos_flip_rate.txt).  It replaces the general library routine, whose large-argument
// path alone took the shade kernel from 11 to 34 spilled VGPRs.  No large-argument path here:
// the reduction stays accurate to ~1e-29 absolute for |x| up to ~1e4, far beyond any caller.
PT_HD void pt_sincos(double x, double* s, double* c) {
#if (defined(__HIP_DEVICE_COMPILE__) || defined(PT_DEVICE_SINCOS)) && !defined(PT_LIB_SINCOS)
    const double hi = 1.5707963267948966, lo = 6.123233995736766e-17, two_over_pi = 0.63661977236758134;
    const double k = rint(x * two_over_pi);
    const double ph = k * hi;
    const double pe = fma(k, hi, -ph);
    const double r = x - ph;
    const double cc = pe + k * lo;
    const double y0 = r - cc, y1 = (r - y0) - cc;
    double ks, kc;
    sincos_kernel(y0, y1, ks, kc);
    const int q = (int)k & 3;
    double so = (q & 1) ? kc : ks, co = (q & 1) ? ks : kc;
    if (q == 1 || q == 2) co = -co;
    if (q >= 2) so = -so;
    *s = so; *c = co;
#else
    sincos(x, s, c);
#endif
}
// Vector.RandomUnitVector (Vector.cs:339-347)
PT_HD v3 random_unit_vector(uint64_t key, uint32_t dz, uint32_t da) {
    double z = draw(key, dz) * 2.0 - 1.0;
    double a = draw(key, da) * 2.0 * kPi;
    double r = sqrt(1.0 - z * z);
    double x, y;
    pt_sincos(a, &x, &y);
    return mk(r * x, r * y, z);
}
// Vector.Reflect / Refract / Reflectance with `this` = the surface normal (Vector.cs:497-536)
PT_HD v3 reflect(v3 n, v3 i) { return sub(i, muls(n, 2 * dot(n, i))); }
PT_HD v3 refract(v3 n, v3 i, double n1, double n2) {
    double nr = n1 / n2;
    double cosI = -dot(n, i);
    double sinT2 = nr * nr * (1 - cosI * cosI);
    if (sinT2 > 1) return zero3();
    double cosT = sqrt(1 - sinT2);
    return add(muls(i, nr), muls(n, nr * cosI - cosT));
}
PT_HD double reflectance(v3 n, v3 i, double n1, double n2) {
    double nr2 = (n1 * n1) / (n2 * n2);
    double cosI = -dot(n, i);
    double sinT2 = nr2 * (1 - cosI * cosI);
    if (sinT2 > 1) return 1;
    double cosT = sqrt(1 - sinT2);
    double cosI_n1 = n1 * cosI;
    double cosT_n2 = n2 * cosT;
    double rOrth = (cosI_n1 - cosT_n2) / (cosI_n1 + cosT_n2);
    double rPar = (cosT_n2 - cosI_n1) / (cosT_n2 + cosI_n1);
    return (rOrth * rOrth + rPar * rPar) / 2;
}

// ------------------------------------------------------------------ primitives
// Sphere.Intersect (Sphere.cs:40-60)
PT_HD double isect_sphere(v3 center, double radius, v3 o, v3 d) {
    v3 to = sub(o, center);
    double b = dot(to, d);
    double c = dot(to, to) - radius * radius;
    double disc = b * b - c;
    if (disc > 0) {
        disc = sqrt(disc);
        double t1 = -b - disc;
        if (t1 > kEps) return t1;
        double t2 = -b + disc;
        if (t2 > kEps) return t2;
    }
    return kHitInf;
}
// Cube.Intersect (Cube.cs:35-47): entry face only.
PT_HD double isect_cube(v3 mn, v3 mx, v3 o, v3 d) {
    v3 n = divv(sub(mn, o), d);
    v3 f = divv(sub(mx, o), d);
    v3 n2 = vmin(n, f), f2 = vmax(n, f);
    double t0 = net_max(net_max(n2.x, n2.y), n2.z);
    double t1 = net_min(net_min(f2.x, f2.y), f2.z);
    if (t0 > 0 && t0 < t1) return t0;
    return kHitInf;
}
// Plane.Intersect (Plane.cs:36-50)
PT_HD double isect_plane(v3 point, v3 normal, v3 o, v3 d) {
    double dd = dot(normal, d);
    if (fabs(dd) < kEps) return kHitInf;
    v3 a = sub(point, o);
    double t = dot(a, normal) / dd;
    if (t < kEps) return kHitInf;
    return t;
}
// Triangle.Intersect, Möller–Trumbore (Triangle.cs:95-124) on precomputed
// e1 = V2-V1, e2 = V3-V1 (bit-identical to the per-call Sub in the reference).
PT_HD double isect_tri(v3 v1, v3 e1, v3 e2, v3 o, v3 d) {
    v3 h = cross(d, e2);
    const float det = dotf(e1, h);
    if ((double)det > -kEps && (double)det < kEps) return kHitInf;
    // det, u·det, v·det and t·det are fp32 dot products, so most rejections are
    // decided here, before the fp64 division: a sign test is exact (the fp64
    // product of nonzero finite values never rounds to 0), and "> 1" is only
    // taken with a 1e-4 margin, far beyond the fp64 products' 2^-52 error.  Every
    // triangle not rejected here takes the reference's own fp64 sequence below.
    v3 s = sub(o, v1);
    const float a = dotf(s, h), ad = fabsf(det), lim = ad * 1.0001f;
    const bool neg = det < 0;
    const float as = neg ? -a : a;
    if (as < 0 || as > lim) return kHitInf;           // u < 0 or u > 1
    v3 q = cross(s, e1);
    const float b = dotf(d, q), c = dotf(e2, q);
    const float bs = neg ? -b : b, cs = neg ? -c : c;
    if (bs < 0 || as + bs > lim || cs < 0) return kHitInf;  // v < 0, u + v > 1, t < 0
    double invDet = 1.0 / det;
    double u = (double)a * invDet;
    if (u < 0 || u > 1) return kHitInf;
    double v = (double)b * invDet;
    if (v < 0 || (u + v) > 1) return kHitInf;
    double t = (double)c * invDet;
    if (t < kEps) return kHitInf;
    return t;
}
// Cube.NormalAt (Cube.cs:57-69) with the |p - face| < EPS quirk.
PT_HD v3 cube_normal(v3 mn, v3 mx, v3 p) {
    if (fabs((double)p.x - (double)mn.x) < kEps) return mk(-1, 0, 0);
    if (fabs((double)p.x - (double)mx.x) < kEps) return mk(1, 0, 0);
    if (fabs((double)p.y - (double)mn.y) < kEps) return mk(0, -1, 0);
    if (fabs((double)p.y - (double)mx.y) < kEps) return mk(0, 1, 0);
    if (fabs((double)p.z - (double)mn.z) < kEps) return mk(0, 0, -1);
    if (fabs((double)p.z - (double)mx.z) < kEps) return mk(0, 0, 1);
    return mk(0, 1, 0);
}
// Triangle.Barycentric (Triangle.cs:208-223) with e1 = V2-V1, e2 = V3-V1.
PT_HD void barycentric(v3 v1, v3 e1, v3 e2, v3 p, double& bu, double& bv, double& bw) {
    v3 w2 = sub(p, v1);
    double d00 = dot(e1, e1);
    double d01 = dot(e1, e2);
    double d11 = dot(e2, e2);
    double d20 = dot(w2, e1);
    double d21 = dot(w2, e2);
    double den = d00 * d11 - d01 * d01;
    bv = (d11 * d20 - d01 * d21) / den;
    bw = (d00 * d21 - d01 * d20) / den;
    bu = 1 - bv - bw;
}
// Triangle.NormalAt without maps (Triangle.cs:142-145, 186-188).
PT_HD v3 tri_normal(v3 v1, v3 e1, v3 e2, v3 n1, v3 n2, v3 n3, v3 p) {
    double bu, bv, bw;
    barycentric(v1, e1, e2, p, bu, bv, bw);
    v3 n = add(add(muls(n1, bu), muls(n2, bv)), muls(n3, bw));
    return normalize(n);
}

}  // namespace pt
