// pt_ext.h — §8f row 4 shapes on the render path: SDFShape (SDF.cs), Volume
// (Volume.cs) and TransformedShape (TransformedShape.cs).
//
// Layout in HBM (pt_api.hip builds it):
//   SDF trees are compiled on the host into one postfix program per SDFShape: point-
//   stack pushes for TransformSDF / ScaleSDF / RepeatSDF, a leaf op per primitive SDF
//   and a binary fold per Union / Difference / Intersection child, so the device
//   evaluates SDF.Evaluate's recursion with two small stacks and no calls.
//   Volumes keep the C# voxel grid (fp64 Data[x + y*W + z*W*H]) and windows.
//   A TransformedShape holds Matrix (3 rows) and Inverse (3 rows) in fp64 and points
//   at an object-space record of its inner shape (the analytic-record format).
//
// Every function restates its reference lines with the same fp32 Vector / fp64
// scalar rounding sequence (pt_math.h); host and device share them (PT_HD).
#pragma once
#include <stdint.h>

#include "pt_math.h"

#pragma clang fp contract(off)

namespace pt {

enum SdfOp : int32_t {
    SDF_LEAF_SPHERE = 0, SDF_LEAF_CUBE, SDF_LEAF_CYLINDER, SDF_LEAF_CAPSULE, SDF_LEAF_TORUS,
    SDF_PUSH_TRANSFORM,   // point ← Inverse.MulPosition(point)          (TransformSDF, SDF.cs:338-342)
    SDF_PUSH_SCALE,       // point ← point.DivScalar(Factor)             (ScaleSDF, SDF.cs:369-372)
    SDF_PUSH_REPEAT,      // point ← point.Mod(Step).Sub(Step / 2)       (RepeatSDF, SDF.cs:549-553)
    SDF_POP_POINT,
    SDF_MUL,              // value ← value · Factor                      (ScaleSDF)
    SDF_UNION,            // fold: d < result ? d : result               (SDF.cs:398-411)
    SDF_DIFFERENCE,       // fold: -d > result ? -d : result             (SDF.cs:451-468)
    SDF_INTERSECTION,     // fold: d > result ? d : result               (SDF.cs:493-507)
    SDF_CONST0            // an empty Union / Difference / Intersection returns 0
};
constexpr int kSdfStack = 8;   // point / value stack depth of a compiled program (host-checked)

struct DevSdfIns {
    int32_t op;
    int32_t param;   // offset into sdf_params (doubles)
};
struct DevSdfShape {
    int32_t begin, len;   // program range
    int32_t mat;
    int32_t chain;        // 1: one leaf under point ops and value scalings only (no fold): sdf_eval_chain
    float bmin[3], bmax[3];   // SDFShape.BoundingBox (SDF.BoundingBox of the root)
};
struct DevWindow {
    double lo, hi;
    int32_t mat, _pad;
};
struct DevVolume {
    const double* data;   // [d][h][w]
    const DevWindow* windows;
    int32_t w, h, d, nwin;
    double zscale;
    double zinv;          // RN(1 / zscale) for vol_zdiv; 0: divide (host views, a zscale without a normal reciprocal)
    float bmin[3], bmax[3];
    // Uniform cells (vol_build_runs): per cell (x0, y0, z0) of Sample's lattice, indices -1..w-1
    // etc., the Sign every sample inside it has (1 or nwin + 1), or 0 when it cannot be vouched
    // for; null: no skipping.  zero_sign: the Sign of a cell with every corner outside the grid.
    const int8_t* runs;
    int32_t zero_sign, _pad;
    // The eight corners of every cell of the runs table's lattice, cell-major (vol_build_cells: 64 B per cell,
    // v000 v001 v010 v011 v100 v101 v110 v111, Volume.Get's values), so a march position's corners are one
    // half-line read instead of eight reads on four lines; null: read data.
    const double* cells;
};
constexpr size_t kVolLdsHeader = 128;   // a DevVolume staged in LDS (pt_wavefront.hip stage_vol), padded
struct DevBlas {          // object-space BVH4 of a mesh instanced by TransformedShape
    int32_t node_off;     // first node in blas_nodes
    int32_t num_nodes;
    int32_t rec_off;      // first triangle in blas_recs / blas_shade / blas_uv
    int32_t _pad;
};
struct DevXform {
    double m[12];     // Matrix rows 1-3 (row 4 is 0 0 0 1 for affine transforms; MulPosition ignores it)
    double inv[12];   // Inverse rows 1-3
    int32_t kind;     // inner shape kind (KIND_SPHERE, KIND_CUBE, KIND_PLANE, KIND_SDF, KIND_VOLUME, KIND_MESH)
    int32_t rec;      // its record in ext_recs (analytic-record format); KIND_MESH: its DevBlas
};

// ---------------------------------------------------------------- Matrix (Matrix.cs)
// MulPosition (Matrix.cs:134-141): fp64 rows, then a Vector (fp32).
PT_HD v3 mat_position(const double* m, v3 b) {
    double x = m[0] * b.x + m[1] * b.y + m[2] * b.z + m[3];
    double y = m[4] * b.x + m[5] * b.y + m[6] * b.z + m[7];
    double z = m[8] * b.x + m[9] * b.y + m[10] * b.z + m[11];
    return mk(x, y, z);
}
// MulDirection (Matrix.cs:144-150), normalised
PT_HD v3 mat_direction(const double* m, v3 b) {
    double x = m[0] * b.x + m[1] * b.y + m[2] * b.z;
    double y = m[4] * b.x + m[5] * b.y + m[6] * b.z;
    double z = m[8] * b.x + m[9] * b.y + m[10] * b.z;
    return normalize(mk(x, y, z));
}
// Transpose().MulDirection (Matrix.cs:176, 144-150) on the 3x3 part
PT_HD v3 mat_direction_t(const double* m, v3 b) {
    double x = m[0] * b.x + m[4] * b.y + m[8] * b.z;
    double y = m[1] * b.x + m[5] * b.y + m[9] * b.z;
    double z = m[2] * b.x + m[6] * b.y + m[10] * b.z;
    return normalize(mk(x, y, z));
}
// MulBox (Matrix.cs:156-173)
PT_HD void mat_box(const double* m, v3 mn, v3 mx, v3& omn, v3& omx) {
    v3 r = mk(m[0], m[4], m[8]), u = mk(m[1], m[5], m[9]), b = mk(m[2], m[6], m[10]), t = mk(m[3], m[7], m[11]);
    v3 xa = muls(r, mn.x), xb = muls(r, mx.x), ya = muls(u, mn.y), yb = muls(u, mx.y), za = muls(b, mn.z),
       zb = muls(b, mx.z);
    omn = add(add(add(vmin(xa, xb), vmin(ya, yb)), vmin(za, zb)), t);
    omx = add(add(add(vmax(xa, xb), vmax(ya, yb)), vmax(za, zb)), t);
}
// Box.Intersect (Box.cs:72-94), fp64
PT_HD void box_span(const float* mn, const float* mx, v3 o, v3 d, double& tmin, double& tmax) {
    double x1 = ((double)mn[0] - (double)o.x) / (double)d.x, y1 = ((double)mn[1] - (double)o.y) / (double)d.y;
    double z1 = ((double)mn[2] - (double)o.z) / (double)d.z;
    double x2 = ((double)mx[0] - (double)o.x) / (double)d.x, y2 = ((double)mx[1] - (double)o.y) / (double)d.y;
    double z2 = ((double)mx[2] - (double)o.z) / (double)d.z;
    if (x1 > x2) { double t = x1; x1 = x2; x2 = t; }
    if (y1 > y2) { double t = y1; y1 = y2; y2 = t; }
    if (z1 > z2) { double t = z1; z1 = z2; z2 = t; }
    tmin = net_max(net_max(x1, y1), z1);
    tmax = net_min(net_min(x2, y2), z2);
}

// ---------------------------------------------------------------- SDF leaves (SDF.cs)
// Vector.LengthN (Vector.cs:359-367)
PT_HD double length_n(v3 a, double n) {
    if (n == 2) return (double)lengthf(a);
    const double x = fabs((double)a.x), y = fabs((double)a.y), z = fabs((double)a.z);   // Abs (Vector.cs:402-405)
    return pow(pow(x, n) + pow(y, n) + pow(z, n), 1 / n);
}
PT_HD double sdf_leaf(int op, const double* P, v3 p) {
    switch (op) {
        case SDF_LEAF_SPHERE: return length_n(p, P[1]) - P[0];   // SDF.cs:131-134
        case SDF_LEAF_CUBE: {                                     // SDF.cs:157-189
            double x = p.x, y = p.y, z = p.z;
            if (x < 0) x = -x;
            if (y < 0) y = -y;
            if (z < 0) z = -z;
            x -= P[0] / 2;
            y -= P[1] / 2;
            z -= P[2] / 2;
            double a = x;
            if (y > a) a = y;
            if (z > a) a = z;
            if (a > 0) a = 0;
            if (x < 0) x = 0;
            if (y < 0) y = 0;
            if (z < 0) z = 0;
            return a + sqrt(x * x + y * y + z * z);
        }
        case SDF_LEAF_CYLINDER: {                                 // SDF.cs:226-251
            double x = sqrt((double)p.x * p.x + (double)p.z * p.z);
            double y = p.y;
            if (x < 0) x = -x;
            if (y < 0) y = -y;
            x -= P[0];
            y -= P[1] / 2;
            double a = x;
            if (y > a) a = y;
            if (a > 0) a = 0;
            if (x < 0) x = 0;
            if (y < 0) y = 0;
            return a + sqrt(x * x + y * y);
        }
        case SDF_LEAF_CAPSULE: {                                  // SDF.cs:273-279
            v3 A = mk(P[0], P[1], P[2]), B = mk(P[3], P[4], P[5]);
            v3 pa = sub(p, A), ba = sub(B, A);
            double h = net_max(0, net_min(1, dot(pa, ba) / dot(ba, ba)));
            return length_n(sub(pa, muls(ba, h)), P[7]) - P[6];
        }
        default: {                                                // SDF_LEAF_TORUS, SDF.cs:307-311
            v3 q = mk(length_n(v3{p.x, p.y, 0.f}, P[2]) - P[0], p.z, 0);
            return length_n(q, P[3]) - P[1];
        }
    }
}

// SDF.Evaluate of a compiled program (see the header comment).
PT_HD double sdf_eval(const DevSdfIns* prog, const double* params, int begin, int len, v3 p) {
    v3 pts[kSdfStack];
    double vals[kSdfStack];
    int ps = 0, vs = 0;
    pts[0] = p;
    for (int i = begin; i < begin + len; i++) {
        const DevSdfIns I = prog[i];
        const double* P = params + I.param;
        const v3 q = pts[ps];
        switch (I.op) {
            case SDF_PUSH_TRANSFORM: pts[++ps] = mat_position(P, q); break;
            case SDF_PUSH_SCALE: pts[++ps] = mk((double)q.x / P[0], (double)q.y / P[0], (double)q.z / P[0]); break;
            case SDF_PUSH_REPEAT: {   // Vector.Mod (Vector.cs:420-426), then Sub(Step.DivScalar(2))
                v3 st = mk(P[0], P[1], P[2]);
                v3 m = mk((double)q.x - (double)st.x * floor((double)q.x / (double)st.x),
                          (double)q.y - (double)st.y * floor((double)q.y / (double)st.y),
                          (double)q.z - (double)st.z * floor((double)q.z / (double)st.z));
                pts[++ps] = sub(m, mk((double)st.x / 2, (double)st.y / 2, (double)st.z / 2));
                break;
            }
            case SDF_POP_POINT: ps--; break;
            case SDF_MUL: vals[vs - 1] = vals[vs - 1] * P[0]; break;
            case SDF_UNION: { double b = vals[--vs]; if (b < vals[vs - 1]) vals[vs - 1] = b; break; }
            case SDF_DIFFERENCE: { double b = vals[--vs]; if (-b > vals[vs - 1]) vals[vs - 1] = -b; break; }
            case SDF_INTERSECTION: { double b = vals[--vs]; if (b > vals[vs - 1]) vals[vs - 1] = b; break; }
            case SDF_CONST0: vals[vs++] = 0.0; break;
            default: vals[vs++] = sdf_leaf(I.op, P, q); break;
        }
    }
    return vals[0];
}

// SDF.Evaluate of a chain program (DevSdfShape::chain: Transform / Scale / Repeat nodes above one
// leaf, no Union / Difference / Intersection): after the leaf only value scalings and point pops
// follow, so no saved point is read again and the one value needs no stack.  The same operations as
// sdf_eval in the same order, with the point and the value in registers (sdf_eval's stacks, indexed
// at run time, live in scratch memory).
PT_HD double sdf_eval_chain(const DevSdfIns* prog, const double* params, int begin, int len, v3 p) {
    v3 q = p;
    double v = 0.0;
    for (int i = begin; i < begin + len; i++) {
        const DevSdfIns I = prog[i];
        const double* P = params + I.param;
        switch (I.op) {
            case SDF_PUSH_TRANSFORM: q = mat_position(P, q); break;
            case SDF_PUSH_SCALE: q = mk((double)q.x / P[0], (double)q.y / P[0], (double)q.z / P[0]); break;
            case SDF_PUSH_REPEAT: {
                v3 st = mk(P[0], P[1], P[2]);
                v3 m = mk((double)q.x - (double)st.x * floor((double)q.x / (double)st.x),
                          (double)q.y - (double)st.y * floor((double)q.y / (double)st.y),
                          (double)q.z - (double)st.z * floor((double)q.z / (double)st.z));
                q = sub(m, mk((double)st.x / 2, (double)st.y / 2, (double)st.z / 2));
                break;
            }
            case SDF_POP_POINT: break;
            case SDF_MUL: v = v * P[0]; break;
            default: v = sdf_leaf(I.op, P, q); break;
        }
    }
    return v;
}
PT_HD double sdf_value(const DevSdfIns* prog, const double* params, const DevSdfShape& sh, v3 p) {
    return sh.chain ? sdf_eval_chain(prog, params, sh.begin, sh.len, p) : sdf_eval(prog, params, sh.begin, sh.len, p);
}

// SDFShape.Intersect (SDF.cs:32-76): sphere tracing within the bounding box.
// `evals` (instrumentation, may be null): the SDF evaluations the march made.
PT_HD double sdf_t(const DevSdfIns* prog, const double* params, const DevSdfShape& sh, v3 o, v3 d,
                   uint32_t* evals = nullptr) {
    const double epsilon = (double)0.00001f, start = (double)0.0001f, jump_size = (double)0.001f;
    double t1, t2;
    box_span(sh.bmin, sh.bmax, o, d, t1, t2);
    if (t2 < t1 || t2 < 0) return kHitInf;
    double t = net_max(start, t1);
    bool jump = true;
    uint32_t n = 0;
    double r = kHitInf;
    for (int i = 0; i < 1000; i++) {
        double dist = sdf_value(prog, params, sh, add(o, muls(d, t)));
        n++;
        if (jump && dist < 0) {
            t -= jump_size;
            jump = false;
            continue;
        }
        if (dist < epsilon) { r = t; break; }
        if (jump && dist < jump_size) dist = jump_size;
        t += dist;
        if (t > t2) break;
    }
    if (evals) *evals = n;
    return r;
}
// SDFShape.NormalAt (SDF.cs:83-92)
PT_HD v3 sdf_normal(const DevSdfIns* prog, const double* params, const DevSdfShape& sh, v3 p) {
    const double e = 0.0001;
    const double x = p.x, y = p.y, z = p.z;
    double nx = sdf_value(prog, params, sh, mk(x - e, y, z)) - sdf_value(prog, params, sh, mk(x + e, y, z));
    double ny = sdf_value(prog, params, sh, mk(x, y - e, z)) - sdf_value(prog, params, sh, mk(x, y + e, z));
    double nz = sdf_value(prog, params, sh, mk(x, y, z - e)) - sdf_value(prog, params, sh, mk(x, y, z + e));
    return normalize(mk(nx, ny, nz));
}

// ---------------------------------------------------------------- Volume (Volume.cs)
// z / zscale (Volume.Sample's `z /= ZScale`, Volume.cs:76), correctly rounded, from the reciprocal y =
// RN(1/zscale): q0 = RN(z·y) is within 1.5 ulp of z/zscale, the first correction makes it faithful, and
// Markstein's theorem makes the second, RN(q1 + (z − zscale·q1)·y) with the residual exact by the FMA,
// the correctly rounded quotient.  Five dependent fp64 operations instead of the division's sequence;
// tests/native/vol_skip_check.cpp compares it with the division (also on divisors with all-ones and
// few-bit significands).  A zero z gives +0 for −0, which Sample's next step (z + 1, z + 2) erases.
PT_HD double vol_zdiv(const DevVolume& v, double z) {
    if (v.zinv == 0.0) return z / v.zscale;
    const double b = v.zscale, y = v.zinv;
    double q = z * y;
    double r = fma(-q, b, z);
    q = fma(r, y, q);
    r = fma(-q, b, z);
    return fma(r, y, q);
}
// The reciprocal vol_zdiv takes: normal zscale and 1/zscale only (no overflow or underflow in the steps).
inline double vol_zinv(double zscale) {
    const double y = 1.0 / zscale;
    return (isnormal(zscale) && isnormal(y)) ? y : 0.0;
}
PT_HD double vol_get(const DevVolume& v, int x, int y, int z) {   // Volume.Get (Volume.cs:40-46)
    if (x < 0 || y < 0 || z < 0 || x >= v.w || y >= v.h || z >= v.d) return 0;
    return v.data[(size_t)x + (size_t)y * (size_t)v.w + (size_t)z * (size_t)v.w * (size_t)v.h];
}
struct alignas(16) VolPair {
    double lo, hi;
};
// The eight corners of cell (x0, y0, z0): Volume.Get's values, from the cell-major copy when the cell is on it.
PT_HD void vol_corners(const DevVolume& v, int x0, int y0, int z0, double c[8]) {
    if (v.cells && x0 >= -1 && y0 >= -1 && z0 >= -1 && x0 < v.w && y0 < v.h && z0 < v.d) {
        PT_GLOBAL(VolPair) p = (PT_GLOBAL(VolPair))(
            v.cells + 8 * ((size_t)(x0 + 1) + (size_t)(y0 + 1) * (v.w + 1) + (size_t)(z0 + 1) * (v.w + 1) * (v.h + 1)));
        const VolPair a = p[0], b = p[1], e = p[2], f = p[3];   // four 16-B loads of one half-line
        c[0] = a.lo; c[1] = a.hi; c[2] = b.lo; c[3] = b.hi; c[4] = e.lo; c[5] = e.hi; c[6] = f.lo; c[7] = f.hi;
        return;
    }
    c[0] = vol_get(v, x0, y0, z0); c[1] = vol_get(v, x0, y0, z0 + 1);
    c[2] = vol_get(v, x0, y0 + 1, z0); c[3] = vol_get(v, x0, y0 + 1, z0 + 1);
    c[4] = vol_get(v, x0 + 1, y0, z0); c[5] = vol_get(v, x0 + 1, y0, z0 + 1);
    c[6] = vol_get(v, x0 + 1, y0 + 1, z0); c[7] = vol_get(v, x0 + 1, y0 + 1, z0 + 1);
}
// Volume.Sample (Volume.cs:73-105), with its y-from-z slip (:77).  Coordinates outside
// the int range (an OverflowException in the reference) sample 0, as in the oracle.
PT_HD double vol_sample(const DevVolume& v, double x, double y, double z) {
    (void)y;
    z = vol_zdiv(v, z);
    x = ((x + 1) / 2) * (double)v.w;
    y = ((z + 1) / 2) * (double)v.h;
    z = ((z + 2) / 2) * (double)v.d;
    const double lim = 2147483647.0;
    if (!(fabs(x) < lim && fabs(y) < lim && fabs(z) < lim)) return 0;
    const int x0 = (int)floor(x), y0 = (int)floor(y), z0 = (int)floor(z);
    const int x1 = x0 + 1, y1 = y0 + 1, z1 = z0 + 1;
    const double v000 = vol_get(v, x0, y0, z0), v001 = vol_get(v, x0, y0, z1), v010 = vol_get(v, x0, y1, z0);
    const double v011 = vol_get(v, x0, y1, z1), v100 = vol_get(v, x1, y0, z0), v101 = vol_get(v, x1, y0, z1);
    const double v110 = vol_get(v, x1, y1, z0), v111 = vol_get(v, x1, y1, z1);
    x -= (double)x0;
    y -= (double)y0;
    z -= (double)z0;
    const double c00 = v000 * (1 - x) + v100 * x;
    const double c01 = v001 * (1 - x) + v101 * x;
    const double c10 = v010 * (1 - x) + v110 * x;
    const double c11 = v011 * (1 - x) + v111 * x;
    const double c0 = c00 * (1 - y) + c10 * y;
    const double c1 = c01 * (1 - y) + c11 * y;
    return c0 * (1 - z) + c1 * z;
}
// The eight corner values of the last cell Volume.Intersect's march sampled: its steps (1/512
// of a unit) cross a cell (2/W of a unit, before the instance transform) tens of steps apart,
// so the march re-reads the grid only when the cell changes.  The values and the arithmetic
// after them are Volume.Sample's, bit for bit.
struct VolCell {
    int x0, y0, z0;
    double c[8];   // v000 v001 v010 v011 v100 v101 v110 v111
};
PT_HD double vol_sample_cell(const DevVolume& v, double x, double y, double z, VolCell& k) {
    (void)y;
    z = vol_zdiv(v, z);
    x = ((x + 1) / 2) * (double)v.w;
    y = ((z + 1) / 2) * (double)v.h;
    z = ((z + 2) / 2) * (double)v.d;
    const double lim = 2147483647.0;
    if (!(fabs(x) < lim && fabs(y) < lim && fabs(z) < lim)) return 0;
    const int x0 = (int)floor(x), y0 = (int)floor(y), z0 = (int)floor(z);
    if (x0 != k.x0 || y0 != k.y0 || z0 != k.z0) {
        vol_corners(v, x0, y0, z0, k.c);
        k.x0 = x0; k.y0 = y0; k.z0 = z0;
    }
    x -= (double)x0;
    y -= (double)y0;
    z -= (double)z0;
    const double c00 = k.c[0] * (1 - x) + k.c[4] * x;
    const double c01 = k.c[1] * (1 - x) + k.c[5] * x;
    const double c10 = k.c[2] * (1 - x) + k.c[6] * x;
    const double c11 = k.c[3] * (1 - x) + k.c[7] * x;
    const double c0 = c00 * (1 - y) + c10 * y;
    const double c1 = c01 * (1 - y) + c11 * y;
    return c0 * (1 - z) + c1 * z;
}
// Volume.Sign (Volume.cs:114-131) of a sample value: its `i` is never incremented, so
// "below a window" is 1.
PT_HD int vol_sign_of(const DevVolume& v, double s) {
    for (int i = 0; i < v.nwin; i++) {
        if (s < v.windows[i].lo) return 1;
        if (s > v.windows[i].hi) continue;
        return 0;
    }
    return v.nwin + 1;
}
PT_HD int vol_sign(const DevVolume& v, v3 a) { return vol_sign_of(v, vol_sample(v, a.x, a.y, a.z)); }
// Volume.NormalAt (Volume.cs:138-145)
PT_HD v3 vol_normal(const DevVolume& v, v3 p) {
    const double eps = (double)0.001f;
    return normalize(mk(vol_sample(v, p.x - eps, p.y, p.z) - vol_sample(v, p.x + eps, p.y, p.z),
                        vol_sample(v, p.x, p.y - eps, p.z) - vol_sample(v, p.x, p.y + eps, p.z),
                        vol_sample(v, p.x, p.y, p.z - eps) - vol_sample(v, p.x, p.y, p.z + eps)));
}
// Volume.MaterialAt (Volume.cs:148-166): the window holding the sample, else the nearest
// (`new Material()` = default_mat when none is nearer than 1e9F).
PT_HD int vol_material(const DevVolume& v, v3 p, int default_mat) {
    double be = (double)1e9f;
    int bm = default_mat;
    const double s = vol_sample(v, p.x, p.y, p.z);
    for (int i = 0; i < v.nwin; i++) {
        const DevWindow w = v.windows[i];
        if (s >= w.lo && s <= w.hi) return w.mat;
        const double e = net_min(fabs(s - w.lo), fabs(s - w.hi));
        if (e < be) { be = e; bm = w.mat; }
    }
    return bm;
}
// ---------------------------------------------------------------- uniform Volume cells
// Volume.Intersect acts at a march position only when its Sign is 0 or differs from the last
// one.  Sample is a convex combination of its cell's eight corners, so a cell whose corner range
// lies inside one Sign band (with a margin far above the interpolation's rounding) gives every
// position in it that band's Sign: the cooperative march (pt_device.h coop_vol_t) reads such a
// cell's Sign from a table and passes runs of such cells at once, at the exact positions (the
// reference's own repeated additions, t_after, and fp32 Ray.Position), so the t returned is the
// loop's, bit for bit.  In the reference's own volume scene (Example.volume) Sample's y-from-z slip
// puts most of the box beyond the grid's last slice, where every sample is exactly 0.
//
// The band of a value: 2i for "below window i's lo" (i = nwin: above every window), 2i + 1 for
// "inside window i" (Sign 0); bands 2i all have Sign 1 except 2·nwin (Sign nwin + 1).
PT_HD int vol_band(const DevVolume& v, double s) {
    for (int i = 0; i < v.nwin; i++) {
        if (s < v.windows[i].lo) return 2 * i;
        if (s <= v.windows[i].hi) return 2 * i + 1;
    }
    return 2 * v.nwin;
}
// Host: fill out[(x0+1) + (y0+1)(w+1) + (z0+1)(w+1)(h+1)] for cells x0 in -1..w-1, y0 in -1..h-1,
// z0 in -1..d-1 (a cell outside that range has every corner outside the grid: zero_sign).
inline void vol_build_runs(const DevVolume& v, int8_t* out, int32_t& zero_sign) {
    const int sx = v.w + 1, sy = v.h + 1;
    auto sign_of_band = [&](int b) { return (b & 1) ? 0 : (b == 2 * v.nwin ? v.nwin + 1 : 1); };
    zero_sign = sign_of_band(vol_band(v, 0.0));
    for (int z0 = -1; z0 < v.d; z0++)
        for (int y0 = -1; y0 < v.h; y0++)
            for (int x0 = -1; x0 < v.w; x0++) {
                double mn = 0, mx = 0;
                bool first = true, finite = true;   // a NaN / infinite corner can interpolate to NaN (Sign 0)
                for (int c = 0; c < 8; c++) {
                    const double g = vol_get(v, x0 + (c >> 2 & 1), y0 + (c >> 1 & 1), z0 + (c & 1));
                    finite = finite && isfinite(g);
                    if (first || g < mn) mn = g;
                    if (first || g > mx) mx = g;
                    first = false;
                }
                const double margin = 1e-9 * (1.0 + fabs(mn) + fabs(mx));
                const int b0 = vol_band(v, mn - margin), b1 = vol_band(v, mx + margin);
                const int sg = (finite && b0 == b1) ? sign_of_band(b0) : 0;
                // a Sign past int8 (above every window of 127 or more) is stored as 0: "no shortcut"
                out[(x0 + 1) + (size_t)(y0 + 1) * sx + (size_t)(z0 + 1) * sx * sy] = (int8_t)(sg > 127 ? 0 : sg);
            }
}
// t after k more additions of step (a power of two) made one at a time, as Volume.Intersect's
// `t += step`: inside one binade, with t's ulp dividing step, every partial sum is exact, so k·step
// is added at once; the addition that crosses into the next binade rounds, and is made alone.
PT_HD double t_after(double t, double step, long long k) {
    while (k > 0) {
        int e;
        (void)frexp(t, &e);   // t in [2^(e-1), 2^e), t > 0
        if (ldexp(1.0, e - 53) > step) {   // every addition rounds (t >= 2^44 at 1/512): one by one
            for (; k > 0; k--) t += step;
            break;
        }
        const double lim = ldexp(1.0, e);
        // additions that stay below lim; step is a power of two, so multiplying by its reciprocal is the division
        const long long room = (long long)ceil((lim - t) * (1.0 / step)) - 1;
        if (room >= k) return t + (double)k * step;
        t = t + (double)room * step;
        t += step;   // into the next binade: rounded, as the reference's
        k -= room + 1;
    }
    return t;
}
// The cell of march position t, with each index clamped to the band -2..dim (a clamped index is
// a cell outside the grid); clamping keeps every index monotone along the ray.
struct VolKey {
    int x, y, z;
};
PT_HD VolKey vol_key(const DevVolume& v, v3 o, v3 d, double t) {
    const v3 a = add(o, muls(d, t));   // Ray.Position, as vol_t's positions
    double x = a.x, z = a.z;
    z = vol_zdiv(v, z);
    x = ((x + 1) / 2) * (double)v.w;
    const double y = ((z + 1) / 2) * (double)v.h;
    z = ((z + 2) / 2) * (double)v.d;
    auto cl = [](double c, int n) {   // floor, clamped to -2..n (non-finite: outside)
        if (!(c > -2.0)) return -2;
        if (!(c < (double)n)) return n;
        return (int)floor(c);
    };
    return VolKey{cl(x, v.w), cl(y, v.h), cl(z, v.d)};
}
PT_HD int vol_key_sign(const DevVolume& v, VolKey k) {
    if (k.x < -1 || k.y < -1 || k.z < -1 || k.x >= v.w || k.y >= v.h || k.z >= v.d) return v.zero_sign;
    return v.runs[(k.x + 1) + (size_t)(k.y + 1) * (v.w + 1) + (size_t)(k.z + 1) * (v.w + 1) * (v.h + 1)];
}
// Host: fill out[8·((x0+1) + (y0+1)(w+1) + (z0+1)(w+1)(h+1)) + c] = corner c of cell (x0, y0, z0), the runs table's
// cells, c = 4·dx + 2·dy + dz (vol_sample's v000 v001 v010 v011 v100 v101 v110 v111).
inline void vol_build_cells(const DevVolume& v, double* out) {
    size_t i = 0;
    for (int z0 = -1; z0 < v.d; z0++)
        for (int y0 = -1; y0 < v.h; y0++)
            for (int x0 = -1; x0 < v.w; x0++, i++)
                for (int c = 0; c < 8; c++) out[8 * i + (size_t)c] = vol_get(v, x0 + (c >> 2), y0 + (c >> 1 & 1), z0 + (c & 1));
}
// The Sign of march position t (vol_key_sign of a uniform cell, else Volume.Sign of the sample) with the
// lattice coordinates computed once: vol_key and Volume.Sample (vol_sample) scale the same position by
// the same operations, so the key and the sample share them (one fp64 division by zscale, not two).
PT_HD int vol_sign_at(const DevVolume& v, v3 o, v3 d, double t) {
    const v3 a = add(o, muls(d, t));   // Ray.Position
    double x = a.x, z = a.z;
    z = vol_zdiv(v, z);
    x = ((x + 1) / 2) * (double)v.w;
    double y = ((z + 1) / 2) * (double)v.h;   // Sample's y-from-z slip (Volume.cs:77)
    z = ((z + 2) / 2) * (double)v.d;
    if (v.runs) {
        auto cl = [](double c, int n) {   // vol_key's floor, clamped to -2..n
            if (!(c > -2.0)) return -2;
            if (!(c < (double)n)) return n;
            return (int)floor(c);
        };
        const int s = vol_key_sign(v, VolKey{cl(x, v.w), cl(y, v.h), cl(z, v.d)});
        if (s > 0) return s;
    }
    const double lim = 2147483647.0;   // vol_sample from the scaled coordinates on
    if (!(fabs(x) < lim && fabs(y) < lim && fabs(z) < lim)) return vol_sign_of(v, 0.0);
    const int x0 = (int)floor(x), y0 = (int)floor(y), z0 = (int)floor(z);
    double k[8];
    vol_corners(v, x0, y0, z0, k);
    x -= (double)x0;
    y -= (double)y0;
    z -= (double)z0;
    const double c00 = k[0] * (1 - x) + k[4] * x;
    const double c01 = k[1] * (1 - x) + k[5] * x;
    const double c10 = k[2] * (1 - x) + k[6] * x;
    const double c11 = k[3] * (1 - x) + k[7] * x;
    const double c0 = c00 * (1 - y) + c10 * y;
    const double c1 = c01 * (1 - y) + c11 * y;
    return vol_sign_of(v, c0 * (1 - z) + c1 * z);
}
// Volume.Intersect (Volume.cs:168-197).  The reference loop has no bound; 2^24 steps
// stand in for it (a ray that needs more never finishes in the reference either).
// `samples` (instrumentation, may be null): the Volume.Sample calls the march made.  Each position
// reads its cell's corners once per cell (vol_sample_cell).  A serial search for the end of a run of
// uniform cells measured slower than the wave's strided pass.
PT_HD double vol_t(const DevVolume& v, v3 o, v3 d, uint32_t* samples = nullptr) {
    double tmin, tmax;
    box_span(v.bmin, v.bmax, o, d, tmin, tmax);
    double step = (double)(1.0f / 512.0f);
    const double start = net_max(step, tmin);
    int sign = -1;
    int iters = 0;
    VolCell k;
    k.x0 = k.y0 = k.z0 = -2147483647 - 1;   // no cell: floor() of an in-range coordinate is above it
    uint32_t n = 0;
    auto done = [&](double r) {
        if (samples) *samples = n;
        return r;
    };
    auto sign_at = [&](double t) {
        n++;
        const v3 a = add(o, muls(d, t));
        return vol_sign_of(v, vol_sample_cell(v, a.x, a.y, a.z, k));
    };
    for (double t = start; t <= tmax && iters < (1 << 24); t += step, iters++) {
        const int sg = sign_at(t);
        if (sg == 0 || (sign >= 0 && sg != sign)) {
            t -= step;
            step /= 64;
            t += step;
            for (int i = 0; i < 64; i++) {
                if (sign_at(t) == 0) return done(t - step);
                t += step;
            }
        }
        sign = sg;
    }
    return done(kHitInf);
}

}  // namespace pt
