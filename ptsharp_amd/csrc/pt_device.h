// pt_device.h — device functions shared by both render engines (the per-pixel
// megakernel in pt_render.hip and the wavefront kernels in pt_wavefront.hip),
// so both run bit-identical arithmetic for every Scene.Intersect, Hit.Info,
// Ray.Bounce and sampleLight.
#pragma once
#include <hip/hip_runtime.h>

#include "pt_bvh.h"
#include "pt_math.h"
#include "pt_scene.h"

#pragma clang fp contract(off)

namespace pt {

struct HitRec {
    double t;
    int32_t kind;   // KIND_* of the primitive hit; -1 = miss
    int32_t idx;    // record position: tri_recs / ana_recs / planes
    double tx = 0;  // KIND_XFORM (FULL): the inner shape's object-space t, so Hit.Info need not intersect again
};

// A whole traversal stack in a private array (scratch): the nested traversal of an instanced mesh, whose
// object-space BVH4 keeps every path within kStack4Budget pushes (pack_nodes checks it).  Sized by that bound,
// not by the triangle BVH8's kStackMax (64 since round 5: 128 B more scratch per lane for no use).
struct LocalStack {
    static constexpr int kLds = kStack4Budget;
    static constexpr int kStride = 1;
    uint32_t* lds;
    __device__ __forceinline__ void put(int i, uint32_t v) const { lds[i] = v; }
    __device__ __forceinline__ uint32_t get(int i) const { return lds[i]; }
};

struct Counters {
    uint32_t rays, nodes, prims, shades;
};


__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }

// Round a hit distance up so the fp32 cull never drops an equal-t candidate.
__device__ __forceinline__ float tmax_bound(double t) {
    float f = (float)t;
    return (double)f < t ? __uint_as_float(f2u(f) + 1u) : f;
}

__device__ __forceinline__ double rec_radius(const float4* r) {
    const float4 c = r[2];
    return __hiloint2double((int)f2u(c.z), (int)f2u(c.y));
}
__device__ __forceinline__ int32_t rec_ext(const float4* r) { return (int32_t)f2u(r[2].y); }   // SDF / volume / xform index

// Intersect of a shape that can sit inside a TransformedShape: Sphere, Cube, Plane,
// SDFShape, Volume (analytic-record format).
__device__ __noinline__ double inner_t(const DevScene& S, const float4* r, int32_t kind, v3 o, v3 d) {
    const float4 a = r[0], b = r[1];
    switch (kind) {
        case KIND_SPHERE: return isect_sphere(v3{a.x, a.y, a.z}, rec_radius(r), o, d);
        case KIND_CUBE: return isect_cube(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
        case KIND_PLANE: return isect_plane(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
        case KIND_SDF:
        case KIND_VOLUME: {   // the marches; a counted pass adds their steps (S.march)
            uint32_t n = 0;
            const double t = kind == KIND_SDF ? sdf_t(S.sdf_prog, S.sdf_params, S.sdf_shapes[rec_ext(r)], o, d, &n)
                                              : vol_t(S.volumes[rec_ext(r)], o, d, &n);
            if (S.march) atomicAdd(S.march + (kind == KIND_SDF ? 1 : 0), (unsigned long long)n);
            return t;
        }
    }
    return kHitInf;
}
struct HitRec;
__device__ __noinline__ HitRec blas_hit(const DevScene& S, int b, v3 o, v3 d);   // below, after traverse()

// TransformedShape.Intersect (TransformedShape.cs:43-73) up to hit.T: the inner hit mapped
// back to world space, T = |position - origin| (fp32 Length).
__device__ __noinline__ double xform_t(const DevScene& S, const DevXform& X, v3 o, v3 d, double* tobj = nullptr);

// Intersect one record; returns t (kHitInf = miss) and the primitive kind.  FULL adds
// the §8f row 4 kinds of the analytic BVH (SDF, volume, transformed shape).
// tx (FULL, may be null): a TransformedShape's inner object-space t (HitRec::tx).
template <bool TRI, bool FULL = false>
__device__ __forceinline__ double prim_t(const DevScene& S, const float4* __restrict__ recs, uint32_t pos, v3 o, v3 d,
                                         int32_t& kind, double* tx = nullptr) {
    const float4* r = recs + 3 * (size_t)pos;
    if (TRI) {
        float4 a = r[0], b = r[1], c = r[2];
        kind = KIND_TRI;
        return isect_tri(v3{a.x, a.y, a.z}, v3{a.w, b.x, b.y}, v3{b.z, b.w, c.x}, o, d);
    }
    float4 a = r[0], b = r[1];
    kind = (int32_t)f2u(a.w);
    if (kind == KIND_SPHERE) return isect_sphere(v3{a.x, a.y, a.z}, rec_radius(r), o, d);
    if (!FULL || kind == KIND_CUBE) return isect_cube(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
    if (kind == KIND_XFORM) return xform_t(S, S.xforms[rec_ext(r)], o, d, tx);
    return inner_t(S, r, kind, o, d);
}

// Is this analytic record a Volume march (a Volume, or a TransformedShape of one)?
__device__ __forceinline__ bool march_deferred(const DevScene& S, const float4* r) {
    const int32_t kind = (int32_t)f2u(r[0].w);
    if (kind == KIND_VOLUME) return true;
    return kind == KIND_XFORM && S.xforms[rec_ext(r)].kind == KIND_VOLUME;
}

// Per-lane traversal stacks.  LdsStack: all kStackMax entries in LDS (column
// `lds`, entries STRIDE words apart).  SpillStack: the first LDSN entries in LDS
// and the rarely used deeper ones in a per-thread global column (entries
// `ostride` words apart, coalesced across lanes), so a traversal kernel's LDS
// footprint no longer caps its occupancy.
// push_hits() pushes the hit children after the nearest, far-to-near.  While
// the three slots above sp are in LDS (nearly always) it stores all three
// unconditionally and advances sp by predicate: no per-push branch.
template <int STRIDE>
struct LdsStack {
    static constexpr int kLds = kStackMax;
    static constexpr int kStride = STRIDE;
    uint32_t* lds;
    __device__ __forceinline__ void put(int i, uint32_t v) const { lds[i * STRIDE] = v; }
    __device__ __forceinline__ uint32_t get(int i) const { return lds[i * STRIDE]; }
};

template <int STRIDE, int LDSN>
struct SpillStack {
    static constexpr int kLds = LDSN;
    static constexpr int kStride = STRIDE;
    uint32_t* lds;
    uint32_t* ovf;
    uint32_t ostride;
    __device__ __forceinline__ void put(int i, uint32_t v) const {
        if (i < LDSN) lds[i * STRIDE] = v;
        else ovf[(size_t)(i - LDSN) * ostride] = v;
    }
    __device__ __forceinline__ uint32_t get(int i) const {
        if (__builtin_expect(i >= LDSN, 0)) return ovf[(size_t)(i - LDSN) * ostride];
        return lds[i * STRIDE];
    }
};

template <class STK>
__device__ __forceinline__ void push_hits(const STK& st, int& sp, int n, uint32_t v1, uint32_t v2, uint32_t v3) {
    if (__builtin_expect(sp <= STK::kLds - 3, 1)) {
        st.lds[sp * STK::kStride] = v3;
        sp += n > 3;
        st.lds[sp * STK::kStride] = v2;
        sp += n > 2;
        st.lds[sp * STK::kStride] = v1;
        sp += n > 1;
    } else {
        if (n > 3) { st.put(sp, v3); sp++; }
        if (n > 2) { st.put(sp, v2); sp++; }
        if (n > 1) { st.put(sp, v1); sp++; }
    }
}

// Conservative fp32 slab test of one child box: (b - o) * (1/d) carries <= 3 ulp
// of relative error, so the far distance is widened by 2^-21 relative; NaN slabs
// (o on a plane with d = 0) drop out of fminf/fmaxf, which only widens the interval.
__device__ __forceinline__ float slab1(float lx, float hx, float ly, float hy, float lz, float hz, v3 o, v3 invd,
                                       float tmax) {
    float tx1 = (lx - o.x) * invd.x, tx2 = (hx - o.x) * invd.x;
    float ty1 = (ly - o.y) * invd.y, ty2 = (hy - o.y) * invd.y;
    float tz1 = (lz - o.z) * invd.z, tz2 = (hz - o.z) * invd.z;
    float tn = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fmaxf(fminf(tz1, tz2), 0.0f));
    float tf = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fminf(fmaxf(tz1, tz2), tmax));
    return tn <= tf * 1.0000005f ? tn : __int_as_float(0x7f800000);  // entry distance, +inf = miss
}

__device__ __forceinline__ void cswap(float& ka, uint32_t& va, float& kb, uint32_t& vb) {
    const bool s = kb < ka;
    const float k = s ? kb : ka;
    kb = s ? ka : kb;
    ka = k;
    const uint32_t v = s ? vb : va;
    vb = s ? va : vb;
    va = v;
}

// The four child slabs of a BVH4 node line (pt_bvh.h: seven pieces, lo.x[4] hi.x[4] lo.y[4] hi.y[4]
// lo.z[4] hi.z[4] refs[4]) → entry distances k0..k3 (+inf = miss or empty slot) and child refs v0..v3.
// Compressed lines (8-bit and binary16 child bounds) measured slower: the decode costs more than the
// loads it saves.
__device__ __forceinline__ void node4_test(float4 q0, float4 q1, float4 q2, float4 q3, float4 q4, float4 q5, float4 q6,
                                           v3 o, v3 invd, float tmax, float& k0, float& k1, float& k2, float& k3,
                                           uint32_t& v0, uint32_t& v1, uint32_t& v2, uint32_t& v3r) {
    k0 = slab1(q0.x, q1.x, q2.x, q3.x, q4.x, q5.x, o, invd, tmax);
    k1 = slab1(q0.y, q1.y, q2.y, q3.y, q4.y, q5.y, o, invd, tmax);
    k2 = slab1(q0.z, q1.z, q2.z, q3.z, q4.z, q5.z, o, invd, tmax);
    k3 = slab1(q0.w, q1.w, q2.w, q3.w, q4.w, q5.w, o, invd, tmax);
    v0 = __float_as_uint(q6.x); v1 = __float_as_uint(q6.y); v2 = __float_as_uint(q6.z); v3r = __float_as_uint(q6.w);
    const float inf = __int_as_float(0x7f800000);
    if (v1 == kEmpty4) k1 = inf;  // slot 0 is never empty
    if (v2 == kEmpty4) k2 = inf;
    if (v3r == kEmpty4) k3 = inf;
}

// ---- The triangle BVH as 8-wide nodes with quantized child boxes (pt_bvh.h collapse_bvh8q: one 128-B line,
// eight 16-B pieces q0..q7).  A child's slab distances are fma(q, step/d, (origin - o)/d) per axis, the near
// and far bounds chosen once per node by the ray's direction signs (an empty slot's +inf / -inf bounds give
// an entry distance of +inf on every axis whose direction is not 0, so it never hits).  The hit children's
// entry distances (fp32 bits, non-negative, so ordered as integers) carry the slot in their low 3 bits: the
// nearest is a 3-input-min tree away, and it is descended; the other hits are pushed in slot order (popped
// lowest slot first).  Sorting them far-to-near measured no fewer steps in the C4 ray mix
// (tools/bvh_quality.cpp PUSH_ORDER: closest hit 6.08 vs 6.21 steps, shadow 8.33 vs 8.29) and cost a
// 19-comparator network per step.  The slab test keeps slab1's widening of the far distance (the fma
// form's rounding is of the same order).
typedef _Float16 pt_half2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void halves(float w, float& a, float& b) {
    const pt_half2 h = __builtin_bit_cast(pt_half2, w);
    a = (float)h.x;
    b = (float)h.y;
}
// The ref of slot k (inner children first: base_in + k; leaf chunks after them: base_leaf - n_in + k, the
// count in the chunk's word 0).
__device__ __forceinline__ uint32_t node8_ref(uint32_t k, uint32_t nin, uint32_t base_in, uint32_t leaf0) {
    return k < nin ? base_in + k : leaf0 + k;
}
template <class STK>
__device__ __forceinline__ bool node8_step(float4 q0, float4 q1, float4 q2, float4 q3, float4 q4, float4 q5, float4 q6,
                                           float4 q7, v3 o, v3 invd, float tmax, const STK& st, int& sp, uint32_t& ref) {
    const uint32_t hdr = __float_as_uint(q0.w);
    const float sx = __uint_as_float((hdr & 0xFFu) << 23), sy = __uint_as_float(((hdr >> 8) & 0xFFu) << 23);
    const float sz = __uint_as_float(((hdr >> 16) & 0xFFu) << 23);
    const float ax = (q0.x - o.x) * invd.x, ay = (q0.y - o.y) * invd.y, az = (q0.z - o.z) * invd.z;
    const float bx = sx * invd.x, by = sy * invd.y, bz = sz * invd.z;
    const bool fx = invd.x < 0.f, fy = invd.y < 0.f, fz = invd.z < 0.f;   // the near bound is hi on that axis
    const float4 nx = fx ? q3 : q2, gx = fx ? q2 : q3;
    const float4 ny = fy ? q5 : q4, gy = fy ? q4 : q5;
    const float4 nz = fz ? q7 : q6, gz = fz ? q6 : q7;
    uint32_t key[8];
    auto slab = [&](int k, float wnx, float wgx, float wny, float wgy, float wnz, float wgz, bool hi) {
        float a0, a1, b0, b1, c0, c1, d0, d1, e0, e1, f0, f1;
        halves(wnx, a0, a1); halves(wgx, b0, b1);
        halves(wny, c0, c1); halves(wgy, d0, d1);
        halves(wnz, e0, e1); halves(wgz, f0, f1);
        const float tnx = fmaf(hi ? a1 : a0, bx, ax), tfx = fmaf(hi ? b1 : b0, bx, ax);
        const float tny = fmaf(hi ? c1 : c0, by, ay), tfy = fmaf(hi ? d1 : d0, by, ay);
        const float tnz = fmaf(hi ? e1 : e0, bz, az), tfz = fmaf(hi ? f1 : f0, bz, az);
        const float tn = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, 0.0f));
        const float tf = fminf(fminf(tfx, tfy), fminf(tfz, tmax));
        key[k] = tn <= tf * 1.0000005f ? ((__float_as_uint(tn) & 0x7FFFFFF8u) | (uint32_t)k) : 0xFFFFFFFFu;
    };
    slab(0, nx.x, gx.x, ny.x, gy.x, nz.x, gz.x, false);
    slab(1, nx.x, gx.x, ny.x, gy.x, nz.x, gz.x, true);
    slab(2, nx.y, gx.y, ny.y, gy.y, nz.y, gz.y, false);
    slab(3, nx.y, gx.y, ny.y, gy.y, nz.y, gz.y, true);
    slab(4, nx.z, gx.z, ny.z, gy.z, nz.z, gz.z, false);
    slab(5, nx.z, gx.z, ny.z, gy.z, nz.z, gz.z, true);
    slab(6, nx.w, gx.w, ny.w, gy.w, nz.w, gz.w, false);
    slab(7, nx.w, gx.w, ny.w, gy.w, nz.w, gz.w, true);
    const uint32_t kmin = min(min(min(key[0], key[1]), min(key[2], key[3])), min(min(key[4], key[5]), min(key[6], key[7])));
    if (kmin == 0xFFFFFFFFu) return false;
    const uint32_t near = kmin & 7u;
    const uint32_t nin = (hdr >> 24) & 15u, base_in = __float_as_uint(q1.x), leaf0 = __float_as_uint(q1.y);
    ref = node8_ref(near, nin, base_in, leaf0);
    if (__builtin_expect(sp <= STK::kLds - 8, 1)) {   // every slot written, sp advanced by the other hits
#pragma unroll
        for (int j = 7; j >= 0; j--) {
            st.lds[sp * STK::kStride] = node8_ref((uint32_t)j, nin, base_in, leaf0);
            sp += (key[j] != 0xFFFFFFFFu && (uint32_t)j != near) ? 1 : 0;
        }
    } else {
#pragma unroll
        for (int j = 7; j >= 0; j--)
            if (key[j] != 0xFFFFFFFFu && (uint32_t)j != near) { st.put(sp, node8_ref((uint32_t)j, nin, base_in, leaf0)); sp++; }
    }
    return true;
}

// SDF records (an SDFShape, or a TransformedShape of one): their sphere tracing runs up to 1000
// dependent steps, taken by the lane whose traversal meets the leaf.  The analytic half of a split
// closest hit (k_wf_trace<.., SPLIT>) and of split shadow rays leaves the first SDF record of a ray in a
// compact queue instead (pend_sdf → sdf_out), and k_wf_sdf_hits / k_wf_sdf_shadow trace the queue
// with every lane busy (deferring it to the end of the traversal, every such lane of the wave at
// once, measured slower: DESIGN.md §9c).
__device__ __forceinline__ bool sdf_deferred(const DevScene& S, const float4* r) {
    const int32_t kind = (int32_t)f2u(r[0].w);
    if (kind == KIND_SDF) return true;
    return kind == KIND_XFORM && S.xforms[rec_ext(r)].kind == KIND_SDF;
}
// Intersect of an SDF record (an SDFShape, or a TransformedShape of one): prim_t's t for the SDF
// queues (k_wf_sdf_hits / k_wf_sdf_shadow) without prim_t's other kinds (their calls and stacks).
__device__ __forceinline__ double sdf_record_t(const DevScene& S, uint32_t p, v3 o, v3 d, int32_t& kind, double& tx) {
    const float4* r = S.ana_recs + 3 * (size_t)p;
    kind = (int32_t)f2u(r[0].w);
    uint32_t n = 0;
    double t;
    if (kind == KIND_SDF) {
        t = sdf_t(S.sdf_prog, S.sdf_params, S.sdf_shapes[rec_ext(r)], o, d, &n);
    } else {   // TransformedShape.Intersect (TransformedShape.cs:43-73) of an SDFShape, as xform_t
        const DevXform& X = S.xforms[rec_ext(r)];
        const v3 so = mat_position(X.inv, o), sd = mat_direction(X.inv, d);
        t = sdf_t(S.sdf_prog, S.sdf_params, S.sdf_shapes[rec_ext(S.ext_recs + 3 * (size_t)X.rec)], so, sd, &n);
        if (t < kHitInf) {
            tx = t;
            const v3 position = mat_position(X.m, add(so, muls(sd, t)));
            t = (double)lengthf(sub(position, o));
        } else {
            t = kHitInf;
        }
    }
    if (S.march) atomicAdd(S.march + 1, (unsigned long long)n);
    return t;
}
template <bool ANY>
__device__ __forceinline__ void sdf_pending(const DevScene& S, v3 o, v3 d, int32_t p, HitRec& best, bool* blocked = nullptr) {
    if (p < 0) return;
    int32_t kind;
    double tx = 0;
    const double t = prim_t<false, true>(S, S.ana_recs, (uint32_t)p, o, d, kind, &tx);
    if (ANY) {
        if (t < best.t) *blocked = true;
    } else if (t < best.t || (t == best.t && best.kind == KIND_TRI)) {
        best.t = t; best.kind = kind; best.idx = p; best.tx = tx;
    }
}

// Stack-based BVH4 traversal (node layout: pt_bvh.h, collapse_bvh4).  A node is
// one 128-byte line fetched with seven independent 16-byte loads; the four
// child slabs are tested, hits sorted nearest-first with a 5-comparator network,
// the nearest descended and the others pushed far-to-near on the per-lane stack
// (LdsStack / SpillStack).  The collapse bounds every path's pushes by kStackMax.
// ANY: stop at the first primitive with t < best.t (shadow visibility).
// pend (FULL, analytic BVH): the first Volume record reached is not marched here but left in
// *pend for the wave's cooperative march after the traversal (march_pending).
template <bool TRI, bool COUNT, bool ANY, bool FULL, class STK>
__device__ __forceinline__ bool traverse(const DevScene& S, const float4* __restrict__ nodes, int32_t num_nodes,
                                         const float4* __restrict__ recs, v3 o, v3 d, v3 invd, HitRec& best,
                                         const STK& stack, Counters& ctr, int32_t* pend = nullptr,
                                         int32_t* pend_sdf = nullptr) {
    if (num_nodes <= 0) return false;
    uint32_t ref = 0;  // root: always an inner node
    int sp = 0;
    float tmax = tmax_bound(best.t);  // fp32 cull bound, refreshed when best.t changes
    for (;;) {
        if (!(ref & 0x80000000u)) {
            const float4* c = nodes + 8 * (size_t)ref;
            const float4 q0 = c[0], q1 = c[1], q2 = c[2], q3 = c[3], q4 = c[4], q5 = c[5], q6 = c[6];
            if (COUNT) ctr.nodes++;
            const float inf = __int_as_float(0x7f800000);
            float k0, k1, k2, k3;
            uint32_t v0, v1, v2, v3r;
            node4_test(q0, q1, q2, q3, q4, q5, q6, o, invd, tmax, k0, k1, k2, k3, v0, v1, v2, v3r);
            cswap(k0, v0, k1, v1);
            cswap(k2, v2, k3, v3r);
            cswap(k0, v0, k2, v2);
            cswap(k1, v1, k3, v3r);
            cswap(k1, v1, k2, v2);
            if (k0 != inf) {
                push_hits(stack, sp, 1 + (k1 != inf) + (k2 != inf) + (k3 != inf), v1, v2, v3r);
                ref = v0;
                continue;
            }
        } else {
            const uint32_t first = ref & 0x1FFFFFFFu, cnt = ((ref >> 29) & 3u) + 1u;
            for (uint32_t k = 0; k < cnt; k++) {
                if (COUNT) ctr.prims++;
                int32_t kind;
                if (FULL && pend && *pend < 0 && march_deferred(S, recs + 3 * (size_t)(first + k))) {
                    *pend = (int32_t)(first + k);
                    continue;
                }
                if (FULL && pend_sdf && *pend_sdf < 0 &&
                    sdf_deferred(S, recs + 3 * (size_t)(first + k))) {
                    *pend_sdf = (int32_t)(first + k);
                    continue;
                }
                double tx = 0;
                double t = prim_t<TRI, FULL>(S, recs, first + k, o, d, kind, FULL ? &tx : nullptr);
                if (t < best.t) {
                    if (ANY) return true;
                    best.t = t; best.kind = kind; best.idx = (int32_t)(first + k);
                    if (FULL) best.tx = tx;
                    tmax = tmax_bound(t);
                }
            }
        }
        if (sp == 0) break;
        sp--;
        ref = stack.get(sp);
    }
    return false;
}

// Pin loaded values so the compiler keeps each aligned 16-B load whole (left alone it
// re-splits them along the consumers' 12-B vertex fields into unaligned pieces).
#define PT_PIN4(q) asm volatile("" : "+v"((q).x), "+v"((q).y), "+v"((q).z), "+v"((q).w))
// Two loads pinned together: both are issued before the one wait the pin needs (a pin of one value
// after its load makes the compiler wait for it before it issues the next)
#define PT_PIN44(p, q) asm volatile("" : "+v"((p).x), "+v"((p).y), "+v"((p).z), "+v"((p).w), \
                                         "+v"((q).x), "+v"((q).y), "+v"((q).z), "+v"((q).w))


// The triangles of a leaf chunk (pt_api.hip build_tri_bvh): word 0 = the first triangle
// record, triangle k = words 1 + 9k .. 9 + 9k as {v1, e1, e2}; a0..a2 is the first, b the
// second, c the third (shifted down after each test).  A chunk of cnt triangles is read with its
// first 1 + 2·cnt 16-B pieces; the rest of q is stale and never tested.
#define PT_CHUNK_TRIS(q0, q1, q2, q3, q4, q5, q6)                                          \
    v3 a0{q0.y, q0.z, q0.w}, a1{q1.x, q1.y, q1.z}, a2{q1.w, q2.x, q2.y};                  \
    v3 b0{q2.z, q2.w, q3.x}, b1{q3.y, q3.z, q3.w}, b2{q4.x, q4.y, q4.z};                  \
    const v3 c0{q4.w, q5.x, q5.y}, c1{q5.z, q5.w, q6.x}, c2{q6.y, q6.z, q6.w}

// Triangle-BVH traversal over leaf chunks (pt_api.hip build_tri_bvh).  The node step is
// node8_step's (8-wide quantized nodes); a leaf ref points at a 128-B chunk of up to three
// triangles, so an inner step and a leaf step read the same 128-B line's 16-B pieces and a
// wave whose lanes are split between nodes and leaves pays for one set of load
// instructions, not for the node loads plus a per-triangle load loop.
template <bool COUNT, bool ANY, class STK>
__device__ __forceinline__ bool traverse_tri(const DevScene& S, v3 o, v3 d, v3 invd, HitRec& best, const STK& stack,
                                             Counters& ctr) {
    if (S.tri_num_nodes <= 0) return false;
    uint32_t ref = 0;  // root: always an inner node
    int sp = 0;
    float tmax = tmax_bound(best.t);
    for (;;) {
        const bool leaf = (ref & 0x80000000u) != 0;
        const float4* c = (leaf ? S.tri_chunks : S.tri_nodes) + 8 * (size_t)(ref & 0x1FFFFFFFu);
        float4 q0 = c[0], q1 = c[1], q2 = c[2], q3 = c[3], q4 = c[4], q5 = c[5], q6 = c[6], q7 = c[7];
        PT_PIN4(q0); PT_PIN4(q1); PT_PIN4(q2); PT_PIN4(q3); PT_PIN4(q4); PT_PIN4(q5); PT_PIN4(q6); PT_PIN4(q7);
        if (!leaf) {
            if (COUNT) ctr.nodes++;
            if (node8_step(q0, q1, q2, q3, q4, q5, q6, q7, o, invd, tmax, stack, sp, ref)) continue;
        } else {
            const uint32_t w0 = __float_as_uint(q0.x), cnt = (w0 >> 29) + 1u, first = w0 & 0x1FFFFFFFu;   // chunk word 0
            PT_CHUNK_TRIS(q0, q1, q2, q3, q4, q5, q6);
#pragma unroll 1
            for (uint32_t k = 0; k < cnt; k++) {
                if (COUNT) ctr.prims++;
                const double t = isect_tri(a0, a1, a2, o, d);
                if (t < best.t) {
                    if (ANY) return true;
                    best.t = t; best.kind = KIND_TRI; best.idx = (int32_t)(first + k);
                    tmax = tmax_bound(t);
                }
                a0 = b0; a1 = b1; a2 = b2;
                b0 = c0; b1 = c1; b2 = c2;
            }
        }
        if (sp == 0) break;
        sp--;
        ref = stack.get(sp);
    }
    return false;
}

// Mesh.Intersect of an instanced mesh: its own object-space BVH4 (Mesh.cs:83-86, 122-125);
// idx is the triangle's position in the mesh's BLAS records.
__device__ __noinline__ HitRec blas_hit(const DevScene& S, int b, v3 o, v3 d) {
    const DevBlas B = S.blas[b];
    uint32_t st[kStack4Budget];
    const LocalStack stack{st};
    HitRec best{kHitInf, -1, -1};
    Counters ctr{0, 0, 0, 0};
    const v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    traverse<true, false, false, false>(S, S.blas_nodes + 8 * (size_t)B.node_off, B.num_nodes,
                                        S.blas_recs + 3 * (size_t)B.rec_off, o, d, invd, best, stack, ctr);
    return best;
}

__device__ __noinline__ double xform_t(const DevScene& S, const DevXform& X, v3 o, v3 d, double* tobj) {
    const v3 so = mat_position(X.inv, o), sd = mat_direction(X.inv, d);   // Matrix.Inverse().MulRay
    double t;
    if (X.kind == KIND_MESH) t = blas_hit(S, X.rec, so, sd).t;
    else t = inner_t(S, S.ext_recs + 3 * (size_t)X.rec, X.kind, so, sd);
    if (!(t < kHitInf)) return kHitInf;
    if (tobj) *tobj = t;
    const v3 position = mat_position(X.m, add(so, muls(sd, t)));
    return (double)lengthf(sub(position, o));
}

// ---------------------------------------------------------------- cooperative Volume march
// Volume.Intersect (Volume.cs:168-197) marches a ray in fixed 1/512 steps, hundreds per ray
// that crosses the grid's box.  Marched by the lane that meets it (vol_t), the rest of the
// wave waits that long with one lane active.  Here the active lanes march one ray together:
// lane of rank k takes the k-th next sample position, the ballots find the first sample where
// the reference's loop would act (a window, or a sign change), and the 64 fine steps of that
// refinement are taken the same way.  Every position is the reference's own repeated fp64
// addition (each lane repeats k additions of the step from the chunk's first t), and the
// actions are the sequential loop's, so the t returned is vol_t's, bit for bit.
__device__ __forceinline__ int nth_lane(uint64_t m, int r) {   // the lane of the r-th set bit of m
    for (int k = 0; k < r; k++) m &= m - 1ull;
    return __builtin_ctzll(m);
}
// t plus k steps, k = 0..63, as k repeated fp64 additions of `step` give it (a power of two: the
// march's 1/512, divided by 64 at each refinement).  When t's ulp divides the step and t + 63
// steps stays in t's binade, every partial sum is exact, so one addition of k·step (exact) gives
// the same bits; otherwise the k additions are made.
__device__ __forceinline__ double march_pos(double t, double step, int k, bool exact) {
    if (exact) return t + (double)k * step;
    double u = t;
    for (int j = 0; j < k; j++) u += step;
    return u;
}
__device__ __forceinline__ bool march_exact(double t, double step) {   // t > 0
    int e;
    (void)frexp(t, &e);   // t in [2^(e-1), 2^e), ulp 2^(e-53)
    return ldexp(1.0, e - 53) <= step && t + 63.0 * step < ldexp(1.0, e);
}
// The Sign of march position t: a uniform cell's (pt_ext.h vol_build_runs: every sample in it has
// that Sign) without the eight corner loads and the interpolation, else Volume.Sign of the sample.
__device__ __forceinline__ int vol_sign_fast(const DevVolume& v, v3 o, v3 d, double t) {
    return vol_sign_at(v, o, d, t);   // the key and the sample from one scaling of the position
}
// vol_sign_at with the shader clock read between its phases (counted passes only, pt_trace_counters
// march_clock): dt[0] += the position, its scaling, the key and the uniform-cell table read; dt[1] += the
// corner reads and the interpolation; dt[2] += the window loop (Volume.Sign).  Each phase's end waits for its
// loads (the asm statements use their values), so the clocks bracket the latencies.  Same result.
__device__ __forceinline__ int vol_sign_at_timed(const DevVolume& v, v3 o, v3 d, double t, uint64_t dt[3]) {
    const uint64_t c0 = clock64();
    const v3 a = add(o, muls(d, t));   // Ray.Position
    double x = a.x, z = a.z;
    z = vol_zdiv(v, z);
    x = ((x + 1) / 2) * (double)v.w;
    double y = ((z + 1) / 2) * (double)v.h;
    z = ((z + 2) / 2) * (double)v.d;
    if (v.runs) {
        auto cl = [](double c, int n) {
            if (!(c > -2.0)) return -2;
            if (!(c < (double)n)) return n;
            return (int)floor(c);
        };
        const int st = vol_key_sign(v, VolKey{cl(x, v.w), cl(y, v.h), cl(z, v.d)});
        asm volatile("" ::"v"(st));
        const uint64_t c1 = clock64();
        dt[0] += c1 - c0;
        if (st > 0) return st;
    } else {
        dt[0] += clock64() - c0;
    }
    const uint64_t c1 = clock64();
    double smp = 0.0;
    const double lim = 2147483647.0;
    if (fabs(x) < lim && fabs(y) < lim && fabs(z) < lim) {
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
        const double cc0 = c00 * (1 - y) + c10 * y;
        const double cc1 = c01 * (1 - y) + c11 * y;
        smp = cc0 * (1 - z) + cc1 * z;
    }
    asm volatile("" ::"v"(smp));
    const uint64_t c2 = clock64();
    dt[1] += c2 - c1;
    const int sg = vol_sign_of(v, smp);
    asm volatile("" ::"v"(sg));
    dt[2] += clock64() - c2;
    return sg;
}
// the wave's time of a phase: the longest of its lanes' (lanes outside the phase read 0)
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t y = ((uint64_t)(uint32_t)__shfl_xor((int)(x >> 32), off, 64) << 32) | (uint32_t)__shfl_xor((int)x, off, 64);
        x = x > y ? x : y;
    }
    return x;
}
// Every cell of the index box spanned by cells a and b (at most one step apart per axis) has
// Sign `sign`: then every position between a position in a and a later one in b lies in such a
// cell (each index is monotone along the ray, so the cells between lie in that box).
__device__ __forceinline__ bool vol_box_sign(const DevVolume& v, VolKey a, VolKey b, int sign) {
    const int x0 = min(a.x, b.x), y0 = min(a.y, b.y), z0 = min(a.z, b.z);
    const int nx = max(a.x, b.x) - x0, ny = max(a.y, b.y) - y0, nz = max(a.z, b.z) - z0;
    if (nx > 1 || ny > 1 || nz > 1) return false;
    for (int c = 0; c < 8; c++) {
        const int dx = c & 1, dy = (c >> 1) & 1, dz = c >> 2;
        if (dx > nx || dy > ny || dz > nz) continue;
        if (vol_key_sign(v, VolKey{x0 + dx, y0 + dy, z0 + dz}) != sign) return false;
    }
    return true;
}
constexpr int kVolStride = 16;   // the strided pass's positions per lane (8 / 32 measured: no better)
// Every active lane passes the same (v, o, d); returns vol_t(v, o, d) to all of them and, in
// `samples`, the Volume.Sample calls vol_t makes (instrumentation).
// clk (counted passes, else null): the phase clocks of pt_trace_counters::march_clock, added by the first
// active lane at the end.
template <bool TIMED>
__device__ inline double coop_vol_t(const DevVolume& v, v3 o, v3 d, uint32_t& samples, unsigned long long* clk) {
    const uint64_t act = __ballot(true);
    const int lane = threadIdx.x & 63;
    const uint64_t lower = act & ((1ull << lane) - 1ull);
    const int rank = __popcll(lower), nact = __popcll(act);
    const int prev_lane = lower ? 63 - __builtin_clzll(lower) : lane;
    const int last_lane = 63 - __builtin_clzll(act);
    double tmin, tmax;
    box_span(v.bmin, v.bmax, o, d, tmin, tmax);
    double step = (double)(1.0f / 512.0f);
    double t = net_max(step, tmin);
    int sign = -1, iters = 0;
    samples = 0;
    auto sign_at = [&](double tt) { return vol_sign_fast(v, o, d, tt); };
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // clk: strided, table, corners, windows, rest, refinements, rounds x2
    auto flush = [&]() {
        if (TIMED && clk && lane == __builtin_ctzll(act))
            for (int k = 0; k < 8; k++) atomicAdd(clk + k, (unsigned long long)ph[k]);
    };
    for (;;) {   // wave-uniform: every branch below is on ballots
        const uint64_t cs = TIMED ? clock64() : 0;
        // Strided pass over runs of uniform cells: lane of rank r looks at position (r + 1)·S from
        // t; when the cells of consecutive looked-at positions (and of position 0) span only cells
        // of the running Sign, no position up to there can act, and the march moves past them,
        // 64·S positions per round.  The positions are the reference's repeated additions (t_after).
        while (v.runs) {   // wave-uniform
            const VolKey k0 = vol_key(v, o, d, t);
            const int s0 = vol_key_sign(v, k0);
            if (s0 <= 0 || (sign >= 0 && s0 != sign)) break;
            const int off = (rank + 1) * kVolStride;
            const double tr = t_after(t, step, off);
            const bool valid = tr <= tmax && iters + off < (1 << 24);
            const VolKey kr = vol_key(v, o, d, tr);
            VolKey kp{__shfl(kr.x, prev_lane, 64), __shfl(kr.y, prev_lane, 64), __shfl(kr.z, prev_lane, 64)};
            if (rank == 0) kp = k0;
            const uint64_t unsafe = __ballot(!(valid && vol_box_sign(v, kp, kr, s0)));
            const int f = unsafe ? __popcll(act & ((1ull << __builtin_ctzll(unsafe)) - 1ull)) : nact;   // safe ranks
            if (f == 0) break;
            const int k = f * kVolStride + 1;   // positions 0 .. f·S: all of Sign s0
            samples += (uint32_t)k;   // counted: the reference samples them
            t = t_after(t, step, k);
            iters += k;
            sign = s0;
            if (TIMED) ph[7]++;
            if (f < nact) break;
        }
        uint64_t cd = 0, dt[3] = {0, 0, 0};
        if (TIMED) {
            cd = clock64();
            ph[0] += cd - cs;
            ph[6]++;
        }
        const double tk = march_pos(t, step, rank, march_exact(t, step));
        const bool valid = tk <= tmax && iters + rank < (1 << 24);   // a prefix of the ranks (t grows)
        const int sg = valid ? (TIMED ? vol_sign_at_timed(v, o, d, tk, dt) : sign_at(tk)) : 0;
        const int sp = __shfl(sg, prev_lane, 64);
        const int prev = rank == 0 ? sign : sp;
        const uint64_t evb = __ballot(valid && (sg == 0 || (prev >= 0 && sg != prev)));
        if (TIMED) {   // this round's phases (the wave's: its longest lane's), the rest of it is bookkeeping
            const uint64_t t0 = wave_max_u64(dt[0]), t1 = wave_max_u64(dt[1]), t2 = wave_max_u64(dt[2]);
            const uint64_t all = clock64() - cd;
            ph[1] += t0; ph[2] += t1; ph[3] += t2;
            ph[4] += all > t0 + t1 + t2 ? all - (t0 + t1 + t2) : 0;
        }
        if (evb == 0ull) {
            const uint64_t vb = __ballot(valid);
            if (vb != act) {   // the loop's condition ended it first
                samples += (uint32_t)__popcll(vb);
                flush();
                return kHitInf;
            }
            samples += (uint32_t)nact;
            t = __shfl(tk, last_lane, 64) + step;
            sign = __shfl(sg, last_lane, 64);
            iters += nact;
            continue;
        }
        const uint64_t cr = TIMED ? clock64() : 0;
        const int ke = __builtin_ctzll(evb);
        const int re = __popcll(act & ((1ull << ke) - 1ull));
        samples += (uint32_t)(re + 1);
        double tr = __shfl(tk, ke, 64);
        const int sge = __shfl(sg, ke, 64);
        tr -= step;   // the refinement (Volume.cs:183-191)
        step /= 64;
        tr += step;
        for (int j0 = 0; j0 < 64; j0 += nact) {
            const double u = march_pos(tr, step, rank, march_exact(tr, step));
            const bool in = j0 + rank < 64;
            const uint64_t zb = __ballot(in && sign_at(u) == 0);
            if (zb) {
                const int kz = __builtin_ctzll(zb);
                samples += (uint32_t)(__popcll(act & ((1ull << kz) - 1ull)) + 1);
                if (TIMED) { ph[5] += clock64() - cr; flush(); }
                return __shfl(u, kz, 64) - step;
            }
            const int cnt = min(nact, 64 - j0);
            samples += (uint32_t)cnt;
            tr = __shfl(u, cnt == nact ? last_lane : nth_lane(act, cnt - 1), 64) + step;
        }
        t = tr + step;   // the outer loop's t += step, with the refined step
        sign = sge;
        iters += re + 1;
        if (TIMED) ph[5] += clock64() - cr;
    }
}
// Intersect of analytic record p (march_deferred) by the active lanes together: prim_t's t.
// TIMED (counted passes): the march's phase clocks (pt_trace_counters::march_clock); the timed passes' kernels
// are built without them (their registers: the FULL kernels spilled 31 more VGPRs with the clocks inline).
template <bool TIMED>
__device__ __forceinline__ double coop_record_t_body(const DevScene& S, int32_t p, v3 o, v3 d, int32_t& kind,
                                                    double& tobj) {
    const float4* r = S.ana_recs + 3 * (size_t)p;
    kind = (int32_t)f2u(r[0].w);
    uint32_t n = 0;
    double t;
    // S.march = word 9; this wave's slot of the phase clocks
    unsigned long long* const clk = TIMED && S.march
        ? S.march + (kMarchClockWord - 9) + 8 * (((blockIdx.x * blockDim.x + threadIdx.x) >> 6) & (kMarchSlots - 1)) : nullptr;
    if (kind == KIND_VOLUME) {
        t = coop_vol_t<TIMED>(S.volumes[rec_ext(r)], o, d, n, clk);
        tobj = t;
    } else {   // xform_t over an inner Volume (TransformedShape.cs:43-73)
        const DevXform& X = S.xforms[rec_ext(r)];
        const v3 so = mat_position(X.inv, o), sd = mat_direction(X.inv, d);
        t = coop_vol_t<TIMED>(S.volumes[rec_ext(S.ext_recs + 3 * (size_t)X.rec)], so, sd, n, clk);
        tobj = t;
        if (t < kHitInf) {
            const v3 position = mat_position(X.m, add(so, muls(sd, t)));
            t = (double)lengthf(sub(position, o));
        }
    }
    if (S.march && (threadIdx.x & 63) == __builtin_ctzll(__ballot(true))) atomicAdd(S.march, (unsigned long long)n);
    return t;
}
// Out of line in the FULL traversal kernels (their registers), inlined in k_wf_vol_* (INL).
template <bool TIMED>
__device__ __noinline__ double coop_record_t(const DevScene& S, int32_t p, v3 o, v3 d, int32_t& kind, double& tobj) {
    return coop_record_t_body<TIMED>(S, p, o, d, kind, tobj);
}
// The lanes' pending Volume records, one ray at a time by all active lanes (at least S.coop_min_lanes):
// march_pending's merge, without its few-lanes fallback (k_wf_vol_hits / k_wf_vol_shadow run full waves).
template <bool ANY, bool INL, bool TIMED>
__device__ inline void march_coop(const DevScene& S, v3 o, v3 d, int32_t pend, HitRec& best, bool* blocked) {
    const int lane = threadIdx.x & 63;
    for (uint64_t todo = __ballot(pend >= 0); todo; todo &= todo - 1ull) {   // wave-uniform
        const int src = __builtin_ctzll(todo);
        const int32_t p = __shfl(pend, src, 64);
        const v3 so{__shfl(o.x, src, 64), __shfl(o.y, src, 64), __shfl(o.z, src, 64)};
        const v3 sd{__shfl(d.x, src, 64), __shfl(d.y, src, 64), __shfl(d.z, src, 64)};
        int32_t kind;
        double tx = 0;
        const double t = INL ? coop_record_t_body<TIMED>(S, p, so, sd, kind, tx) : coop_record_t<TIMED>(S, p, so, sd, kind, tx);
        if (lane == src) {
            if (ANY) {
                if (t < best.t) *blocked = true;
            } else if (t < best.t || (t == best.t && best.kind == KIND_TRI)) {
                best.t = t; best.kind = kind; best.idx = p; best.tx = tx;
            }
        }
    }
}
// The lanes' pending Volume records (traverse's pend), one ray at a time by all active lanes.
// Closest hit: the march's t replaces the best when nearer, and on a tie with a triangle (the
// analytic BVH is traversed before the triangles, which replace only a strictly farther best);
// any-hit (ANY): *blocked when nearer than the light.
template <bool ANY, bool TIMED>
__device__ inline void march_pending(const DevScene& S, v3 o, v3 d, int32_t pend, HitRec& best, bool* blocked = nullptr) {
    auto merge = [&](double t, int32_t kind, int32_t p, double tx) {
        if (ANY) {
            if (t < best.t) *blocked = true;
        } else if (t < best.t || (t == best.t && best.kind == KIND_TRI)) {
            best.t = t; best.kind = kind; best.idx = p; best.tx = tx;
        }
    };
    if (__popcll(__ballot(true)) < S.coop_min_lanes) {   // too few lanes to share a march: each its own
        if (pend >= 0) {
            int32_t kind;
            double tx = 0;
            const double t = prim_t<false, true>(S, S.ana_recs, (uint32_t)pend, o, d, kind, &tx);
            merge(t, kind, pend, tx);
        }
        return;
    }
    march_coop<ANY, false, TIMED>(S, o, d, pend, best, blocked);
}

// Scene.Intersect (Scene.cs:75-79): closest hit over planes, analytic BVH, triangle BVH.
template <bool COUNT, bool FULL, class STK>
__device__ __forceinline__ HitRec trace(const DevScene& S, v3 o, v3 d, const STK& stack, Counters& ctr) {
    ctr.rays++;
    HitRec best{kHitInf, -1, -1};
    for (int i = 0; i < S.num_planes; i++) {
        float4 a = S.planes[2 * i], b = S.planes[2 * i + 1];
        double t = isect_plane(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
        if (t < best.t) { best.t = t; best.kind = KIND_PLANE; best.idx = i; }
    }
    v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    int32_t pend = -1;   // FULL: a Volume left for the cooperative march
    if (S.ana_linear) {   // a few analytic shapes, one by one (as the refill kernels test them; pt_scene.h)
        for (int p = 0; p < S.ana_count; p++) {
            if (COUNT) ctr.prims++;
            int32_t kind;
            double tx = 0;
            const double t = prim_t<false, FULL>(S, S.ana_recs, (uint32_t)p, o, d, kind, FULL ? &tx : nullptr);
            if (t < best.t) { best.t = t; best.kind = kind; best.idx = p; if (FULL) best.tx = tx; }
        }
    } else {
        traverse<false, COUNT, false, FULL>(S, S.ana_nodes, S.ana_num_nodes, S.ana_recs, o, d, invd, best, stack, ctr,
                                            FULL ? &pend : nullptr);
    }
    traverse_tri<COUNT, false>(S, o, d, invd, best, stack, ctr);
    if (FULL) march_pending<false, COUNT>(S, o, d, pend, best);
    return best;
}

// trace() for the scenes whose shapes are a few analytic records and planes, and no triangle BVH (lean, ana_linear,
// tri_num_nodes 0): the same tests in the same order, so the same hit; for k_wf_trace_linear, which holds no
// traversal state.
// recs / planes: S.ana_recs / S.planes or copies of them (k_wf_trace_linear stages them in LDS).
template <bool COUNT>
__device__ __forceinline__ HitRec trace_linear(const DevScene& S, const float4* recs, const float4* planes, v3 o, v3 d,
                                               Counters& ctr) {
    ctr.rays++;
    HitRec best{kHitInf, -1, -1};
    for (int i = 0; i < S.num_planes; i++) {
        float4 a = planes[2 * i], b = planes[2 * i + 1];
        double t = isect_plane(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
        if (t < best.t) { best.t = t; best.kind = KIND_PLANE; best.idx = i; }
    }
    for (int p = 0; p < S.ana_count; p++) {
        if (COUNT) ctr.prims++;
        int32_t kind;
        const double t = prim_t<false, false>(S, recs, (uint32_t)p, o, d, kind);
        if (t < best.t) { best.t = t; best.kind = kind; best.idx = p; }
    }
    return best;
}

// t of the light's own primitive along (o, d), exactly as the closest-hit query computes it.
template <bool FULL>
// lrec (may be null): the light's own record (3 float4), staged in LDS by the shadow kernels
__device__ __forceinline__ double light_t(const DevScene& S, const DevLight& L, v3 o, v3 d, const float4* lrec = nullptr) {
    if (L.kind == KIND_PLANE) {
        float4 a = S.planes[2 * L.index], b = S.planes[2 * L.index + 1];
        return isect_plane(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
    }
    int32_t kind;
    if (lrec) return prim_t<false, FULL>(S, lrec, 0u, o, d, kind);
    return prim_t<false, FULL>(S, S.ana_recs, (uint32_t)L.index, o, d, kind);
}

// Is any primitive strictly nearer than tl along (o, d)?  The any-hit half of the shadow query
// (light_visible) after the light's own t; pt_occluded runs it for a host's rays.
template <bool COUNT, bool FULL, class STK>
__device__ __forceinline__ bool any_nearer(const DevScene& S, v3 o, v3 d, double tl, const STK& stack, Counters& ctr) {
    HitRec best{tl, -1, -1};
    for (int i = 0; i < S.num_planes; i++) {
        float4 a = S.planes[2 * i], b = S.planes[2 * i + 1];
        if (isect_plane(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d) < tl) return true;
    }
    v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    int32_t pend = -1;   // FULL: a Volume left for the cooperative march
    if (S.ana_linear) {
        for (int p = 0; p < S.ana_count; p++) {
            if (COUNT) ctr.prims++;
            int32_t kind;
            if (prim_t<false, FULL>(S, S.ana_recs, (uint32_t)p, o, d, kind) < tl) return true;
        }
    } else if (traverse<false, COUNT, true, FULL>(S, S.ana_nodes, S.ana_num_nodes, S.ana_recs, o, d, invd, best, stack,
                                                 ctr, FULL ? &pend : nullptr)) {
        return true;
    }
    if (traverse_tri<COUNT, true>(S, o, d, invd, best, stack, ctr)) return true;
    if (FULL) {   // the lanes still unblocked march their pending Volume together
        bool blocked = false;
        march_pending<true, COUNT>(S, o, d, pend, best, &blocked);
        if (blocked) return true;
    }
    return false;
}

// Shadow visibility (Sampler.cs:261-265): the reference takes the nearest hit and
// compares it with the light by reference.  Equivalent query: the light's own t,
// then "is any primitive strictly nearer" (any-hit, early exit).  Counts one ray.
template <bool COUNT, bool FULL, class STK>
__device__ __forceinline__ bool light_visible(const DevScene& S, const DevLight& L, v3 o, v3 d, const STK& stack,
                                              Counters& ctr, const float4* lrec = nullptr) {
    ctr.rays++;
    if (L.phantom) {
        // a struct Triangle light never equals the re-boxed hit shape; the reference still
        // traces the ray, so trace it (the answer is "not visible" either way)
        HitRec h{kHitInf, -1, -1};
        v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        traverse_tri<COUNT, true>(S, o, d, invd, h, stack, ctr);
        return false;
    }
    const double tl = light_t<FULL>(S, L, o, d, lrec);
    if (!(tl < kHitInf)) return false;
    return !any_nearer<COUNT, FULL>(S, o, d, tl, stack, ctr);
}
// light_visible() for the same scenes as trace_linear (no triangles: a phantom light's ray has nothing to
// trace); k_wf_shadow_linear.
template <bool COUNT>
__device__ __forceinline__ bool light_visible_linear(const DevScene& S, const float4* recs, const float4* planes,
                                                     const DevLight& L, v3 o, v3 d, Counters& ctr, const float4* lrec) {
    ctr.rays++;
    if (L.phantom) return false;
    double tl;
    if (L.kind == KIND_PLANE) {   // light_t
        const float4 a = planes[2 * L.index], b = planes[2 * L.index + 1];
        tl = isect_plane(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
    } else {
        int32_t kind;
        tl = prim_t<false, false>(S, lrec ? lrec : recs + 3 * (size_t)L.index, 0u, o, d, kind);
    }
    if (!(tl < kHitInf)) return false;
    for (int i = 0; i < S.num_planes; i++) {
        float4 a = planes[2 * i], b = planes[2 * i + 1];
        if (isect_plane(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d) < tl) return false;
    }
    for (int p = 0; p < S.ana_count; p++) {
        if (COUNT) ctr.prims++;
        int32_t kind;
        if (prim_t<false, false>(S, recs, (uint32_t)p, o, d, kind) < tl) return false;
    }
    return true;
}
// Split traversal (scenes with §8f row 4 shapes and a large triangle BVH, pt_wavefront.hip
// "split"): the lean refill kernels take the planes and the triangle BVH, then the FULL kernel
// takes the analytic BVH of the same ray, starting from that hit.  Scene.Intersect visits planes,
// the analytic BVH, then the triangles, each replacing the best only when strictly nearer, so an
// analytic hit beats a triangle at an equal t and loses to a plane at an equal t: with a triangle
// best its t is raised by one ulp for the analytic pass (no double lies between), and restored
// when no analytic hit took it.  The triangles the refill kernel found without the analytic
// hit's tighter bound are the same: a bound only prunes, it never reorders the visits.
// sdf_out: the SDF record left for k_wf_sdf_hits (-1: none), not merged here; vol_out: likewise the
// Volume record left for k_wf_vol_hits, which merges it first.
template <bool COUNT, class STK>
__device__ __forceinline__ void trace_ana(const DevScene& S, v3 o, v3 d, const STK& stack, Counters& ctr, HitRec& best,
                                          int32_t* sdf_out = nullptr, int32_t* vol_out = nullptr) {
    const double t_in = best.t;
    const bool tri_best = best.kind == KIND_TRI;
    if (tri_best) best.t = nextafter(best.t, (double)INFINITY);
    v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    int32_t pend = -1, pend_sdf = -1;
    if (S.ana_linear) {
        for (int p = 0; p < S.ana_count; p++) {
            if (COUNT) ctr.prims++;
            int32_t kind;
            double tx = 0;
            const double t = prim_t<false, true>(S, S.ana_recs, (uint32_t)p, o, d, kind, &tx);
            if (t < best.t) { best.t = t; best.kind = kind; best.idx = p; best.tx = tx; }
        }
    } else {
        traverse<false, COUNT, false, true>(S, S.ana_nodes, S.ana_num_nodes, S.ana_recs, o, d, invd, best, stack, ctr, &pend,
                                            sdf_out ? &pend_sdf : nullptr);
    }
    if (vol_out) *vol_out = pend;
    else march_pending<false, COUNT>(S, o, d, pend, best);
    if (sdf_out) *sdf_out = pend_sdf;
    else sdf_pending<false>(S, o, d, pend_sdf, best);
    if (best.kind == KIND_TRI && tri_best) best.t = t_in;
}
// The analytic half of a split shadow query (light_visible's analytic part): is any analytic
// primitive strictly nearer than the light?  The refill kernel already cleared the planes and
// the triangles.
// sdf_out: the SDF record left for k_wf_sdf_shadow (-1: none), with the light's t; vol_out: the
// Volume record left for k_wf_vol_shadow.
template <bool COUNT, class STK>
__device__ __forceinline__ bool ana_blocked(const DevScene& S, const DevLight& L, v3 o, v3 d, const STK& stack,
                                            Counters& ctr, int32_t* sdf_out = nullptr, double* tl_out = nullptr,
                                            int32_t* vol_out = nullptr) {
    const double tl = light_t<true>(S, L, o, d);
    if (!(tl < kHitInf)) return true;   // (the refill kernel found it lit, so tl is finite)
    HitRec best{tl, -1, -1};
    v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    int32_t pend = -1, pend_sdf = -1;
    if (S.ana_linear) {
        for (int p = 0; p < S.ana_count; p++) {
            if (COUNT) ctr.prims++;
            int32_t kind;
            if (prim_t<false, true>(S, S.ana_recs, (uint32_t)p, o, d, kind) < tl) return true;
        }
    } else if (traverse<false, COUNT, true, true>(S, S.ana_nodes, S.ana_num_nodes, S.ana_recs, o, d, invd, best, stack, ctr,
                                                   &pend, sdf_out ? &pend_sdf : nullptr)) {
        return true;
    }
    if (vol_out) {
        *vol_out = pend;
    } else {
        bool blocked = false;
        march_pending<true, COUNT>(S, o, d, pend, best, &blocked);
        if (blocked) return true;
    }
    if (sdf_out) {   // left for k_wf_sdf_shadow
        *sdf_out = pend_sdf;
        *tl_out = tl;
        return false;
    }
    bool blocked = false;
    sdf_pending<true>(S, o, d, pend_sdf, best, &blocked);
    return blocked;
}

// ---- Routed split (DevScene::route).  The refill kernels test the lean analytic records (spheres,
// cubes) themselves; a ray whose segment [0, best] reaches the BVH box of a row-4 ("heavy") record is
// the only kind that goes on to the FULL kernels, which test just those records.  The boxes are the
// ones the analytic BVH holds (widened by the march pads, so every reference hit lies inside), and a
// record the BVH would reach lies inside every box on its path: testing its own box prunes exactly
// the records that cannot give a nearer hit, as the split's bound does.
__device__ __forceinline__ bool heavy_reach(const DevScene& S, v3 o, v3 invd, float tmax) {
    for (int h = 0; h < S.heavy_count; h++) {
        const float4 lo = S.heavy[2 * h], hi = S.heavy[2 * h + 1];
        if (slab1(lo.x, hi.x, lo.y, hi.y, lo.z, hi.z, o, invd, tmax) != __int_as_float(0x7f800000)) return true;
    }
    return false;
}
// trace_ana over the heavy records only (the refill kernel took the planes, the lean analytic records
// and the triangles): the same merge rules, the same deferred Volume march and SDF queue.
template <bool COUNT>
__device__ __forceinline__ void trace_heavy(const DevScene& S, v3 o, v3 d, Counters& ctr, HitRec& best,
                                            int32_t* sdf_out, int32_t* vol_out) {
    const double t_in = best.t;
    const bool tri_best = best.kind == KIND_TRI;
    if (tri_best) best.t = nextafter(best.t, (double)INFINITY);
    const v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    int32_t pend = -1, pend_sdf = -1;
    for (int h = 0; h < S.heavy_count; h++) {
        const float4 lo = S.heavy[2 * h], hi = S.heavy[2 * h + 1];
        if (slab1(lo.x, hi.x, lo.y, hi.y, lo.z, hi.z, o, invd, tmax_bound(best.t)) == __int_as_float(0x7f800000)) continue;
        const uint32_t p = f2u(lo.w);
        if (COUNT) ctr.prims++;
        const float4* r = S.ana_recs + 3 * (size_t)p;
        if (pend < 0 && march_deferred(S, r)) { pend = (int32_t)p; continue; }
        if (sdf_out && pend_sdf < 0 && sdf_deferred(S, r)) { pend_sdf = (int32_t)p; continue; }
        int32_t kind;
        double tx = 0;
        const double t = prim_t<false, true>(S, S.ana_recs, p, o, d, kind, &tx);
        if (t < best.t) { best.t = t; best.kind = kind; best.idx = (int32_t)p; best.tx = tx; }
    }
    if (vol_out) *vol_out = pend;
    else march_pending<false, COUNT>(S, o, d, pend, best);
    if (sdf_out) *sdf_out = pend_sdf;
    else sdf_pending<false>(S, o, d, pend_sdf, best);
    if (best.kind == KIND_TRI && tri_best) best.t = t_in;
}
// ana_blocked over the heavy records only.
template <bool COUNT>
__device__ __forceinline__ bool heavy_blocked(const DevScene& S, const DevLight& L, v3 o, v3 d, Counters& ctr,
                                              int32_t* sdf_out, double* tl_out, int32_t* vol_out) {
    const double tl = light_t<true>(S, L, o, d);
    if (!(tl < kHitInf)) return true;
    HitRec best{tl, -1, -1};
    const v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const float tmax = tmax_bound(tl);
    int32_t pend = -1, pend_sdf = -1;
    for (int h = 0; h < S.heavy_count; h++) {
        const float4 lo = S.heavy[2 * h], hi = S.heavy[2 * h + 1];
        if (slab1(lo.x, hi.x, lo.y, hi.y, lo.z, hi.z, o, invd, tmax) == __int_as_float(0x7f800000)) continue;
        const uint32_t p = f2u(lo.w);
        if (COUNT) ctr.prims++;
        const float4* r = S.ana_recs + 3 * (size_t)p;
        if (pend < 0 && march_deferred(S, r)) { pend = (int32_t)p; continue; }
        if (sdf_out && pend_sdf < 0 && sdf_deferred(S, r)) { pend_sdf = (int32_t)p; continue; }
        int32_t kind;
        if (prim_t<false, true>(S, S.ana_recs, p, o, d, kind) < tl) return true;
    }
    if (vol_out) {
        *vol_out = pend;
    } else {
        bool blocked = false;
        march_pending<true, COUNT>(S, o, d, pend, best, &blocked);
        if (blocked) return true;
    }
    if (sdf_out) {
        *sdf_out = pend_sdf;
        *tl_out = tl;
        return false;
    }
    bool blocked = false;
    sdf_pending<true>(S, o, d, pend_sdf, best, &blocked);
    return blocked;
}

// ---------------------------------------------------------------- textures (§8f row 3)
// Util.Modf / ColorTexture.Fract (Util.cs:108-113, Texture.cs:218-222): fractional part, sign kept.
__device__ __forceinline__ double fract_d(double x) { return x - trunc(x); }

// ColorTexture.BilinearSample (Texture.cs:188-216), fp64 over the C# texels.  The
// reference's int conversions throw OverflowException on non-finite coordinates; such a
// lookup is black here and in the oracle.
__device__ inline void tex_bilinear(const DevTexture& T, double u, double v, double c[3]) {
    if (u == 1) u -= kEps;
    if (v == 1) v -= kEps;
    const double w = (double)T.w - 1, h = (double)T.h - 1;
    const double uw = u * w, vh = v * h;
    c[0] = 0.0; c[1] = 0.0; c[2] = 0.0;
    if (!isfinite(uw) || !isfinite(vh)) return;
    const double X = trunc(uw), x = uw - X, Y = trunc(vh), y = vh - Y;
    PT_GLOBAL(double) r0 = (PT_GLOBAL(double))(T.data + 3 * ((size_t)(int)Y * (size_t)T.w + (size_t)(int)X));
    PT_GLOBAL(double) r1 = r0 + 3 * (size_t)T.w;
    const double w00 = (1 - x) * (1 - y), w10 = x * (1 - y), w01 = (1 - x) * y, w11 = x * y;
    for (int k = 0; k < 3; k++) {   // Black.Add(c00·w00).Add(c10·w10).Add(c01·w01).Add(c11·w11)
        double a = 0.0;
        a = a + r0[k] * w00;
        a = a + r0[3 + k] * w10;
        a = a + r1[k] * w01;
        a = a + r1[3 + k] * w11;
        c[k] = a;
    }
}
// ITexture.Sample (Texture.cs:224-229)
__device__ inline void tex_sample(const DevTexture& T, double u, double v, double c[3]) {
    u = fract_d(fract_d(u) + 1);
    v = fract_d(fract_d(v) + 1);
    tex_bilinear(T, u, 1 - v, c);
}
// ITexture.NormalSample (Texture.cs:231-237)
__device__ inline v3 tex_normal_sample(const DevTexture& T, double u, double v) {
    double c[3];
    tex_sample(T, u, v, c);
    return normalize(mk(c[0] * 2 - 1, c[1] * 2 - 1, c[2] * 2 - 1));
}
// ITexture.BumpSample (Texture.cs:239-251); row Height (v == 0, an IndexOutOfRange in the
// reference) is clamped, as in the oracle.
__device__ inline v3 tex_bump_sample(const DevTexture& T, double u, double v) {
    u = fract_d(fract_d(u) + 1);
    v = 1 - fract_d(fract_d(v) + 1);
    const double fx = u * T.w, fy = v * T.h;
    if (!isfinite(fx) || !isfinite(fy)) return zero3();
    const int x = min((int)fx, T.w - 1), y = min((int)fy, T.h - 1);
    const int x1 = max(x - 1, 0), x2 = min(x + 1, T.w - 1), y1 = max(y - 1, 0), y2 = min(y + 1, T.h - 1);
    const double* d = T.data;
    const size_t W = (size_t)T.w;
    const double cx = d[3 * ((size_t)y * W + x1)] - d[3 * ((size_t)y * W + x2)];
    const double cy = d[3 * ((size_t)y1 * W + x)] - d[3 * ((size_t)y2 * W + x)];
    return mk(cx, cy, 0);
}
__device__ __forceinline__ bool nonzero3(v3 a) { return !(a.x == 0 && a.y == 0 && a.z == 0); }

__device__ __forceinline__ void tri_uvs(const DevScene& S, int idx, v3& t1, v3& t2, v3& t3) {
    const float4* u = S.tri_uv + (size_t)S.tri_ustride * idx;
    const float4 A = u[0], B = u[1];
    t1 = v3{A.x, A.y, 0.f}; t2 = v3{A.z, A.w, 0.f}; t3 = v3{B.x, B.y, 0.f};
}

// IShape.UVector (Sphere.cs:62-69 with its p.Y-for-p.Z slip, Cube.cs:49-53, Plane.cs:52-55,
// Triangle.cs:127-136; SDFShape / Volume give 0) of the primitive at record `idx` of `recs`
// (default: the analytic records).
__device__ inline v3 shape_uv(const DevScene& S, int kind, int idx, v3 p, const float4* recs = nullptr) {
    if (kind == KIND_TRI) {
        const float4* r = S.tri_recs + (size_t)S.tri_rstride * idx;
        const float4 a = r[0], b = r[1], c = r[2];
        double u, v, w;
        barycentric(v3{a.x, a.y, a.z}, v3{a.w, b.x, b.y}, v3{b.z, b.w, c.x}, p, u, v, w);
        v3 t1, t2, t3;
        tri_uvs(S, idx, t1, t2, t3);
        const v3 n = add(add(add(zero3(), muls(t1, u)), muls(t2, v)), muls(t3, w));
        return v3{n.x, n.y, 0.f};
    }
    if (kind != KIND_SPHERE && kind != KIND_CUBE) return zero3();
    const float4* r = (recs ? recs : S.ana_recs) + 3 * (size_t)idx;
    const float4 a = r[0], b = r[1];
    if (kind == KIND_SPHERE) {
        const v3 q = sub(p, v3{a.x, a.y, a.z});
        double u = atan2((double)q.z, (double)q.x);
        double v = atan2((double)q.y, (double)lengthf(v3{q.x, 0.f, q.y}));
        u = 1 - (u + kPi) / (2 * kPi);
        v = (v + kPi / 2) / kPi;
        return mk(u, v, 0);
    }
    const v3 q = divv(sub(p, v3{a.x, a.y, a.z}), sub(v3{b.x, b.y, b.z}, v3{a.x, a.y, a.z}));
    return v3{q.x, q.z, 0.f};
}

// Material.MaterialAt (Material.cs:124-138): the colour and gloss seen at p.  FULL = the
// scene has textures: kernels are instantiated both ways, so untextured scenes run the
// shading code without any texture path (no extra registers in the hot kernels).
template <bool FULL>
__device__ __forceinline__ void surface_at(const DevScene& S, const DevMaterial& m, int kind, int idx, v3 p,
                                           double col[3], double& gloss, const float4* recs = nullptr) {
    col[0] = m.color[0]; col[1] = m.color[1]; col[2] = m.color[2];
    gloss = m.gloss;
    if (!FULL || (m.tex < 0 && m.gtex < 0)) return;
    const v3 uv = shape_uv(S, kind, idx, p, recs);
    double c[3];
    if (m.tex >= 0) {
        tex_sample(S.texs[m.tex], uv.x, uv.y, c);
        col[0] = c[0]; col[1] = c[1]; col[2] = c[2];
    }
    if (m.gtex >= 0) {
        tex_sample(S.texs[m.gtex], uv.x, uv.y, c);
        gloss = (c[0] + c[1] + c[2]) / 3;
    }
}

// Triangle.NormalAt with NormalTexture / BumpTexture (Triangle.cs:142-189).
__device__ __noinline__ v3 tri_normal_mapped(const DevScene& S, const DevMaterial& m, int idx, v3 v1, v3 e1, v3 e2,
                                             v3 n1, v3 n2, v3 n3, v3 p) {
    double u, v, w;
    barycentric(v1, e1, e2, p, u, v, w);
    v3 n = add(add(muls(n1, u), muls(n2, v)), muls(n3, w));
    v3 t1, t2, t3;
    tri_uvs(S, idx, t1, t2, t3);
    const v3 dt1 = sub(t2, t1), dt2 = sub(t3, t1);   // dv1 = V2 - V1 = e1, dv2 = V3 - V1 = e2
    if (m.ntex >= 0) {
        const v3 b = add(add(muls(t1, u), muls(t2, v)), muls(t3, w));
        const v3 ns = tex_normal_sample(S.texs[m.ntex], b.x, b.y);
        if (nonzero3(ns)) {
            const v3 T = normalize(sub(muls(e1, dt2.y), muls(e2, dt1.y)));
            const v3 B = normalize(sub(muls(e2, dt1.x), muls(e1, dt2.x)));
            const v3 N = cross(T, B);
            // Matrix(T.X, B.X, N.X, 0, ...).MulDirection(ns) (Matrix.cs:144-150)
            const double x = (double)T.x * ns.x + (double)B.x * ns.y + (double)N.x * ns.z;
            const double y = (double)T.y * ns.x + (double)B.y * ns.y + (double)N.y * ns.z;
            const double z = (double)T.z * ns.x + (double)B.z * ns.y + (double)N.z * ns.z;
            n = normalize(mk(x, y, z));
        }
    }
    if (m.btex >= 0) {
        const v3 b = add(add(muls(t1, u), muls(t2, v)), muls(t3, w));
        const v3 bump = tex_bump_sample(S.texs[m.btex], b.x, b.y);
        if (nonzero3(bump)) {
            const v3 tangent = normalize(sub(muls(e1, dt2.y), muls(e2, dt1.y)));
            const v3 bitangent = normalize(sub(muls(e2, dt1.x), muls(e1, dt2.x)));
            n = add(n, muls(tangent, (double)bump.x * m.bump_multiplier));
            n = add(n, muls(bitangent, (double)bump.y * m.bump_multiplier));
        }
    }
    return normalize(n);
}

// sampleEnvironment (Sampler.cs:177-189)
template <bool FULL>
__device__ __forceinline__ double3 environment(const DevScene& S, v3 d) {
    if (!FULL || S.env_tex < 0) return make_double3(S.env[0], S.env[1], S.env[2]);
    double u = atan2((double)d.z, (double)d.x) + S.env_angle;
    double v = atan2((double)d.y, (double)lengthf(v3{d.x, 0.f, d.z}));
    u = (u + kPi) / (2 * kPi);
    v = (v + kPi / 2) / kPi;
    double c[3];
    tex_sample(S.texs[S.env_tex], u, v, c);
    return make_double3(c[0], c[1], c[2]);
}

struct Shade {
    v3 pos, nrm;
    int32_t mat;
    int32_t inside;
    double col[3];   // Material.MaterialAt colour (texture applied), fp64 Colour
    double gloss;    // and gloss (gloss texture applied)
};

// Triangle.NormalAt (maps included) and its material id, for triangle record idx of S.tri_recs / tri_shade.
__device__ inline v3 tri_normal_at(const DevScene& S, int idx, v3 p, int32_t& mat) {
    const float4* r = S.tri_recs + (size_t)S.tri_rstride * idx;
    const float4* q = S.tri_shade + (size_t)S.tri_rstride * idx;
    const float4 a = r[0], b = r[1], c = r[2];
    const float4 x = q[0], y = q[1], z = q[2];
    mat = (int32_t)f2u(z.y);
    const DevMaterial& m = S.mats[mat];
    const v3 v1{a.x, a.y, a.z}, e1{a.w, b.x, b.y}, e2{b.z, b.w, c.x};
    const v3 n1{x.x, x.y, x.z}, n2{x.w, y.x, y.y}, n3{y.z, y.w, z.x};
    if (m.ntex < 0 && m.btex < 0) return tri_normal(v1, e1, e2, n1, n2, n3, p);
    return tri_normal_mapped(S, m, idx, v1, e1, e2, n1, n2, n3, p);
}

// NormalAt / MaterialAt of an analytic-format record (kinds that can be a TransformedShape's inner shape).
__device__ inline v3 inner_normal(const DevScene& S, const float4* r, int32_t kind, v3 p) {
    const float4 a = r[0], b = r[1];
    switch (kind) {
        case KIND_SPHERE: return normalize(sub(p, v3{a.x, a.y, a.z}));                 // Sphere.NormalAt
        case KIND_CUBE: return cube_normal(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, p);    // Cube.NormalAt
        case KIND_PLANE: return v3{b.x, b.y, b.z};                                      // Plane.NormalAt
        case KIND_SDF: return sdf_normal(S.sdf_prog, S.sdf_params, S.sdf_shapes[rec_ext(r)], p);
        default: return vol_normal(S.volumes[rec_ext(r)], p);
    }
}
__device__ inline int32_t inner_material(const DevScene& S, const float4* r, int32_t kind, v3 p) {
    if (kind == KIND_VOLUME) return vol_material(S.volumes[rec_ext(r)], p, S.default_mat);
    return (int32_t)f2u(r[2].x);
}

// Hit.Info for the §8f row 4 kinds.  SDFShape / Volume: the normal flips but `inside`
// stays false (Hit.cs:42-49).  TransformedShape: the HitInfo its Intersect builds
// (TransformedShape.cs:52-70), recomputed from the same inner intersect.
__device__ __noinline__ void ext_hit_info(const DevScene& S, const HitRec& h, v3 o, v3 d, Shade& s) {
    const float4* r = S.ana_recs + 3 * (size_t)h.idx;
    v3 n;
    if (h.kind == KIND_XFORM) {
        const DevXform& X = S.xforms[rec_ext(r)];
        const v3 so = mat_position(X.inv, o), sd = mat_direction(X.inv, d);
        v3 sp, sn;
        if (X.kind == KIND_MESH) {   // hit.Shape is the mesh's Triangle: shade it from the BLAS records
            const HitRec ih = blas_hit(S, X.rec, so, sd);
            const int off = S.blas[X.rec].rec_off;
            DevScene T = S;
            T.tri_recs = S.blas_recs + 3 * (size_t)off;
            T.tri_shade = S.blas_shade + 3 * (size_t)off;
            T.tri_uv = S.blas_uv ? S.blas_uv + 2 * (size_t)off : nullptr;
            T.tri_rstride = 3;
            T.tri_ustride = 2;
            sp = add(so, muls(sd, ih.t));
            sn = tri_normal_at(T, ih.idx, sp, s.mat);
            surface_at<true>(T, S.mats[s.mat], KIND_TRI, ih.idx, sp, s.col, s.gloss);
        } else {
            const float4* ir = S.ext_recs + 3 * (size_t)X.rec;
            // the inner intersect's t as the closest-hit query found it (HitRec::tx), not a second
            // intersect here (for a Volume, a whole march per hit)
            const double t = h.tx;
            sp = add(so, muls(sd, t));
            sn = inner_normal(S, ir, X.kind, sp);
            s.mat = inner_material(S, ir, X.kind, sp);
            surface_at<true>(S, S.mats[s.mat], X.kind, X.rec, sp, s.col, s.gloss, S.ext_recs);
        }
        s.pos = mat_position(X.m, sp);
        n = mat_direction_t(X.inv, sn);   // Matrix.Inverse().Transpose().MulDirection
        s.inside = 0;
        if (dot(sn, sd) > 0) { n = neg(n); s.inside = 1; }
        s.nrm = n;
        return;
    }
    s.pos = add(o, muls(d, h.t));
    n = inner_normal(S, r, h.kind, s.pos);
    s.mat = inner_material(S, r, h.kind, s.pos);
    surface_at<true>(S, S.mats[s.mat], h.kind, h.idx, s.pos, s.col, s.gloss);
    s.inside = 0;
    if (dot(n, d) > 0) n = neg(n);
    s.nrm = n;
}

// Hit.Info (Hit.cs:26-55): position (fp32 re-rounded), NormalAt, MaterialAt, flip.
template <bool COUNT, bool FULL>
__device__ __forceinline__ Shade hit_info(const DevScene& S, const HitRec& h, v3 o, v3 d, Counters& ctr) {
    Shade s;
    s.pos = add(o, muls(d, h.t));
    v3 n;
    if (h.kind == KIND_TRI) {
        if (COUNT) ctr.shades++;
        const float4* r = S.tri_recs + (size_t)S.tri_rstride * h.idx;
        const float4* q = S.tri_shade + (size_t)S.tri_rstride * h.idx;
        float4 a = r[0], b = r[1], c = r[2];
        float4 x = q[0], y = q[1], z = q[2];
        s.mat = (int32_t)f2u(z.y);
        const DevMaterial& m = S.mats[s.mat];
        const v3 v1{a.x, a.y, a.z}, e1{a.w, b.x, b.y}, e2{b.z, b.w, c.x};
        const v3 n1{x.x, x.y, x.z}, n2{x.w, y.x, y.y}, n3{y.z, y.w, z.x};
        if (!FULL || (m.ntex < 0 && m.btex < 0)) n = tri_normal(v1, e1, e2, n1, n2, n3, s.pos);
        else n = tri_normal_mapped(S, m, h.idx, v1, e1, e2, n1, n2, n3, s.pos);
    } else if (h.kind == KIND_PLANE) {
        float4 a = S.planes[2 * h.idx], b = S.planes[2 * h.idx + 1];
        n = v3{b.x, b.y, b.z};
        s.mat = (int32_t)f2u(a.w);
    } else if (!FULL || h.kind == KIND_SPHERE || h.kind == KIND_CUBE) {
        const float4* r = S.ana_recs + 3 * (size_t)h.idx;
        float4 a = r[0], b = r[1], c = r[2];
        if (h.kind == KIND_SPHERE) n = normalize(sub(s.pos, v3{a.x, a.y, a.z}));   // Sphere.NormalAt
        else n = cube_normal(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, s.pos);           // Cube.NormalAt
        s.mat = (int32_t)f2u(c.x);
    } else {
        ext_hit_info(S, h, o, d, s);
        return s;
    }
    surface_at<FULL>(S, S.mats[s.mat], h.kind, h.idx, s.pos, s.col, s.gloss);
    s.inside = 0;
    if (dot(n, d) > 0) { n = neg(n); s.inside = 1; }
    s.nrm = n;
    return s;
}

// Util.Cone (Util.cs:17-32)
__device__ __forceinline__ v3 cone(v3 direction, double theta, double u, double v, uint64_t key) {
    if (theta < kEps) return direction;
    theta = theta * (1 - (2 * acos(u) / kPi));
    double m1, m2;
    pt_sincos(theta, &m1, &m2);
    double a = v * 2 * kPi;
    double sa, ca;
    pt_sincos(a, &sa, &ca);
    v3 q = random_unit_vector(key, D_RUV_Z, D_RUV_A);
    v3 s = cross(direction, q);
    v3 t = cross(direction, s);
    v3 dd = add(add(add(zero3(), muls(s, m1 * ca)), muls(t, m1 * sa)), muls(direction, m2));
    return normalize(dd);
}

// Ray.Bounce (Ray.cs:44-85); btype 0 Any, 1 Diffuse, 2 Specular.  Returns the new
// ray in (no, nd); `reflected` and `p` as the reference's tuple.
__device__ __forceinline__ void bounce_dir(const DevMaterial& m, const Shade& sh, v3 indir, double u, double v, bool refl,
                                           double n1, double n2, uint64_t key, v3& no, v3& nd);

// Fresnel / fixed reflectivity of a vertex (Ray.cs:170-177): the same for every child.
__device__ __forceinline__ double vertex_p(const DevMaterial& m, const Shade& sh, v3 indir, double& n1, double& n2) {
    n1 = 1.0;
    n2 = m.index;
    if (sh.inside) { double t = n1; n1 = n2; n2 = t; }
    return m.reflectivity >= 0 ? m.reflectivity : reflectance(sh.nrm, indir, n1, n2);
}

__device__ __forceinline__ void bounce(const DevMaterial& m, const Shade& sh, v3 indir, double u, double v, int btype,
                                       uint64_t key, v3& no, v3& nd, bool& reflected, double& p) {
    double n1, n2;
    p = vertex_p(m, sh, indir, n1, n2);
    bool refl = btype == 2 || (btype == 0 && draw(key, D_REFLECT) < p);
    bounce_dir(m, sh, indir, u, v, refl, n1, n2, key, no, nd);
    reflected = refl || m.transparent;
    if (!refl) p = 1 - p;
}

// The new ray of Ray.Bounce once the reflect decision is made (Ray.cs:192-205).
__device__ __forceinline__ void bounce_dir(const DevMaterial& m, const Shade& sh, v3 indir, double u, double v, bool refl,
                                           double n1, double n2, uint64_t key, v3& no, v3& nd) {
    if (refl) {
        no = sh.pos;
        nd = cone(reflect(sh.nrm, indir), sh.gloss, u, v, key);
    } else if (m.transparent) {
        v3 rd = refract(sh.nrm, indir, n1, n2);
        no = add(sh.pos, muls(rd, 1e-4));
        nd = cone(rd, sh.gloss, u, v, key);
    } else {
        // Ray.WeightedBounce (Ray.cs:28-35) around the normal
        double radius = sqrt(u);
        double theta = 2 * kPi * v;
        double st, ct;
        pt_sincos(theta, &st, &ct);
        v3 s = normalize(cross(sh.nrm, random_unit_vector(key, D_RUV_Z, D_RUV_A)));
        v3 t = cross(sh.nrm, s);
        no = sh.pos;
        nd = add(add(add(zero3(), muls(s, radius * ct)), muls(t, radius * st)), muls(sh.nrm, sqrt(1 - u)));
    }
}

// Sampler.sampleLight (Sampler.cs:212-296) up to the shadow query: the sampled
// direction and the colour the light contributes if it is the nearest hit
// (coverage depends only on the light centre/radius, so it is computed here).
// Returns false when diffuse <= 0 (no shadow ray is cast).
template <bool FULL>
__device__ __forceinline__ bool light_setup(const DevScene& S, const DevSampler& smp, const DevLight& L, v3 o, v3 n,
                                            uint64_t key, v3& dir, double3& contrib) {
    v3 center{L.center[0], L.center[1], L.center[2]};
    double radius = L.radius;
    v3 point = center;
    if (smp.ss) {
        for (uint32_t k = 0; k < 256; k++) {
            double x = draw(key, D_SS_XY + 2 * k) * 2 - 1;
            double y = draw(key, D_SS_XY + 2 * k + 1) * 2 - 1;
            if (x * x + y * y <= 1) {
                v3 l = normalize(sub(center, o));
                v3 u = normalize(cross(l, random_unit_vector(key, D_SS_RUV_Z, D_SS_RUV_A)));
                v3 v = cross(l, u);
                point = add(add(center, muls(u, x * radius)), muls(v, y * radius));
                break;
            }
        }
    }
    dir = normalize(sub(point, o));
    double diffuse = dot(dir, n);
    if (diffuse <= 0) return false;
    // coverage (Sampler.cs:278-288): θ = asin(s), adj = radius/tanθ, d = cosθ·adj,
    // r = sinθ·adj, coverage = r²/d² = tan²θ = s²/(1-s²) with s = radius/hyp.  It only
    // scales the colour, so the closed form replaces the asin/tan/cos/sin round trip
    // (difference ~1e-15 relative).
    double hyp = (double)lengthf(sub(center, o));
    double s = radius / hyp;
    double coverage = (s * s) / (1 - s * s);
    if (hyp < radius) coverage = 1;
    coverage = net_min(coverage, 1);
    // Material.MaterialAt(light, point) (Sampler.cs:292): a textured light's colour, a volume
    // light's window, at the sampled point
    int32_t mat = L.mat;
    if (FULL && L.kind == KIND_VOLUME)
        mat = vol_material(S.volumes[rec_ext(S.ana_recs + 3 * (size_t)L.index)], point, S.default_mat);
    const DevMaterial& m = S.mats[mat];
    double col[3] = {m.color[0], m.color[1], m.color[2]};
    double gl;
    if (!L.phantom) surface_at<FULL>(S, m, L.kind, L.index, point, col, gl);
    const double mm = m.emittance * diffuse * coverage;   // material.Color.MulScalar(m) (Sampler.cs:293-295)
    contrib = make_double3(col[0] * mm, col[1] * mm, col[2] * mm);
    return true;
}

// Camera.CastRay (Camera.cs:98-119), u/v as passed by RenderParallel (jitter bug kept).
__device__ __forceinline__ void cast_ray(const DevCamera& cam, int x, int y, int w, int h, double u, double v,
                                         uint64_t key, v3& o, v3& d) {
    double aspect = w / (double)h;
    double px = ((x + u - 0.5) / (w - 1.0)) * 2 - 1;
    double py = ((y + v - 0.5) / (h - 1.0)) * 2 - 1;
    v3 cu{cam.u[0], cam.u[1], cam.u[2]}, cv{cam.v[0], cam.v[1], cam.v[2]};
    v3 cw{cam.w[0], cam.w[1], cam.w[2]}, cp{cam.p[0], cam.p[1], cam.p[2]};
    d = normalize(add(add(add(zero3(), muls(cu, -px * aspect)), muls(cv, -py)), muls(cw, cam.m)));
    o = cp;
    if (cam.aperture_radius > 0) {
        v3 focal = add(cp, muls(d, cam.focal_distance));
        double angle = draw(key, D_LENS_ANGLE) * 2 * kPi;
        double radius = draw(key, D_LENS_RADIUS) * cam.aperture_radius;
        double sa, ca;
        pt_sincos(angle, &sa, &ca);
        o = add(o, muls(cu, ca * radius));
        o = add(o, muls(cv, sa * radius));
        d = normalize(sub(focal, o));
    }
}

// Pixel.AddSample (Buffer.cs:33-44)
// buf.StandardDeviation(x, y).MaxComponent() > FireflyThreshold (= 1; Renderer.cs:48, 426,
// Buffer.cs:48-57): black below 2 samples, else sqrt(V / (N-1)) (Pow(0.5) correctly rounded).
__device__ __forceinline__ bool firefly_candidate(const DevBuffer& B, size_t i) {
    const int32_t n = B.n[i];
    if (n < 2) return false;
    const double* V = B.v + 3 * i;
    double r = sqrt(V[0] / (double)(n - 1)), g = sqrt(V[1] / (double)(n - 1)), b = sqrt(V[2] / (double)(n - 1));
    return net_max(net_max(r, g), b) > 1.0;
}

// Render's adaptive branch (Renderer.cs:155-158, AdaptiveThreshold = AdaptiveExponent = 1,
// Renderer.cs:45-46): v = clamp(σmax / 1, 0, 1)^1 and AdaptiveSamples · (int)v samples, so a
// pixel takes them all when σmax ≥ 1 and none otherwise (NaN: (int)NaN · AdaptiveSamples ≤ 0).
__device__ __forceinline__ bool adaptive_serial_candidate(const DevBuffer& B, size_t i) {
    const int32_t n = B.n[i];
    if (n < 2) return false;
    const double* V = B.v + 3 * i;
    double r = sqrt(V[0] / (double)(n - 1)), g = sqrt(V[1] / (double)(n - 1)), b = sqrt(V[2] / (double)(n - 1));
    return net_max(net_max(r, g), b) >= 1.0;
}

// IsFirefly + CalculateLocalDeviation (Renderer.cs:473-537): brightness > 0.9 and the
// 3x3 (image-clipped) neighbourhood mean deviates by > 0.2.  Neighbours from `snap`
// (M at the start of the firefly phase), the pixel's own M live.
__device__ __forceinline__ bool is_firefly(double sr, double sg, double sb, int x, int y, int w, int h,
                                           const double* __restrict__ snap, const double* own) {
    double brightness = sr * 0.2126 + sg * 0.7152 + sb * 0.0722;
    if (!(brightness > 0.9)) return false;
    const int sx = max(0, x - 1), sy = max(0, y - 1), ex = min(w - 1, x + 1), ey = min(h - 1, y + 1);
    double tr = 0, tg = 0, tb = 0;
    int count = 0;
    for (int j = sy; j <= ey; j++)
        for (int i = sx; i <= ex; i++) {
            const double* c = (i == x && j == y) ? own : snap + 3 * ((size_t)j * (size_t)w + (size_t)i);
            tr += c[0]; tg += c[1]; tb += c[2];
            count++;
        }
    double ar = tr / count, ag = tg / count, ab = tb / count;
    double dr = fabs(sr - ar), dg = fabs(sg - ag), db = fabs(sb - ab);
    return sqrt(dr * dr + dg * dg + db * db) > 0.2;
}

__device__ __forceinline__ void welford(const DevBuffer& B, size_t i, double r, double g, double b) {
    int32_t n = B.n[i] + 1;
    B.n[i] = n;
    double* M = B.m + 3 * i;
    double* V = B.v + 3 * i;
    if (n == 1) { M[0] = r; M[1] = g; M[2] = b; return; }
    double s[3] = {r, g, b};
    for (int k = 0; k < 3; k++) {
        double mo = M[k];
        double mn = mo + (s[k] - mo) / (double)n;
        V[k] = V[k] + (s[k] - mo) * (s[k] - mn);
        M[k] = mn;
    }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Pixel (x, y) of slot `local` (0..1023) of a 32x32 tile: 8x8 blocks per wave,
// 16x16 quarters, so consecutive slots are screen-space neighbours.
__device__ __forceinline__ void tile_pixel(int tile, int local, int tiles_x, int& x, int& y) {
    const int quarter = local >> 8, wave = (local >> 6) & 3, lane = local & 63;
    x = (tile % tiles_x) * 32 + (quarter & 1) * 16 + (wave & 1) * 8 + (lane & 7);
    y = (tile / tiles_x) * 32 + (quarter >> 1) * 16 + (wave >> 1) * 8 + (lane >> 3);
}

}  // namespace pt
