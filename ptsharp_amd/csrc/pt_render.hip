// pt_render.hip — gfx950 kernels for PTSharp's per-pixel render hot path.
//
// k_render_pass: one wave64 per 8x8 pixel block (4 waves = a 16x16 quarter of
// a 32x32 tile, 4 blocks per tile).  Each lane owns one pixel for the whole
// pass: spp camera samples (Renderer.RenderParallel, Renderer.cs:287-310), each
// expanded from DefaultSampler.sample's recursion (Sampler.cs:55-145) into an
// iterative depth-first walk.  Branching vertices (the n²·modes first-hit
// strata, and every vertex under SpecularModeAll) live on a small per-lane
// frame stack; chain vertices (one child) are processed inline.  The estimator
// is linear, so the recursion becomes throughput-weighted accumulation
// ("Recursion → iteration").
// Every Scene.Intersect is a closest-hit query over planes (linear), a BVH2 over
// spheres/cubes and a BVH2 over all triangles, with the per-lane traversal stack
// in LDS.  The Welford update (Pixel.AddSample, Buffer.cs:33-44) is done by the
// owning lane: no atomics on the Buffer.
#include <hip/hip_runtime.h>

#include "pt_bvh.h"
#include "pt_math.h"
#include "pt_scene.h"

#pragma clang fp contract(off)

namespace pt {

constexpr int kBlock = 256;
constexpr int kMaxFrames = 34;   // MaxBounces <= 32 under SpecularModeAll (checked on the host)

struct HitRec {
    double t;
    int32_t kind;   // KIND_* of the primitive hit; -1 = miss
    int32_t idx;    // record position: tri_recs / ana_recs / planes
};

struct Counters {
    uint32_t rays, nodes, prims, shades;
};

__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }

// Conservative fp32 slab test: (b - o) * (1/d) carries <= 3 ulp of relative error,
// so the far distance is widened by 2^-21 relative; NaN slabs (o on a plane with
// d = 0) drop out of fminf/fmaxf, which only widens the interval.
__device__ __forceinline__ bool slab(float4 lo, float4 hi, v3 o, v3 invd, float tmax, float& tentry) {
    float tx1 = (lo.x - o.x) * invd.x, tx2 = (hi.x - o.x) * invd.x;
    float ty1 = (lo.y - o.y) * invd.y, ty2 = (hi.y - o.y) * invd.y;
    float tz1 = (lo.z - o.z) * invd.z, tz2 = (hi.z - o.z) * invd.z;
    float tn = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fmaxf(fminf(tz1, tz2), 0.0f));
    float tf = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fminf(fmaxf(tz1, tz2), tmax));
    tentry = tn;
    return tn <= tf * 1.0000005f;
}

// Round the closest-hit distance up so the fp32 cull never drops an equal-t candidate.
__device__ __forceinline__ float tmax_bound(double t) {
    float f = (float)t;
    return (double)f < t ? __uint_as_float(f2u(f) + 1u) : f;
}

template <bool TRI, bool COUNT>
__device__ __forceinline__ void leaf_hits(const float4* __restrict__ recs, uint32_t first, uint32_t cnt, v3 o, v3 d,
                                          HitRec& best, Counters& ctr) {
    for (uint32_t k = 0; k < cnt; k++) {
        const uint32_t pos = first + k;
        const float4* r = recs + 3 * (size_t)pos;
        if (COUNT) ctr.prims++;
        if (TRI) {
            float4 a = r[0], b = r[1], c = r[2];
            double t = isect_tri(v3{a.x, a.y, a.z}, v3{a.w, b.x, b.y}, v3{b.z, b.w, c.x}, o, d);
            if (t < best.t) { best.t = t; best.kind = KIND_TRI; best.idx = (int32_t)pos; }
        } else {
            float4 a = r[0], b = r[1];
            int32_t kind = (int32_t)f2u(a.w);
            double t;
            if (kind == KIND_SPHERE) {
                float4 c = r[2];
                double radius = __hiloint2double((int)f2u(c.z), (int)f2u(c.y));
                t = isect_sphere(v3{a.x, a.y, a.z}, radius, o, d);
            } else {
                t = isect_cube(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
            }
            if (t < best.t) { best.t = t; best.kind = kind; best.idx = (int32_t)pos; }
        }
    }
}

// Stack-based BVH2 traversal.  A child pair is fetched together (64 B, one
// line); the nearer child is descended, the farther pushed on the LDS stack.
// Node ref (host encoding, pt_api.hip): bit31 = 0 → inner, value = index of the
// pair's left node; bit31 = 1 → leaf, bits 29..30 = count-1, bits 0..28 = first.
template <bool TRI, bool COUNT>
__device__ __forceinline__ void traverse(const float4* __restrict__ nodes, int32_t num_nodes,
                                         const float4* __restrict__ recs, v3 o, v3 d, v3 invd, HitRec& best,
                                         uint32_t* __restrict__ stack, Counters& ctr) {
    if (num_nodes <= 0) return;
    float4 r0 = nodes[0], r1 = nodes[1];
    float te;
    if (!slab(r0, r1, o, invd, tmax_bound(best.t), te)) return;
    uint32_t ref = f2u(r0.w);
    int sp = 0;
    for (;;) {
        if (!(ref & 0x80000000u)) {
            const float4* c = nodes + 2 * (size_t)ref;
            float4 l0 = c[0], l1 = c[1], q0 = c[2], q1 = c[3];
            if (COUNT) ctr.nodes++;
            float tmax = tmax_bound(best.t);
            float tl, tr;
            bool hl = slab(l0, l1, o, invd, tmax, tl);
            bool hr = slab(q0, q1, o, invd, tmax, tr);
            if (hl && hr) {
                uint32_t nearr = f2u(l0.w), farr = f2u(q0.w);
                if (tr < tl) { uint32_t s = nearr; nearr = farr; farr = s; }
                stack[sp * kBlock] = farr;
                sp++;
                ref = nearr;
                continue;
            }
            if (hl) { ref = f2u(l0.w); continue; }
            if (hr) { ref = f2u(q0.w); continue; }
        } else {
            leaf_hits<TRI, COUNT>(recs, ref & 0x1FFFFFFFu, ((ref >> 29) & 3u) + 1u, o, d, best, ctr);
        }
        if (sp == 0) break;
        sp--;
        ref = stack[sp * kBlock];
    }
}

// Scene.Intersect (Scene.cs:75-79): closest hit over planes, analytic BVH, triangle BVH.
template <bool COUNT>
__device__ HitRec trace(const DevScene& S, v3 o, v3 d, uint32_t* stack, Counters& ctr) {
    ctr.rays++;
    HitRec best{kHitInf, -1, -1};
    for (int i = 0; i < S.num_planes; i++) {
        float4 a = S.planes[2 * i], b = S.planes[2 * i + 1];
        double t = isect_plane(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, o, d);
        if (t < best.t) { best.t = t; best.kind = KIND_PLANE; best.idx = i; }
    }
    v3 invd{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    traverse<false, COUNT>(S.ana_nodes, S.ana_num_nodes, S.ana_recs, o, d, invd, best, stack, ctr);
    traverse<true, COUNT>(S.tri_nodes, S.tri_num_nodes, S.tri_recs, o, d, invd, best, stack, ctr);
    return best;
}

struct Shade {
    v3 pos, nrm;
    int32_t mat;
    int32_t inside;
};

// Hit.Info (Hit.cs:26-55): position (fp32 re-rounded), NormalAt, MaterialAt, flip.
template <bool COUNT>
__device__ __forceinline__ Shade hit_info(const DevScene& S, const HitRec& h, v3 o, v3 d, Counters& ctr) {
    Shade s;
    s.pos = add(o, muls(d, h.t));
    v3 n;
    if (h.kind == KIND_TRI) {
        if (COUNT) ctr.shades++;
        const float4* r = S.tri_recs + 3 * (size_t)h.idx;
        const float4* q = S.tri_shade + 3 * (size_t)h.idx;
        float4 a = r[0], b = r[1], c = r[2];
        float4 x = q[0], y = q[1], z = q[2];
        n = tri_normal(v3{a.x, a.y, a.z}, v3{a.w, b.x, b.y}, v3{b.z, b.w, c.x}, v3{x.x, x.y, x.z},
                       v3{x.w, y.x, y.y}, v3{y.z, y.w, z.x}, s.pos);
        s.mat = (int32_t)f2u(z.y);
    } else if (h.kind == KIND_PLANE) {
        float4 a = S.planes[2 * h.idx], b = S.planes[2 * h.idx + 1];
        n = v3{b.x, b.y, b.z};
        s.mat = (int32_t)f2u(a.w);
    } else {
        const float4* r = S.ana_recs + 3 * (size_t)h.idx;
        float4 a = r[0], b = r[1], c = r[2];
        if (h.kind == KIND_SPHERE) n = normalize(sub(s.pos, v3{a.x, a.y, a.z}));   // Sphere.NormalAt
        else n = cube_normal(v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, s.pos);           // Cube.NormalAt
        s.mat = (int32_t)f2u(c.x);
    }
    s.inside = 0;
    if (dot(n, d) > 0) { n = neg(n); s.inside = 1; }
    s.nrm = n;
    return s;
}

// Util.Cone (Util.cs:17-32)
__device__ __forceinline__ v3 cone(v3 direction, double theta, double u, double v, uint64_t key) {
    if (theta < kEps) return direction;
    theta = theta * (1 - (2 * acos(u) / kPi));
    double m1 = sin(theta);
    double m2 = cos(theta);
    double a = v * 2 * kPi;
    v3 q = random_unit_vector(key, D_RUV_Z, D_RUV_A);
    v3 s = cross(direction, q);
    v3 t = cross(direction, s);
    v3 dd = add(add(add(zero3(), muls(s, m1 * cos(a))), muls(t, m1 * sin(a))), muls(direction, m2));
    return normalize(dd);
}

// Ray.Bounce (Ray.cs:44-85); btype 0 Any, 1 Diffuse, 2 Specular.  Returns the new
// ray in (no, nd); `reflected` and `p` as the reference's tuple.
__device__ __forceinline__ void bounce(const DevMaterial& m, const Shade& sh, v3 indir, double u, double v, int btype,
                                       uint64_t key, v3& no, v3& nd, bool& reflected, double& p) {
    double n1 = 1.0, n2 = m.index;
    if (sh.inside) { double t = n1; n1 = n2; n2 = t; }
    p = m.reflectivity >= 0 ? m.reflectivity : reflectance(sh.nrm, indir, n1, n2);
    bool refl = btype == 2 || (btype == 0 && draw(key, D_REFLECT) < p);
    if (refl) {
        no = sh.pos;
        nd = cone(reflect(sh.nrm, indir), m.gloss, u, v, key);
        reflected = true;
    } else if (m.transparent) {
        v3 rd = refract(sh.nrm, indir, n1, n2);
        no = add(sh.pos, muls(rd, 1e-4));
        nd = cone(rd, m.gloss, u, v, key);
        reflected = true;
        p = 1 - p;
    } else {
        // Ray.WeightedBounce (Ray.cs:28-35) around the normal
        double radius = sqrt(u);
        double theta = 2 * kPi * v;
        v3 s = normalize(cross(sh.nrm, random_unit_vector(key, D_RUV_Z, D_RUV_A)));
        v3 t = cross(sh.nrm, s);
        no = sh.pos;
        nd = add(add(add(zero3(), muls(s, radius * cos(theta))), muls(t, radius * sin(theta))),
                 muls(sh.nrm, sqrt(1 - u)));
        reflected = false;
        p = 1 - p;
    }
}

// Sampler.sampleLight (Sampler.cs:212-296) for light L from the normal ray (o, n).
template <bool COUNT>
__device__ __noinline__ float3 sample_light(const DevScene& S, const DevSampler& smp, const DevLight& L, v3 o, v3 n,
                                            uint64_t key, uint32_t* stack, Counters& ctr) {
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
    v3 dir = normalize(sub(point, o));
    double diffuse = dot(dir, n);
    if (diffuse <= 0) return make_float3(0.f, 0.f, 0.f);
    HitRec h = trace<COUNT>(S, o, dir, stack, ctr);
    // hit.Shape != light is a reference compare; struct Triangle lights never match.
    if (!(h.t < kHitInf) || L.phantom || h.kind != L.kind || h.idx != L.index) return make_float3(0.f, 0.f, 0.f);
    double hyp = (double)lengthf(sub(center, o));
    double theta = asin(radius / hyp);
    double adj = radius / tan(theta);
    double dd = cos(theta) * adj;
    double rr = sin(theta) * adj;
    double coverage = (rr * rr) / (dd * dd);
    if (hyp < radius) coverage = 1;
    coverage = net_min(coverage, 1);
    const DevMaterial& m = S.mats[L.mat];
    float mm = (float)((double)m.emittance * diffuse * coverage);
    return make_float3(m.color[0] * mm, m.color[1] * mm, m.color[2] * mm);
}

// Sampler.sampleLights (Sampler.cs:191-210)
template <bool COUNT>
__device__ __forceinline__ float3 sample_lights(const DevScene& S, const DevSampler& smp, v3 o, v3 n, uint64_t key,
                                                uint32_t* stack, Counters& ctr) {
    int nl = S.num_lights;
    if (nl == 0) return make_float3(0.f, 0.f, 0.f);
    if (smp.light_mode == 1) {
        float3 acc = make_float3(0.f, 0.f, 0.f);
        for (int i = 0; i < nl; i++) {
            float3 c = sample_light<COUNT>(S, smp, S.lights[i], o, n, light_key(key, (uint32_t)i), stack, ctr);
            acc.x += c.x; acc.y += c.y; acc.z += c.z;
        }
        float inv = 1.0f / (float)nl;
        return make_float3(acc.x * inv, acc.y * inv, acc.z * inv);
    }
    int idx = (int)(draw(key, D_LIGHT) * nl);
    if (idx >= nl) idx = nl - 1;
    float3 c = sample_light<COUNT>(S, smp, S.lights[idx], o, n, key, stack, ctr);
    float fn = (float)nl;
    return make_float3(c.x * fn, c.y * fn, c.z * fn);
}

// A branching vertex of the sampler tree (pending children).
struct Frame {
    v3 pos, nrm, indir;
    float thr[3];        // throughput into this vertex already divided by n²
    uint64_t node;
    int32_t mat, inside, depth, n, nm, next;
};

// Child c of a vertex: one iteration of the u/v/mode loop of Sampler.cs:96-131.
// Adds the vertex' direct-light term to acc and returns the child's ray/throughput.
template <bool COUNT>
__device__ __forceinline__ bool child_step(const DevScene& S, const DevSampler& smp, const Shade& sh, v3 indir,
                                           const float thr[3], uint64_t node, int n, int nm, int c, float3& acc,
                                           v3& no, v3& nd, bool& emission, float nthr[3], uint64_t& nkey,
                                           uint32_t* stack, Counters& ctr) {
    const DevMaterial& m = S.mats[sh.mat];
    int ma = nm == 2 ? 1 : 0;
    int mode = ma + c % nm;
    int stratum = c / nm;
    int u = stratum / n, v = stratum % n;
    uint64_t E = child_key(node, (uint32_t)c);
    double fu = ((double)u + draw(E, D_STRATUM_U)) / (double)n;
    double fv = ((double)(float)v + draw(E, D_STRATUM_V)) / (double)n;
    bool reflected;
    double p;
    bounce(m, sh, indir, fu, fv, mode, E, no, nd, reflected, p);
    if (mode == 0) p = 1;
    if (!(p > 0)) return false;
    float fp = (float)p;
    float w[3];
    if (reflected) {
        // specular: tinted = indirect.Mix(Color*indirect, Tint) (Sampler.cs:112-114)
        for (int k = 0; k < 3; k++) w[k] = fp * ((1.0f - m.tint) + m.tint * m.color[k]);
    } else {
        for (int k = 0; k < 3; k++) w[k] = fp * m.color[k];
        if (smp.dl) {
            float3 dl = sample_lights<COUNT>(S, smp, sh.pos, sh.nrm, E, stack, ctr);
            acc.x += thr[0] * w[0] * dl.x;
            acc.y += thr[1] * w[1] * dl.y;
            acc.z += thr[2] * w[2] * dl.z;
        }
    }
    for (int k = 0; k < 3; k++) nthr[k] = thr[k] * w[k];
    emission = reflected;
    nkey = E;
    return true;
}

// DefaultSampler.Sample(scene, ray) for one camera ray; returns the sample colour.
template <bool COUNT>
__device__ float3 sample_path(const DevScene& S, const DevSampler& smp, v3 o, v3 d, uint64_t root_key,
                              uint32_t* stack, Frame* frames, Counters& ctr) {
    float3 acc = make_float3(0.f, 0.f, 0.f);
    // current vertex to visit
    bool have = true;
    bool emission = true;
    int samples = smp.fh;
    int depth = 0;
    uint64_t node = root_key;
    float thr[3] = {1.f, 1.f, 1.f};
    int sp = 0;
    for (;;) {
        if (have) {
            have = false;
            if (depth <= smp.mb) {
                HitRec h = trace<COUNT>(S, o, d, stack, ctr);
                if (!(h.t < kHitInf)) {
                    acc.x += thr[0] * S.env[0];
                    acc.y += thr[1] * S.env[1];
                    acc.z += thr[2] * S.env[2];
                } else {
                    Shade sh = hit_info<COUNT>(S, h, o, d, ctr);
                    const DevMaterial& m = S.mats[sh.mat];
                    int n = (int)sqrt((double)samples);
                    float inv_n2 = 1.0f / (float)(n * n);
                    bool alive = true;
                    if (m.emittance > 0) {
                        if (smp.dl && !emission) {
                            alive = false;
                        } else {
                            float e = (float)((double)m.emittance * samples) * inv_n2;
                            acc.x += thr[0] * m.color[0] * e;
                            acc.y += thr[1] * m.color[1] * e;
                            acc.z += thr[2] * m.color[2] * e;
                        }
                    }
                    if (alive) {
                        int nm = (smp.spec_mode == 2 || (depth == 0 && smp.spec_mode == 1)) ? 2 : 1;
                        float t2[3] = {thr[0] * inv_n2, thr[1] * inv_n2, thr[2] * inv_n2};
                        if (n * n * nm == 1) {
                            // chain vertex: its only child is processed inline
                            float nthr[3];
                            uint64_t nkey;
                            v3 no, nd;
                            bool em;
                            if (child_step<COUNT>(S, smp, sh, d, t2, node, 1, 1, 0, acc, no, nd, em, nthr, nkey, stack,
                                                  ctr)) {
                                o = no; d = nd; emission = em; samples = 1; depth = depth + 1; node = nkey;
                                thr[0] = nthr[0]; thr[1] = nthr[1]; thr[2] = nthr[2];
                                have = true;
                                continue;
                            }
                        } else if (n > 0 && sp < kMaxFrames) {
                            Frame& F = frames[sp++];
                            F.pos = sh.pos; F.nrm = sh.nrm; F.indir = d;
                            F.thr[0] = t2[0]; F.thr[1] = t2[1]; F.thr[2] = t2[2];
                            F.node = node; F.mat = sh.mat; F.inside = sh.inside; F.depth = depth;
                            F.n = n; F.nm = nm; F.next = 0;
                        }
                    }
                }
            }
        }
        // next pending child of the innermost branching vertex
        while (!have && sp > 0) {
            Frame& F = frames[sp - 1];
            int c = F.next++;
            int nch = F.n * F.n * F.nm;
            Shade sh{F.pos, F.nrm, F.mat, F.inside};
            v3 indir = F.indir;
            float t2[3] = {F.thr[0], F.thr[1], F.thr[2]};
            uint64_t fnode = F.node;
            int fdepth = F.depth, fn = F.n, fnm = F.nm;
            if (F.next >= nch) sp--;
            float nthr[3];
            uint64_t nkey;
            v3 no, nd;
            bool em;
            if (child_step<COUNT>(S, smp, sh, indir, t2, fnode, fn, fnm, c, acc, no, nd, em, nthr, nkey, stack, ctr)) {
                o = no; d = nd; emission = em; samples = 1; depth = fdepth + 1; node = nkey;
                thr[0] = nthr[0]; thr[1] = nthr[1]; thr[2] = nthr[2];
                have = true;
            }
        }
        if (!have) break;
    }
    return acc;
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
        o = add(o, muls(cu, cos(angle) * radius));
        o = add(o, muls(cv, sin(angle) * radius));
        d = normalize(sub(focal, o));
    }
}

// Pixel.AddSample (Buffer.cs:33-44)
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

template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_render_pass(DevScene S, DevCamera cam, DevSampler smp, DevPass P,
                                                        DevBuffer B) {
    __shared__ uint32_t s_stack[kMaxDepth * kBlock];
    uint32_t* stack = s_stack + threadIdx.x;
    const int tile_slot = blockIdx.x >> 2;
    const int quarter = blockIdx.x & 3;
    const int tile = P.tiles ? P.tiles[tile_slot] : tile_slot;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int x = (tile % P.tiles_x) * 32 + (quarter & 1) * 16 + (wave & 1) * 8 + (lane & 7);
    const int y = (tile / P.tiles_x) * 32 + (quarter >> 1) * 16 + (wave >> 1) * 8 + (lane >> 3);
    Counters ctr{0, 0, 0, 0};
    Frame local_frames[kMaxFrames];
    if (x < P.width && y < P.height) {
        const int w = P.width, h = P.height;
        const uint64_t pix = (uint64_t)y * (uint64_t)w + (uint64_t)x;
        if (P.stratified) {
            int root = (int)sqrt((double)P.spp);
            for (int u = 0; u < root; u++)
                for (int v = 0; v < root; v++) {
                    uint64_t K = camera_key(P.seed, P.pass_index, pix, (uint32_t)(u * root + v));
                    v3 o, d;
                    cast_ray(cam, x, y, w, h, ((double)u + 0.5) / (double)root, ((double)v + 0.5) / (double)root,
                             K, o, d);
                    float3 c = sample_path<COUNT>(S, smp, o, d, K, stack, local_frames, ctr);
                    welford(B, (size_t)pix, (double)c.x, (double)c.y, (double)c.z);
                }
        } else {
            float cr = 0.f, cg = 0.f, cb = 0.f;
            for (int p = 0; p < P.spp; p++) {
                uint64_t K = camera_key(P.seed, P.pass_index, pix, (uint32_t)p);
                double fu = (x + draw(K, D_JX)) / w;
                double fv = (y + draw(K, D_JY)) / h;
                v3 o, d;
                cast_ray(cam, x, y, w, h, fu, fv, K, o, d);
                float3 c = sample_path<COUNT>(S, smp, o, d, K, stack, local_frames, ctr);
                cr += c.x; cg += c.y; cb += c.z;
            }
            double inv = (double)P.spp;
            welford(B, (size_t)pix, (double)cr / inv, (double)cg / inv, (double)cb / inv);
        }
    }
    uint32_t rays = wave_sum(ctr.rays);
    if (COUNT) {
        uint32_t nodes = wave_sum(ctr.nodes), prims = wave_sum(ctr.prims), shades = wave_sum(ctr.shades);
        if (lane == 0) {
            atomicAdd(&B.counters[1], (unsigned long long)nodes);
            atomicAdd(&B.counters[2], (unsigned long long)prims);
            atomicAdd(&B.counters[3], (unsigned long long)shades);
        }
    }
    if (lane == 0) atomicAdd(&B.counters[0], (unsigned long long)rays);
}

// Host-side launch (called from pt_api.hip).
hipError_t launch_render_pass(const DevScene& S, const DevCamera& cam, const DevSampler& smp, const DevPass& P,
                              const DevBuffer& B, int num_tiles, bool count, hipStream_t stream) {
    dim3 grid((unsigned)num_tiles * 4u), block(kBlock);
    if (count)
        hipLaunchKernelGGL(k_render_pass<true>, grid, block, 0, stream, S, cam, smp, P, B);
    else
        hipLaunchKernelGGL(k_render_pass<false>, grid, block, 0, stream, S, cam, smp, P, B);
    return hipGetLastError();
}

}  // namespace pt
