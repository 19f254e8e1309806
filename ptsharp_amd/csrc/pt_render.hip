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
// Every Scene.Intersect is a closest-hit query over planes (linear), a 4-wide
// BVH over spheres/cubes and one over all triangles, with the per-lane traversal
// stack in LDS.  The Welford update (Pixel.AddSample, Buffer.cs:33-44) is done by the
// owning lane: no atomics on the Buffer.  Colour terms are fp64 and summed in the
// fixed-point form of pt_accum.h, term by term as the wavefront engine adds them, so
// both engines produce the same bits.
#include <hip/hip_runtime.h>

#include "pt_accum.h"
#include "pt_device.h"

#pragma clang fp contract(off)

namespace pt {

constexpr int kBlock = 256;
// The megakernel's per-lane traversal stack: all kStackMax entries in LDS (64 KiB per 256-thread block).  The
// deepest stack the CPU model saw on C4 is 17 entries, but 24 entries in LDS and the rest in the lane's scratch
// ran 3 % slower (C4 960x540, 1 spp: 589 -> 571 Mrays/s, gpurun_out/r06a/mega.txt): the kernel's registers,
// not its LDS, bound its occupancy, and the scratch column cost the difference.
using MStack = LdsStack<kBlock>;
constexpr int kMaxFrames = 34;   // MaxBounces <= 32 under SpecularModeAll (checked on the host)

// Sampler.sampleLight (Sampler.cs:212-296): the megakernel keeps the reference's
// nearest-hit + identity structure for the shadow query.  Returns false (black) when
// no ray is cast or the light is not the nearest hit.
template <bool COUNT, bool FULL>
__device__ __noinline__ bool sample_light(const DevScene& S, const DevSampler& smp, const DevLight& L, v3 o, v3 n,
                                          uint64_t key, MStack stack, Counters& ctr, double3& contrib) {
    v3 dir;
    if (!light_setup<FULL>(S, smp, L, o, n, key, dir, contrib)) return false;
    HitRec h = trace<COUNT, FULL>(S, o, dir, stack, ctr);
    // hit.Shape != light is a reference compare; struct Triangle lights never match.
    return (h.t < kHitInf) && !L.phantom && h.kind == L.kind && h.idx == L.index;
}

// Sampler.sampleLights (Sampler.cs:191-210) times the child's throughput·weight tw, each
// light's term added to acc on its own, as the wavefront's shadow rays add them.
template <bool COUNT, bool FULL>
__device__ __forceinline__ void sample_lights(const DevScene& S, const DevSampler& smp, v3 o, v3 n, uint64_t key,
                                              const double tw[3], FixReg& acc, MStack stack, Counters& ctr) {
    const int nl = S.num_lights;
    if (nl == 0) return;
    const bool all = smp.light_mode == 1;
    const int first = all ? 0 : min((int)(draw(key, D_LIGHT) * nl), nl - 1);
    const int count = all ? nl : 1;
    for (int j = 0; j < count; j++) {
        const int li = first + j;
        double3 lc;
        if (!sample_light<COUNT, FULL>(S, smp, S.lights[li], o, n, all ? light_key(key, (uint32_t)li) : key, stack, ctr, lc))
            continue;
        if (all) { lc.x /= nl; lc.y /= nl; lc.z /= nl; }
        else { lc.x *= nl; lc.y *= nl; lc.z *= nl; }
        fixreg_add3(acc, tw[0] * lc.x, tw[1] * lc.y, tw[2] * lc.z);
    }
}

// A branching vertex of the sampler tree (pending children).
struct Frame {
    v3 pos, nrm, indir;
    double thr[3];       // throughput into this vertex already divided by n²
    double col[3];       // Material.MaterialAt colour / gloss of the vertex
    double gloss;
    uint64_t node;
    int32_t mat, inside, depth, n, nm, next;
};

// Child c of a vertex: one iteration of the u/v/mode loop of Sampler.cs:96-131.
// Adds the vertex' direct-light term to acc and returns the child's ray/throughput.
template <bool COUNT, bool FULL>
__device__ __forceinline__ bool child_step(const DevScene& S, const DevSampler& smp, const Shade& sh, v3 indir,
                                           const double thr[3], uint64_t node, int n, int nm, int c, FixReg& acc,
                                           v3& no, v3& nd, bool& emission, double nthr[3], uint64_t& nkey,
                                           MStack stack, Counters& ctr) {
    const DevMaterial& m = S.mats[sh.mat];
    int ma = nm == 2 ? 1 : 0;
    int mode = ma + c % nm;
    int stratum = c / nm;
    int u = stratum / n, v = stratum % n;
    uint64_t E = child_key(node, (uint32_t)c);
    const double rn = strata_recip(n);   // pt_math.h div_strata
    double fu = div_strata((double)u + draw(E, D_STRATUM_U), n, rn);
    double fv = div_strata((double)(float)v + draw(E, D_STRATUM_V), n, rn);
    bool reflected;
    double p;
    bounce(m, sh, indir, fu, fv, mode, E, no, nd, reflected, p);
    if (mode == 0) p = 1;
    if (!(p > 0)) return false;
    const double fp = p;
    double w[3];
    if (reflected) {
        // specular: tinted = indirect.Mix(Color*indirect, Tint) (Sampler.cs:112-114)
        for (int k = 0; k < 3; k++) w[k] = fp * ((1.0 - m.tint) + m.tint * sh.col[k]);
    } else {
        for (int k = 0; k < 3; k++) w[k] = fp * sh.col[k];
        if (smp.dl) {
            const double tw[3] = {thr[0] * w[0], thr[1] * w[1], thr[2] * w[2]};
            sample_lights<COUNT, FULL>(S, smp, sh.pos, sh.nrm, E, tw, acc, stack, ctr);
        }
    }
    for (int k = 0; k < 3; k++) nthr[k] = thr[k] * w[k];
    emission = reflected;
    nkey = E;
    return true;
}

// DefaultSampler.Sample(scene, ray) for one camera ray; adds the sample's terms to acc.
template <bool COUNT, bool FULL>
__device__ void sample_path(const DevScene& S, const DevSampler& smp, v3 o, v3 d, uint64_t root_key,
                            MStack stack, Frame* frames, Counters& ctr, FixReg& acc) {
    // current vertex to visit
    bool have = true;
    bool emission = true;
    int samples = smp.fh;
    int depth = 0;
    uint64_t node = root_key;
    double thr[3] = {1.0, 1.0, 1.0};
    int sp = 0;
    for (;;) {
        if (have) {
            have = false;
            if (depth <= smp.mb) {
                HitRec h = trace<COUNT, FULL>(S, o, d, stack, ctr);
                if (!(h.t < kHitInf)) {
                    const double3 env = environment<FULL>(S, d);   // sampleEnvironment (Sampler.cs:177-189)
                    fixreg_add3(acc, thr[0] * env.x, thr[1] * env.y, thr[2] * env.z);
                } else {
                    Shade sh = hit_info<COUNT, FULL>(S, h, o, d, ctr);
                    const DevMaterial& m = S.mats[sh.mat];
                    int n = (int)sqrt((double)samples);
                    const double rsq = strata_recip(n * n);   // pt_math.h div_strata
                    bool alive = true;
                    if (m.emittance > 0) {
                        if (smp.dl && !emission) {
                            alive = false;
                        } else {
                            const double e = m.emittance * samples;
                            fixreg_add3(acc, thr[0] * div_strata(sh.col[0] * e, n * n, rsq),
                                        thr[1] * div_strata(sh.col[1] * e, n * n, rsq),
                                        thr[2] * div_strata(sh.col[2] * e, n * n, rsq));
                        }
                    }
                    if (alive) {
                        int nm = (smp.spec_mode == 2 || (depth == 0 && smp.spec_mode == 1)) ? 2 : 1;
                        double t2[3] = {div_strata(thr[0], n * n, rsq), div_strata(thr[1], n * n, rsq), div_strata(thr[2], n * n, rsq)};
                        if (n * n * nm == 1) {
                            // chain vertex: its only child is processed inline
                            double nthr[3];
                            uint64_t nkey;
                            v3 no, nd;
                            bool em;
                            if (child_step<COUNT, FULL>(S, smp, sh, d, t2, node, 1, 1, 0, acc, no, nd, em, nthr, nkey, stack,
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
                            F.col[0] = sh.col[0]; F.col[1] = sh.col[1]; F.col[2] = sh.col[2]; F.gloss = sh.gloss;
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
            Shade sh{F.pos, F.nrm, F.mat, F.inside, {F.col[0], F.col[1], F.col[2]}, F.gloss};
            v3 indir = F.indir;
            double t2[3] = {F.thr[0], F.thr[1], F.thr[2]};
            uint64_t fnode = F.node;
            int fdepth = F.depth, fn = F.n, fnm = F.nm;
            if (F.next >= nch) sp--;
            double nthr[3];
            uint64_t nkey;
            v3 no, nd;
            bool em;
            if (child_step<COUNT, FULL>(S, smp, sh, indir, t2, fnode, fn, fnm, c, acc, no, nd, em, nthr, nkey, stack, ctr)) {
                o = no; d = nd; emission = em; samples = 1; depth = fdepth + 1; node = nkey;
                thr[0] = nthr[0]; thr[1] = nthr[1]; thr[2] = nthr[2];
                have = true;
            }
        }
        if (!have) break;
    }
}

template <bool COUNT, bool FULL>
__global__ __launch_bounds__(kBlock) void k_render_pass(DevScene S, DevCamera cam, DevSampler smp, DevPass P,
                                                        DevBuffer B) {
    __shared__ uint32_t s_stack[kStackMax * kBlock];
    const MStack stack{s_stack + threadIdx.x};
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
                    FixReg acc;
                    fixreg_clear(acc);
                    sample_path<COUNT, FULL>(S, smp, o, d, K, stack, local_frames, ctr, acc);
                    welford(B, (size_t)pix, fixreg_value(acc, 0), fixreg_value(acc, 1), fixreg_value(acc, 2));
                }
        } else {
            FixReg acc;   // the pixel's spp samples (c += sampler.Sample(...), Renderer.cs:304)
            fixreg_clear(acc);
            for (int p = 0; p < P.spp; p++) {
                uint64_t K = camera_key(P.seed, P.pass_index, pix, (uint32_t)p);
                double fu = (x + draw(K, D_JX)) / w;
                double fv = (y + draw(K, D_JY)) / h;
                v3 o, d;
                cast_ray(cam, x, y, w, h, fu, fv, K, o, d);
                sample_path<COUNT, FULL>(S, smp, o, d, K, stack, local_frames, ctr, acc);
            }
            const double spp = (double)P.spp;   // c /= spp (Renderer.cs:308)
            welford(B, (size_t)pix, fixreg_value(acc, 0) / spp, fixreg_value(acc, 1) / spp, fixreg_value(acc, 2) / spp);
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

// Scene.Intersect (Scene.cs:75-79) of a host's rays (pt_intersect), or the any-hit shadow query against
// a given t (pt_occluded, light_visible's any_nearer): one lane per ray, the megakernel's trace() with its
// LDS stack.  S.coop_min_lanes (set by the host) picks how a pending Volume is marched.
template <bool FULL, bool ANY>
__global__ __launch_bounds__(kBlock) void k_intersect(DevScene S, uint32_t n, const float* __restrict__ o3,
                                                      const float* __restrict__ d3, const double* __restrict__ tl,
                                                      double* __restrict__ out_t, int32_t* __restrict__ out_kind) {
    __shared__ uint32_t s_stack[kStackMax * kBlock];
    const MStack stack{s_stack + threadIdx.x};
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const v3 o{o3[3 * (size_t)i], o3[3 * (size_t)i + 1], o3[3 * (size_t)i + 2]};
    const v3 d{d3[3 * (size_t)i], d3[3 * (size_t)i + 1], d3[3 * (size_t)i + 2]};
    Counters ctr{0, 0, 0, 0};
    if (ANY) {
        out_kind[i] = any_nearer<false, FULL>(S, o, d, tl[i], stack, ctr) ? 1 : 0;
    } else {
        const HitRec h = trace<false, FULL>(S, o, d, stack, ctr);
        out_t[i] = h.t;
        out_kind[i] = h.t < kHitInf ? h.kind : -1;
    }
}

hipError_t launch_intersect(const DevScene& S, uint32_t n, const float* o3, const float* d3, const double* tl,
                            double* out_t, int32_t* out_kind, hipStream_t stream) {
    const dim3 grid((n + kBlock - 1) / kBlock), block(kBlock);
    const bool full = S.full_geom != 0;
    if (tl && full) hipLaunchKernelGGL((k_intersect<true, true>), grid, block, 0, stream, S, n, o3, d3, tl, out_t, out_kind);
    else if (tl) hipLaunchKernelGGL((k_intersect<false, true>), grid, block, 0, stream, S, n, o3, d3, tl, out_t, out_kind);
    else if (full) hipLaunchKernelGGL((k_intersect<true, false>), grid, block, 0, stream, S, n, o3, d3, tl, out_t, out_kind);
    else hipLaunchKernelGGL((k_intersect<false, false>), grid, block, 0, stream, S, n, o3, d3, tl, out_t, out_kind);
    return hipGetLastError();
}

// Host-side launch (called from pt_api.hip).
hipError_t launch_render_pass(const DevScene& S, const DevCamera& cam, const DevSampler& smp, const DevPass& P,
                              const DevBuffer& B, int num_tiles, bool count, hipStream_t stream) {
    dim3 grid((unsigned)num_tiles * 4u), block(kBlock);
    const bool tex = S.full != 0;
    if (count && tex) hipLaunchKernelGGL((k_render_pass<true, true>), grid, block, 0, stream, S, cam, smp, P, B);
    else if (count) hipLaunchKernelGGL((k_render_pass<true, false>), grid, block, 0, stream, S, cam, smp, P, B);
    else if (tex) hipLaunchKernelGGL((k_render_pass<false, true>), grid, block, 0, stream, S, cam, smp, P, B);
    else hipLaunchKernelGGL((k_render_pass<false, false>), grid, block, 0, stream, S, cam, smp, P, B);
    return hipGetLastError();
}

}  // namespace pt
