// pt_scene.h — device-resident scene layout (HBM) shared by the host runtime
// and the gfx950 kernels.
//
// Hot / cold split: traversal touches only node pairs (64 B) and primitive
// records (48 B, three 16-B loads from one line); shading data (normals,
// material id: 48 B) is fetched once per closest hit.  Everything is laid out as
// arrays of float4 so every lane issues dwordx4 loads.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#include "pt_ext.h"

namespace pt {

enum PrimKind : int32_t { KIND_SPHERE = 0, KIND_CUBE = 1, KIND_PLANE = 2, KIND_TRI = 3, KIND_MESH = 4,
                          KIND_SDF = 5, KIND_VOLUME = 6, KIND_XFORM = 7 };

// Material (Material.cs:8-62), every scalar fp64 as in the reference (Colour is fp64,
// Colour.cs:10-12): colour, emittance and tint feed the fp64 path throughput.
struct DevMaterial {
    double color[3];
    double emittance;
    double tint;
    double index;
    double gloss;
    double reflectivity;
    double bump_multiplier;
    int32_t transparent;
    int32_t tex, ntex, btex, gtex;   // Texture / NormalTexture / BumpTexture / GlossTexture (-1 = null)
    int32_t _pad[3];
};

// ColorTexture (Texture.cs:96-252): fp64 Colour texels [h][w][3], exactly the C# Data,
// so bilinear weights, gloss and normal-map decisions reproduce the reference's fp64 sums.
struct DevTexture {
    const double* data;
    int32_t w, h;
};

// Scene.Lights entry (Scene.cs:33-37) with the centre/radius sampleLight derives
// (Sampler.cs:218-234), precomputed on the host with the same fp32 ops.
struct DevLight {
    int32_t kind;        // KIND_SPHERE / KIND_CUBE / KIND_PLANE / KIND_TRI
    int32_t index;       // scene index of that kind (identity test, Sampler.cs:264)
    int32_t mat;
    int32_t phantom;     // struct Triangle light: identity never matches (boxing)
    float center[3];
    float _pad;
    double radius;
};

struct DevScene {
    // triangle BVH (world-space mesh + directly-added triangles)
    const float4* tri_nodes;   // 2 float4 per node (pt::BvhNode)
    int32_t tri_num_nodes;
    const float4* tri_recs;    // 3 float4 per triangle: {v1.xyz,e1.x} {e1.yz,e2.xy} {e2.z,-,-,-}
    const float4* tri_chunks;  // 8 float4 per triangle leaf (pt_api.hip build_tri_bvh)
    const float4* tri_shade;   // 3 float4 per triangle: {n1.xyz,n2.x} {n2.yz,n3.xy} {n3.z,mat,-,-}
    // analytic BVH (spheres, cubes)
    const float4* ana_nodes;
    int32_t ana_num_nodes;
    const float4* ana_recs;    // 3 float4: {a.xyz,kind} {b.xyz,scene index} {mat, radius(double) | ext index, -}
    // ana_nodes, tri_nodes and tri_chunks are one allocation of 128-B lines (in that order), so
    // the cooperative fetch (pt_wavefront.hip coop_line) names any traversal line by a 32-bit index
    const float4* lines;
    uint32_t tri_node_line0, tri_chunk_line0, lines_n;   // lines_n: 128-B lines in `lines`
    // the triangle BVH's root box (the union of the root node's child boxes): a refill traversal
    // whose ray misses it skips the triangle phase instead of spending a step on the root node
    float tri_box[6];          // lo.xyz, hi.xyz
    // planes (unbounded: tested outside the BVHs)
    const float4* planes;      // 2 float4: {point.xyz, mat} {normal.xyz, scene index}
    int32_t num_planes;
    const DevMaterial* mats;
    const DevLight* lights;
    int32_t num_lights;
    int32_t num_mats;          // entries of mats (k_wf_shade stages a small table in LDS)
    double env[3];              // Scene.Color (fp64 Colour)
    // textures (§8f row 3)
    const DevTexture* texs;
    const float4* tri_uv;      // 2 float4 per triangle: {t1.xy, t2.xy} {t3.xy, -, -}; null without textured triangles
    // float4 stride between consecutive triangles of tri_recs / tri_shade / tri_uv: the
    // world mesh interleaves the three into one 128-B shading record per triangle (8:
    // recs at +0, shade at +3, uv at +6), a BLAS keeps separate arrays (3, 3, 2)
    int32_t tri_rstride, tri_ustride;
    int32_t env_tex;           // Scene.Texture (-1 = null)
    double env_angle;          // Scene.TextureAngle
    // SDF shapes, volumes, transformed shapes (§8f row 4; pt_ext.h)
    const DevSdfIns* sdf_prog;
    const double* sdf_params;
    int32_t sdf_lds;           // LDS bytes k_wf_sdf_* stage sdf_prog and sdf_params in (8-B aligned halves); 0: none
    int32_t vol_lds;           // LDS bytes k_wf_vol_* stage the scene's one Volume in (its DevVolume, windows and
                               // uniform-cell table: pt_wavefront.hip stage_vol); 0: none
    int32_t sdf_prog_n;        // entries of sdf_prog
    const DevSdfShape* sdf_shapes;
    const DevVolume* volumes;
    const DevXform* xforms;
    const float4* ext_recs;    // object-space records of transformed shapes' inner shapes (ana format)
    const DevBlas* blas;       // instanced meshes: object-space BVH4s over their own triangle records
    const float4* blas_nodes;
    const float4* blas_recs;   // tri_recs / tri_shade / tri_uv formats
    const float4* blas_shade;
    const float4* blas_uv;
    int32_t default_mat;       // `new Material()` (Volume.MaterialAt with no window near)
    int32_t full;              // textures or §8f row 4 shapes present: kernels run their FULL instantiation
    int32_t full_geom;         // §8f row 4 shapes present: the traversal kernels need FULL (textures alone do not)
    // a few analytic shapes (spheres / cubes only): the per-lane refill kernels test them one by one at
    // refill, every lane the same record (scalar loads), instead of an analytic-BVH phase
    int32_t ana_count;         // records in ana_recs
    int32_t ana_linear;        // 1: test ana_recs linearly in the refill kernels
    int32_t lights_lean;       // 1: every light's own t is a lean intersect (no SDF / Volume light): split shadow rays
    int32_t num_sdf;           // SDFShapes (the split closest hit queues their records: k_wf_sdf_hits)
    int32_t num_vol;           // Volumes (likewise: k_wf_vol_hits)
    // Routed split traversal (a scene with §8f row-4 shapes, at most 8 analytic records, lean lights and a
    // large triangle BVH): the refill kernels test the lean analytic records (spheres, cubes) linearly and
    // the row-4 ("heavy") records' boxes; only rays whose segment reaches such a box take the FULL half
    int32_t route;
    // Routed shade (a FULL scene whose materials carry no textures: only the environment texture or the
    // row-4 shapes make it FULL): vertices hitting spheres, cubes, planes and triangles go to the lean
    // shade kernel, the rest (row-4 hits, environment-texture misses) to the FULL one
    int32_t shade_route;
    int32_t heavy_count;
    const float4* heavy;       // 2 float4 per heavy record: {box lo.xyz, record index (bits)} {box hi.xyz, 0}
    // march_pending: a wave with fewer active lanes than this marches each pending Volume by its own lane
    // (vol_t, one grid read per cell), else by all active lanes together (coop_vol_t).  8 in every render;
    // pt_intersect / pt_occluded set 65 (every lane its own) or 1 (always together) to test both forms
    int32_t coop_min_lanes = 8;
    // counted passes only (else null): [0] Volume.Sample calls and [1] SDF evaluations of the
    // Volume / SDFShape intersect marches (DevBuffer::counters words 9 and 10)
    unsigned long long* march;
};

struct DevCamera {
    float p[3], u[3], v[3], w[3];
    double m, focal_distance, aperture_radius;
};

struct DevSampler {
    int32_t fh, mb, dl, ss, light_mode, spec_mode;
};

struct DevPass {
    int32_t width, height, spp, stratified;
    uint64_t seed;
    uint32_t pass_index;
    int32_t tiles_x;           // ceil(W/32)
    const int32_t* tiles;      // nullptr: tile = blockIdx.x / 4
    int32_t num_tiles;
    // A batch of `passes` consecutive passes (pass_index .. pass_index + passes - 1) in one
    // launch sequence (wavefront engine): pass p's samples add into accumulator p·acc_stride +
    // pixel, and k_wf_finalize applies the passes' Welford updates per pixel in pass order.
    int32_t passes = 1;
    uint32_t acc_stride = 0;   // accumulators per pass (W·H)
};

constexpr int kCounterWords = 32;    // DevBuffer::counters words
// Counted passes: the cooperative Volume march's phase clocks, 8 words per slot, kMarchSlots slots after the
// counters (a march adds its clocks to its wave's slot: one set of 8 words hit by every march serialised the
// counted pass' march kernels on those lines, C5 13 s per counted pass); the host sums the slots.
constexpr int kMarchClockWord = kCounterWords;
constexpr int kMarchSlots = 2048;
constexpr int kCounterAllocWords = kCounterWords + 8 * kMarchSlots;
struct DevBuffer {
    double* m;                 // [P][3] Welford mean   (Pixel.M, Buffer.cs:21)
    double* v;                 // [P][3] Welford M2     (Pixel.V, Buffer.cs:22)
    int32_t* n;                // [P]    sample count   (Pixel.Samples)
    unsigned long long* counters;  // [0..2] closest-hit rays/nodes/prims, [3] shading fetches, [4..6] shadow
                                   // rays/nodes/prims, [7] lit shadow rays, [8] their accumulation runs,
                                   // [9] volume samples, [10] SDF evaluations (DevScene::march),
                                   // [11] shadow-ray tail hand-offs (k_wf_shadow_lanes helpers, uncounted
                                   // passes), [15] wavefront queue overflow flag; counted passes also hold
                                   // the Volume march's phase clocks from word kMarchClockWord on, kMarchSlots
                                   // slots of 8 words (pt_device.h coop_vol_t)
};

}  // namespace pt
