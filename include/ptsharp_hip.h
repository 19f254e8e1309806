/*
 * ptsharp_hip.h — C-ABI of libptsharp_hip.so, the MI355X (gfx950) render hot path
 * that drops in for PTSharp's CPU `Renderer` (reference: akav/PTSharp).
 *
 * Boundary.  The C# side keeps scene construction (Example.*,
 * IShape/Material/Camera/Scene objects) and the `Buffer` output; it flattens the
 * scene once and calls these entry points through P/Invoke, following the same
 * create / commit / execute / release lifecycle and out-string error convention
 * the reference already uses for its only other native library, OIDN
 * (PTSharpCore/OIDN.cs:43-95, used at Renderer.cs:614-677).
 *
 * Which reference interface each entry point replaces:
 *   pt_create          Renderer.NewRenderer(scene,camera,sampler,w,h,mt)   Renderer.cs:35-56
 *                      (+ new Buffer(w,h)                                  Buffer.cs:67-80)
 *   pt_upload_scene    Scene.Compile() → Tree.NewTree / Mesh.Compile        Scene.cs:48-68, Tree.cs:22-29, Mesh.cs:45-57
 *                      (lights registered as in Scene.Add                  Scene.cs:29-38)
 *   pt_render_pass     one Renderer.RenderParallel() pass                  Renderer.cs:199-338
 *                      (flag PT_PASS_SERIAL: one Renderer.Render() pass  Renderer.cs:80-198)
 *                      = spp × Camera.CastRay → DefaultSampler.Sample      Camera.cs:98-119, Sampler.cs:40-145,191-296
 *                        → Scene.Intersect → Tree/IShape.Intersect        Scene.cs:75-79, Tree.cs:31-128
 *                        → Buffer.AddSample (Welford)                     Buffer.cs:33-44,94-97
 *   pt_read_buffer     reading Renderer.PBuffer pixels {Samples, M, V}     Buffer.cs:18-58, Renderer.cs:20
 *   pt_reset_buffer    Renderer.PBuffer = new Buffer(w,h)                  Renderer.cs:41
 *   pt_write_buffer    resuming IterativeRender from a saved PBuffer       Renderer.cs:702-765
 *   pt_read_tiles /    (new) a tile list's pixels, packed: progressive    SURVEY.md §8e
 *   pt_write_tiles     display of a rank's tiles, host-side gathers
 *   pt_intersect /     Scene.Intersect of a host's rays; the shadow query   Scene.cs:75-79, Sampler.cs:261-265
 *   pt_occluded
 *   pt_stats           Scene.rays (Interlocked counter, never printed)     Scene.cs:70-79
 *                      + the "time elapsed" stopwatch                      Renderer.cs:212-213,470
 *   pt_last_error      oidnGetDeviceError(device, out msg)                 OIDN.cs:85-86
 *   pt_destroy         oidnReleaseDevice                                   OIDN.cs:55-56
 *   pt_comm_*          (new) Buffer gather across GPUs over RCCL/xGMI      SURVEY.md §8e
 *                      (one process per GPU, or one process on all GPUs:  Renderer.cs:257-333 is one
 *                       pt_comm_init_all / pt_comm_gather_all)            process on all cores)
 *
 * Conventions: every function returns PT_OK (0) or a negative pt_status; the
 * detail string of the last failure on the calling thread is pt_last_error().
 * All structs are blittable POD (C# [StructLayout(LayoutKind.Sequential)]).
 * Geometry is float (the reference stores Vector as System.Numerics.Vector3,
 * Vector.cs:201), material/colour/camera scalars are double (Colour.cs:10-12,
 * Camera.cs:12-14).  Host arrays are caller-owned and are copied during the call.
 * A context is used by one host thread at a time; contexts are independent.
 */
#ifndef PTSHARP_HIP_H
#define PTSHARP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 9

typedef enum pt_status {
    PT_OK = 0,
    PT_ERR_INVALID_ARG = -1,
    PT_ERR_HIP = -2,          /* a HIP runtime call failed (detail in pt_last_error) */
    PT_ERR_NO_SCENE = -3,     /* pt_render_pass before pt_upload_scene */
    PT_ERR_UNSUPPORTED = -4,  /* a shape/material feature the GPU path does not cover */
    PT_ERR_OUT_OF_MEMORY = -5,
    PT_ERR_RCCL = -6,
    PT_ERR_NO_DEVICE = -7
} pt_status;

/* Shape kinds in Scene.Shapes order (Scene.cs:19,29-38). */
typedef enum pt_shape_kind {
    PT_SHAPE_SPHERE = 0,    /* Sphere.cs   */
    PT_SHAPE_CUBE = 1,      /* Cube.cs     */
    PT_SHAPE_PLANE = 2,     /* Plane.cs    */
    PT_SHAPE_TRIANGLE = 3,  /* Triangle.cs, added directly to the scene (a boxed struct) */
    PT_SHAPE_MESH = 4,      /* Mesh.cs, a range of triangles with its own tree */
    PT_SHAPE_SDF = 5,       /* SDF.cs SDFShape (sphere-traced signed distance tree) */
    PT_SHAPE_VOLUME = 6,    /* Volume.cs (voxel grid, iso-window marching) */
    PT_SHAPE_TRANSFORMED = 7 /* TransformedShape.cs (instancing of one inner shape) */
} pt_shape_kind;

/* ---- §8f row 4: SDF.cs, Volume.cs, TransformedShape.cs ----------------------
 * SDF nodes form a tree (children listed in pt_scene_desc.sdf_children).  Vector-
 * valued parameters are the reference's fp32 Vector fields widened to double. */
typedef enum pt_sdf_op {
    PT_SDF_SPHERE = 0,        /* SphereSDF       params: Radius, Exponent                 SDF.cs:115-140 */
    PT_SDF_CUBE = 1,          /* CubeSDF         params: Size.xyz                          SDF.cs:142-195 */
    PT_SDF_CYLINDER = 2,      /* CylinderSDF     params: Radius, Height                    SDF.cs:197-252 */
    PT_SDF_CAPSULE = 3,       /* CapsuleSDF      params: A.xyz, B.xyz, Radius, Exponent    SDF.cs:254-285 */
    PT_SDF_TORUS = 4,         /* TorusSDF        params: MajorRadius, MinRadius, MajorExponent, MinorExponent  SDF.cs:287-319 */
    PT_SDF_TRANSFORM = 5,     /* TransformSDF    matrix, inverse; 1 child                  SDF.cs:321-353 */
    PT_SDF_SCALE = 6,         /* ScaleSDF        params: Factor; 1 child                   SDF.cs:355-382 */
    PT_SDF_UNION = 7,         /* UnionSDF        n children                                SDF.cs:384-435 */
    PT_SDF_DIFFERENCE = 8,    /* DifferenceSDF   n >= 1 children                           SDF.cs:437-477 */
    PT_SDF_INTERSECTION = 9,  /* IntersectionSDF n children                                SDF.cs:479-531 */
    PT_SDF_REPEAT = 10        /* RepeatSDF       params: Step.xyz; 1 child                 SDF.cs:533-559 */
} pt_sdf_op;

typedef struct pt_sdf_node {
    int32_t op;               /* pt_sdf_op */
    int32_t num_children;
    int32_t first_child;      /* children: sdf_children[first_child .. first_child + num_children) */
    int32_t _pad;
    double params[8];
    double matrix[16];        /* PT_SDF_TRANSFORM: Matrix M11..M44, row-major */
    double inverse[16];       /* and the Inverse TransformSDF stores */
} pt_sdf_node;

typedef struct pt_sdf_shape {  /* SDFShape.NewSDFShape(sdf, material), SDF.cs:12-113 */
    int32_t root;             /* node index */
    int32_t material;
} pt_sdf_shape;

typedef struct pt_volume_window {  /* Volume.VolumeWindow, Volume.cs:8-19 */
    double lo, hi;
    int32_t material;
    int32_t _pad;
} pt_volume_window;

typedef struct pt_volume {    /* Volume fields W, H, D, ZScale, Data, Windows, Box (Volume.cs:21-38) */
    int32_t w, h, d;
    int32_t num_windows;
    double zscale;
    const double* data;       /* [d][h][w] */
    const pt_volume_window* windows;
    float box_min[3];
    float box_max[3];
} pt_volume;

typedef struct pt_transformed_shape {  /* TransformedShape(Shape, Matrix, Inverse), TransformedShape.cs:9-24 */
    int32_t shape_kind;       /* inner IShape: SPHERE, CUBE, PLANE, SDF or VOLUME */
    int32_t shape_index;      /* index into that kind's arrays */
    double matrix[16];
    double inverse[16];
} pt_transformed_shape;

/* ColorTexture (Texture.cs:96-252): Width x Height Colour texels, row-major, as the
 * C# object holds them (Data[y * Width + x], already through Pow(2.2) and any
 * ITexture.Pow / MulScalar the scene applied).  Width and Height must be >= 2
 * (BilinearSample reads texel x0 + 1 and y0 + 1, Texture.cs:198-206). */
typedef struct pt_texture {
    int32_t width;
    int32_t height;
    const double* data;   /* [height][width][3] */
} pt_texture;

/* Material (Material.cs:8-62).  Texture slots are 1-based references into
 * pt_scene_desc.textures: 0 = null (no map), k = textures[k - 1], so a zeroed
 * pt_material is a valid untextured material. */
typedef struct pt_material {
    double color[3];      /* Colour Color            */
    double emittance;     /* Emittance               */
    double index;         /* Index (IOR)             */
    double gloss;         /* Gloss (radians)         */
    double tint;          /* Tint                    */
    double reflectivity;  /* Reflectivity (<0: Fresnel) */
    int32_t transparent;  /* Transparent             */
    int32_t texture;          /* Texture       → Color (Material.MaterialAt, Material.cs:124-138)  */
    int32_t normal_texture;   /* NormalTexture → Triangle.NormalAt normal map (Triangle.cs:147-168) */
    int32_t bump_texture;     /* BumpTexture   → Triangle.NormalAt bump (Triangle.cs:170-184)       */
    int32_t gloss_texture;    /* GlossTexture  → Gloss = mean of the sampled colour               */
    int32_t _pad;
    double bump_multiplier;   /* BumpMultiplier */
} pt_material;

/* Flattened Scene.  Triangle arrays hold every triangle: directly-added ones
 * (shape_kind TRIANGLE, shape_index = triangle index) and mesh triangles
 * (mesh_first/mesh_count ranges).  Per-element arrays are [n][3] row-major. */
typedef struct pt_scene_desc {
    int32_t num_materials;
    const pt_material* materials;

    int32_t num_shapes;
    const int32_t* shape_kind;    /* pt_shape_kind, Scene.Shapes order */
    const int32_t* shape_index;   /* index into the per-kind arrays    */

    int32_t num_spheres;
    const float* sphere_center;   /* [n][3]  Sphere.Center (Vector) */
    const double* sphere_radius;  /* [n]     Sphere.Radius (double) */
    const int32_t* sphere_material;

    int32_t num_cubes;
    const float* cube_min;        /* [n][3] */
    const float* cube_max;        /* [n][3] */
    const int32_t* cube_material;

    int32_t num_planes;
    const float* plane_point;     /* [n][3] */
    const float* plane_normal;    /* [n][3], already normalised as Plane.NewPlane does */
    const int32_t* plane_material;

    int32_t num_triangles;
    const float* tri_v1;          /* [n][3] V1,V2,V3 */
    const float* tri_v2;
    const float* tri_v3;
    const float* tri_n1;          /* [n][3] N1,N2,N3 (after FixNormals / SmoothNormals) */
    const float* tri_n2;
    const float* tri_n3;
    const int32_t* tri_material;

    int32_t num_meshes;
    const int32_t* mesh_first;    /* first triangle of each mesh */
    const int32_t* mesh_count;

    double env_color[3];          /* Scene.Color (Scene.cs:25), returned on a miss */

    /* textures (§8f row 3); all optional */
    int32_t num_textures;
    const pt_texture* textures;
    const float* tri_t1;          /* [n][3] Triangle.T1..T3 texture coordinates; NULL = all zero */
    const float* tri_t2;
    const float* tri_t3;
    int32_t env_texture;          /* Scene.Texture (1-based, 0 = null): sampleEnvironment, Sampler.cs:177-189 */
    int32_t _pad;
    double env_texture_angle;     /* Scene.TextureAngle */

    /* SDF shapes, volumes, transformed shapes (§8f row 4); all optional */
    int32_t num_sdf_nodes;
    const pt_sdf_node* sdf_nodes;
    const int32_t* sdf_children;
    int32_t num_sdf_shapes;
    const pt_sdf_shape* sdf_shapes;
    int32_t num_volumes;
    const pt_volume* volumes;
    int32_t num_transformed;
    const pt_transformed_shape* transformed;
} pt_scene_desc;

/* Camera struct fields (Camera.cs:11-14) as produced by Camera.LookAt/SetFocus. */
typedef struct pt_camera {
    float p[3], u[3], v[3], w[3];
    double m;
    double focal_distance;
    double aperture_radius;
} pt_camera;

typedef enum pt_light_mode { PT_LIGHT_RANDOM = 0, PT_LIGHT_ALL = 1 } pt_light_mode;        /* LightMode.cs */
typedef enum pt_specular_mode { PT_SPEC_NAIVE = 0, PT_SPEC_FIRST = 1, PT_SPEC_ALL = 2 } pt_specular_mode; /* SpecularMode.cs */

/* DefaultSampler parameters (Sampler.cs:13-18).  FirstHitSamples/MaxBounces/
 * DirectLighting/SoftShadows are private in C#, so the drop-in passes them explicitly. */
typedef struct pt_sampler {
    int32_t first_hit_samples;
    int32_t max_bounces;
    int32_t direct_lighting;
    int32_t soft_shadows;
    int32_t light_mode;      /* pt_light_mode    */
    int32_t specular_mode;   /* pt_specular_mode */
} pt_sampler;

/* One render pass (one RenderParallel call).  Random.Shared is replaced by a
 * counter-based stream keyed (seed, pass_index, pixel, sample, path node, dim). */
typedef struct pt_pass_params {
    int32_t spp;             /* Renderer.SamplesPerPixel                         */
    int32_t stratified;      /* Renderer.StratifiedSampling (Renderer.cs:231-253) */
    uint64_t seed;
    uint32_t pass_index;     /* IterativeRender iteration i (Renderer.cs:709)    */
    int32_t num_tiles;       /* 0 = whole image; else render only these 32x32 tiles */
    const int32_t* tiles;    /* tile id = ty * ceil(W/32) + tx                   */
    int32_t engine;          /* pt_engine                                        */
    int32_t flags;           /* PT_PASS_KERNEL_TIMING: per-kernel hipEvent timing; PT_PASS_SERIAL */
    int32_t adaptive_samples;/* Renderer.AdaptiveSamples (Renderer.cs:340-410): per-sample AddSample x N */
    int32_t firefly_samples; /* Renderer.FireflySamples (Renderer.cs:412-470, FireflyThreshold = 1) */
    int32_t passes;          /* 0 or 1: one pass.  K > 1: K consecutive IterativeRender passes
                              * (pass_index .. pass_index + K - 1) in one call, the Buffer as after K
                              * separate calls, bit for bit.  Plain RenderParallel passes on the
                              * wavefront engine run as one batch: every pass' samples in one launch
                              * sequence, each pass' Welford update applied per pixel in order (a
                              * small tile share fills the GPU like a whole frame); other passes run
                              * one by one.  pt_stats then covers the K passes. */
} pt_pass_params;

#define PT_PASS_KERNEL_TIMING 1
/* Renderer.Render semantics (Renderer.cs:80-198, taken by IterativeRender when NumCPU == 1,
 * Renderer.cs:712-719) instead of RenderParallel's: the main samples are the same; then per
 * pixel AdaptiveSamples individual samples when StandardDeviation().MaxComponent() >= 1
 * (AdaptiveSamples * (int)v, AdaptiveThreshold = AdaptiveExponent = 1, :153-175), then
 * FireflySamples individual samples when it exceeds 1 (:177-191; no IsFirefly stop, jitter
 * (x + NextDouble()) * (1.0f / w)). */
#define PT_PASS_SERIAL 2

/* Kernel classes reported by pt_stats.kernel_ms / kernel_launches. */
typedef enum pt_kernel_class {
    PT_K_CAMERA = 0, PT_K_TRACE = 1, PT_K_SHADE = 2, PT_K_SHADOW = 3, PT_K_FINALIZE = 4, PT_K_MEGAKERNEL = 5,
    PT_K_ACCUM = 6,            /* k_wf_nee_accum: the visible shadow rays' light terms into the pixel sums */
    PT_K_COUNT = 7
} pt_kernel_class;
#define PT_K_SLOTS 8           /* length of pt_stats.kernel_ms / kernel_launches */

/* Both engines compute identical per-ray arithmetic; they differ in scheduling. */
typedef enum pt_engine {
    PT_ENGINE_AUTO = 0,        /* wavefront, megakernel when the queues cannot hold a useful chunk */
    PT_ENGINE_MEGAKERNEL = 1,  /* one lane per pixel runs the whole sampler recursion */
    PT_ENGINE_WAVEFRONT = 2    /* depth-by-depth ray queues in HBM (trace / shade / shadow kernels) */
} pt_engine;

typedef struct pt_device_opts {
    int32_t device;          /* HIP device ordinal */
    int32_t width;
    int32_t height;
} pt_device_opts;

typedef struct pt_stats {
    uint64_t rays;           /* Scene.Intersect calls, last pass (Scene.cs:77) */
    uint64_t rays_total;     /* since pt_create / pt_reset_buffer             */
    double last_pass_ms;     /* device time of the last pass (hipEvent)       */
    double total_ms;
    uint64_t bvh_nodes;      /* acceleration structure size                   */
    uint64_t bvh_bytes;
    double build_ms;         /* host BVH build time of the last upload        */
    uint64_t passes;
    uint64_t shadow_rays;    /* of `rays`: shadow-visibility queries (sampleLight)     */
    double kernel_ms[PT_K_SLOTS];     /* last pass, device time per pt_kernel_class (flag PT_PASS_KERNEL_TIMING) */
    uint32_t kernel_launches[PT_K_SLOTS];
    uint64_t traversal_bytes; /* of bvh_bytes: BVH nodes + leaf chunks, what the traversal kernels read */
    uint64_t tail_handoffs;   /* last pass (ABI 9): stack entries the shadow refill kernel's idle lanes took from
                               * busy lanes' rays in its tail (k_wf_shadow_lanes helpers; wavefront engine) */
} pt_stats;

int pt_get_version(void);
int pt_device_count(int32_t* out_count);
int pt_create(const pt_device_opts* opts, void** out_ctx);
int pt_upload_scene(void* ctx, const pt_scene_desc* scene);
int pt_render_pass(void* ctx, const pt_camera* camera, const pt_sampler* sampler,
                   const pt_pass_params* pass);
int pt_synchronize(void* ctx);
int pt_reset_buffer(void* ctx);
/* Welford state of every pixel, row-major: M,V [H*W][3] (Colour, double), N [H*W]. */
int pt_read_buffer(void* ctx, double* out_m, double* out_v, int32_t* out_n);
/* Replace the Welford state (same layout; NULL leaves that array as it is): resume an
 * IterativeRender from a saved Buffer (Renderer.cs:702-765 keeps accumulating into
 * Renderer.PBuffer pass after pass; a checkpoint is that Buffer). */
int pt_write_buffer(void* ctx, const double* m, const double* v, const int32_t* n);

/* The Buffer pixels of `num_tiles` 32x32 tiles, packed: m, v [num_tiles][32][32][3], n
 * [num_tiles][32][32], row-major inside a tile (entry (t, r, c) = pixel (32·(tiles[t] mod
 * ceil(W/32)) + c, 32·(tiles[t] div ceil(W/32)) + r)).  Pixels outside the image read as 0
 * and are ignored on write.  The same packing carries pt_comm_gather's tiles; a host that
 * moves Buffers over its own transport (gloo, MPI, sockets) gathers with these two calls. */
int pt_read_tiles(void* ctx, const int32_t* tiles, int32_t num_tiles, double* out_m, double* out_v, int32_t* out_n);
int pt_write_tiles(void* ctx, const int32_t* tiles, int32_t num_tiles, const double* m, const double* v,
                   const int32_t* n);
int pt_stats_get(void* ctx, pt_stats* out_stats);
const char* pt_last_error(void);
void pt_destroy(void* ctx);

/* ---- Mesh ingest (host only; no device needed).  OBJ.Load (OBJ.cs:11-165) with its
 * quirks: lower-cased lines split on ' ', the dummy normal 0, "v//n"
 * read as a texture index, fan triangulation, Triangle.FixNormals.  Arrays are [n][3]
 * float, allocated by the library; release them with pt_mesh_free. */
typedef struct pt_mesh_data {
    int32_t num_triangles;
    float *v1, *v2, *v3;   /* Triangle.V1..V3 */
    float *n1, *n2, *n3;   /* Triangle.N1..N3 (after FixNormals) */
    float *t1, *t2, *t3;   /* Triangle.T1..T3 (u, v, 0) */
} pt_mesh_data;
int pt_obj_load(const char* path, pt_mesh_data* out);
void pt_mesh_free(pt_mesh_data* mesh);
const char* pt_obj_last_error(void);
/* Mesh.SmoothNormals (Mesh.cs:191-229), in place on n1..n3. */
int pt_mesh_smooth_normals(int32_t n, const float* v1, const float* v2, const float* v3, float* n1, float* n2,
                           float* n3);

/* Multi-GPU: one context per GPU.  Each context renders its tile list
 * (pt_pass_params.tiles; the ranks' lists must be disjoint), and pt_comm_gather assembles
 * them on rank `root`: every other rank packs the {M, V, N} of its last pass' tiles and sends
 * them with the tile ids (RCCL send/recv over xGMI, after an all-gather of the tile counts);
 * root writes them into its Buffer.  For disjoint tiles that is the sum of the ranks'
 * Buffers, at 1/N of a full frame's bytes per rank.  Two ways to form the communicator:
 *   - one process per GPU: rank 0 makes the id (pt_comm_unique_id), ships it to the other
 *     processes, and every rank calls pt_comm_init (it blocks until all ranks joined);
 *   - one process driving G GPUs (the .NET host): G contexts on G devices, joined by ONE
 *     call pt_comm_init_all from any thread, gathered by pt_comm_gather_all.  Render the G
 *     contexts from G host threads at once (one thread per context): a pass with
 *     firefly_samples > 0 all-reduces the firefly snapshot across the group.
 * After a gather, root's pt_read_buffer returns the whole frame; root's next pass first
 * clears the pixels outside its own tiles again, so gathers can repeat every pass (so does any
 * rank's next tile-subset pass after pt_write_buffer or pt_write_tiles put other ranks' pixels in
 * its Buffer, e.g. every rank resuming from the whole checkpoint).  Root refuses a gather whose
 * tile ids repeat (two ranks rendered one tile) before it writes anything. */
int pt_comm_unique_id(uint8_t out_id[128]);
int pt_comm_init(void* ctx, int32_t nranks, int32_t rank, const uint8_t id[128]);
int pt_comm_gather(void* ctx, int32_t root);
int pt_comm_destroy(void* ctx);
int pt_comm_init_all(void* const* ctxs, int32_t n);            /* ncclCommInitAll over the contexts' devices */
int pt_comm_gather_all(void* const* ctxs, int32_t n, int32_t root);   /* the group's gathers, issued together */
/* The gather's host-side arithmetic, exported so a host can check its tile assignment before any
 * RCCL call (pure functions: no device, no context).  pt_gather_layout: where rank p's packed
 * tiles land in root's receive buffers (tile offset; -1 for root and for ranks with no tiles),
 * and the tiles root receives; PT_ERR_INVALID_ARG if a count is out of range or the counts sum
 * past image_tiles (overlapping lists).  pt_tile_lists_check: every id in [0, image_tiles), none
 * twice.  (Renderer.cs:257-333 deals disjoint sub-tiles to tasks; these keep the ranks disjoint.) */
int pt_gather_layout(int32_t nranks, int32_t root, const int32_t* counts, int32_t image_tiles,
                     int64_t* out_offsets, int64_t* out_total);
int pt_tile_lists_check(const int32_t* ids, int64_t n, int32_t image_tiles);

/* Ray queries on the uploaded scene, one lane per ray (the megakernel's traversal).  Rays are
 * [n][3] float origins and directions (Ray.Origin / Ray.Direction, Vector = Vector3).
 *   pt_intersect  Scene.Intersect (Scene.cs:75-79 → Tree.Intersect, Tree.cs:31-42): out_t[i] the
 *                 nearest hit's T (Hit.T, 1e9 = Hit.INF on a miss, Hit.cs:6), out_kind[i] its
 *                 pt_shape_kind (a mesh triangle is PT_SHAPE_TRIANGLE) or -1.
 *   pt_occluded   the shadow query after the light's own t (Sampler.cs:261-265 as the wavefront engine
 *                 answers it): out_blocked[i] = 1 if some shape is hit strictly nearer
 *                 than t_max[i].
 * flags choose how a ray's Volume (Volume.Intersect, Volume.cs:168-197) is marched; every choice
 * returns the same bits, which is what the flags are for: 0 as in a render (a wave's lanes march
 * together unless fewer than 8 are active), PT_MARCH_LANE every lane its own march, PT_MARCH_WAVE
 * always together. */
#define PT_MARCH_LANE 1
#define PT_MARCH_WAVE 2
int pt_intersect(void* ctx, int64_t n, const float* origins, const float* dirs, int32_t flags, double* out_t,
                 int32_t* out_kind);
int pt_occluded(void* ctx, int64_t n, const float* origins, const float* dirs, const double* t_max, int32_t flags,
                int32_t* out_blocked);

/* The triangle BVH is built once per process for identical geometry: N contexts that upload the same
 * scene (one process driving N GPUs) share one host build (Scene.Compile once, Scene.cs:48-68) and upload
 * its bytes; a context that uploads while another builds waits for that build.  Host only (no device):
 * out[0] a 64-bit digest of the BVH bytes a context of this scene receives (node lines, leaf chunks,
 * triangle order), out[1] their size in bytes, out[2] / out[3] the builds made / builds reused so far. */
int pt_scene_bvh_digest(const pt_scene_desc* scene, uint64_t out[4]);

/* Instrumentation (bench / roofline): last pass' traversal counters, summed. */
typedef struct pt_trace_counters {
    uint64_t rays;            /* all Scene.Intersect calls                     */
    uint64_t nodes_visited;   /* BVH child-pair fetches (64 B each), all rays  */
    uint64_t prims_tested;    /* triangle/sphere/cube records tested (48 B)     */
    uint64_t shading_fetches; /* closest-hit shading records (40 B)            */
    uint64_t shadow_rays;     /* the shadow-visibility part of the above ...   */
    uint64_t shadow_nodes;
    uint64_t shadow_prims;
    uint64_t lit_shadow_rays; /* shadow rays whose light was the nearest hit (terms added)   */
    uint64_t accum_runs;      /* their per-pixel runs after wave aggregation (atomic sets)  */
    uint64_t volume_samples;  /* Volume.Sample calls of Volume.Intersect's march (Volume.cs:168-197) */
    uint64_t sdf_evals;       /* SDF evaluations of SDFShape.Intersect's sphere tracing (SDF.cs:32-76) */
    /* The cooperative Volume march's time by phase, shader-clock cycles summed over the marching waves
     * (s_memtime around each phase, so they run ~10 % slower in a counted pass): [0] strided passes over
     * uniform cells, [1] a dense round's position and uniform-cell table read, [2] its corner reads and
     * interpolation, [3] its window loop (Volume.Sign), [4] its ballots and bookkeeping, [5] refinements;
     * [6] dense rounds, [7] strided-pass rounds (counts). */
    uint64_t march_clock[8];
} pt_trace_counters;
int pt_render_pass_counted(void* ctx, const pt_camera* camera, const pt_sampler* sampler,
                           const pt_pass_params* pass, pt_trace_counters* out);

#ifdef __cplusplus
}
#endif
#endif /* PTSHARP_HIP_H */
