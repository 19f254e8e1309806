/*
 * oracle.h — CPU restatement of PTSharp's render hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so, and only as the checker / CPU baseline.
 * The product (libptsharp_hip.so, ptsharp_amd/) never links or calls it.
 *
 * Parity status: UNPINNED against the reference itself — PTSharp is C#/.NET 9
 * (no dotnet/mono in this image), ships no tests, fixtures or
 * golden images, and draws every random number from the unseedable
 * Random.Shared.  The restatement is pinned instead by analytic known-answer
 * tests derived from the reference's semantics (tests/test_oracle.py) and by
 * the golden fixtures it generates (tests/golden/, generating script committed).
 *
 * The scene/camera/sampler/pass structs have the same layout as the product's
 * C-ABI (include/ptsharp_hip.h) so one host-side flattening feeds both.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_texture {
    int32_t width, height;
    const double* data;   /* [h][w][3] ColorTexture.Data */
} or_texture;

typedef struct or_material {
    double color[3];
    double emittance, index, gloss, tint, reflectivity;
    int32_t transparent;
    int32_t texture, normal_texture, bump_texture, gloss_texture;  /* 1-based, 0 = null */
    int32_t _pad;
    double bump_multiplier;
} or_material;

typedef struct or_sdf_node {
    int32_t op, num_children, first_child, _pad;
    double params[8];
    double matrix[16], inverse[16];
} or_sdf_node;
typedef struct or_sdf_shape { int32_t root, material; } or_sdf_shape;
typedef struct or_volume_window { double lo, hi; int32_t material, _pad; } or_volume_window;
typedef struct or_volume {
    int32_t w, h, d, num_windows;
    double zscale;
    const double* data;
    const or_volume_window* windows;
    float box_min[3], box_max[3];
} or_volume;
typedef struct or_transformed_shape {
    int32_t shape_kind, shape_index;
    double matrix[16], inverse[16];
} or_transformed_shape;

typedef struct or_scene_desc {
    int32_t num_materials; const or_material* materials;
    int32_t num_shapes; const int32_t* shape_kind; const int32_t* shape_index;
    int32_t num_spheres; const float* sphere_center; const double* sphere_radius; const int32_t* sphere_material;
    int32_t num_cubes; const float* cube_min; const float* cube_max; const int32_t* cube_material;
    int32_t num_planes; const float* plane_point; const float* plane_normal; const int32_t* plane_material;
    int32_t num_triangles;
    const float *tri_v1, *tri_v2, *tri_v3, *tri_n1, *tri_n2, *tri_n3;
    const int32_t* tri_material;
    int32_t num_meshes; const int32_t* mesh_first; const int32_t* mesh_count;
    double env_color[3];
    int32_t num_textures; const or_texture* textures;
    const float *tri_t1, *tri_t2, *tri_t3;
    int32_t env_texture, _pad;
    double env_texture_angle;
    int32_t num_sdf_nodes; const or_sdf_node* sdf_nodes; const int32_t* sdf_children;
    int32_t num_sdf_shapes; const or_sdf_shape* sdf_shapes;
    int32_t num_volumes; const or_volume* volumes;
    int32_t num_transformed; const or_transformed_shape* transformed;
} or_scene_desc;

typedef struct or_camera {
    float p[3], u[3], v[3], w[3];
    double m, focal_distance, aperture_radius;
} or_camera;

typedef struct or_sampler {
    int32_t first_hit_samples, max_bounces, direct_lighting, soft_shadows, light_mode, specular_mode;
} or_sampler;

typedef struct or_pass_params {
    int32_t spp, stratified;
    uint64_t seed;
    uint32_t pass_index;
    int32_t num_tiles;
    const int32_t* tiles;
    int32_t engine, flags;  /* engine, and flags other than OR_PASS_SERIAL: product-only, ignored here */
    int32_t adaptive_samples, firefly_samples;  /* Renderer.AdaptiveSamples / FireflySamples */
    int32_t passes;  /* product-only (a batch of passes in one call); the oracle renders one pass per call */
} or_pass_params;
/* flags: Renderer.Render's extra phases (Renderer.cs:80-198) instead of RenderParallel's */
#define OR_PASS_SERIAL 2

/* Build the scene (k-d trees as Scene.Compile/Tree.NewTree do).  Returns NULL on error. */
void* or_scene_create(const or_scene_desc* desc);
void or_scene_destroy(void* scene);
/* Number of k-d tree nodes (top-level + per-mesh trees). */
int64_t or_scene_tree_nodes(void* scene);

/* One RenderParallel pass into caller-owned Welford arrays (M,V: [H*W][3], N: [H*W]).
 * brute_force != 0 replaces the k-d tree by a linear nearest-hit loop.
 * num_threads <= 0: all hardware threads.  Returns Scene.Intersect calls. */
int64_t or_render_pass(void* scene, int32_t width, int32_t height, const or_camera* cam,
                       const or_sampler* smp, const or_pass_params* pass,
                       double* m, double* v, int32_t* n, int32_t num_threads, int32_t brute_force);

/* Render only pixels [pix_begin, pix_end) in row-major order (CPU-baseline sampling). */
int64_t or_render_pixels(void* scene, int32_t width, int32_t height, const or_camera* cam,
                         const or_sampler* smp, const or_pass_params* pass,
                         int64_t pix_begin, int64_t pix_end, int64_t pix_stride,
                         double* m, double* v, int32_t* n, int32_t num_threads);

/* Known-answer helpers. */
/* Nearest hit: returns t (1e9 = miss), writes hit kind (-1 none) and index. */
double or_intersect(void* scene, const float origin[3], const float dir[3], int32_t brute_force,
                    int32_t* out_kind, int32_t* out_index);
/* Full Hit.Info: position, normal (after flip), inside flag, material id. */
int32_t or_hit_info(void* scene, const float origin[3], const float dir[3],
                    float out_pos[3], float out_normal[3], int32_t* out_inside, int32_t* out_mat);
void or_cast_ray(const or_camera* cam, int32_t x, int32_t y, int32_t w, int32_t h,
                 double u, double v, uint64_t key, float out_origin[3], float out_dir[3]);
/* Primitive-level intersect on a standalone primitive (kind 0..3), for KAT tables. */
double or_prim_intersect(int32_t kind, const float* a, const float* b, const float* c, double radius,
                         const float origin[3], const float dir[3]);
void or_prim_normal(int32_t kind, const float* a, const float* b, const float* c,
                    const float* n1, const float* n2, const float* n3,
                    const float pos[3], float out_normal[3]);

/* Texture KATs (Texture.cs:188-251): kind 0 Sample -> colour, 1 NormalSample, 2 BumpSample
 * -> vector; texture is 1-based as in or_material. */
void or_texture_sample(void* scene, int32_t texture, int32_t kind, double u, double v, double out[3]);
/* IShape.UVector of scene primitive (kind K_*, index into the per-kind arrays) at p. */
void or_shape_uv(void* scene, int32_t kind, int32_t index, const float p[3], float out_uv[3]);
/* sampleEnvironment (Sampler.cs:177-189) for a ray direction. */
void or_environment(void* scene, const float dir[3], double out[3]);
/* Hit.Info's material after Material.MaterialAt (Material.cs:124-138): colour and gloss. */
int32_t or_hit_surface(void* scene, const float origin[3], const float dir[3], double out_color[3], double* out_gloss);

/* SDF.Evaluate of node `node` at p (SDF.cs), Volume.Sample (Volume.cs:73-105). */
double or_sdf_evaluate(void* scene, int32_t node, const float p[3]);
double or_volume_sample(void* scene, int32_t volume, double x, double y, double z);
/* Bounding box of scene primitive (kind, index): IShape.BoundingBox. */
void or_shape_box(void* scene, int32_t kind, int32_t index, float out_min[3], float out_max[3]);

/* Bounce and light-sampling KATs (checked against tests/sampler_ref.py, a separate Python
 * restatement of the same C# lines). */
/* Ray.Bounce (Ray.cs:44-85) at the nearest hit of (origin, dir): 0 on a miss. */
int32_t or_bounce(void* scene, const float origin[3], const float dir[3], double u, double v, int32_t btype,
                  uint64_t key, float out_origin[3], float out_dir[3], int32_t* out_reflected, double* out_p);
/* Util.Cone (Util.cs:17-32). */
void or_cone(const float dir[3], double theta, double u, double v, uint64_t key, float out[3]);
/* Scene.Lights (Scene.cs:33-37): returns the count, fills (kind, index) of the first `cap`. */
int32_t or_lights(void* scene, int32_t* kinds, int32_t* indices, int32_t cap);
/* Sampler.sampleLight (Sampler.cs:212-296) of Scene.Lights[light] from the normal ray
 * (origin, normal); returns the Scene.Intersect calls made (0 or 1). */
int64_t or_sample_light(void* scene, const float origin[3], const float normal[3], int32_t light, uint64_t key,
                        int32_t soft_shadows, double out[3]);
/* Sampler.sampleLights (Sampler.cs:191-210); returns the Scene.Intersect calls made. */
int64_t or_sample_lights(void* scene, const float origin[3], const float normal[3], uint64_t key, int32_t light_mode,
                         int32_t soft_shadows, double out[3]);
/* The any-hit form of the shadow query the GPU runs: 1 if some scene shape
 * (brute force) is hit strictly nearer than t_light along (origin, dir). */
int32_t or_any_nearer(void* scene, const float origin[3], const float dir[3], double t_light);

/* Counter-based RNG that replaces Random.Shared (spec in DESIGN.md §RNG). */
uint64_t or_camera_key(uint64_t seed, uint32_t pass, uint64_t pixel, uint32_t sample);
uint64_t or_child_key(uint64_t key, uint32_t child);
uint64_t or_light_key(uint64_t key, uint32_t light);
double or_draw(uint64_t key, uint32_t dim);

#ifdef __cplusplus
}
#endif
#endif
