// HipRenderer.cs — drop-in for PTSharpCore.Renderer that runs the per-pixel hot
// path on an MI355X through libptsharp_hip.so (include/ptsharp_hip.h).
//
// Add this file to PTSharpCore/ (same namespace).  It mirrors the reference's
// Renderer factory and knobs (Renderer.cs:35-56), its IterativeRender contract
// (Renderer.cs:702-765) and writes into the same static Buffer (Renderer.PBuffer,
// Buffer.cs:60-97).  P/Invoke follows the conventions the reference already uses
// for its only native dependency, OIDN (OIDN.cs:43-95): Cdecl, IntPtr handles,
// create / commit / execute / release, error strings fetched after a failure.
//
// NOTE: this file is not compiled in this repository (no .NET SDK in the build
// image); the same ABI is exercised from Python/ctypes by tests/test_abi.py and
// the GPU parity suite.  Struct layouts below match ptsharp_hip.h field by field.
using System;
using System.Collections.Generic;
using System.Runtime.InteropServices;
using System.Threading.Tasks;
using SkiaSharp;

namespace PTSharpCore
{
    internal static class PtHip
    {
        const string Lib = "ptsharp_hip";   // libptsharp_hip.so on Linux

        public const int PT_OK = 0;
        public const int PT_ERR_UNSUPPORTED = -4;
        public const int PT_PASS_KERNEL_TIMING = 1, PT_PASS_SERIAL = 2;
        public const int PT_MARCH_LANE = 1, PT_MARCH_WAVE = 2;   // pt_intersect / pt_occluded flags
        public const int SHAPE_SPHERE = 0, SHAPE_CUBE = 1, SHAPE_PLANE = 2, SHAPE_TRIANGLE = 3, SHAPE_MESH = 4;
        public const int SHAPE_SDF = 5, SHAPE_VOLUME = 6, SHAPE_TRANSFORMED = 7;

        [StructLayout(LayoutKind.Sequential)]
        public struct pt_texture
        {
            public int width; public int height; public IntPtr data;   // ColorTexture.Data as [h][w][3] double
        }

        [StructLayout(LayoutKind.Sequential)]
        public unsafe struct pt_material
        {
            public fixed double color[3];
            public double emittance, index, gloss, tint, reflectivity;
            public int transparent;
            public int texture, normal_texture, bump_texture, gloss_texture;   // 1-based into textures, 0 = null
            public int _pad;
            public double bump_multiplier;
        }

        [StructLayout(LayoutKind.Sequential)]
        public unsafe struct pt_sdf_node
        {
            public int op, num_children, first_child, _pad;
            public fixed double @params[8];
            public fixed double matrix[16];
            public fixed double inverse[16];
        }

        [StructLayout(LayoutKind.Sequential)]
        public struct pt_sdf_shape { public int root, material; }

        [StructLayout(LayoutKind.Sequential)]
        public struct pt_volume_window { public double lo, hi; public int material, _pad; }

        [StructLayout(LayoutKind.Sequential)]
        public unsafe struct pt_volume
        {
            public int w, h, d;
            public int num_windows;
            public double zscale;
            public IntPtr data;
            public IntPtr windows;
            public fixed float box_min[3];
            public fixed float box_max[3];
        }

        [StructLayout(LayoutKind.Sequential)]
        public unsafe struct pt_transformed_shape
        {
            public int shape_kind, shape_index;
            public fixed double matrix[16];
            public fixed double inverse[16];
        }

        [StructLayout(LayoutKind.Sequential)]
        public unsafe struct pt_scene_desc
        {
            public int num_materials; public IntPtr materials;
            public int num_shapes; public IntPtr shape_kind; public IntPtr shape_index;
            public int num_spheres; public IntPtr sphere_center; public IntPtr sphere_radius; public IntPtr sphere_material;
            public int num_cubes; public IntPtr cube_min; public IntPtr cube_max; public IntPtr cube_material;
            public int num_planes; public IntPtr plane_point; public IntPtr plane_normal; public IntPtr plane_material;
            public int num_triangles; public IntPtr tri_v1, tri_v2, tri_v3, tri_n1, tri_n2, tri_n3; public IntPtr tri_material;
            public int num_meshes; public IntPtr mesh_first; public IntPtr mesh_count;
            public fixed double env_color[3];
            public int num_textures; public IntPtr textures;
            public IntPtr tri_t1, tri_t2, tri_t3;
            public int env_texture; public int _pad; public double env_texture_angle;
            public int num_sdf_nodes; public IntPtr sdf_nodes; public IntPtr sdf_children;
            public int num_sdf_shapes; public IntPtr sdf_shapes;
            public int num_volumes; public IntPtr volumes;
            public int num_transformed; public IntPtr transformed;
        }

        [StructLayout(LayoutKind.Sequential)]
        public unsafe struct pt_camera
        {
            public fixed float p[3]; public fixed float u[3]; public fixed float v[3]; public fixed float w[3];
            public double m, focal_distance, aperture_radius;
        }

        [StructLayout(LayoutKind.Sequential)]
        public struct pt_sampler
        {
            public int first_hit_samples, max_bounces, direct_lighting, soft_shadows, light_mode, specular_mode;
        }

        [StructLayout(LayoutKind.Sequential)]
        public struct pt_pass_params
        {
            public int spp, stratified;
            public ulong seed;
            public uint pass_index;
            public int num_tiles;
            public IntPtr tiles;
            public int engine, flags;
            public int adaptive_samples, firefly_samples;   // Renderer.AdaptiveSamples / FireflySamples
            public int passes;                              // K consecutive passes in one call (0/1: one)
        }

        [StructLayout(LayoutKind.Sequential)]
        public struct pt_device_opts { public int device, width, height; }

        [StructLayout(LayoutKind.Sequential)]
        public unsafe struct pt_stats
        {
            public ulong rays, rays_total; public double last_pass_ms, total_ms;
            public ulong bvh_nodes, bvh_bytes; public double build_ms; public ulong passes;
            public ulong shadow_rays;
            public fixed double kernel_ms[8];       // PT_K_SLOTS
            public fixed uint kernel_launches[8];
            public ulong traversal_bytes;           // BVH nodes + leaf chunks (what traversal reads)
            public ulong tail_handoffs;             // shadow refill kernel's tail hand-offs, last pass (ABI 9)
        }

        [StructLayout(LayoutKind.Sequential)]
        public unsafe struct pt_trace_counters
        {
            public ulong rays, nodes_visited, prims_tested, shading_fetches, shadow_rays, shadow_nodes, shadow_prims;
            public ulong lit_shadow_rays, accum_runs;
            public ulong volume_samples, sdf_evals;   // Volume.Intersect / SDFShape.Intersect march steps
            public fixed ulong march_clock[8];   // the Volume march's phase clocks (counted passes)
        }

        [StructLayout(LayoutKind.Sequential)]
        public struct pt_mesh_data
        {
            public int num_triangles;
            public IntPtr v1, v2, v3, n1, n2, n3, t1, t2, t3;   // [n][3] float, owned by the library
        }

        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_get_version();
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_device_count(out int count);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_create(ref pt_device_opts opts, out IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_upload_scene(IntPtr ctx, ref pt_scene_desc scene);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_render_pass(IntPtr ctx, ref pt_camera cam, ref pt_sampler smp, ref pt_pass_params pass);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_render_pass_counted(IntPtr ctx, ref pt_camera cam, ref pt_sampler smp, ref pt_pass_params pass, out pt_trace_counters counters);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_synchronize(IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_read_buffer(IntPtr ctx, double[] m, double[] v, int[] n);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_write_buffer(IntPtr ctx, double[] m, double[] v, int[] n);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_read_tiles(IntPtr ctx, int[] tiles, int num_tiles, double[] m, double[] v, int[] n);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_write_tiles(IntPtr ctx, int[] tiles, int num_tiles, double[] m, double[] v, int[] n);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_reset_buffer(IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_stats_get(IntPtr ctx, out pt_stats stats);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_scene_bvh_digest(ref pt_scene_desc scene, ulong[] out4);
        // Scene.Intersect of a batch of rays / the shadow query against a t (PT_MARCH_* flags: the Volume march form)
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_intersect(IntPtr ctx, long n, float[] origins, float[] dirs, int flags, double[] t, int[] kind);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_occluded(IntPtr ctx, long n, float[] origins, float[] dirs, double[] tMax, int flags, int[] blocked);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern IntPtr pt_last_error();
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern void pt_destroy(IntPtr ctx);
        // multi-GPU (include/ptsharp_hip.h "Multi-GPU"): one process per GPU (unique id + init per rank) or
        // one process driving G contexts (init_all / gather_all)
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_comm_unique_id(byte[] id128);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_comm_init(IntPtr ctx, int nranks, int rank, byte[] id128);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_comm_gather(IntPtr ctx, int root);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_comm_destroy(IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_comm_init_all(IntPtr[] ctxs, int n);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_comm_gather_all(IntPtr[] ctxs, int n, int root);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_gather_layout(int nranks, int root, int[] counts, int imageTiles, long[] offsets, out long total);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_tile_lists_check(int[] ids, long n, int imageTiles);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl, CharSet = CharSet.Ansi)] public static extern int pt_obj_load(string path, out pt_mesh_data mesh);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern void pt_mesh_free(ref pt_mesh_data mesh);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern IntPtr pt_obj_last_error();
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)] public static extern int pt_mesh_smooth_normals(int n, float[] v1, float[] v2, float[] v3, float[] n1, float[] n2, float[] n3);

        public static void Check(int rc, string where)
        {
            if (rc != PT_OK)
                throw new InvalidOperationException($"{where} failed ({rc}): {Marshal.PtrToStringAnsi(pt_last_error())}");
        }
    }

    /// <summary>Renderer drop-in: same factory, knobs and IterativeRender contract as Renderer.</summary>
    class HipRenderer : IDisposable
    {
        Scene Scene; Camera Camera; DefaultSampler Sampler;
        public int SamplesPerPixel = 2;           // Renderer.cs:42
        public bool StratifiedSampling = false;   // Renderer.cs:44
        public int AdaptiveSamples = 0;           // Renderer.cs:23, phase at :340-410
        public int FireflySamples = 0;            // Renderer.cs:26, phase at :412-470
        public ulong Seed = 0;                     // Random.Shared is unseedable; this keys the GPU stream
        public int NumCPU = Environment.ProcessorCount;   // Renderer.cs:51-54: 1 selects Render() in IterativeRender
        /// <summary>32x32 tiles this renderer draws (tile id = ty * ceil(W/32) + tx); null = the whole
        /// image.  A multi-GPU rank draws TilesForRank(W, H, rank, world) (SURVEY.md §8e).</summary>
        public int[] Tiles = null;
        internal IntPtr ctx;
        int W, H, pass;
        internal int Width => W;
        internal int Height => H;
        bool uploaded;
        readonly List<GCHandle> pins = new();

        // DefaultSampler keeps FirstHitSamples/MaxBounces/DirectLighting/SoftShadows private
        // (Sampler.cs:13-16): the caller passes the values it constructed the sampler with.
        int firstHit, maxBounces; bool directLighting = true, softShadows = true;

        public static HipRenderer NewRenderer(Scene scene, Camera camera, DefaultSampler sampler, int firstHitSamples,
                                              int maxBounces, int w, int h, int device = 0, bool multithreaded = true)
        {
            var r = new HipRenderer { Scene = scene, Camera = camera, Sampler = sampler, W = w, H = h,
                                      firstHit = firstHitSamples, maxBounces = maxBounces,
                                      NumCPU = multithreaded ? Environment.ProcessorCount : 1 };
            Renderer.PBuffer = new Buffer(w, h);
            var opts = new PtHip.pt_device_opts { device = device, width = w, height = h };
            PtHip.Check(PtHip.pt_create(ref opts, out r.ctx), "pt_create");
            return r;
        }

        IntPtr Pin(Array a) { var g = GCHandle.Alloc(a, GCHandleType.Pinned); pins.Add(g); return g.AddrOfPinnedObject(); }

        /// <summary>Static interleaved tile ownership: tile t belongs to rank t % world.  Every pixel's
        /// random stream is keyed by the pixel, so the union of the ranks' Buffers is the 1-GPU Buffer, bit
        /// for bit (pt_comm_gather sums the disjoint tiles).</summary>
        public static int[] TilesForRank(int w, int h, int rank, int world)
        {
            int n = ((w + 31) / 32) * ((h + 31) / 32);
            var t = new List<int>();
            for (int i = rank; i < n; i += world) t.Add(i);
            return t.ToArray();
        }

        // Flatten Scene.Shapes (Scene.cs:19) with a type switch; returns PT_ERR_UNSUPPORTED kinds as exceptions
        // so the caller can fall back to the CPU Renderer.
        unsafe void Upload()
        {
            // ColorTexture instances (Texture.cs:96-252) by reference; 1-based ids, 0 = null.
            var texs = new List<PtHip.pt_texture>(); var texIds = new Dictionary<ITexture, int>(ReferenceEqualityComparer.Instance);
            int Tid(ITexture t)
            {
                if (t == null) return 0;
                if (t is not ColorTexture ct) throw new NotSupportedException($"{t.GetType().Name} is not on the GPU path");
                if (!texIds.TryGetValue(t, out int id))
                {
                    var data = new double[3 * ct.Data.Length];
                    for (int i = 0; i < ct.Data.Length; i++) { data[3 * i] = ct.Data[i].r; data[3 * i + 1] = ct.Data[i].g; data[3 * i + 2] = ct.Data[i].b; }
                    texs.Add(new PtHip.pt_texture { width = ct.Width, height = ct.Height, data = Pin(data) });
                    id = texs.Count; texIds[t] = id;
                }
                return id;
            }
            var mats = new List<PtHip.pt_material>(); var matIds = new Dictionary<Material, int>();
            int Mid(Material m)
            {
                if (!matIds.TryGetValue(m, out int id))
                {
                    id = mats.Count; matIds[m] = id;
                    var pm = new PtHip.pt_material { emittance = m.Emittance, index = m.Index, gloss = m.Gloss, tint = m.Tint,
                        reflectivity = m.Reflectivity, transparent = m.Transparent ? 1 : 0,
                        texture = Tid(m.Texture), normal_texture = Tid(m.NormalTexture), bump_texture = Tid(m.BumpTexture),
                        gloss_texture = Tid(m.GlossTexture), bump_multiplier = m.BumpMultiplier };
                    pm.color[0] = m.Color.r; pm.color[1] = m.Color.g; pm.color[2] = m.Color.b;
                    mats.Add(pm);
                }
                return id;
            }
            var kind = new List<int>(); var index = new List<int>();
            var sc = new List<float>(); var sr = new List<double>(); var sm = new List<int>();
            var cmin = new List<float>(); var cmax = new List<float>(); var cm = new List<int>();
            var pp = new List<float>(); var pn = new List<float>(); var pm = new List<int>();
            var v1 = new List<float>(); var v2 = new List<float>(); var v3 = new List<float>();
            var n1 = new List<float>(); var n2 = new List<float>(); var n3 = new List<float>(); var tm = new List<int>();
            var t1 = new List<float>(); var t2 = new List<float>(); var t3 = new List<float>();
            var mf = new List<int>(); var mc = new List<int>();
            void Add3(List<float> l, Vector v) { l.Add((float)v.X); l.Add((float)v.Y); l.Add((float)v.Z); }
            // SDF trees, volumes and transformed shapes (§8f row 4).  SDF / Volume / TransformedShape keep
            // their fields private in the reference (SDF.cs, Volume.cs:21-27, TransformedShape.cs:11-13):
            // the integration marks them `internal` (INTEGRATION.md), as for Plane.
            var sdfNodes = new List<PtHip.pt_sdf_node>(); var sdfKids = new List<int>(); var sdfIds = new Dictionary<SDF, int>(ReferenceEqualityComparer.Instance);
            var meshIds = new Dictionary<IShape, int>(ReferenceEqualityComparer.Instance);
            var sdfShapes = new List<PtHip.pt_sdf_shape>(); var vols = new List<PtHip.pt_volume>(); var xfs = new List<PtHip.pt_transformed_shape>();
            void Mat16(double* dst, Matrix m)
            {
                double[] a = { m.M11, m.M12, m.M13, m.M14, m.M21, m.M22, m.M23, m.M24, m.M31, m.M32, m.M33, m.M34, m.M41, m.M42, m.M43, m.M44 };
                for (int k = 0; k < 16; k++) dst[k] = a[k];
            }
            int Sdf(SDF n)
            {
                if (sdfIds.TryGetValue(n, out int id)) return id;
                var node = new PtHip.pt_sdf_node();
                SDF[] kids = n switch
                {
                    TransformSDF t => new[] { t.SDF }, ScaleSDF sc => new[] { sc.SDF }, RepeatSDF r => new[] { r.SDF },
                    UnionSDF u => u.Items, DifferenceSDF df => df.Items, IntersectionSDF i => i.Items, _ => Array.Empty<SDF>(),
                };
                var kidIds = new List<int>(); foreach (var k in kids) kidIds.Add(Sdf(k));
                node.num_children = kidIds.Count; node.first_child = sdfKids.Count; sdfKids.AddRange(kidIds);
                switch (n)
                {
                    case SphereSDF sp: node.op = 0; node.@params[0] = sp.Radius; node.@params[1] = sp.Exponent; break;
                    case CubeSDF cu: node.op = 1; node.@params[0] = cu.Size.X; node.@params[1] = cu.Size.Y; node.@params[2] = cu.Size.Z; break;
                    case CylinderSDF cy: node.op = 2; node.@params[0] = cy.Radius; node.@params[1] = cy.Height; break;
                    case CapsuleSDF ca: node.op = 3; node.@params[0] = ca.A.X; node.@params[1] = ca.A.Y; node.@params[2] = ca.A.Z;
                        node.@params[3] = ca.B.X; node.@params[4] = ca.B.Y; node.@params[5] = ca.B.Z; node.@params[6] = ca.Radius; node.@params[7] = ca.Exponent; break;
                    case TorusSDF to: node.op = 4; node.@params[0] = to.MajorRadius; node.@params[1] = to.MinRadius;
                        node.@params[2] = to.MajorExponent; node.@params[3] = to.MinorExponent; break;
                    case TransformSDF tr: node.op = 5; Mat16(node.matrix, tr.Matrix); Mat16(node.inverse, tr.Inverse); break;
                    case ScaleSDF sc: node.op = 6; node.@params[0] = sc.Factor; break;
                    case UnionSDF: node.op = 7; break;
                    case DifferenceSDF: node.op = 8; break;
                    case IntersectionSDF: node.op = 9; break;
                    case RepeatSDF re: node.op = 10; node.@params[0] = re.Step.X; node.@params[1] = re.Step.Y; node.@params[2] = re.Step.Z; break;
                    default: throw new NotSupportedException($"{n.GetType().Name} is not on the GPU path");
                }
                id = sdfNodes.Count; sdfIds[n] = id; sdfNodes.Add(node);
                return id;
            }
            (int, int) Inner(IShape s)
            {
                switch (s)
                {
                    case Sphere sp: Add3(sc, sp.Center); sr.Add(sp.Radius); sm.Add(Mid(sp.Material)); return (PtHip.SHAPE_SPHERE, sr.Count - 1);
                    case Cube cu: Add3(cmin, cu.Min); Add3(cmax, cu.Max); cm.Add(Mid(cu.Material)); return (PtHip.SHAPE_CUBE, cm.Count - 1);
                    case Plane pl: Add3(pp, pl.Point); Add3(pn, pl.Normal); pm.Add(Mid(pl.Material)); return (PtHip.SHAPE_PLANE, pm.Count - 1);
                    case SDFShape sd: sdfShapes.Add(new PtHip.pt_sdf_shape { root = Sdf(sd.SDF), material = Mid(sd.Material) }); return (PtHip.SHAPE_SDF, sdfShapes.Count - 1);
                    case Volume vo:
                    {
                        var wins = new PtHip.pt_volume_window[vo.Windows.Length];
                        for (int k = 0; k < wins.Length; k++)
                            wins[k] = new PtHip.pt_volume_window { lo = vo.Windows[k].Lo, hi = vo.Windows[k].Hi, material = Mid(vo.Windows[k].VolumeWindowMaterial) };
                        var v = new PtHip.pt_volume { w = vo.W, h = vo.H, d = vo.D, num_windows = wins.Length, zscale = vo.ZScale,
                                                      data = Pin(vo.Data), windows = Pin(wins) };
                        v.box_min[0] = (float)vo.Box.Min.X; v.box_min[1] = (float)vo.Box.Min.Y; v.box_min[2] = (float)vo.Box.Min.Z;
                        v.box_max[0] = (float)vo.Box.Max.X; v.box_max[1] = (float)vo.Box.Max.Y; v.box_max[2] = (float)vo.Box.Max.Z;
                        vols.Add(v);
                        return (PtHip.SHAPE_VOLUME, vols.Count - 1);
                    }
                    case Mesh me:   // instanced: the mesh's triangles in object space, one BLAS per distinct mesh
                    {
                        if (!meshIds.TryGetValue(s, out int id))
                        {
                            id = mf.Count; mf.Add(tm.Count); mc.Add(me.Triangles.Length);
                            foreach (var t in me.Triangles) AddTri(t);
                            meshIds[s] = id;
                        }
                        return (PtHip.SHAPE_MESH, id);
                    }
                    default: throw new NotSupportedException($"{s.GetType().Name} inside a TransformedShape is not on the GPU path");
                }
            }
            void AddTri(Triangle t)
            {
                Add3(v1, t.V1); Add3(v2, t.V2); Add3(v3, t.V3); Add3(n1, t.N1); Add3(n2, t.N2); Add3(n3, t.N3);
                Add3(t1, t.T1); Add3(t2, t.T2); Add3(t3, t.T3);
                tm.Add(Mid(t.Material));
            }
            foreach (var s in Scene.Shapes)
            {
                switch (s)
                {
                    case Sphere sp: kind.Add(PtHip.SHAPE_SPHERE); index.Add(sr.Count); Add3(sc, sp.Center); sr.Add(sp.Radius); sm.Add(Mid(sp.Material)); break;
                    case Cube cu: kind.Add(PtHip.SHAPE_CUBE); index.Add(cm.Count); Add3(cmin, cu.Min); Add3(cmax, cu.Max); cm.Add(Mid(cu.Material)); break;
                    // Plane.Point/Normal/Material are private in the reference (Plane.cs:9-11): the integration
                    // marks them `internal`, the same visibility Sphere and Cube already use (INTEGRATION.md).
                    case Plane pl: kind.Add(PtHip.SHAPE_PLANE); index.Add(pm.Count); Add3(pp, pl.Point); Add3(pn, pl.Normal); pm.Add(Mid(pl.Material)); break;
                    case Triangle tr: kind.Add(PtHip.SHAPE_TRIANGLE); index.Add(tm.Count); AddTri(tr); break;
                    case SDFShape or Volume: { var (k, i) = Inner(s); kind.Add(k); index.Add(i); break; }
                    case TransformedShape ts:
                    {
                        var (k, i) = Inner(ts.Shape);
                        var x = new PtHip.pt_transformed_shape { shape_kind = k, shape_index = i };
                        Mat16(x.matrix, ts.Matrix); Mat16(x.inverse, ts.Inverse);
                        kind.Add(PtHip.SHAPE_TRANSFORMED); index.Add(xfs.Count); xfs.Add(x);
                        break;
                    }
                    case Mesh me: kind.Add(PtHip.SHAPE_MESH); index.Add(mf.Count); mf.Add(tm.Count); mc.Add(me.Triangles.Length); foreach (var t in me.Triangles) AddTri(t); break;
                    default: throw new NotSupportedException($"{s.GetType().Name} is not on the GPU path");
                }
            }
            var d = new PtHip.pt_scene_desc
            {
                num_materials = mats.Count, materials = Pin(mats.ToArray()),
                num_shapes = kind.Count, shape_kind = Pin(kind.ToArray()), shape_index = Pin(index.ToArray()),
                num_spheres = sr.Count, sphere_center = Pin(sc.ToArray()), sphere_radius = Pin(sr.ToArray()), sphere_material = Pin(sm.ToArray()),
                num_cubes = cm.Count, cube_min = Pin(cmin.ToArray()), cube_max = Pin(cmax.ToArray()), cube_material = Pin(cm.ToArray()),
                num_planes = pm.Count, plane_point = Pin(pp.ToArray()), plane_normal = Pin(pn.ToArray()), plane_material = Pin(pm.ToArray()),
                num_triangles = tm.Count, tri_v1 = Pin(v1.ToArray()), tri_v2 = Pin(v2.ToArray()), tri_v3 = Pin(v3.ToArray()),
                tri_n1 = Pin(n1.ToArray()), tri_n2 = Pin(n2.ToArray()), tri_n3 = Pin(n3.ToArray()), tri_material = Pin(tm.ToArray()),
                num_meshes = mf.Count, mesh_first = Pin(mf.ToArray()), mesh_count = Pin(mc.ToArray()),
                tri_t1 = Pin(t1.ToArray()), tri_t2 = Pin(t2.ToArray()), tri_t3 = Pin(t3.ToArray()),
                env_texture = Tid(Scene.Texture), env_texture_angle = Scene.TextureAngle,
            };
            d.env_color[0] = Scene.Color.r; d.env_color[1] = Scene.Color.g; d.env_color[2] = Scene.Color.b;
            d.num_textures = texs.Count; d.textures = Pin(texs.ToArray());
            d.num_sdf_nodes = sdfNodes.Count; d.sdf_nodes = Pin(sdfNodes.ToArray()); d.sdf_children = Pin(sdfKids.ToArray());
            d.num_sdf_shapes = sdfShapes.Count; d.sdf_shapes = Pin(sdfShapes.ToArray());
            d.num_volumes = vols.Count; d.volumes = Pin(vols.ToArray());
            d.num_transformed = xfs.Count; d.transformed = Pin(xfs.ToArray());
            try { PtHip.Check(PtHip.pt_upload_scene(ctx, ref d), "pt_upload_scene"); }
            finally { foreach (var g in pins) g.Free(); pins.Clear(); }   // arrays are copied during the call
            uploaded = true;
        }

        unsafe PtHip.pt_camera Cam()
        {
            var c = new PtHip.pt_camera { m = Camera.m, focal_distance = Camera.focalDistance, aperture_radius = Camera.apertureRadius };
            c.p[0] = (float)Camera.p.X; c.p[1] = (float)Camera.p.Y; c.p[2] = (float)Camera.p.Z;
            c.u[0] = (float)Camera.u.X; c.u[1] = (float)Camera.u.Y; c.u[2] = (float)Camera.u.Z;
            c.v[0] = (float)Camera.v.X; c.v[1] = (float)Camera.v.Y; c.v[2] = (float)Camera.v.Z;
            c.w[0] = (float)Camera.w.X; c.w[1] = (float)Camera.w.Y; c.w[2] = (float)Camera.w.Z;
            return c;
        }

        /// <summary>One Renderer.RenderParallel pass on the GPU (Renderer.cs:199-338).</summary>
        public void RenderParallel() => Pass(0);

        /// <summary>One Renderer.Render pass (Renderer.cs:80-198, the NumCPU == 1 twin): the same main
        /// samples, then per pixel its adaptive and firefly samples (PT_PASS_SERIAL).</summary>
        public void Render() => Pass(PtHip.PT_PASS_SERIAL);

        /// <summary>k consecutive RenderParallel passes in one call (pt_pass_params.passes): the Buffer
        /// k RenderParallel() calls leave, bit for bit; plain passes run as one GPU batch, so a rank's
        /// tile share fills the device like a whole frame.  (IterativeRender keeps one pass per PNG.)</summary>
        public void RenderPasses(int k) => Pass(0, k);

        void Pass(int flags, int passes = 1)
        {
            if (!uploaded) Upload();
            var cam = Cam();
            var smp = new PtHip.pt_sampler { first_hit_samples = firstHit, max_bounces = maxBounces,
                direct_lighting = directLighting ? 1 : 0, soft_shadows = softShadows ? 1 : 0,
                light_mode = (int)Sampler.LightMode, specular_mode = (int)Sampler.SpecularMode };
            var pass = new PtHip.pt_pass_params { spp = SamplesPerPixel, stratified = StratifiedSampling ? 1 : 0,
                seed = Seed, pass_index = (uint)(this.pass + 1), adaptive_samples = AdaptiveSamples,
                firefly_samples = FireflySamples, flags = flags, passes = passes };
            this.pass += passes;
            GCHandle tiles = default;
            if (Tiles != null)
            {
                tiles = GCHandle.Alloc(Tiles, GCHandleType.Pinned);
                pass.num_tiles = Tiles.Length; pass.tiles = tiles.AddrOfPinnedObject();
            }
            try { PtHip.Check(PtHip.pt_render_pass(ctx, ref cam, ref smp, ref pass), "pt_render_pass"); }
            finally { if (tiles.IsAllocated) tiles.Free(); }
        }

        /// <summary>Resume: load a saved Buffer (e.g. Renderer.PBuffer of an earlier IterativeRender) into
        /// the GPU's Welford state; later passes keep accumulating into it (Renderer.cs:702-765).  `passesDone`
        /// continues the pass numbering the random streams are keyed by.</summary>
        public void LoadBuffer(Buffer b, int passesDone)
        {
            int P = W * H;
            var m = new double[3 * P]; var v = new double[3 * P]; var n = new int[P];
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++)
                {
                    int i = y * W + x; var px = b.Pixels[(x, y)];
                    n[i] = px.Samples;
                    m[3 * i] = px.M.r; m[3 * i + 1] = px.M.g; m[3 * i + 2] = px.M.b;
                    v[3 * i] = px.V.r; v[3 * i + 1] = px.V.g; v[3 * i + 2] = px.V.b;
                }
            PtHip.Check(PtHip.pt_write_buffer(ctx, m, v, n), "pt_write_buffer");
            pass = passesDone;
        }

        /// <summary>The Buffer pixels of 32x32 tiles, packed row-major inside each tile (pt_read_tiles):
        /// m, v [tiles][32][32][3], n [tiles][32][32].  With WriteTiles, a host that moves Buffers over
        /// its own transport assembles a sharded frame (pt_comm_gather's protocol).</summary>
        public (double[] m, double[] v, int[] n) ReadTiles(int[] tiles)
        {
            var m = new double[tiles.Length * 3072]; var v = new double[tiles.Length * 3072]; var n = new int[tiles.Length * 1024];
            PtHip.Check(PtHip.pt_read_tiles(ctx, tiles, tiles.Length, m, v, n), "pt_read_tiles");
            return (m, v, n);
        }

        public void WriteTiles(int[] tiles, double[] m, double[] v, int[] n) =>
            PtHip.Check(PtHip.pt_write_tiles(ctx, tiles, tiles.Length, m, v, n), "pt_write_tiles");

        /// <summary>Copy the HBM Welford state into Renderer.PBuffer's Pixel objects (Buffer.cs:18-58).</summary>
        public void ReadBuffer()
        {
            int P = W * H;
            var m = new double[3 * P]; var v = new double[3 * P]; var n = new int[P];
            PtHip.Check(PtHip.pt_read_buffer(ctx, m, v, n), "pt_read_buffer");
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++)
                {
                    int i = y * W + x;
                    Renderer.PBuffer.Pixels[(x, y)] = new Pixel(n[i], new Colour(m[3 * i], m[3 * i + 1], m[3 * i + 2]),
                                                                 new Colour(v[3 * i], v[3 * i + 1], v[3 * i + 2]));
                }
        }

        /// <summary>Renderer.IterativeRender (Renderer.cs:702-765): N passes, a PNG after each.</summary>
        public SKBitmap IterativeRender(string pathTemplate, int iter)
        {
            SKBitmap colour = null;
            for (int i = 1; i <= iter; i++)
            {
                Console.WriteLine("Iteration " + i + " of " + iter);
                if (NumCPU == 1) Render(); else RenderParallel();   // Renderer.cs:712-719
                ReadBuffer();
                colour = Renderer.PBuffer.Image(Channel.ColorChannel);
                using var stream = System.IO.File.OpenWrite(string.Format(pathTemplate, i));
                colour.Encode(SKEncodedImageFormat.Png, 100).SaveTo(stream);
            }
            return colour;
        }

        public void Dispose() { if (ctx != IntPtr.Zero) { PtHip.pt_destroy(ctx); ctx = IntPtr.Zero; } }
    }

    /// <summary>One .NET process driving G GPUs (the reference's Renderer is one process on all cores,
    /// Renderer.cs:257-333): one HipRenderer per device drawing its interleaved tiles, one RCCL
    /// communicator over the G contexts (pt_comm_init_all), passes issued from G host threads at once
    /// (a firefly pass all-reduces its snapshot across the group), the Buffer gathered onto device 0
    /// (pt_comm_gather_all) and copied into Renderer.PBuffer.</summary>
    class HipRendererGroup : IDisposable
    {
        readonly HipRenderer[] parts;
        readonly IntPtr[] ctxs;

        HipRendererGroup(HipRenderer[] p)
        {
            parts = p;
            ctxs = Array.ConvertAll(p, r => r.ctx);
            // the ranks' tile lists must be disjoint: checked once, before any RCCL call
            var all = new System.Collections.Generic.List<int>();
            foreach (var r in p) if (r.Tiles != null) all.AddRange(r.Tiles);
            PtHip.Check(PtHip.pt_tile_lists_check(all.ToArray(), all.Count, ((p[0].Width + 31) / 32) * ((p[0].Height + 31) / 32)),
                        "pt_tile_lists_check");
            PtHip.Check(PtHip.pt_comm_init_all(ctxs, ctxs.Length), "pt_comm_init_all");
        }

        public static HipRendererGroup NewRenderer(Scene scene, Camera camera, DefaultSampler sampler, int firstHitSamples,
                                                   int maxBounces, int w, int h, int[] devices)
        {
            var p = new HipRenderer[devices.Length];
            for (int i = 0; i < devices.Length; i++)
            {
                p[i] = HipRenderer.NewRenderer(scene, camera, sampler, firstHitSamples, maxBounces, w, h, devices[i]);
                p[i].Tiles = HipRenderer.TilesForRank(w, h, i, devices.Length);
            }
            return new HipRendererGroup(p);
        }

        public int SamplesPerPixel { set { foreach (var r in parts) r.SamplesPerPixel = value; } }
        public int AdaptiveSamples { set { foreach (var r in parts) r.AdaptiveSamples = value; } }
        public int FireflySamples { set { foreach (var r in parts) r.FireflySamples = value; } }
        public bool StratifiedSampling { set { foreach (var r in parts) r.StratifiedSampling = value; } }
        public ulong Seed { set { foreach (var r in parts) r.Seed = value; } }
        public int NumCPU { get => parts[0].NumCPU; set { foreach (var r in parts) r.NumCPU = value; } }

        /// <summary>One RenderParallel pass on every GPU, one host thread per context.</summary>
        public void RenderParallel() => Parallel.For(0, parts.Length, new ParallelOptions { MaxDegreeOfParallelism = parts.Length },
                                                     i => parts[i].RenderParallel());

        /// <summary>One Render pass (the NumCPU == 1 twin, Renderer.cs:80-198) on every GPU: its extra
        /// phases decide per pixel, so the tile split renders exactly the one-GPU frame.</summary>
        public void Render() => Parallel.For(0, parts.Length, new ParallelOptions { MaxDegreeOfParallelism = parts.Length },
                                             i => parts[i].Render());

        /// <summary>Sum the ranks' disjoint tiles onto device 0 and copy them into Renderer.PBuffer.</summary>
        public void ReadBuffer()
        {
            // device 0 then holds every rank's tiles; its next pass clears the others' pixels again
            // (ptsharp_hip.h "Multi-GPU"), so the gather can follow every pass
            PtHip.Check(PtHip.pt_comm_gather_all(ctxs, ctxs.Length, 0), "pt_comm_gather_all");
            parts[0].ReadBuffer();
        }

        public SKBitmap IterativeRender(string pathTemplate, int iter)
        {
            SKBitmap colour = null;
            for (int i = 1; i <= iter; i++)
            {
                Console.WriteLine("Iteration " + i + " of " + iter);
                if (NumCPU == 1) Render(); else RenderParallel();   // Renderer.cs:712-719
                ReadBuffer();
                colour = Renderer.PBuffer.Image(Channel.ColorChannel);
                using var stream = System.IO.File.OpenWrite(string.Format(pathTemplate, i));
                colour.Encode(SKEncodedImageFormat.Png, 100).SaveTo(stream);
            }
            return colour;
        }

        public void Dispose() { foreach (var r in parts) r.Dispose(); }
    }

    /// <summary>OBJ.Load (OBJ.cs:11-165) parsed natively, same quirks; the Triangle[] is then
    /// built as Mesh.NewMesh does.  Replaces `OBJ.Load(path, material)` in Example.*.</summary>
    static class HipObj
    {
        static Vector V(float[] a, int i) => new Vector(a[3 * i], a[3 * i + 1], a[3 * i + 2]);

        internal static Mesh Load(string path, Material parent)
        {
            var rc = PtHip.pt_obj_load(path, out var md);
            if (rc != PtHip.PT_OK)
                throw new InvalidOperationException($"pt_obj_load failed ({rc}): {Marshal.PtrToStringAnsi(PtHip.pt_obj_last_error())}");
            try
            {
                int n = md.num_triangles;
                float[] Copy(IntPtr p) { var a = new float[3 * n]; if (n > 0) Marshal.Copy(p, a, 0, 3 * n); return a; }
                float[] v1 = Copy(md.v1), v2 = Copy(md.v2), v3 = Copy(md.v3), n1 = Copy(md.n1), n2 = Copy(md.n2),
                        n3 = Copy(md.n3), t1 = Copy(md.t1), t2 = Copy(md.t2), t3 = Copy(md.t3);
                var tris = new Triangle[n];
                for (int i = 0; i < n; i++)
                {
                    var t = new Triangle { V1 = V(v1, i), V2 = V(v2, i), V3 = V(v3, i), N1 = V(n1, i), N2 = V(n2, i),
                                           N3 = V(n3, i), T1 = V(t1, i), T2 = V(t2, i), T3 = V(t3, i), Material = parent };
                    tris[i] = t;   // FixNormals already applied by the loader
                }
                return Mesh.NewMesh(tris);
            }
            finally { PtHip.pt_mesh_free(ref md); }
        }
    }
}
