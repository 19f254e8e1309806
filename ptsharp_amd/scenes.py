"""Scenes for the BASELINE.json configs, built through the mirrored API exactly
as PTSharpCore/Example.cs builds them.  No model assets ship with the reference
(SURVEY.md fact 6), so meshes come from a seeded generator.

  gopher3          Example.gopher (Example.cs:1542-1564) with the OBJ mesh replaced
                   by two spheres                       → C1, C2
  bunny_frame(n)   Example.bunny (Example.cs:1084-1102) with a seeded displaced
                   sphere of ~n triangles in place of models/bunny.obj  → C3 (70k), C4 (1M)
  materialspheres  Example.materialspheres (Example.cs:1204-1227)
  simplesphere     Example.simplesphere (Example.cs:1670-1697)
  example1         Example.example1 (Example.cs:341-359), no adaptive/firefly passes
  example3         Example.example3 (Example.cs:387-418), the scene Program.cs:97 renders: 840 thin
                   cubes and a Cube light; the renderer runs AdaptiveSamples 32, FireflySamples 64
  textured         §8f row 3: colour / gloss / normal / bump maps, a textured light and an
                   environment map with TextureAngle, on seeded synthetic textures (no
                   texture assets ship with the reference either)
  sdf              Example.sdf (Example.cs:1398-1424), §8f row 4
  sdf_zoo          every other SDF node (capsule, torus, scale, union, repeat) and an SDF light
  volume           Example.volume (Example.cs:1426-1471) on seeded synthetic slices
  transformed      TransformedShape over spheres (Example.go's stones, Translate quirk kept),
                   a cube, a plane, an SDF shape and a volume, and a transformed light
  instances        one Mesh instanced six times through TransformedShape
"""
from __future__ import annotations

import math

import numpy as np

from .geometry import Box, Colour, Matrix, Util, Vector
from .scene import (Camera, CapsuleSDF, ColorTexture, Cube, CubeSDF, CylinderSDF, DefaultSampler, DifferenceSDF,
                    IntersectionSDF, LightMode, Material, Mesh, Plane, RepeatSDF, ScaleSDF, Scene, SDFShape,
                    SpecularMode, Sphere, SphereSDF, TorusSDF, TransformedShape, TransformSDF, Triangle, UnionSDF,
                    Volume, VolumeWindow)

F = lambda x: float(np.float32(x))  # C# float literal (e.g. 0.75F)


def gopher3():
    scene = Scene()
    wall = Material.GlossyMaterial(Colour.HexColor(0xFCFAE1), 1.5, Util.Radians(10))
    light = Material.LightMaterial(Colour.White, 80)
    scene.Add(Cube.NewCube(Vector(-10, -1, -10), Vector(-2, 10, 10), wall))
    scene.Add(Cube.NewCube(Vector(-10, -1, -10), Vector(10, 0, 10), wall))
    scene.Add(Sphere.NewSphere(Vector(4, 10, 1), 1, light))
    scene.Add(Sphere.NewSphere(Vector(0, 1, 0), 1, Material.GlossyMaterial(Colour.Black, 1.2, Util.Radians(30))))
    scene.Add(Sphere.NewSphere(Vector(0, 0.5, 1.5), 0.5, Material.SpecularMaterial(Colour.HexColor(0x334D5C), 2)))
    camera = Camera.LookAt(Vector(4, 1, 0), Vector(0, 0.9, 0), Vector(0, 1, 0), 40)
    sampler = DefaultSampler.NewSampler(16, 16)
    return scene, camera, sampler


def materialspheres():
    scene = Scene()
    r = F(0.4)
    scene.Add(Sphere.NewSphere(Vector(-2, r, 0), r, Material.DiffuseMaterial(Colour.HexColor(0x334D5C))))
    scene.Add(Sphere.NewSphere(Vector(-1, r, 0), r, Material.SpecularMaterial(Colour.HexColor(0x334D5C), 2)))
    scene.Add(Sphere.NewSphere(Vector(0, r, 0), r, Material.GlossyMaterial(Colour.HexColor(0x334D5C), 2,
                                                                          Util.Radians(50))))
    scene.Add(Sphere.NewSphere(Vector(1, r, 0), r, Material.TransparentMaterial(Colour.HexColor(0x334D5C), 2,
                                                                               Util.Radians(20), 1)))
    scene.Add(Sphere.NewSphere(Vector(2, r, 0), r, Material.ClearMaterial(2, 0)))
    scene.Add(Sphere.NewSphere(Vector(0, F(1.5), -4), F(1.5), Material.MetallicMaterial(Colour.HexColor(0xFFFFFF), 0, 1)))
    scene.Add(Cube.NewCube(Vector(-1000, -1, -1000), Vector(1000, 0, 1000),
                           Material.GlossyMaterial(Colour.HexColor(0xFFFFFF), F(1.4), Util.Radians(20))))
    scene.Add(Sphere.NewSphere(Vector(0, 5, 0), 1, Material.LightMaterial(Colour.White, 25)))
    camera = Camera.LookAt(Vector(0, 3, 6), Vector(0, 1, 0), Vector(0, 1, 0), 30)
    sampler = DefaultSampler.NewSampler(16, 16)
    return scene, camera, sampler


def simplesphere():
    scene = Scene()
    material = Material.DiffuseMaterial(Colour.White)
    scene.Add(Plane.NewPlane(Vector(0, 0, 0), Vector(0, 0, 1), material))
    scene.Add(Sphere.NewSphere(Vector(0, 0, 1), F(1.0), material))
    scene.Add(Sphere.NewSphere(Vector(0, 0, F(5.0)), F(1.0), Material.LightMaterial(Colour.White, 8)))
    camera = Camera.LookAt(Vector(3, 3, 3), Vector(0, 0, F(0.5)), Vector(0, 0, 1), 50)
    sampler = DefaultSampler.NewSampler(16, 4)
    return scene, camera, sampler


def example1():
    scene = Scene()
    scene.Add(Sphere.NewSphere(Vector(1.5, 1.25, 0), 1.25, Material.SpecularMaterial(Colour.HexColor(0x004358), 1.3)))
    scene.Add(Sphere.NewSphere(Vector(-1, 1, 2), 1, Material.SpecularMaterial(Colour.HexColor(0xFFE11A), 1.3)))
    scene.Add(Sphere.NewSphere(Vector(-2.5, 0.75, 0), 0.75, Material.SpecularMaterial(Colour.HexColor(0xFD7400), 1.3)))
    scene.Add(Sphere.NewSphere(Vector(-0.75, 0.5, -1), 0.5, Material.ClearMaterial(1.5, 0)))
    scene.Add(Cube.NewCube(Vector(-10, -1, -10), Vector(10, 0, 10), Material.GlossyMaterial(Colour.White, 1.1,
                                                                                          Util.Radians(10))))
    scene.Add(Sphere.NewSphere(Vector(-1.5, 4, 0), 0.5, Material.LightMaterial(Colour.White, 30)))
    camera = Camera.LookAt(Vector(0, 2, -5), Vector(0, 0.25, 3), Vector(0, 1, 0), 45)
    camera.SetFocus(Vector(-0.75, 1, -1), 0.1)
    sampler = DefaultSampler.NewSampler(8, 10)
    sampler.SpecularMode = SpecularMode.SpecularModeFirst
    return scene, camera, sampler


def example3():
    """Example.example3 (Example.cs:387-418): a floor cube, the 840 cubes of the 41x41 grid whose
    x + z is odd ((x + z) % 2 == 0 skips, C#'s % keeps the sign so odd negatives are kept too), a
    Cube light, LookAt((20,10,0), (8,0,0), up, 45), NewSampler(4,4).  The reference renders it with
    AdaptiveSamples = 32 and FireflySamples = 64 (pass those to the Renderer)."""
    scene = Scene()
    material = Material.DiffuseMaterial(Colour.HexColor(0xFCFAE1))
    scene.Add(Cube.NewCube(Vector(-1000, -1, -1000), Vector(1000, 0, 1000), material))
    for x in range(-20, 21):
        for z in range(-20, 21):
            if math.fmod(x + z, 2) == 0:
                continue
            sz = 0.1
            scene.Add(Cube.NewCube(Vector(float(x) - sz, 0, float(z) - sz), Vector(float(x) + sz, 2, float(z) + sz),
                                   material))
    scene.Add(Cube.NewCube(Vector(-5, 10, -5), Vector(5, 11, 5), Material.LightMaterial(Colour.White, 5)))
    camera = Camera.LookAt(Vector(20, 10, 0), Vector(8, 0, 0), Vector(0, 1, 0), 45)
    sampler = DefaultSampler.NewSampler(4, 4)
    return scene, camera, sampler


def _blob_geometry(n_target: int, seed: int = 1234, amplitude: float = 0.05):
    """blob_mesh's shared vertex list (float32 [V,3]), per-vertex texture coordinates (float32 [V,3])
    and triangle vertex indices ([T,3], 0-based)."""
    # tris = 2*ns + 2*ns*(nr-2) = 2*ns*(nr-1);  choose nr ≈ ns/2
    ns = max(8, int(round(math.sqrt(n_target))))
    nr = max(3, int(round(n_target / (2 * ns))) + 1)
    rng = np.random.default_rng(seed)
    k = 24
    dirs = rng.normal(size=(k, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    freq = rng.uniform(2.0, 9.0, size=k)
    phase = rng.uniform(0, 2 * math.pi, size=k)
    amp = rng.uniform(0.3, 1.0, size=k) / freq

    theta = np.pi * np.arange(1, nr) / nr
    phi = 2 * np.pi * np.arange(ns) / ns
    th, ph = np.meshgrid(theta, phi, indexing="ij")
    unit = np.stack([np.sin(th) * np.cos(ph), np.cos(th), np.sin(th) * np.sin(ph)], axis=-1).reshape(-1, 3)
    unit = np.concatenate([unit, [[0, 1, 0], [0, -1, 0]]])
    noise = (amp[None, :] * np.sin(unit @ dirs.T * freq[None, :] + phase[None, :])).sum(axis=1)
    noise /= np.abs(noise).max() + 1e-12
    # quantise to 2^-20 so last-ulp differences between numpy's SIMD sin/cos paths on
    # different CPUs cannot change the mesh (fixtures are generated on one host, checked on another)
    verts = (np.round(unit * (1.0 + amplitude * noise)[:, None] * 2.0**20) / 2.0**20).astype(np.float32)
    north, south = len(verts) - 2, len(verts) - 1
    ring = lambda i, j: i * ns + (j % ns)
    tris = []
    j = np.arange(ns)
    tris.append(np.stack([np.full(ns, north), ring(0, j + 1), ring(0, j)], axis=1))
    for i in range(nr - 2):
        a, b, c, d = ring(i, j), ring(i, j + 1), ring(i + 1, j), ring(i + 1, j + 1)
        tris.append(np.stack([a, b, d], axis=1))
        tris.append(np.stack([a, d, c], axis=1))
    tris.append(np.stack([np.full(ns, south), ring(nr - 2, j), ring(nr - 2, j + 1)], axis=1))
    t = np.concatenate(tris)
    # texture coordinates: the sphere parametrisation (u = φ/2π, v = θ/π), poles at the ring's u
    uv = np.stack([ph.reshape(-1) / (2 * np.pi), th.reshape(-1) / np.pi, np.zeros(th.size)], axis=-1)
    uv = np.concatenate([uv, [[0.5, 0, 0], [0.5, 1, 0]]]).astype(np.float32)
    return verts, uv, t


def blob_mesh(n_target: int, seed: int = 1234, amplitude: float = 0.05) -> Mesh:
    """Seeded displaced UV sphere with ~n_target triangles (fan caps + quad bands), per-vertex
    radius 1 + amplitude·noise, zero normals (FixNormals → face normals), consistent winding."""
    verts, uv, t = _blob_geometry(n_target, seed, amplitude)
    z = np.zeros((len(t), 3), np.float32)
    m = Mesh(verts[t[:, 0]], verts[t[:, 1]], verts[t[:, 2]], z, z, z, t1=uv[t[:, 0]], t2=uv[t[:, 1]], t3=uv[t[:, 2]])
    from .scene import fix_normals_arrays
    m.n1, m.n2, m.n3 = fix_normals_arrays(m.v1, m.v2, m.v3, m.n1, m.n2, m.n3)
    return m


def blob_obj_text(n_target: int, seed: int = 1234, amplitude: float = 0.05) -> str:
    """blob_mesh's mesh as Wavefront OBJ text, the form Example.bunny loads (OBJ.Load("models/bunny.obj"),
    Example.cs:1088): one `v` per vertex and one `vt` per vertex (the same index), faces
    `f a/a b/b c/c` (1-based, no normal index: OBJ.cs:104 then reads the dummy normal and
    Triangle.FixNormals puts the face normal in, as blob_mesh does).  Numbers are written with 9
    significant digits, which float.Parse / strtof read back to the same float32 bits."""
    verts, uv, t = _blob_geometry(n_target, seed, amplitude)
    out = [f"# seeded displaced sphere: {len(t)} triangles, blob_mesh({n_target}, seed={seed})\n"]

    def rows(fmt, a, k=8192):   # one %-format call per block of rows
        for i in range(0, len(a), k):
            blk = a[i:i + k]
            out.append((fmt * len(blk)) % tuple(blk.reshape(-1).tolist()))
    rows("v %.9g %.9g %.9g\n", verts.astype(np.float64))
    rows("vt %.9g %.9g\n", uv[:, :2].astype(np.float64))
    rows("f %d/%d %d/%d %d/%d\n", np.repeat(t + 1, 2, axis=1))
    return "".join(out)


def write_blob_obj(path: str, n_target: int, seed: int = 1234) -> str:
    with open(path, "w") as f:
        f.write(blob_obj_text(n_target, seed))
    return path


def bunny_frame(n_tris: int = 69_451, seed: int = 1234, mesh: Mesh = None):
    """Example.bunny's scene around a synthetic mesh (SURVEY.md §8d mesh70k / mesh1M)."""
    scene = Scene()
    material = Material.GlossyMaterial(Colour.HexColor(0xF2EBC7), F(1.5), Util.Radians(0))
    if mesh is None:
        mesh = blob_mesh(n_tris, seed)
    mesh.SetMaterial(material)
    mesh.SmoothNormals()
    mesh.FitInside(Box(Vector(-1, 0, -1), Vector(1, 2, 1)), Vector(F(0.5), 0, F(0.5)))
    scene.Add(mesh)
    floor = Material.GlossyMaterial(Colour.HexColor(0x33332D), F(1.2), Util.Radians(20))
    scene.Add(Cube.NewCube(Vector(-10000, -10000, -10000), Vector(10000, 0, 10000), floor))
    scene.Add(Sphere.NewSphere(Vector(0, 5, 0), 1, Material.LightMaterial(Colour.White, 10)))
    scene.Add(Sphere.NewSphere(Vector(4, 5, 4), 1, Material.LightMaterial(Colour.White, 10)))
    camera = Camera.LookAt(Vector(-1, 2, 3), Vector(0, F(0.75), 0), Vector(0, 1, 0), 50)
    sampler = DefaultSampler.NewSampler(4, 4)
    sampler.SetSpecularMode(SpecularMode.SpecularModeFirst)
    return scene, camera, sampler


def furnace(albedo: float = 0.5):
    """Analytic 'floor furnace' (SURVEY.md §4): a huge diffuse cube seen from above, scene.Color = 1,
    no lights → every floor pixel is exactly `albedo`, every sky pixel exactly 1."""
    scene = Scene()
    scene.Color = Colour(1, 1, 1)
    scene.Add(Cube.NewCube(Vector(-1000, -1, -1000), Vector(1000, 0, 1000),
                           Material.DiffuseMaterial(Colour(albedo, albedo, albedo))))
    camera = Camera.LookAt(Vector(0, 2, 3), Vector(0, 1.5, 0), Vector(0, 1, 0), 60)
    sampler = DefaultSampler.NewSampler(4, 4)
    return scene, camera, sampler


def emitter(fh: int = 16):
    """A lone light sphere in a black environment: a camera hit returns Color·Emittance·FH/⌊√FH⌋²."""
    scene = Scene()
    scene.Add(Sphere.NewSphere(Vector(0, 0, 0), 1, Material.LightMaterial(Colour(0.25, 0.5, 1.0), 2)))
    camera = Camera.LookAt(Vector(0, 0, 4), Vector(0, 0, 0), Vector(0, 1, 0), 40)
    sampler = DefaultSampler.NewSampler(fh, 4)
    return scene, camera, sampler


def seeded_texture(w: int, h: int, seed: int, kind: str = "color") -> ColorTexture:
    """ColorTexture.NewTexture over seeded 8-bit pixels: 'color' uniform noise, 'normal' a
    tangent-space normal map around (128, 128, 255), 'bump' smooth grey noise."""
    rng = np.random.default_rng(seed)
    if kind == "normal":
        px = np.stack([rng.integers(88, 168, (h, w)), rng.integers(88, 168, (h, w)), rng.integers(200, 256, (h, w))], -1)
    elif kind == "bump":
        g = rng.integers(0, 256, (h, w))
        g = (g + np.roll(g, 1, 0) + np.roll(g, 1, 1) + np.roll(g, (1, 1), (0, 1))) // 4
        px = np.repeat(g[:, :, None], 3, axis=2)
    else:
        px = rng.integers(0, 256, (h, w, 3))
    return ColorTexture.NewTexture(px.astype(np.uint8))


def textured(mesh_tris: int = 2000):
    """§8f row 3 on one scene: Material.Texture on a cube, spheres, a light sphere and a mesh;
    GlossTexture on a glossy sphere; NormalTexture + BumpTexture on the mesh (Triangle.NormalAt);
    Scene.Texture (environment map) with a TextureAngle; a directly added textured Triangle."""
    scene = Scene()
    scene.Texture = seeded_texture(64, 32, 11)
    scene.TextureAngle = Util.Radians(30)
    floor = Material.GlossyMaterial(Colour.White, F(1.2), Util.Radians(20)).with_(Texture=seeded_texture(32, 32, 12))
    scene.Add(Cube.NewCube(Vector(-12, -1, -12), Vector(12, 0, 12), floor))
    scene.Add(Sphere.NewSphere(Vector(-1.6, 0.7, 0.4), 0.7,
                               Material.DiffuseMaterial(Colour.White).with_(Texture=seeded_texture(24, 12, 13))))
    glossy = Material.GlossyMaterial(Colour.HexColor(0x334D5C), 1.5, Util.Radians(10))
    scene.Add(Sphere.NewSphere(Vector(1.6, 0.6, 0.6), 0.6, glossy.with_(GlossTexture=seeded_texture(16, 8, 14))))
    light = Material.LightMaterial(Colour.White, 12).with_(Texture=seeded_texture(8, 8, 15))
    scene.Add(Sphere.NewSphere(Vector(0, 4.5, 1), 0.8, light))
    mesh = blob_mesh(mesh_tris, seed=16, amplitude=0.1)
    mat = Material.GlossyMaterial(Colour.White, 1.4, Util.Radians(15)).with_(
        Texture=seeded_texture(32, 16, 17), NormalTexture=seeded_texture(32, 16, 18, "normal"),
        BumpTexture=seeded_texture(32, 16, 19, "bump"), BumpMultiplier=0.5)
    mesh.SetMaterial(mat)
    mesh.SmoothNormals()
    mesh.FitInside(Box(Vector(-0.8, 0, -0.8), Vector(0.8, 1.6, 0.8)), Vector(F(0.5), 0, F(0.5)))
    scene.Add(mesh)
    scene.Add(Triangle.NewTriangle(Vector(-3, 0.01, -2), Vector(3, 0.01, -2), Vector(0, 2.5, -2.5),
                                   Vector(0, 0, 0), Vector(1, 0, 0), Vector(0.5, 1, 0),
                                   Material.DiffuseMaterial(Colour.White).with_(Texture=seeded_texture(16, 16, 20))))
    camera = Camera.LookAt(Vector(0, 2.2, 5), Vector(0, 0.8, 0), Vector(0, 1, 0), 45)
    sampler = DefaultSampler.NewSampler(4, 4)
    sampler.SetSpecularMode(SpecularMode.SpecularModeFirst)
    return scene, camera, sampler


def sdf():
    """Example.sdf (Example.cs:1398-1424)."""
    scene = Scene()
    light = Material.LightMaterial(Colour.White, 180)
    d = F(4.0)
    for v in (Vector(-1, -1, F(0.5)), Vector(0, -1, F(0.25)), Vector(-1, 1, 0)):
        scene.Add(Sphere.NewSphere(v.Normalize().MulScalar(d), F(0.25), light))
    material = Material.GlossyMaterial(Colour.HexColor(0x468966), F(1.2), Util.Radians(20))
    sphere = SphereSDF.NewSphereSDF(F(0.65))
    cube = CubeSDF.NewCubeSDF(Vector(1, 1, 1))
    rounded = IntersectionSDF.NewIntersectionSDF([sphere, cube])
    a = CylinderSDF.NewCylinderSDF(F(0.25), F(1.1))
    b = TransformSDF.NewTransformSDF(a, Matrix.RotateM(Vector(1, 0, 0), Util.Radians(90)))
    c = TransformSDF.NewTransformSDF(a, Matrix.RotateM(Vector(0, 0, 1), Util.Radians(90)))
    difference = DifferenceSDF.NewDifferenceSDF([rounded, a, b, c])
    shape = TransformSDF.NewTransformSDF(difference, Matrix.RotateM(Vector(0, 0, 1), Util.Radians(30)))
    scene.Add(SDFShape.NewSDFShape(shape, material))
    floor = Material.GlossyMaterial(Colour.HexColor(0xFFF0A5), F(1.2), Util.Radians(20))
    scene.Add(Plane.NewPlane(Vector(0, 0, F(-0.5)), Vector(0, 0, 1), floor))
    camera = Camera.LookAt(Vector(-3, 0, 1), Vector(0, 0, 0), Vector(0, 0, 1), 35)
    sampler = DefaultSampler.NewSampler(4, 4)
    sampler.LightMode = LightMode.LightModeAll
    sampler.SpecularMode = SpecularMode.SpecularModeAll
    return scene, camera, sampler


def sdf_zoo():
    """The SDF nodes Example.sdf does not use: CapsuleSDF, TorusSDF (with its flat bounding box,
    SDF.cs:314-318), ScaleSDF, UnionSDF, RepeatSDF (zero box, so only inside an intersection), a
    non-2 LengthN exponent, and an emissive SDF shape (a class shape: a real light)."""
    scene = Scene()
    scene.Color = Colour(0.05, 0.05, 0.08)
    glossy = Material.GlossyMaterial(Colour.HexColor(0xBEDB39), F(1.3), Util.Radians(15))
    capsule = CapsuleSDF.NewCapsuleSDF(Vector(-0.6, -0.3, 0.2), Vector(0.4, 0.5, 0.6), F(0.2))
    torus = TransformSDF.NewTransformSDF(TorusSDF.NewTorusSDF(F(0.5), F(0.15)), Matrix.TranslateM(Vector(0.3, 0.2, -0.25)))
    blob = ScaleSDF.NewScaleSDF(SphereSDF(( F(0.5), 3.0)), F(0.8))       # LengthN with exponent 3
    union = UnionSDF.NewUnionSDF([capsule, torus, TransformSDF.NewTransformSDF(blob, Matrix.TranslateM(Vector(0.6, -0.5, 0.3)))])
    scene.Add(SDFShape.NewSDFShape(union, glossy))
    grid = IntersectionSDF.NewIntersectionSDF([CubeSDF.NewCubeSDF(Vector(2.4, 2.4, 0.3)),
                                               RepeatSDF.NewRepeaterSDF(SphereSDF.NewSphereSDF(F(0.12)), Vector(0.3, 0.3, 0.3))])
    scene.Add(SDFShape.NewSDFShape(TransformSDF.NewTransformSDF(grid, Matrix.TranslateM(Vector(0, 0, -0.55))),
                                   Material.DiffuseMaterial(Colour.HexColor(0xFD7400))))
    lamp = SphereSDF.NewSphereSDF(F(0.3))
    scene.Add(SDFShape.NewSDFShape(TransformSDF.NewTransformSDF(lamp, Matrix.TranslateM(Vector(-0.5, 1.2, 1.6))),
                                   Material.LightMaterial(Colour.White, 30)))
    scene.Add(Plane.NewPlane(Vector(0, 0, -0.8), Vector(0, 0, 1), Material.DiffuseMaterial(Colour(0.6, 0.6, 0.6))))
    camera = Camera.LookAt(Vector(-3, -1, 1.6), Vector(0, 0, -0.1), Vector(0, 0, 1), 40)
    sampler = DefaultSampler.NewSampler(4, 3)
    return scene, camera, sampler


def volume_slices(w: int = 48, h: int = 48, d: int = 24, seed: int = 7):
    """Seeded 8-bit slices standing in for Example.volume's images/ folder: a smooth density
    blob (rings through every window of the scene) plus noise, as SKBitmap red channels."""
    rng = np.random.default_rng(seed)
    z, y, x = np.meshgrid(np.linspace(-1, 1, d), np.linspace(-1, 1, h), np.linspace(-1, 1, w), indexing="ij")
    r = np.sqrt(x * x + 1.3 * y * y + 0.8 * z * z)
    dens = 0.75 * np.exp(-1.5 * r * r) + 0.08 * rng.standard_normal((d, h, w))
    return [np.clip(np.round(sl * 255), 0, 255).astype(np.uint8) for sl in dens]


def volume(w: int = 48, h: int = 48, d: int = 24, seed: int = 7):
    """Example.volume (Example.cs:1426-1471) on volume_slices()."""
    scene = Scene()
    scene.Color = Colour.White
    colors = [Colour.HexColor(c) for c in (0x004358, 0x1F8A70, 0xBEDB39, 0xFFE11A, 0xFD7400)]
    start, size, step = F(0.2), F(0.01), F(0.1)
    windows = []
    for i, col in enumerate(colors):
        lo = start + step * float(i)
        windows.append(VolumeWindow(lo, lo + size, Material.GlossyMaterial(col, F(1.3), Util.Radians(0))))
    box = Box(Vector(-1, -1, F(-0.2)), Vector(1, 1, 1))
    scene.Add(Volume.NewVolume(box, volume_slices(w, h, d, seed), F(3.4) / F(0.9765625), windows))
    camera = Camera.LookAt(Vector(0, -3, -3), Vector(0, 0, 0), Vector(0, 0, -1), 35)
    sampler = DefaultSampler.NewSampler(4, 4)
    return scene, camera, sampler


def transformed():
    """TransformedShape (TransformedShape.cs) over every inner kind on the GPU path."""
    scene = Scene()
    scene.Color = Colour(0.3, 0.3, 0.35)
    black = Material.GlossyMaterial(Colour.HexColor(0x111111), 1.5, Util.Radians(45))
    white = Material.GlossyMaterial(Colour.HexColor(0xFFFFFF), 1.6, Util.Radians(20))
    # Example.go's stones: `new Matrix().Scale(..).Translate(..)` keeps only the translation (Matrix.cs:33-36)
    for i, (px, pz) in enumerate([(-1.2, 0.3), (0.0, -0.4), (1.1, 0.5), (-0.4, 1.3)]):
        m = Matrix.TranslateM(Vector(px, 0, pz))
        scene.Add(TransformedShape.NewTransformedShape(Sphere.NewSphere(Vector(), 0.45, black if i % 2 else white), m))
    squash = Matrix.ScaleM(Vector(0.9, 0.35, 0.6)).Mul(Matrix.RotateM(Vector(0, 1, 0), Util.Radians(25)))
    scene.Add(TransformedShape.NewTransformedShape(
        Sphere.NewSphere(Vector(), 1, Material.SpecularMaterial(Colour.HexColor(0x334D5C), 2)),
        Matrix.TranslateM(Vector(0.2, 0.35, -1.4)).Mul(squash)))
    cube_m = Matrix.TranslateM(Vector(1.6, 0.4, -0.6)).Mul(Matrix.RotateM(Vector(1, 1, 0), Util.Radians(35)))
    scene.Add(TransformedShape.NewTransformedShape(
        Cube.NewCube(Vector(-0.3, -0.3, -0.3), Vector(0.3, 0.3, 0.3), Material.DiffuseMaterial(Colour.HexColor(0xFFE11A))),
        cube_m))
    tor = SDFShape.NewSDFShape(TorusSDF(( F(0.45), F(0.12), 2, 2)), Material.GlossyMaterial(Colour.HexColor(0x1F8A70), 1.4, 0.2))
    scene.Add(TransformedShape.NewTransformedShape(
        tor, Matrix.TranslateM(Vector(-1.5, 0.6, -0.9)).Mul(Matrix.RotateM(Vector(1, 0, 0), Util.Radians(70)))))
    vol, _, _ = volume(16, 16, 8, seed=3)
    scene.Add(TransformedShape.NewTransformedShape(
        vol.Shapes[0], Matrix.TranslateM(Vector(0.2, 1.2, 0.9)).Mul(Matrix.ScaleM(Vector(0.4, 0.4, 0.4)))))
    floor = Plane.NewPlane(Vector(0, 0, 0), Vector(0, 1, 0), Material.GlossyMaterial(Colour.HexColor(0xEFECCA), 1.2,
                                                                                       Util.Radians(30)))
    scene.Add(TransformedShape.NewTransformedShape(floor, Matrix.TranslateM(Vector(0, -0.45, 0))
                                                   .Mul(Matrix.RotateM(Vector(0, 0, 1), Util.Radians(4)))))
    lamp = Sphere.NewSphere(Vector(), 0.5, Material.LightMaterial(Colour.White, 20))
    scene.Add(TransformedShape.NewTransformedShape(lamp, Matrix.TranslateM(Vector(-1, 3, 1))))   # phantom light
    scene.Add(Sphere.NewSphere(Vector(1.5, 3.5, 1.5), 0.5, Material.LightMaterial(Colour.White, 25)))
    camera = Camera.LookAt(Vector(0, 2.4, 4.2), Vector(0, 0.2, 0), Vector(0, 1, 0), 45)
    sampler = DefaultSampler.NewSampler(4, 4)
    sampler.SetSpecularMode(SpecularMode.SpecularModeFirst)
    return scene, camera, sampler


def instances(copies: int = 6, mesh_tris: int = 3000):
    """TransformedShape over one Mesh, several times (Example.cs:1016, 1274, 1339 instance meshes
    this way): one object-space BVH shared by every instance."""
    scene = Scene()
    scene.Color = Colour(0.4, 0.45, 0.5)
    mesh = blob_mesh(mesh_tris, seed=21, amplitude=0.15)
    mesh.SetMaterial(Material.GlossyMaterial(Colour.HexColor(0xBEDB39), 1.4, Util.Radians(10)))
    mesh.SmoothNormals()
    rng = np.random.default_rng(5)
    for i in range(copies):
        m = Matrix.TranslateM(Vector(rng.uniform(-2, 2), rng.uniform(0.3, 1.2), rng.uniform(-2, 1))).Mul(
            Matrix.RotateM(Vector(*rng.normal(size=3)), rng.uniform(0, 3))).Mul(
            Matrix.ScaleM(Vector(*rng.uniform(0.3, 0.6, size=3))))
        scene.Add(TransformedShape.NewTransformedShape(mesh, m))
    scene.Add(Cube.NewCube(Vector(-20, -1, -20), Vector(20, 0, 20), Material.DiffuseMaterial(Colour(0.7, 0.7, 0.7))))
    scene.Add(Sphere.NewSphere(Vector(2, 5, 3), 1, Material.LightMaterial(Colour.White, 15)))
    camera = Camera.LookAt(Vector(0, 3, 5), Vector(0, 0.6, -0.5), Vector(0, 1, 0), 50)
    sampler = DefaultSampler.NewSampler(4, 4)
    return scene, camera, sampler


def mixed(n_tris: int = 1_000_000, seed: int = 1234, mesh: Mesh = None):
    """BASELINE.json configs[4]'s kind of scene (C5): the C4 mesh frame plus an SDF shape, a
    voxel Volume (iso-windows) and an environment texture standing in for the HDRI (the
    reference's environment is an 8-bit ColorTexture lookup, Sampler.cs:177-189)."""
    scene, camera, sampler = bunny_frame(n_tris, seed=seed, mesh=mesh)
    scene.Texture = seeded_texture(512, 256, 21)
    scene.TextureAngle = Util.Radians(40)
    ring = TransformSDF.NewTransformSDF(TorusSDF.NewTorusSDF(F(0.45), F(0.12)),
                                        Matrix.TranslateM(Vector(-1.8, 0.5, 0.4)).Mul(
                                            Matrix.RotateM(Vector(1, 0, 0), Util.Radians(70))))
    scene.Add(SDFShape.NewSDFShape(ring, Material.GlossyMaterial(Colour.HexColor(0x1F8A70), F(1.4), Util.Radians(10))))
    vol, _, _ = volume(32, 32, 16, seed=5)
    scene.Add(TransformedShape.NewTransformedShape(
        vol.Shapes[0], Matrix.TranslateM(Vector(1.6, 0.55, -0.6)).Mul(Matrix.ScaleM(Vector(0.5, 0.5, 0.5)))))
    return scene, camera, sampler


SCENES = {
    "gopher3": gopher3,
    "materialspheres": materialspheres,
    "simplesphere": simplesphere,
    "example1": example1,
    "example3": example3,
    "bunny70k": lambda: bunny_frame(69_451),
    "mesh1m": lambda: bunny_frame(1_000_000),
    "furnace": furnace,
    "emitter": emitter,
    "textured": textured,
    "sdf": sdf,
    "sdf_zoo": sdf_zoo,
    "volume": volume,
    "transformed": transformed,
    "instances": instances,
    "mixed": mixed,
}
