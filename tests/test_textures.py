"""§8f row 3 — textures on the oracle: ColorTexture sampling (Texture.cs:188-251),
IShape.UVector (Sphere.cs:62-69, Cube.cs:49-53, Plane.cs:52-55, Triangle.cs:127-136),
Material.MaterialAt (Material.cs:124-138) and sampleEnvironment (Sampler.cs:177-189).

Each known answer is restated here in plain Python from the reference lines (fp64
scalars, np.float32 where the reference builds a Vector) and compared bit-exactly
with the oracle.  Parity against C# itself stays unpinned (no runtime).
"""
import math

import numpy as np
import pytest

import oracle_lib as O
from ptsharp_amd import Camera, ColorTexture, Colour, Cube, DefaultSampler, Material, Plane, Scene, Sphere, Triangle
from ptsharp_amd import Util, Vector, scenes

f32 = lambda x: float(np.float32(x))
EPS = 1e-9


def fract(x):  # Util.Modf's fractional part (Util.cs:108-113)
    return x - math.trunc(x)


def ref_bilinear(t: ColorTexture, u, v):  # Texture.cs:188-216
    if u == 1:
        u -= EPS
    if v == 1:
        v -= EPS
    w, h = t.Width - 1.0, t.Height - 1.0
    X, x = math.trunc(u * w), u * w - math.trunc(u * w)
    Y, y = math.trunc(v * h), v * h - math.trunc(v * h)
    x0, y0 = int(X), int(Y)
    D = t.Data
    c00, c01, c10, c11 = D[y0 * t.Width + x0], D[(y0 + 1) * t.Width + x0], D[y0 * t.Width + x0 + 1], \
        D[(y0 + 1) * t.Width + x0 + 1]
    out = []
    for k in range(3):
        a = 0.0
        a = a + c00[k] * ((1 - x) * (1 - y))
        a = a + c10[k] * (x * (1 - y))
        a = a + c01[k] * ((1 - x) * y)
        a = a + c11[k] * (x * y)
        out.append(a)
    return tuple(out)


def ref_sample(t, u, v):  # Texture.cs:224-229
    return ref_bilinear(t, fract(fract(u) + 1), 1 - fract(fract(v) + 1))


def norm32(x, y, z):
    x, y, z = np.float32(x), np.float32(y), np.float32(z)
    l = np.sqrt(np.float32(np.float32(x * x) + np.float32(y * y)) + np.float32(z * z), dtype=np.float32)
    return tuple(float(np.float32(c / l)) for c in (x, y, z))


def tex_scene(*textures, env=None, angle=0.0):
    """A scene whose materials reference the given textures (slots 1..n in that order)."""
    s = Scene()
    for i, t in enumerate(textures):
        s.Add(Sphere.NewSphere(Vector(10 * i, -100, 0), 1, Material.DiffuseMaterial(Colour.White).with_(Texture=t)))
    s.Texture, s.TextureAngle = env, angle
    return s


@pytest.fixture(scope="module")
def tex():
    rng = np.random.default_rng(5)
    return ColorTexture.NewTexture(rng.integers(0, 256, (5, 7, 3)).astype(np.uint8))


def test_new_texture_gamma():
    t = ColorTexture.NewTexture(np.array([[[0, 128, 255], [51, 1, 2]]], np.uint8).repeat(2, axis=0))
    g = float(np.float32(2.2))  # Pow(2.2F)
    assert t.Width == 2 and t.Height == 2
    assert t.Data[0].tolist() == [0.0, (128 / 255) ** g, 1.0]
    assert t.Data[1][0] == (51 / 255) ** g


@pytest.mark.parametrize("u,v", [(0.0, 0.0), (0.3, 0.7), (0.999, 0.001), (0.5, 0.5), (1.0, 1.0), (-0.25, 0.5),
                                 (2.75, -1.5), (0.3, 0.0), (1e-12, 1 - 1e-12)])
def test_sample_bilinear_kat(tex, u, v):
    os = O.OracleScene(tex_scene(tex))
    assert os.texture_sample(1, 0, u, v) == ref_sample(tex, u, v)


def test_sample_wraps_and_eps_rule(tex):
    os = O.OracleScene(tex_scene(tex))
    assert os.texture_sample(1, 0, -0.25, 0.5) == os.texture_sample(1, 0, 0.75, 0.5)
    assert os.texture_sample(1, 0, 3.25, 0.5) == os.texture_sample(1, 0, 0.25, 0.5)
    # v = 0 → BilinearSample(u, 1): the `v == 1 → v -= EPS` rule keeps y0 + 1 inside the image
    assert os.texture_sample(1, 0, 0.4, 0.0) == ref_bilinear(tex, fract(fract(0.4) + 1), 1 - EPS)
    # at a texel centre the sample is that texel (weights 1, 0, 0, 0)
    w, h = tex.Width - 1, tex.Height - 1
    got = os.texture_sample(1, 0, 2 / w, 1 - 3 / h)
    assert np.allclose(got, tex.Data[3 * tex.Width + 2], rtol=0, atol=1e-15)


def test_normal_sample_kat(tex):
    os = O.OracleScene(tex_scene(tex))
    for u, v in [(0.1, 0.2), (0.77, 0.31)]:
        c = ref_sample(tex, u, v)
        assert os.texture_sample(1, 1, u, v) == norm32(f32(c[0] * 2 - 1), f32(c[1] * 2 - 1), f32(c[2] * 2 - 1))


def test_bump_sample_kat(tex):
    os = O.OracleScene(tex_scene(tex))
    W, H, D = tex.Width, tex.Height, tex.Data

    def ref(u, v):  # Texture.cs:239-251 (row Height clamped: the reference indexes past the end)
        u, v = fract(fract(u) + 1), 1 - fract(fract(v) + 1)
        x, y = min(int(u * W), W - 1), min(int(v * H), H - 1)
        cl = lambda a, lo, hi: max(lo, min(hi, a))
        x1, x2, y1, y2 = cl(x - 1, 0, W - 1), cl(x + 1, 0, W - 1), cl(y - 1, 0, H - 1), cl(y + 1, 0, H - 1)
        return (f32(D[y * W + x1][0] - D[y * W + x2][0]), f32(D[y1 * W + x][0] - D[y2 * W + x][0]), 0.0)

    for u, v in [(0.1, 0.2), (0.5, 0.5), (0.99, 0.01), (0.0, 0.999), (0.3, 0.0)]:
        assert os.texture_sample(1, 2, u, v) == ref(u, v)


def test_sphere_uv_keeps_reference_slip():
    """Sphere.UVector measures the latitude against |(p.X, 0, p.Y)| (Sphere.cs:65), not |(p.X, 0, p.Z)|."""
    s = Scene()
    s.Add(Sphere.NewSphere(Vector(1, 2, 3), 2, Material.DiffuseMaterial(Colour.White)))
    os = O.OracleScene(s)
    p = (f32(2.2), f32(3.1), f32(1.4))
    q = [np.float32(p[k]) - np.float32((1, 2, 3)[k]) for k in range(3)]
    u = math.atan2(float(q[2]), float(q[0]))
    ln = float(np.sqrt(np.float32(np.float32(q[0] * q[0]) + np.float32(0)) + np.float32(q[1] * q[1]), dtype=np.float32))
    v = math.atan2(float(q[1]), ln)
    u = 1 - (u + math.pi) / (2 * math.pi)
    v = (v + math.pi / 2) / math.pi
    assert os.shape_uv(0, 0, p) == (f32(u), f32(v), 0.0)


def test_cube_plane_triangle_uv():
    s = Scene()
    s.Add(Cube.NewCube(Vector(-1, -2, -4), Vector(3, 2, 4), Material.DiffuseMaterial(Colour.White)))
    s.Add(Plane.NewPlane(Vector(0, 0, 0), Vector(0, 1, 0), Material.DiffuseMaterial(Colour.White)))
    s.Add(Triangle.NewTriangle(Vector(0, 0, 0), Vector(1, 0, 0), Vector(0, 1, 0), Vector(0.1, 0.2, 0),
                               Vector(0.9, 0.3, 0), Vector(0.4, 0.8, 0), Material.DiffuseMaterial(Colour.White)))
    os = O.OracleScene(s)
    assert os.shape_uv(1, 0, (0.0, 1.0, 2.0)) == (f32(1 / 4), f32(6 / 8), 0.0)   # ((p-Min)/(Max-Min)).X, .Z
    assert os.shape_uv(2, 0, (5.0, 0.0, 7.0)) == (0.0, 0.0, 0.0)                 # Plane.UVector
    # at a vertex the barycentric weights are exact, so UVector returns that vertex's T
    assert os.shape_uv(3, 0, (1.0, 0.0, 0.0)) == (f32(0.9), f32(0.3), 0.0)
    u = os.shape_uv(3, 0, (0.25, 0.25, 0.0))
    assert np.allclose(u[:2], [0.5 * 0.1 + 0.25 * 0.9 + 0.25 * 0.4, 0.5 * 0.2 + 0.25 * 0.3 + 0.25 * 0.8], atol=1e-6)


def test_environment_kat(tex):
    angle = Util.Radians(30)
    os = O.OracleScene(tex_scene(tex, env=tex, angle=angle))
    for d in [(1.0, 0.0, 0.0), (0.0, 0.0, 1.0), norm32(0.3, 0.5, -0.8), norm32(-0.2, -0.9, 0.1)]:
        d = tuple(f32(x) for x in d)
        u = math.atan2(d[2], d[0]) + angle
        ln = float(np.sqrt(np.float32(np.float32(np.float32(d[0]) ** 2) + np.float32(0)) + np.float32(np.float32(d[2]) ** 2),
                           dtype=np.float32))
        v = math.atan2(d[1], ln)
        u, v = (u + math.pi) / (2 * math.pi), (v + math.pi / 2) / math.pi
        assert os.environment(d) == ref_sample(tex, u, v)
    assert O.OracleScene(tex_scene(tex)).environment((1.0, 0, 0)) == (0.0, 0.0, 0.0)  # no Texture: scene.Color


def test_material_at_colour_and_gloss(tex):
    """Hit.Info's material: Texture replaces Color, GlossTexture sets Gloss = mean of the sample."""
    s = Scene()
    m = Material.GlossyMaterial(Colour(0.1, 0.2, 0.3), 1.5, 0.25).with_(Texture=tex, GlossTexture=tex)
    s.Add(Cube.NewCube(Vector(-1, -1, -1), Vector(1, 0, 1), m))
    os = O.OracleScene(s)
    col, gloss = os.hit_surface((0.25, 2.0, -0.5), (0.0, -1.0, 0.0))
    u, v = f32(1.25 / 2), f32(0.5 / 2)   # hit (0.25, 0, -0.5) → ((p-Min)/(Max-Min)).X, .Z
    c = ref_sample(tex, u, v)
    assert col == c and gloss == (c[0] + c[1] + c[2]) / 3
    plain = Scene()
    plain.Add(Cube.NewCube(Vector(-1, -1, -1), Vector(1, 0, 1), Material.GlossyMaterial(Colour(0.1, 0.2, 0.3), 1.5, 0.25)))
    assert O.OracleScene(plain).hit_surface((0.25, 2.0, -0.5), (0.0, -1.0, 0.0)) == ((0.1, 0.2, 0.3), 0.25)


def test_constant_environment_map_furnace():
    """Floor furnace under a constant environment map of value c: sky pixels are the
    bilinear sum of four equal texels (c up to fp64 rounding), floor pixels albedo · that."""
    c = 0.75
    env = ColorTexture(4, 3, np.full((12, 3), c))
    s, cam, smp = scenes.furnace(0.5)
    s.Color = Colour(0, 0, 0)
    s.Texture = env
    b, _ = O.render(O.OracleScene(s), cam, smp, 32, 24, spp=2, seed=4)
    assert np.all(np.isclose(b.M, 0.5 * c, atol=1e-15) | np.isclose(b.M, c, atol=1e-15))


def test_textured_scene_renders_finite():
    s, cam, smp = scenes.textured()
    b, rays = O.render(O.OracleScene(s), cam, smp, 32, 24, spp=1, seed=9)
    assert rays > 32 * 24 and np.isfinite(b.M).all() and (b.N == 1).all()


def test_tiny_texture_rejected_on_host():
    s = tex_scene(ColorTexture(1, 4, np.zeros((4, 3))))
    from ptsharp_amd import _abi
    with pytest.raises(_abi.PTError):
        s.Compile()
