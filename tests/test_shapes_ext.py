"""§8f row 4 on the oracle: SDF.cs (every SDF node), Volume.cs, TransformedShape.cs.

The known answers come from an independent plain-Python restatement of the reference
lines below (fp64 scalars, np.float32 wherever the reference builds a Vector) and
are compared bit-exactly with the oracle.  Parity against C# itself stays unpinned
(no runtime)."""
import math

import numpy as np
import pytest

import oracle_lib as O
from ptsharp_amd import (Box, CapsuleSDF, Colour, Cube, CubeSDF, CylinderSDF, DifferenceSDF, IntersectionSDF,
                         Material, Matrix, RepeatSDF, ScaleSDF, Scene, SDFShape, Sphere, SphereSDF, TorusSDF,
                         TransformedShape, TransformSDF, UnionSDF, Util, Vector, Volume, VolumeWindow, scenes)
from ptsharp_amd.scene import _SDF

f32 = np.float32


def vlen(x, y, z):  # Vector3.Length in fp32
    x, y, z = f32(x), f32(y), f32(z)
    return float(np.sqrt(f32(f32(f32(x * x) + f32(y * y)) + f32(z * z)), dtype=f32))


def length_n(p, n):  # Vector.LengthN (Vector.cs:359-367)
    if n == 2:
        return vlen(*p)
    a = [abs(float(c)) for c in p]
    return (a[0] ** n + a[1] ** n + a[2] ** n) ** (1 / n)


def mulpos(m, p):  # Matrix.MulPosition (Matrix.cs:134-141)
    return tuple(float(f32(((m[r][0] * p[0] + m[r][1] * p[1]) + m[r][2] * p[2]) + m[r][3])) for r in range(3))


def ref_eval(n: _SDF, p):
    """SDF.Evaluate (SDF.cs) restated in Python; p is a tuple of fp32-valued floats."""
    P = n.params
    if isinstance(n, SphereSDF):
        return length_n(p, P[1]) - P[0]
    if isinstance(n, CubeSDF):   # SDF.cs:157-189
        x, y, z = (abs(c) for c in p)
        x, y, z = x - P[0] / 2, y - P[1] / 2, z - P[2] / 2
        a = x
        if y > a:
            a = y
        if z > a:
            a = z
        if a > 0:
            a = 0
        x, y, z = max(x, 0), max(y, 0), max(z, 0)
        return a + math.sqrt(x * x + y * y + z * z)
    if isinstance(n, CylinderSDF):
        x = math.sqrt(p[0] * p[0] + p[2] * p[2]) - P[0]
        y = abs(p[1]) - P[1] / 2
        a = y if y > x else x
        a = 0 if a > 0 else a
        return a + math.sqrt(max(x, 0) * max(x, 0) + max(y, 0) * max(y, 0))
    if isinstance(n, CapsuleSDF):
        A, B = [float(f32(c)) for c in P[0:3]], [float(f32(c)) for c in P[3:6]]
        pa = [float(f32(p[k] - A[k])) for k in range(3)]
        ba = [float(f32(B[k] - A[k])) for k in range(3)]
        dot = lambda u, v: float(f32(f32(f32(u[0] * v[0]) + f32(u[1] * v[1])) + f32(u[2] * v[2])))
        h = max(0.0, min(1.0, dot(pa, ba) / dot(ba, ba)))
        q = [float(f32(pa[k] - float(f32(ba[k] * h)))) for k in range(3)]
        return length_n(q, P[7]) - P[6]
    if isinstance(n, TorusSDF):
        q = (float(f32(length_n((p[0], p[1], 0.0), P[2]) - P[0])), p[2], 0.0)
        return length_n(q, P[3]) - P[1]
    if isinstance(n, TransformSDF):
        return ref_eval(n.children[0], mulpos(n.inverse.m, p))
    if isinstance(n, ScaleSDF):
        return ref_eval(n.children[0], tuple(float(f32(c / P[0])) for c in p)) * P[0]
    if isinstance(n, RepeatSDF):
        st = [float(f32(c)) for c in P[:3]]
        m = [float(f32(p[k] - st[k] * math.floor(p[k] / st[k]))) for k in range(3)]
        return ref_eval(n.children[0], tuple(float(f32(m[k] - float(f32(st[k] / 2)))) for k in range(3)))
    vals = [ref_eval(c, p) for c in n.children]
    r = 0.0
    for i, d in enumerate(vals):
        if isinstance(n, UnionSDF) and (i == 0 or d < r):
            r = d
        elif isinstance(n, IntersectionSDF) and (i == 0 or d > r):
            r = d
        elif isinstance(n, DifferenceSDF):
            r = d if i == 0 else (-d if -d > r else r)
    return r


def zoo():
    sph = SphereSDF.NewSphereSDF(0.65)
    cube = CubeSDF.NewCubeSDF(Vector(1, 0.8, 1.2))
    cyl = CylinderSDF.NewCylinderSDF(0.25, 1.1)
    cap = CapsuleSDF.NewCapsuleSDF(Vector(-0.6, -0.3, 0.2), Vector(0.4, 0.5, 0.6), 0.2)
    tor = TorusSDF.NewTorusSDF(0.5, 0.15)
    rot = TransformSDF.NewTransformSDF(cyl, Matrix.RotateM(Vector(1, 0, 0), Util.Radians(90)))
    sc = ScaleSDF.NewScaleSDF(SphereSDF((0.5, 3.0)), 0.8)
    rep = RepeatSDF.NewRepeaterSDF(SphereSDF.NewSphereSDF(0.12), Vector(0.3, 0.3, 0.3))
    inter = IntersectionSDF.NewIntersectionSDF([sph, cube])
    diff = DifferenceSDF.NewDifferenceSDF([inter, cyl, rot])
    uni = UnionSDF.NewUnionSDF([diff, cap, tor, sc])
    return [sph, cube, cyl, cap, tor, rot, sc, rep, inter, diff, uni]


def test_sdf_nodes_match_python_restatement():
    rng = np.random.default_rng(3)
    for n in zoo():
        s = Scene()
        s.Add(SDFShape.NewSDFShape(n, Material.DiffuseMaterial(Colour.White)))
        os = O.OracleScene(s)
        root = s.Compile().sdf_shapes[0].root
        for p in rng.uniform(-1.2, 1.2, size=(40, 3)).astype(np.float32):
            pt = tuple(float(c) for c in p)
            assert os.sdf_evaluate(root, pt) == ref_eval(n, pt), type(n).__name__


def test_sdf_kat_values():
    s = Scene()
    for n in (SphereSDF.NewSphereSDF(0.25), CubeSDF.NewCubeSDF(Vector(1, 1, 1))):
        s.Add(SDFShape.NewSDFShape(n, Material.DiffuseMaterial(Colour.White)))
    os = O.OracleScene(s)
    r0, r1 = (s.Compile().sdf_shapes[i].root for i in range(2))
    assert os.sdf_evaluate(r0, (0.0, 0.0, 0.0)) == -0.25
    assert os.sdf_evaluate(r1, (2.0, 0.0, 0.0)) == 1.5          # outside: distance to the face
    assert os.sdf_evaluate(r1, (0.0, 0.25, 0.0)) == -0.25       # inside: max(x, y, z) of the offsets
    assert os.sdf_evaluate(r1, (1.5, 1.5, 0.0)) == math.sqrt(2.0)     # corner region: |offsets|


def test_sdf_boxes():
    """SDFShape.BoundingBox: torus box is flat at z = MinRadius (SDF.cs:314-318), a repeat box is empty."""
    s = Scene()
    for n in (TorusSDF.NewTorusSDF(0.5, 0.15), RepeatSDF.NewRepeaterSDF(SphereSDF.NewSphereSDF(0.1), Vector(1, 1, 1)),
              TransformSDF.NewTransformSDF(CubeSDF.NewCubeSDF(Vector(1, 1, 1)), Matrix.TranslateM(Vector(1, 2, 3)))):
        s.Add(SDFShape.NewSDFShape(n, Material.DiffuseMaterial(Colour.White)))
    os = O.OracleScene(s)
    F = lambda x: float(f32(x))
    assert os.shape_box(5, 0) == ((F(-0.65), F(-0.65), F(0.15)), (F(0.65), F(0.65), F(0.15)))
    assert os.shape_box(5, 1) == ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0))
    assert os.shape_box(5, 2) == ((0.5, 1.5, 2.5), (1.5, 2.5, 3.5))


def test_volume_sample_matches_python_restatement():
    """Volume.Sample (Volume.cs:73-105) with its y-from-z slip: the sample does not depend on y."""
    s, _, _ = scenes.volume(12, 10, 6, seed=5)
    vol = s.Shapes[0]
    os = O.OracleScene(s)
    rng = np.random.default_rng(4)
    for x, y, z in rng.uniform(-1.2, 1.2, size=(60, 3)):
        assert os.volume_sample(0, x, y, z) == vol._sample(x, y, z)
        assert os.volume_sample(0, x, y, z) == os.volume_sample(0, x, -y, z)


def test_volume_material_windows():
    """Volume.MaterialAt: the window holding the sample, else the nearest (Volume.cs:148-166).  Scene.Add
    asks at the origin, where Sample reads slice z0 = D (Volume.cs:78), outside the grid: 0."""
    data = np.full((2, 2, 2), 0.5)
    lit, dif = Material.LightMaterial(Colour.White, 3), Material.DiffuseMaterial(Colour.White)
    box = Box(Vector(-1, -1, -1), Vector(1, 1, 1))
    near = Volume(2, 2, 2, 1.0, data, [VolumeWindow(0.1, 0.2, dif), VolumeWindow(0.45, 0.7, lit)], box)
    holds = Volume(2, 2, 2, 1.0, data, [VolumeWindow(0.45, 0.7, dif), VolumeWindow(-0.1, 0.05, lit)], box)
    assert near._sample(0.0, 0.0, 0.0) == 0.0
    s = Scene()
    s.Add(near)
    s.Add(holds)
    assert s.Lights == [holds]
    os = O.OracleScene(s)
    assert os.volume_sample(1, 0.0, 0.0, -1.0) == 0.5            # voxel (1, 0, 1), weights 1, 0, 0
    assert os.volume_sample(1, 0.0, 0.0, -0.5) == 0.25           # z halfway to slice 2, outside the grid (0)


def test_transformed_sphere_hit_and_distance():
    """TransformedShape.Intersect: T = |position - origin| of the inner hit mapped back (TransformedShape.cs:43-73)."""
    s = Scene()
    s.Add(TransformedShape.NewTransformedShape(Sphere.NewSphere(Vector(), 1, Material.DiffuseMaterial(Colour.White)),
                                               Matrix.TranslateM(Vector(0, 0, -5))))
    os = O.OracleScene(s)
    t, kind, idx = os.intersect((0.0, 0.0, 0.0), (0.0, 0.0, -1.0))
    assert kind == 7 and idx == 0 and t == 4.0
    t2, kind2, _ = os.intersect((3.0, 0.0, 0.0), (0.0, 0.0, -1.0))
    assert kind2 == -1


def test_transformed_box_is_mulbox():
    s = Scene()
    m = Matrix.TranslateM(Vector(1, 0, 0)).Mul(Matrix.RotateM(Vector(0, 0, 1), Util.Radians(90)))
    s.Add(TransformedShape.NewTransformedShape(Cube.NewCube(Vector(0, 0, 0), Vector(2, 1, 1),
                                                            Material.DiffuseMaterial(Colour.White)), m))
    os = O.OracleScene(s)
    b = m.MulBox(Box(Vector(0, 0, 0), Vector(2, 1, 1)))
    assert os.shape_box(7, 0) == (b.Min.f32(), b.Max.f32())


def test_transformed_furnace_exact():
    """The floor furnace with the floor cube inside a translating TransformedShape:
    still exactly albedo on the floor and 1 in the sky."""
    s, cam, smp = scenes.furnace(0.5)
    cube = s.Shapes[0]
    s2 = Scene()
    s2.Color = s.Color
    c2 = Cube.NewCube(cube.Min.Sub(Vector(0, 0, 0)), cube.Max, cube.Material)
    s2.Add(TransformedShape.NewTransformedShape(c2, Matrix.TranslateM(Vector(0, 0, 0))))
    b, rays = O.render(O.OracleScene(s2), cam, smp, 32, 24, spp=2, seed=6)
    assert set(np.unique(b.M)) <= {0.5, 1.0} and rays > 0


def test_instanced_mesh_matches_world_space_mesh():
    """A mesh under a pure translation hits where the same mesh moved in world space does
    (up to the fp32 rounding of the two paths), and reports T as a distance."""
    from ptsharp_amd import Mesh
    m = scenes.blob_mesh(800, seed=9)
    s1, s2 = Scene(), Scene()
    s1.Add(TransformedShape.NewTransformedShape(m, Matrix.TranslateM(Vector(0.5, 0.25, -3))))
    moved = m.copy()
    moved.Transform(Matrix.TranslateM(Vector(0.5, 0.25, -3)))
    s2.Add(moved)
    o1, o2 = O.OracleScene(s1), O.OracleScene(s2)
    rng = np.random.default_rng(8)
    hits = 0
    for d in rng.normal(size=(64, 3)) * [0.15, 0.15, 1] - [0, 0, 1]:
        d = d / np.linalg.norm(d)
        t1, k1, _ = o1.intersect((0.5, 0.25, 0.0), d)
        t2, k2, _ = o2.intersect((0.5, 0.25, 0.0), d)
        assert (k1 == 7) == (k2 == 3)
        if k1 == 7:
            hits += 1
            assert abs(t1 - t2) < 1e-5 * t2
    assert hits > 20


@pytest.mark.parametrize("name", ["sdf", "sdf_zoo", "volume", "transformed", "instances"])
def test_row4_scenes_render(name):
    s, cam, smp = scenes.SCENES[name]()
    smp.MaxBounces = min(smp.MaxBounces, 2)
    b, rays = O.render(O.OracleScene(s), cam, smp, 24, 18, spp=1, seed=2)
    assert rays >= 24 * 18 and np.isfinite(b.M).all() and (b.N == 1).all()
