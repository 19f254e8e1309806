"""Host-side mirror: fp32 Vector semantics, Colour/Material factories, Camera.LookAt,
mesh operations, scene flattening, tile sharding and Buffer.Image."""
import math
import os

import numpy as np
import pytest

from ptsharp_amd import (Box, Buffer, Camera, Channel, Colour, Cube, Material, Matrix, Mesh, Plane, Scene, Sphere,
                         Triangle, Vector, tiles_for_rank, write_png)
from ptsharp_amd import _abi, scenes
from ptsharp_amd.scene import DEFAULT_MATERIAL


def test_vector_rounds_to_fp32():
    v = Vector(0.1, 0.2, 0.3)
    assert v.X == float(np.float32(0.1))
    s = v.Add(Vector(0.2, 0.2, 0.2))
    assert s.X == float(np.float32(np.float32(0.1) + np.float32(0.2)))
    m = v.MulScalar(1 / 3)
    assert m.X == float(np.float32(float(np.float32(0.1)) * (1 / 3)))
    d = v.Dot(v)
    assert d == float((np.float32(0.1) * np.float32(0.1) + np.float32(0.2) * np.float32(0.2))
                      + np.float32(0.3) * np.float32(0.3))


def test_normalize_and_cross():
    n = Vector(3, 4, 0).Normalize()
    assert (n.X, n.Y, n.Z) == (0.6000000238418579, 0.800000011920929, 0.0)
    c = Vector(1, 0, 0).Cross(Vector(0, 1, 0))
    assert (c.X, c.Y, c.Z) == (0, 0, 1)


def test_hexcolor():
    c = Colour.HexColor(0xFF8000)
    assert c.r == 1.0
    assert c.b == 0.0
    assert math.isclose(c.g, (128 / 255) ** 2.2, rel_tol=1e-6)


def test_material_factories():
    m = Material.GlossyMaterial(Colour.White, 1.5, 0.2)
    assert (m.Index, m.Gloss, m.Reflectivity, m.Transparent) == (1.5, 0.2, -1, False)
    assert Material.MetallicMaterial(Colour.White, 0, 1).Reflectivity == 1
    assert Material.ClearMaterial(1.5, 0).Transparent
    assert Material.LightMaterial(Colour.White, 3).Emittance == 3


def test_camera_lookat_basis():
    c = Camera.LookAt(Vector(0, 0, 5), Vector(0, 0, 0), Vector(0, 1, 0), 90)
    assert (c.w.X, c.w.Y, c.w.Z) == (0, 0, -1)
    assert (c.u.X, c.u.Y, c.u.Z) == (1, 0, 0) or (c.u.X, c.u.Y, c.u.Z) == (-1, 0, 0)
    assert math.isclose(c.m, 1 / math.tan(math.pi / 4))
    c.SetFocus(Vector(0, 0, 1), 0.1)
    assert c.focalDistance == 4.0 and c.apertureRadius == 0.1


def test_scene_lights_registration():
    s = Scene()
    s.Add(Sphere.NewSphere(Vector(), 1, Material.LightMaterial(Colour.White, 1)))
    s.Add(Cube.NewCube(Vector(), Vector(1, 1, 1), Material.DiffuseMaterial(Colour.White)))
    m = scenes.blob_mesh(200)
    m.SetMaterial(Material.LightMaterial(Colour.White, 5))
    s.Add(m)  # Mesh.MaterialAt is `default` → never a light
    assert len(s.Lights) == 1


def test_flatten_scene_arrays():
    s, c, smp = scenes.bunny_frame(2000, seed=2)
    f = s.Compile()
    assert list(f.shape_kind) == [_abi.SHAPE_MESH, _abi.SHAPE_CUBE, _abi.SHAPE_SPHERE, _abi.SHAPE_SPHERE]
    assert f.num_triangles == f.mesh_count[0]
    assert f.desc.num_triangles == f.num_triangles
    assert f.desc.num_materials == len(f.material_list) == 3
    assert f.tri_v1.dtype == np.float32 and f.tri_v1.flags.c_contiguous


def test_unsupported_shape_rejected():
    s = Scene()
    s.Add(object.__new__(type("Cylinder", (), {"MaterialAt": lambda self, p=None: DEFAULT_MATERIAL})))
    with pytest.raises(_abi.PTError):
        s.Compile()


def test_fit_inside_and_transform():
    m = scenes.blob_mesh(500, seed=1)
    m.FitInside(Box(Vector(-1, 0, -1), Vector(1, 2, 1)), Vector(0.5, 0, 0.5))
    bb = m.BoundingBox()
    assert bb.Min.Y == pytest.approx(0, abs=1e-6)
    assert max(bb.Max.X - bb.Min.X, bb.Max.Y - bb.Min.Y, bb.Max.Z - bb.Min.Z) == pytest.approx(2, rel=1e-6)
    n = np.linalg.norm(m.n1, axis=1)
    assert np.allclose(n, 1, atol=1e-6)


def test_smooth_normals_matches_loop():
    m = scenes.blob_mesh(300, seed=4)
    ref = m.copy()
    m.SmoothNormals()
    # straightforward Mesh.SmoothNormals: dictionary of fp32 sums in triangle order
    acc = {}
    for i in range(len(ref)):
        for v, nn in ((ref.v1, ref.n1), (ref.v2, ref.n2), (ref.v3, ref.n3)):
            key = tuple(float(x) for x in v[i])
            s = acc.get(key, np.zeros(3, np.float32))
            acc[key] = (s + nn[i]).astype(np.float32)
    for i in range(0, len(ref), 7):
        key = tuple(float(x) for x in ref.v1[i])
        s = acc[key]
        l = np.sqrt(np.float32((s[0] * s[0] + s[1] * s[1]) + s[2] * s[2]))
        assert np.array_equal(m.n1[i], (s / l).astype(np.float32))


def test_matrix_rotate_orthonormal():
    r = Matrix.RotateM(Vector(0, 1, 0), 0.3)
    assert np.allclose(r.m[:3, :3] @ r.m[:3, :3].T, np.eye(3))


def test_blob_mesh_size_and_closed():
    m = scenes.blob_mesh(69_451)
    assert abs(len(m) - 69_451) / 69_451 < 0.02
    m1 = scenes.blob_mesh(1_000_000)
    assert abs(len(m1) - 1_000_000) / 1_000_000 < 0.01


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_tiles_partition(world):
    w, h = 1920, 1080
    parts = [tiles_for_rank(w, h, r, world) for r in range(world)]
    allt = np.sort(np.concatenate(parts))
    assert np.array_equal(allt, np.arange(60 * 34))
    sizes = [len(p) for p in parts]
    assert max(sizes) - min(sizes) <= 1


def test_buffer_image_semantics(tmp_path):
    b = Buffer(3, 1)
    b.M[0, 0] = (1.0, 0.5, 0.0)
    b.M[0, 1] = (2.0, np.nan, -1.0)
    b.M[0, 2] = (0.25, 0.25, 0.25)
    img = b.Image(Channel.ColorChannel)
    assert list(img[0, 0]) == [255, int(0.5 ** (1 / 2.2) * 255), 0]
    assert list(img[0, 1]) == [255, 0, 0]
    p = tmp_path / "x.png"
    write_png(str(p), img)
    assert p.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"


def test_buffer_variance_channel():
    b = Buffer(1, 1)
    b.N[0, 0] = 3
    b.V[0, 0] = (0.2, 0.4, 0.6)
    v = b.Variance(0, 0)
    assert (v.r, v.g, v.b) == (0.1, 0.2, 0.3)
    assert b.Samples(0, 0) == 3
