"""Native OBJ ingest (pt_obj_load) and Mesh.SmoothNormals (pt_mesh_smooth_normals):
SURVEY.md §8f row 2.  Host-only entry points of libptsharp_hip.so, so these run on
the CPU.  The checker is tests/obj_ref.py, a line-by-line restatement of OBJ.cs."""
import numpy as np
import pytest

import obj_ref
from ptsharp_amd import _abi, scenes
from ptsharp_amd.scene import OBJ, Mesh

KEYS = ("v1", "v2", "v3", "n1", "n2", "n3", "t1", "t2", "t3")


def _load_both(path):
    m = OBJ.Load(str(path))
    ref = obj_ref.load(str(path))
    got = {"v1": m.v1, "v2": m.v2, "v3": m.v3, "n1": m.n1, "n2": m.n2, "n3": m.n3, "t1": m.t1, "t2": m.t2,
           "t3": m.t3}
    return got, ref


def _same(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_quirks_normal_off_by_one_and_double_slash(tmp_path):
    p = tmp_path / "q.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\n"
                 "vt 0.25 0.5\nvt 0.75 1\n"
                 "vn 0 0 -1\nvn 1 0 0\n"
                 "f 1/1/2 2/2/2 3/1/3\n"   # vn 2 -> file normal 1 (0,0,-1); vn 3 -> file normal 2
                 "f 1//2 2//2 3//1\n"      # '//' : the normal index is read as a texture index
                 "f 1/2/1 2/2/1 3/2/1\n")  # vn 1 -> the dummy (0,0,0) -> FixNormals
    got, ref = _load_both(p)
    for k in KEYS:
        assert _same(got[k], ref[k]), k
    face = np.array([0, 0, 1], np.float32)
    assert np.array_equal(got["n1"][0], [0, 0, -1]) and np.array_equal(got["n3"][0], [1, 0, 0])
    assert np.array_equal(got["n1"][1], face) and np.array_equal(got["t1"][1], [0.75, 1, 0])
    assert np.array_equal(got["n2"][2], face)


def test_fan_triangulation_case_tabs_crlf(tmp_path):
    p = tmp_path / "f.obj"
    p.write_bytes(b"# comment\r\nV 0 0 0\r\nv 1 0 0\r\nv 1 1 0\r\nv 0 1 0\r\nv\t5 5 5\r\nv 0.5 1.5 0\r\n"
                  b"f 1 2 3 4\r\nF 1 2 3 4 5\r\n\r\nusemtl foo\r\nmtllib x.mtl\r\n")
    got, ref = _load_both(p)
    for k in KEYS:
        assert _same(got[k], ref[k]), k
    assert len(got["v1"]) == 2 + 3          # quad -> 2, pentagon -> 3 (the tab line is no vertex)
    assert np.array_equal(got["v3"][1], [0, 1, 0]) and np.array_equal(got["v2"][4], [0, 1, 0])
    assert (got["t1"] == 0).all()            # no vt lines -> zero texture coords


@pytest.mark.parametrize("body,msg", [("v 0 0 0\nf 1 2 3\n", "out of range"), ("v 0 x 0\n", "bad v"),
                                      ("v 0 0 0\nf 1/a 1 1\n", "bad face")])
def test_errors(tmp_path, body, msg):
    p = tmp_path / "e.obj"
    p.write_text(body)
    with pytest.raises(_abi.PTError, match=msg):
        OBJ.Load(str(p))


def test_missing_file(tmp_path):
    with pytest.raises(_abi.PTError, match="does not exist"):
        OBJ.Load(str(tmp_path / "nope.obj"))


def _write_obj(m: Mesh, path, style):
    """Write a mesh with shared vertices; style 'v', 'v/vt/vn' or 'v//vn'."""
    allv = np.concatenate([m.v1, m.v2, m.v3])
    uniq, inv = np.unique(allv, axis=0, return_inverse=True)
    inv = inv.reshape(3, -1).T + 1
    with open(path, "w") as fh:
        for v in uniq:
            fh.write("v %r %r %r\n" % tuple(float(x) for x in v))
        if style != "v":
            fh.write("vt 0.5 0.25\n")
            for n in np.concatenate([m.n1[:50], m.n2[:50]]):
                fh.write("vn %r %r %r\n" % tuple(float(x) for x in n))
        for i, (a, b, c) in enumerate(inv):
            if style == "v":
                fh.write(f"f {a} {b} {c}\n")
            elif style == "v/vt/vn":
                k = 1 + i % 100
                fh.write(f"f {a}/1/{k} {b}/1/{k + 1} {c}/1/{k}\n")
            else:
                fh.write(f"f {a}//1 {b}//1 {c}//1\n")


@pytest.mark.parametrize("style", ["v", "v/vt/vn", "v//vn"])
def test_blob_round_trip(tmp_path, style):
    m = scenes.blob_mesh(4000, seed=3)
    p = tmp_path / "blob.obj"
    _write_obj(m, p, style)
    got, ref = _load_both(p)
    for k in KEYS:
        assert _same(got[k], ref[k]), k
    assert np.array_equal(got["v1"], m.v1) and np.array_equal(got["v3"], m.v3)
    if style == "v":  # FixNormals -> the face normals blob_mesh itself assigns
        assert np.array_equal(got["n1"], m.n1)


def _smooth_ref(m: Mesh):
    """Mesh.SmoothNormals (Mesh.cs:191-229) in numpy: fp32 sums in triangle order per distinct vertex."""
    n = len(m)
    verts = np.stack([m.v1, m.v2, m.v3], axis=1).reshape(-1, 3) + np.float32(0.0)
    norms = np.stack([m.n1, m.n2, m.n3], axis=1).reshape(-1, 3)
    _, inv = np.unique(verts, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    acc = np.zeros((inv.max() + 1, 3), np.float32)
    for k in range(3):
        np.add.at(acc[:, k], inv, norms[:, k])
    x, y, z = acc[:, 0], acc[:, 1], acc[:, 2]
    ln = np.sqrt((x * x + y * y) + z * z)
    unit = (acc / ln[:, None]).astype(np.float32)
    sm = unit[inv].reshape(n, 3, 3)
    return [np.ascontiguousarray(sm[:, k]) for k in range(3)]


def test_smooth_normals_native_equals_numpy():
    m = scenes.blob_mesh(50_000, seed=8)
    ref = _smooth_ref(m)
    m.SmoothNormals()
    for a, b in zip((m.n1, m.n2, m.n3), ref):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_obj_mesh_renders_like_array_mesh(tmp_path):
    """An OBJ-loaded mesh flattens to the same scene arrays as the in-memory mesh."""
    m = scenes.blob_mesh(2000, seed=5)
    p = tmp_path / "m.obj"
    _write_obj(m, p, "v")
    a, _, _ = scenes.bunny_frame(mesh=m.copy())
    b, _, _ = scenes.bunny_frame(mesh=OBJ.Load(str(p)))
    fa, fb = a.Compile(), b.Compile()
    for k in ("tri_v1", "tri_v2", "tri_v3", "tri_n1", "tri_n2", "tri_n3"):
        assert np.array_equal(getattr(fa, k), getattr(fb, k)), k


SCENE_ARRAYS = ("tri_v1", "tri_v2", "tri_v3", "tri_n1", "tri_n2", "tri_n3", "tri_t1", "tri_t2", "tri_t3", "tri_material",
                "shape_kind", "shape_index", "sphere_center", "sphere_radius", "cube_min", "cube_max", "mesh_first",
                "mesh_count")


@pytest.mark.parametrize("n", [4000, 69_451])
def test_bunny_frame_from_obj_equals_generated(tmp_path, n):
    """The C3/C4 scenes as Example.bunny builds them (Example.cs:1084-1102): the mesh written as OBJ by
    scenes.write_blob_obj and read back through pt_obj_load (OBJ.cs quirks: no normal index → the dummy
    normal → FixNormals), then SmoothNormals and FitInside, flatten to the same scene descriptor bit for
    bit as the in-memory generator: the fp32 text round trip (9 significant digits, strtof) is exact."""
    path = scenes.write_blob_obj(str(tmp_path / "blob.obj"), n)
    a = scenes.bunny_frame(n, mesh=OBJ.Load(path))[0].Compile()
    b = scenes.bunny_frame(n)[0].Compile()
    assert a.num_triangles == b.num_triangles > 0
    for k in SCENE_ARRAYS:
        x, y = getattr(a, k), getattr(b, k)
        assert x.dtype == y.dtype and np.array_equal(x.view(np.uint8), y.view(np.uint8)), k
    assert [m.key() for m in a.material_list] == [m.key() for m in b.material_list]


@pytest.mark.slow
def test_c4_obj_1m_equals_generated(tmp_path):
    """The bench's C4 mesh at its full 1,000,000 triangles through the OBJ path (76 MB of text)."""
    path = scenes.write_blob_obj(str(tmp_path / "blob1m.obj"), 1_000_000)
    m, g = OBJ.Load(path), scenes.blob_mesh(1_000_000)
    assert len(m.v1) == 1_000_000
    for k in ("v1", "v2", "v3", "n1", "n2", "n3", "t1", "t2", "t3"):
        assert np.array_equal(getattr(m, k).view(np.uint32), getattr(g, k).view(np.uint32)), k
