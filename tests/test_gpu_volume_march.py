"""The two forms of the Volume march on the GPU against the oracle, ray by ray, bit for bit.

Volume.Intersect (Volume.cs:168-197) runs on the device in two forms:
  * by one lane (vol_t, pt_ext.h): march_pending's fallback when fewer than 8 lanes of a wave are
    active, inner_t for a Volume that is not deferred (a second Volume on the same ray, a Volume
    inside a TransformedShape reached through prim_t), TransformedShape.cs:43-73 around it;
  * by the wave's active lanes together (coop_vol_t, pt_device.h): every deferred Volume.
A render reaches the one-lane form only at wave tails, so a render test cannot show that it is
right.  pt_intersect / pt_occluded run Scene.Intersect and the shadow query for given rays with
the form forced (PT_MARCH_LANE: every lane its own march; PT_MARCH_WAVE: always together); both
must give the oracle's t (or_intersect, the reference loop as written) and the same answers as
the render's own choice, on rays aimed at the Volume of the C5-kind mixed scene and of a scene
with two overlapping Volumes.
"""
import numpy as np
import pytest

import oracle_lib as O
from ptsharp_amd import Renderer, TransformedShape, Vector, _abi, scenes
from ptsharp_amd.geometry import Matrix
from ptsharp_amd.scene import Scene

pytestmark = pytest.mark.gpu

MODES = {"auto": 0, "lane": _abi.MARCH_LANE, "wave": _abi.MARCH_WAVE}


def world_box(shape):
    """World box of a Volume or of a TransformedShape of one (the inner box's corners mapped)."""
    if isinstance(shape, TransformedShape):
        b = shape.Shape.Box
        c = np.array([[x, y, z, 1.0] for x in (b.Min.X, b.Max.X) for y in (b.Min.Y, b.Max.Y) for z in (b.Min.Z, b.Max.Z)])
        w = c @ shape.Matrix.m.T
        return w[:, :3].min(axis=0), w[:, :3].max(axis=0)
    b = shape.Box
    return np.array([b.Min.X, b.Min.Y, b.Min.Z]), np.array([b.Max.X, b.Max.Y, b.Max.Z])


def volume_rays(lo, hi, n, seed):
    """Rays that cross the box [lo, hi]: from a shell around it to a point inside (half), from inside
    the box (a quarter), and grazing its faces (a quarter).  float32, directions normalised."""
    rng = np.random.default_rng(seed)
    c, ext = (lo + hi) / 2, (hi - lo) / 2
    n1, n2 = n // 2, n // 4
    n3 = n - n1 - n2
    u = rng.standard_normal((n1, 3))
    o1 = c + 3.0 * np.abs(ext).max() * u / np.linalg.norm(u, axis=1, keepdims=True)
    t1 = lo + (hi - lo) * rng.random((n1, 3))
    o2 = lo + (hi - lo) * rng.random((n2, 3))
    t2 = o2 + rng.standard_normal((n2, 3))
    face = rng.integers(0, 3, n3)
    t3 = lo + (hi - lo) * rng.random((n3, 3))
    t3[np.arange(n3), face] = np.where(rng.random(n3) < 0.5, lo[face], hi[face])
    tang = rng.standard_normal((n3, 3))
    tang[np.arange(n3), face] *= 0.02   # nearly parallel to the face
    o3 = t3 - 2.5 * tang / np.linalg.norm(tang, axis=1, keepdims=True)
    o = np.concatenate([o1, o2, o3]).astype(np.float32)
    d = (np.concatenate([t1, t2, t3]) - np.concatenate([o1, o2, o3])).astype(np.float32)
    d = d / np.linalg.norm(d.astype(np.float64), axis=1, keepdims=True).astype(np.float32)
    return o, d.astype(np.float32)


def oracle_hits(os_, o, d):
    t = np.empty(len(o), np.float64)
    k = np.empty(len(o), np.int32)
    for i in range(len(o)):
        t[i], k[i], _ = os_.intersect(o[i], d[i])
    return t, k


def check_rays(scene, o, d, vol_kind, min_vol_hits):
    r = Renderer.NewRenderer(scene, None, None, 8, 8, True)
    try:
        res = {m: r.Intersect(o, d, f) for m, f in MODES.items()}
        os_ = O.OracleScene(scene)
        ot, ok = oracle_hits(os_, o, d)
        for m, (t, k) in res.items():
            bad = np.flatnonzero((t.view(np.int64) != ot.view(np.int64)) | (k != ok))
            assert bad.size == 0, (f"{m}: {bad.size} of {len(o)} rays differ from the oracle, first {bad[:5]}: "
                                   f"gpu t {t[bad[:3]]} kind {k[bad[:3]]}, oracle t {ot[bad[:3]]} kind {ok[bad[:3]]}")
        vol_hits = int((ok == vol_kind).sum())
        assert vol_hits >= min_vol_hits, f"only {vol_hits} Volume hits"
        # the shadow query: the hit's own t (nothing strictly nearer unless a tie), one ulp past it,
        # and random bounds before and after it
        rng = np.random.default_rng(7)
        hit = ot < 1e9
        tl = np.where(hit, ot, 5.0)
        for name, tm in {"at_hit": tl, "past_hit": np.nextafter(tl, np.inf),
                         "random": tl * rng.uniform(0.0, 1.6, len(tl))}.items():
            want = np.array([os_.any_nearer(o[i], d[i], tm[i]) for i in range(len(o))], np.int32)
            for m, f in MODES.items():
                got = r.Occluded(o, d, tm, f)
                bad = np.flatnonzero(got != want)
                assert bad.size == 0, f"occluded {name} {m}: {bad.size} rays differ, first {bad[:5]}"
        return vol_hits
    finally:
        r.close()


def test_volume_march_forms_mixed_scene(gpu):
    """The C5-kind mixed scene (scenes.mixed: its Volume inside a TransformedShape, behind the mesh
    and the SDF torus in parts): rays aimed at that Volume."""
    s, _, _ = scenes.mixed(3000, seed=5)
    lo, hi = world_box(s.Shapes[-1])
    o, d = volume_rays(lo, hi, 24000, seed=11)
    check_rays(s, o, d, _abi.SHAPE_TRANSFORMED, 500)


def test_volume_march_forms_two_volumes(gpu):
    """A Volume and a TransformedShape of it above its hittable slab (Sample's y-from-z slip leaves only
    the box's z < 0 part non-zero, Volume.cs:77): a ray that defers the first Volume it reaches meets the
    other in place (prim_t -> xform_t / inner_t -> vol_t) even in the render's own form."""
    a, _, _ = scenes.volume(24, 24, 12, seed=3)
    s = Scene()
    s.Color = a.Color
    s.Add(a.Shapes[0])
    s.Add(TransformedShape.NewTransformedShape(a.Shapes[0], Matrix.TranslateM(Vector(0.3, 0.2, 0.5)).Mul(
        Matrix.ScaleM(Vector(0.9, 0.9, 0.9)))))
    lo0, hi0 = world_box(s.Shapes[0])
    lo1, hi1 = world_box(s.Shapes[1])
    o1, d1 = volume_rays(np.minimum(lo0, lo1), np.maximum(hi0, hi1), 8000, seed=12)
    o2, d2 = volume_rays(np.array([-0.6, -0.7, 0.3]), np.array([1.2, 1.1, 0.5]), 8000, seed=13)   # the second's slab
    o, d = np.concatenate([o1, o2]), np.concatenate([d1, d2])
    check_rays(s, o, d, _abi.SHAPE_VOLUME, 200)
    os_ = O.OracleScene(s)
    _, ok = oracle_hits(os_, o, d)
    assert int((ok == _abi.SHAPE_TRANSFORMED).sum()) >= 200


def test_march_staging_and_cells_equal_plain_grid(gpu, monkeypatch):
    """The Volume queue kernels' two layouts of the grid against the plain one: the Volume staged in LDS
    (stage_vol: header, windows, uniform-cell table) and the corners read cell-major (vol_build_cells), each
    switched off at upload (PT_VOL_LDS=0, PT_VOL_CELLS=0), must leave the same Buffer bits and ray counts as
    both on, on the C5-kind mixed scene at test size (the split traversal, the deferred march)."""
    from parity import render_gpu, same_buffer
    s, c, smp = scenes.mixed(3000, seed=5)
    smp.MaxBounces = 3
    bufs = []
    for lds, cells in (("1", "1"), ("0", "1"), ("1", "0"), ("0", "0")):
        monkeypatch.setenv("PT_VOL_LDS", lds)
        monkeypatch.setenv("PT_VOL_CELLS", cells)
        bufs.append(render_gpu(s, c, smp, 96, 64, 2, passes=1, seed=41, engine=_abi.ENGINE_WAVEFRONT, adaptive=2))
    (a, ra) = bufs[0]
    for b, rb in bufs[1:]:
        assert ra == rb
        same_buffer(a, b)
