"""The oracle's bounce and light sampling pinned by a second restatement (tests/sampler_ref.py,
Python, written line by line from Ray.cs / Util.cs / Vector.cs / Sampler.cs / Box.cs):
Util.Cone, Ray.Bounce (every material kind, every bounce type), Sampler.sampleLight for
sphere and bounding-box lights (and the Cylinder branch standalone), sampleLights in both
light modes: bit-exact.  Also the equivalence the GPU's any-hit shadow query rests on
(DESIGN.md §4): "the nearest hit is the light" == "nothing is hit strictly nearer than the
light's own t", exact except at exact-t ties, whose reference outcome depends on k-d leaf
order (test_exact_t_tie_*)."""

import numpy as np
import pytest

import oracle_lib as O
import sampler_ref as R
from ptsharp_amd import Colour, Cube, Material, Scene, Sphere, Vector, scenes

RNG = np.random.default_rng(20261016)


def v3(t):
    return R.Vec(*t)


def same3(a, b):
    return [np.float32(x) for x in a] == [np.float32(x) for x in b]


def test_cone_bit_exact():
    L = O.lib()
    for _ in range(400):
        d = RNG.normal(size=3)
        d = R.Vec(*d).Normalize()
        theta = float(RNG.choice([0.0, 1e-10, RNG.uniform(0, 1.2)]))
        u, v = float(RNG.uniform()), float(RNG.uniform())
        key = int(RNG.integers(0, 2**63))
        out = (O.C.c_float * 3)()
        L.or_cone(O.f3(d.t()), theta, u, v, key, out)
        assert same3(tuple(out), R.cone(d, theta, u, v, key).t())


def _hits(oscene, camera, n, w=64, h=48, seed=3):
    """Camera rays of the scene that hit: (origin, dir, pos, normal, inside, mat)."""
    L = O.lib()
    cam = camera.to_c()
    out = []
    while len(out) < n:
        x, y = int(RNG.integers(0, w)), int(RNG.integers(0, h))
        o, d = (O.C.c_float * 3)(), (O.C.c_float * 3)()
        L.or_cast_ray(O.C.byref(cam), x, y, w, h, float(RNG.uniform()), float(RNG.uniform()), seed, o, d)
        pos, nrm, inside, mat = (O.C.c_float * 3)(), (O.C.c_float * 3)(), O.C.c_int32(), O.C.c_int32()
        if L.or_hit_info(oscene.h, o, d, pos, nrm, O.C.byref(inside), O.C.byref(mat)):
            out.append((tuple(o), tuple(d), tuple(pos), tuple(nrm), bool(inside.value), mat.value))
    return out


@pytest.mark.parametrize("btype", [0, 1, 2], ids=["any", "diffuse", "specular"])
def test_bounce_bit_exact(btype):
    """Ray.Bounce on materialspheres (diffuse, specular, glossy, transparent with tint, clear,
    metallic with fixed reflectivity) and on transparent spheres seen from inside."""
    s, c, smp = scenes.materialspheres()
    osc = O.OracleScene(s)
    mats = osc.flat.material_list
    kinds = set()
    for o, d, pos, nrm, inside, mi in _hits(osc, c, 300):
        u, v, key = float(RNG.uniform()), float(RNG.uniform()), int(RNG.integers(0, 2**63))
        got = osc.bounce(o, d, u, v, btype, key)
        ro, rd, refl, p = R.bounce(v3(d), v3(pos), v3(nrm), inside, mats[mi], u, v, btype, key)
        assert got is not None
        assert same3(got[0], ro.t()) and same3(got[1], rd.t()), (mats[mi], btype)
        assert got[2] == refl and got[3] == p
        kinds.add((bool(mats[mi].Transparent), mats[mi].Reflectivity >= 0, refl))
    assert len(kinds) >= 3   # the material mix is exercised


def _lights_of(s, osc):
    """sampler_ref Lights for the scene's Scene.Lights, in order, identity by (kind, index)."""
    out = []
    for kind, idx in osc.lights():
        ident = (lambda k, i, kind=kind, idx=idx: k == kind and i == idx)
        if kind == 0:   # K_SPHERE
            sp = [x for x in s.Shapes if isinstance(x, Sphere)][idx]
            m = sp.Material
            out.append(R.Light("sphere", (m.Color.r, m.Color.g, m.Color.b), m.Emittance, ident,
                               center=R.Vec(sp.Center.X, sp.Center.Y, sp.Center.Z), radius=sp.Radius))
        else:           # bounding-box light (Cube, SDF, Volume): light.BoundingBox()
            mn, mx = (O.C.c_float * 3)(), (O.C.c_float * 3)()
            O.lib().or_shape_box(osc.h, kind, idx, mn, mx)
            m = osc.flat.material_list[_mat_of(s, kind, idx)]
            out.append(R.Light("box", (m.Color.r, m.Color.g, m.Color.b), m.Emittance, ident,
                               mn=R.Vec(*mn), mx=R.Vec(*mx)))
    return out


def _mat_of(s, kind, idx):
    osc_flat = s.Compile()
    cubes = [x for x in s.Shapes if isinstance(x, Cube)]
    m = cubes[idx].Material
    return [mm.key() for mm in osc_flat.material_list].index(m.key())


def _intersect(osc):
    def f(o, d):
        t, k, i = osc.intersect(o.t(), d.t())
        return t, k, i
    return f


@pytest.mark.parametrize("name", ["bunny", "example3", "twolights_box"])
@pytest.mark.parametrize("ss", [True, False], ids=["soft", "hard"])
def test_sample_light_bit_exact(name, ss):
    """sampleLight from real shading points: sphere lights (bunny frame), a Cube light through the
    bounding-box branch (Example.example3), and a scene with both kinds."""
    if name == "bunny":
        s, c, smp = scenes.bunny_frame(800, seed=4)
    elif name == "example3":
        s, c, smp = scenes.example3()
    else:
        s, c, smp = scenes.example3()
        s.Add(Sphere.NewSphere(Vector(6, 6, 3), 0.7, Material.LightMaterial(Colour(1, 0.6, 0.3), 9)))
    osc = O.OracleScene(s)
    lights = _lights_of(s, osc)
    assert lights
    isect = _intersect(osc)
    lit = 0
    for _, _, pos, nrm, _, _ in _hits(osc, c, 150):
        for li in range(len(lights)):
            key = int(RNG.integers(0, 2**63))
            got, grays = osc.sample_light(pos, nrm, li, key, ss)
            ref, rrays = R.sample_light(isect, v3(pos), v3(nrm), lights[li], key, ss)
            assert got == ref and grays == rrays
            lit += any(x > 0 for x in ref)
    assert lit > 10


@pytest.mark.parametrize("mode", [0, 1], ids=["random", "all"])
def test_sample_lights_bit_exact(mode):
    s, c, smp = scenes.example3()
    s.Add(Sphere.NewSphere(Vector(6, 6, 3), 0.7, Material.LightMaterial(Colour(1, 0.6, 0.3), 9)))
    osc = O.OracleScene(s)
    lights = _lights_of(s, osc)
    isect = _intersect(osc)
    for _, _, pos, nrm, _, _ in _hits(osc, c, 150):
        key = int(RNG.integers(0, 2**63))
        got, grays = osc.sample_lights(pos, nrm, key, mode, True)
        ref, rrays = R.sample_lights(isect, v3(pos), v3(nrm), lights, key, mode, True)
        assert got == ref and grays == rrays


def test_cylinder_light_branch():
    """Sampler.cs:224-227, 270-274: a Cylinder light's centre is (0, 0, (Z0+Z1)/2) and its coverage 1.
    (Cylinder is not a GPU-path shape; the branch is pinned in the restatement alone.)"""
    L = R.Light("cylinder", (1.0, 0.5, 0.25), 4.0, lambda k, i: True, radius=0.5, z0=1.0, z1=3.0)
    o, n = R.Vec(0, 0, -1), R.Vec(0, 0, 1)
    col, rays = R.sample_light(lambda a, b: (1.0, 9, 0), o, n, L, 1234, soft_shadows=False)
    assert rays == 1
    d = R.Vec(0, 0, 2).Sub(o).Normalize()
    diffuse = d.Dot(n)
    assert col == tuple(x * (4.0 * diffuse * 1.0) for x in (1.0, 0.5, 0.25))


def test_any_hit_equals_nearest_hit_identity():
    """For shadow rays from real shading points towards sampled light points: the reference's rule
    (Scene.Intersect's nearest hit is the light, Sampler.cs:261-265) and the GPU's (no shape strictly
    nearer than the light's own t) agree on every ray without an exact-t tie."""
    s, c, smp = scenes.example3()
    s.Add(Sphere.NewSphere(Vector(6, 6, 3), 0.7, Material.LightMaterial(Colour(1, 0.6, 0.3), 9)))
    osc = O.OracleScene(s)
    lights = _lights_of(s, osc)
    n_rays = n_lit = ties = 0
    for _, _, pos, nrm, _, _ in _hits(osc, c, 200):
        for li, Lt in enumerate(lights):
            key = int(RNG.integers(0, 2**63))
            # the shadow ray sampleLight casts
            captured = []

            def isect(o, d):
                captured.append((o, d))
                return osc.intersect(o.t(), d.t())
            R.sample_light(isect, v3(pos), v3(nrm), Lt, key, True)
            if not captured:
                continue
            o, d = captured[0]
            t, k, i = osc.intersect(o.t(), d.t())
            nearest_is_light = t < 1e9 and Lt.identity(k, i)
            kind, idx = osc.lights()[li]
            tl = _shape_t(s, osc, kind, idx, o, d)
            any_hit_lit = tl < 1e9 and not osc.any_nearer(o.t(), d.t(), tl)
            tie = t < 1e9 and t == tl and not Lt.identity(k, i)
            ties += tie
            if not tie:
                assert nearest_is_light == any_hit_lit
            n_rays += 1
            n_lit += nearest_is_light
    assert n_rays > 200 and n_lit > 20 and ties == 0


def _shape_t(s, osc, kind, idx, o, d):
    """The light's own t along (o, d), by the primitive intersect of the oracle."""
    L = O.lib()
    if kind == 0:
        sp = [x for x in s.Shapes if isinstance(x, Sphere)][idx]
        return L.or_prim_intersect(0, O.f3((sp.Center.X, sp.Center.Y, sp.Center.Z)), O.f3((0, 0, 0)),
                                   O.f3((0, 0, 0)), sp.Radius, O.f3(o.t()), O.f3(d.t()))
    cu = [x for x in s.Shapes if isinstance(x, Cube)][idx]
    return L.or_prim_intersect(1, O.f3((cu.Min.X, cu.Min.Y, cu.Min.Z)), O.f3((cu.Max.X, cu.Max.Y, cu.Max.Z)),
                               O.f3((0, 0, 0)), 0.0, O.f3(o.t()), O.f3(d.t()))


@pytest.mark.parametrize("light_first", [True, False])
def test_exact_t_tie_follows_leaf_order(light_first):
    """A light sphere and an identical non-emissive sphere: every shadow ray hits both at the same t.
    The reference's strict '<' over the k-d leaf's shape list keeps the first one (Tree.cs:115-128),
    so the outcome depends on which sphere comes first in the leaf; the GPU's any-hit query, which
    asks for a shape strictly nearer than the light, always finds the light visible.  This is the
    one place the two formulations differ (DESIGN.md §4 documents it): exact-t ties between
    distinct coincident shapes."""
    s = Scene()
    light = Sphere.NewSphere(Vector(0, 5, 0), 1, Material.LightMaterial(Colour.White, 10))
    twin = Sphere.NewSphere(Vector(0, 5, 0), 1, Material.DiffuseMaterial(Colour.White))
    s.Add(Cube.NewCube(Vector(-10, -1, -10), Vector(10, 0, 10), Material.DiffuseMaterial(Colour.White)))
    for sh in ([light, twin] if light_first else [twin, light]):
        s.Add(sh)
    osc = O.OracleScene(s)
    (kind, idx), = osc.lights()
    pos, nrm = (0.5, 0.0, 0.25), (0.0, 1.0, 0.0)
    col, rays = osc.sample_light(pos, nrm, 0, 77, soft_shadows=False)
    d = R.Vec(0, 5, 0).Sub(R.Vec(*pos)).Normalize()
    t, k, i = osc.intersect(pos, d.t())
    other = 1 - idx
    t_twin = O.lib().or_prim_intersect(0, O.f3((0, 5, 0)), O.f3((0, 0, 0)), O.f3((0, 0, 0)), 1.0, O.f3(pos),
                                       O.f3(d.t()))
    assert t == t_twin                                       # an exact tie
    assert (k, i) in {(kind, idx), (0, other)}
    assert (sum(col) > 0) == ((k, i) == (kind, idx))        # the leaf's first sphere decides
    assert not osc.any_nearer(pos, d.t(), t_twin)            # any-hit: nothing strictly nearer → lit


def test_oracle_keeps_sin_and_cos_separate():
    """.NET's Math.Sin and Math.Cos are two libm calls.  A sincos() fused by the compiler rounds
    differently in the last ulp on this glibc (e.g. sin(0.15142274361170249)), which surfaced as a
    rare sampleLight coverage mismatch; oracle/Makefile builds with -fno-builtin-sin/-cos."""
    import subprocess
    syms = subprocess.run(["nm", "-D", O.build_oracle()], capture_output=True, text=True).stdout
    assert "sincos" not in syms
    L = O.lib()
    assert L is not None
