"""Golden fixtures (tests/golden/golden_v1.npz, made by tools/make_golden.py).

CPU: the oracle reproduces every fixture bit-exactly (RNG stream, primitive
intersect table, seeded renders), so any drift in the restatement is caught.
GPU: libptsharp_hip.so matches the render fixtures (rays, N, M and V) within the parity bar.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
from parity import check, render_gpu
from ptsharp_amd.renderer import Buffer
from ptsharp_amd import _abi

sys_tools = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
import sys  # noqa: E402

sys.path.insert(0, sys_tools)
import make_golden as G  # noqa: E402

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz"))


def test_rng_stream():
    L = O.lib()
    for i in range(len(GOLD["rng_key"])):
        k = L.or_camera_key(int(GOLD["rng_seed"][i]), int(GOLD["rng_pass"][i]), int(GOLD["rng_pixel"][i]),
                            int(GOLD["rng_sample"][i]))
        assert k == int(GOLD["rng_key"][i])
        assert [L.or_draw(k, d) for d in range(12)] == list(GOLD["rng_draws"][i])
        assert [L.or_child_key(k, c) for c in range(8)] == [int(x) for x in GOLD["rng_child"][i]]
        assert [L.or_light_key(k, c) for c in range(3)] == [int(x) for x in GOLD["rng_light"][i]]


@pytest.mark.parametrize("name", ["tri", "sphere", "cube", "plane"])
def test_prim_table(name):
    kind, a, b, c, r = {"tri": (3, (-1, -1, 0), (1, -1, 0.2), (0, 1, -0.1), 0.0),
                        "sphere": (0, (0.2, -0.1, 0.3), (0, 0, 0), (0, 0, 0), 1.3),
                        "cube": (1, (-1, -0.5, -1.5), (0.8, 1.2, 0.5), (0, 0, 0), 0.0),
                        "plane": (2, (0, 0.25, 0), (0, 1, 0), (0, 0, 0), 0.0)}[name]
    L = O.lib()
    t = [L.or_prim_intersect(kind, O.f3(a), O.f3(b), O.f3(c), r, O.f3(o), O.f3(d))
         for o, d in zip(GOLD["kat_origin"], GOLD["kat_dir"])]
    assert np.array_equal(np.array(t), GOLD[f"kat_{name}_t"])
    hits = np.array(t) < 1e9
    assert 0 < hits.sum() < len(t)  # the table exercises both outcomes


@pytest.mark.parametrize("spec", G.RENDERS, ids=[r[0] for r in G.RENDERS])
def test_oracle_render_fixture(spec):
    name, builder, overrides, w, h, spp, npass, seed = spec
    s, c, smp = G.build(name, builder, overrides)
    buf, rays = O.render(O.OracleScene(s), c, smp, w, h, spp, passes=npass, seed=seed)
    assert rays == int(GOLD[f"render_{name}_rays"])
    assert np.array_equal(buf.N, GOLD[f"render_{name}_N"])
    assert np.array_equal(buf.M, GOLD[f"render_{name}_M"])
    assert np.array_equal(buf.V, GOLD[f"render_{name}_V"])


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [_abi.ENGINE_MEGAKERNEL, _abi.ENGINE_WAVEFRONT], ids=["mega", "wave"])
@pytest.mark.parametrize("spec", G.RENDERS, ids=[r[0] for r in G.RENDERS])
def test_gpu_matches_fixture(gpu, spec, engine):
    name, builder, overrides, w, h, spp, npass, seed = spec
    s, c, smp = G.build(name, builder, overrides)
    g, rays = render_gpu(s, c, smp, w, h, spp, passes=npass, seed=seed, engine=engine)
    ref = Buffer(w, h)
    ref.M, ref.V, ref.N = GOLD[f"render_{name}_M"], GOLD[f"render_{name}_V"], GOLD[f"render_{name}_N"]
    check(g, rays, ref, int(GOLD[f"render_{name}_rays"]))
