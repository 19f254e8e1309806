"""§8f row 4 on the GPU (libptsharp_hip.so through the C-ABI) vs the oracle, same seed:
SDF shapes (every node kind), Volume, TransformedShape over each inner kind.  Same bar
as tests/test_gpu_parity.py (tests/parity.py check)."""
import numpy as np
import pytest

from parity import check, render_both
from ptsharp_amd import Cube, Matrix, Scene, TransformedShape, Vector, _abi, scenes

pytestmark = pytest.mark.gpu

ENGINES = pytest.mark.parametrize("engine", [_abi.ENGINE_MEGAKERNEL, _abi.ENGINE_WAVEFRONT], ids=["mega", "wave"])




@ENGINES
@pytest.mark.parametrize("name", ["sdf", "sdf_zoo", "volume", "transformed", "instances"])
def test_row4_scene(gpu, engine, name):
    s, c, smp = scenes.SCENES[name]()
    smp.MaxBounces = min(smp.MaxBounces, 3)
    g, gr, o, orr = render_both(s, c, smp, 48, 36, spp=2, seed=31, engine=engine)
    check(g, gr, o, orr)


@ENGINES
def test_mixed_scene(gpu, engine):
    """The C5-kind scene (mesh + SDF + Volume + environment texture) at a test size."""
    s, c, smp = scenes.mixed(3000, seed=5)
    smp.MaxBounces = 3
    g, gr, o, orr = render_both(s, c, smp, 48, 36, spp=2, seed=33, engine=engine)
    check(g, gr, o, orr)


@ENGINES
def test_transformed_furnace_exact(gpu, engine):
    s, cam, smp = scenes.furnace(0.5)
    cube = s.Shapes[0]
    s2 = Scene()
    s2.Color = s.Color
    s2.Add(TransformedShape.NewTransformedShape(Cube.NewCube(cube.Min, cube.Max, cube.Material),
                                                Matrix.TranslateM(Vector(0, 0, 0))))
    g, gr, o, orr = render_both(s2, cam, smp, 48, 32, spp=2, seed=32, engine=engine)
    assert set(np.unique(g.M)) <= {0.5, 1.0}
    check(g, gr, o, orr, exact=True)


def test_row4_adaptive(gpu):
    s, c, smp = scenes.sdf_zoo()
    smp.MaxBounces = 2
    g, gr, o, orr = render_both(s, c, smp, 40, 30, spp=1, seed=33, engine=_abi.ENGINE_WAVEFRONT, adaptive=2)
    check(g, gr, o, orr)


def test_march_counters(gpu):
    """pt_render_pass_counted reports the Volume / SDFShape march steps (the C5 bench's flop
    model): both present in the mixed scene, neither in a scene without those shapes, and a
    counted pass leaves the same Buffer as an uncounted one."""
    from ptsharp_amd import Renderer
    s, c, smp = scenes.mixed(3000, seed=5)
    smp.MaxBounces = 2
    bufs = []
    for counted in (False, True):
        r = Renderer.NewRenderer(s, c, smp, 48, 36, True)
        r.SamplesPerPixel = 2
        r.Seed = 7
        r.Engine = _abi.ENGINE_WAVEFRONT
        if counted:
            ctr = r.RenderCounted()
        else:
            r.RenderParallel()
        b = r.ReadBuffer()
        bufs.append((b.M.copy(), b.V.copy(), b.N.copy()))
        r.close()
    assert ctr.volume_samples > 0 and ctr.sdf_evals > 0
    for x, y in zip(*bufs):
        assert np.array_equal(x, y)
    s2, c2, smp2 = scenes.gopher3()
    r = Renderer.NewRenderer(s2, c2, smp2, 32, 24, True)
    r.SamplesPerPixel = 1
    ctr2 = r.RenderCounted()
    r.close()
    assert ctr2.rays > 0 and ctr2.volume_samples == 0 and ctr2.sdf_evals == 0


def test_routed_split_equals_full_analytic_half(gpu, monkeypatch):
    """The routed split (only rays that reach a row-4 shape's box take the FULL kernels, which test the
    heavy records in record order) against every ray through the FULL analytic half (PT_ROUTE=0 at
    upload): they differ only at exact-t ties between shapes (class 3), so on C5's
    kind of scene the two Buffers must be the same bits.  C5's 1M-triangle mixed scene at 4K, 4 tiles,
    AdaptiveSamples 8, plus the C5 scene at test size with MaxBounces 3."""
    from parity import render_gpu, same_buffer
    from ptsharp_amd.renderer import tiles_for_rank
    cases = [(scenes.mixed(1_000_000), 3840, 2160, tiles_for_rank(3840, 2160, 5, 2048), 8),
             (scenes.mixed(3000, seed=5), 96, 64, None, 2)]
    for (s, c, smp), w, h, tiles, adaptive in cases:
        smp.MaxBounces = min(smp.MaxBounces, 3)
        bufs = []
        for route in ("1", "0"):
            monkeypatch.setenv("PT_ROUTE", route)
            bufs.append(render_gpu(s, c, smp, w, h, 1, passes=1, seed=77, tiles=tiles,
                                   engine=_abi.ENGINE_WAVEFRONT, adaptive=adaptive))
        (a, ra), (b, rb) = bufs
        assert ra == rb
        same_buffer(a, b)
