"""§8f row 3 on the GPU (libptsharp_hip.so through the C-ABI) vs the oracle, same seed:
colour / gloss / normal / bump maps, a textured light, an environment map with
TextureAngle.  Same bar as tests/test_gpu_parity.py (tests/parity.py check)."""
import numpy as np
import pytest

from parity import check, render_both
from ptsharp_amd import ColorTexture, Colour, LightMode, SpecularMode, _abi, scenes

pytestmark = pytest.mark.gpu

ENGINES = pytest.mark.parametrize("engine", [_abi.ENGINE_MEGAKERNEL, _abi.ENGINE_WAVEFRONT], ids=["mega", "wave"])




@ENGINES
def test_textured_scene(gpu, engine):
    s, c, smp = scenes.textured()
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=2, passes=2, seed=21, engine=engine)
    check(g, gr, o, orr)


@ENGINES
@pytest.mark.parametrize("lm,sm", [(LightMode.LightModeAll, SpecularMode.SpecularModeAll),
                                   (LightMode.LightModeRandom, SpecularMode.SpecularModeNaive)])
def test_textured_sampler_modes(gpu, engine, lm, sm):
    s, c, smp = scenes.textured(mesh_tris=600)
    smp.LightMode, smp.SpecularMode, smp.MaxBounces = lm, sm, 3
    g, gr, o, orr = render_both(s, c, smp, 40, 32, spp=1, seed=22, engine=engine)
    check(g, gr, o, orr)


@ENGINES
def test_constant_environment_map_furnace(gpu, engine):
    env = ColorTexture(4, 3, np.full((12, 3), 0.75))
    s, c, smp = scenes.furnace(0.5)
    s.Color = Colour(0, 0, 0)
    s.Texture = env
    g, gr, o, orr = render_both(s, c, smp, 48, 32, spp=2, seed=23, engine=engine)
    check(g, gr, o, orr)
    assert np.allclose(g.M, o.M, rtol=0, atol=1e-12)


def test_textured_adaptive_firefly(gpu):
    s, c, smp = scenes.textured(mesh_tris=600)
    smp.MaxBounces = 2
    g, gr, o, orr = render_both(s, c, smp, 40, 32, spp=1, seed=24, engine=_abi.ENGINE_WAVEFRONT, adaptive=2, firefly=2)
    check(g, gr, o, orr)   # firefly candidates and stops decided alike: N equal everywhere
