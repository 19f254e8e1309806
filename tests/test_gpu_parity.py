"""GPU (libptsharp_hip.so through the C-ABI) vs the CPU oracle, same seed.

Bar (tests/parity.py): Scene.Intersect counts and Welford sample counts N exact; M and
V within 1e-9·max(1, |ref|) on >= 99.9 % of pixels; PSNR >= 50 dB; the RNG-independent
analytic scenes bit-exact.  Between GPU runs (same seed, either engine, any tile split)
the Buffer is bit-identical: terms are summed in an order-independent fixed-point form
(ptsharp_amd/csrc/pt_accum.h).
"""
import numpy as np
import pytest

import oracle_lib as O
from parity import check, render_both, render_gpu, same_buffer
from ptsharp_amd import LightMode, SpecularMode, _abi, scenes, tiles_for_rank

pytestmark = pytest.mark.gpu

ENGINES = pytest.mark.parametrize("engine", [_abi.ENGINE_MEGAKERNEL, _abi.ENGINE_WAVEFRONT], ids=["mega", "wave"])


@ENGINES
def test_furnace_exact(gpu, engine):
    s, c, smp = scenes.furnace(0.5)
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=2, passes=2, seed=3, engine=engine)
    assert set(np.unique(g.M)) <= {0.5, 1.0}
    check(g, gr, o, orr, exact=True)


@ENGINES
def test_furnace_negative_albedo(gpu, engine):
    """A negative colour (legal in the reference's fp64 Colour): every floor pixel's fixed-point sum is
    negative.  pt_accum.h fix_value converts a total that fits 64 signed bits in one step (ADVICE r02:
    the two-word form rounded the low word of a negative total to 2^11 ulps, ~6e-11 absolute)."""
    s, c, smp = scenes.furnace(-0.3)
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=2, passes=2, seed=3, engine=engine)
    assert gr == orr and np.array_equal(g.N, o.N)
    floor = o.M[..., 0] < 0
    assert floor.any() and (~floor).any()
    assert np.abs(g.M[floor] - o.M[floor]).max() <= 1e-12
    assert np.array_equal(g.M[~floor], o.M[~floor])
    assert np.abs(g.V - o.V).max() <= 1e-12


@ENGINES
@pytest.mark.parametrize("fh", [16, 8, 1])
def test_emitter_exact(gpu, fh, engine):
    s, c, smp = scenes.emitter(fh)
    g, gr, o, orr = render_both(s, c, smp, 48, 40, spp=1, seed=5, engine=engine)
    check(g, gr, o, orr, exact=True)
    n = int(np.sqrt(fh))
    lit = g.M[g.N > 0].reshape(-1, 3)
    assert np.isclose(lit.max(axis=0), np.array([0.25, 0.5, 1.0]) * 2 * fh / (n * n)).all()


@pytest.mark.parametrize("name", ["gopher3", "materialspheres", "simplesphere", "example1"])
@ENGINES
def test_analytic_scenes(gpu, name, engine):
    s, c, smp = scenes.SCENES[name]()
    smp.MaxBounces = min(smp.MaxBounces, 6)
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=2, passes=2, seed=11, engine=engine)
    check(g, gr, o, orr)


@ENGINES
def test_mesh_scene(gpu, engine):
    s, c, smp = scenes.bunny_frame(4000, seed=9)
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=2, passes=2, seed=13, engine=engine)
    check(g, gr, o, orr)


@pytest.mark.parametrize("lm,sm", [(LightMode.LightModeAll, SpecularMode.SpecularModeAll),
                                   (LightMode.LightModeRandom, SpecularMode.SpecularModeFirst),
                                   (LightMode.LightModeAll, SpecularMode.SpecularModeNaive)])
@ENGINES
def test_sampler_modes(gpu, lm, sm, engine):
    s, c, smp = scenes.materialspheres()
    smp.FirstHitSamples, smp.MaxBounces = 4, 3
    smp.LightMode, smp.SpecularMode = lm, sm
    g, gr, o, orr = render_both(s, c, smp, 48, 32, spp=1, passes=2, seed=17, engine=engine)
    check(g, gr, o, orr)


@ENGINES
def test_stratified(gpu, engine):
    s, c, smp = scenes.simplesphere()
    g, gr, o, orr = render_both(s, c, smp, 48, 32, spp=4, seed=19, stratified=True, engine=engine)
    check(g, gr, o, orr)


# ---- determinism: bit-identical Buffers across runs, engines and tile splits
def test_same_seed_bit_identical(gpu):
    """Two same-seed wavefront renders of a mesh scene give the same bits (no fp atomics in the sum)."""
    s, c, smp = scenes.bunny_frame(4000, seed=9)
    a, ra = render_gpu(s, c, smp, 160, 120, spp=4, passes=2, seed=51, engine=_abi.ENGINE_WAVEFRONT)
    b, rb = render_gpu(s, c, smp, 160, 120, spp=4, passes=2, seed=51, engine=_abi.ENGINE_WAVEFRONT)
    assert ra == rb
    same_buffer(a, b)


@ENGINES
def test_tiles_shard_equals_full(gpu, engine):
    """Disjoint tile sets rendered separately sum to the full render, bit for bit (pixel-keyed RNG)."""
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 3
    w, h = 80, 70
    full, _ = render_gpu(s, c, smp, w, h, spp=1, seed=23, engine=engine)
    parts = [render_gpu(s, c, smp, w, h, spp=1, seed=23, tiles=tiles_for_rank(w, h, r, 3), engine=engine)[0]
             for r in range(3)]
    M = sum(p.M for p in parts)
    V = sum(p.V for p in parts)
    N = sum(p.N for p in parts)
    assert np.array_equal(N, full.N)
    assert np.array_equal(M, full.M)
    assert np.array_equal(V, full.V)


@pytest.mark.parametrize("name", ["gopher3", "materialspheres", "mesh"])
def test_engines_bit_identical(gpu, name):
    """Megakernel and wavefront add the same fp64 terms: same rays, same Buffer bits."""
    if name == "mesh":
        s, c, smp = scenes.bunny_frame(4000, seed=9)
    else:
        s, c, smp = scenes.SCENES[name]()
        smp.MaxBounces = 5
    a, ra = render_gpu(s, c, smp, 64, 40, spp=2, passes=2, seed=29, engine=_abi.ENGINE_MEGAKERNEL)
    b, rb = render_gpu(s, c, smp, 64, 40, spp=2, passes=2, seed=29, engine=_abi.ENGINE_WAVEFRONT)
    assert ra == rb
    same_buffer(a, b)


def test_wavefront_many_chunks(gpu, monkeypatch):
    """With the queues held to 4M entries (PT_WF_MAX_CAP) a 640x360 frame at spp 8 with FH 16
    takes ~15 queue chunks; the Buffer is the megakernel's, bit for bit."""
    monkeypatch.setenv("PT_WF_MAX_CAP", str(1 << 22))
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 2
    a, ra = render_gpu(s, c, smp, 640, 360, spp=8, seed=31, engine=_abi.ENGINE_MEGAKERNEL)
    b, rb = render_gpu(s, c, smp, 640, 360, spp=8, seed=31, engine=_abi.ENGINE_WAVEFRONT)
    assert ra == rb
    same_buffer(a, b)


def test_wavefront_full_frame_one_stream(gpu):
    """1920x1080 at 16 spp with 8 first-bounce children: one 33M-sample chunk, above the side-stream
    threshold, so shadow passes run on the main stream (the C4 bench's configuration); the Buffer
    is the megakernel's, bit for bit."""
    s, c, smp = scenes.bunny_frame(4000, seed=9)
    smp.MaxBounces = 2
    a, ra = render_gpu(s, c, smp, 1920, 1080, spp=16, seed=37, engine=_abi.ENGINE_MEGAKERNEL)
    b, rb = render_gpu(s, c, smp, 1920, 1080, spp=16, seed=37, engine=_abi.ENGINE_WAVEFRONT)
    assert ra == rb
    same_buffer(a, b)


def test_side_stream_deep_bvh_spill(gpu, monkeypatch):
    """A chunk small enough for the side stream (shadow passes beside the next closest-hit pass) on a
    1M-triangle BVH whose traversals spill past the 16 LDS stack entries: the shadow kernels' spill
    columns are their own, so the Buffer equals the one-stream render bit for bit."""
    s, c, smp = scenes.bunny_frame(1_000_000)
    smp.MaxBounces = 3
    w, h = 480, 270
    monkeypatch.setenv("PT_SIDE_STREAM", "0")
    a, ra = render_gpu(s, c, smp, w, h, spp=4, seed=41, engine=_abi.ENGINE_WAVEFRONT)
    monkeypatch.setenv("PT_SIDE_STREAM", "1")
    b, rb = render_gpu(s, c, smp, w, h, spp=4, seed=41, engine=_abi.ENGINE_WAVEFRONT)
    assert ra == rb
    same_buffer(a, b)


# ---- adaptive / firefly phases of RenderParallel (Renderer.cs:340-537), wavefront engine
def test_adaptive_phase(gpu):
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 4
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=2, passes=2, seed=21, engine=_abi.ENGINE_WAVEFRONT,
                                adaptive=3)
    assert (g.N == 2 * (1 + 3)).all()   # one averaged sample + 3 individual samples per pass
    check(g, gr, o, orr)


def test_firefly_phase(gpu):
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 4
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=1, passes=3, seed=23, engine=_abi.ENGINE_WAVEFRONT,
                                firefly=4)
    assert (g.N >= 3).all() and (g.N > 3).any(), "no firefly candidates: the test scene exercises nothing"
    check(g, gr, o, orr)   # candidate choice and the IsFirefly stop: N equal on every pixel


def test_serial_render_twin(gpu):
    """Renderer.Render (NumCPU == 1, Renderer.cs:80-198) on the GPU (PT_PASS_SERIAL): per-pixel
    adaptive samples when the deviation reaches 1 and firefly samples when it then exceeds 1,
    against the oracle's Render: M, V, N and the ray count."""
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 4
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=1, passes=3, seed=29, engine=_abi.ENGINE_WAVEFRONT,
                                adaptive=3, firefly=4, serial=True)
    plain = render_gpu(s, c, smp, 64, 48, spp=1, passes=3, seed=29, engine=_abi.ENGINE_WAVEFRONT)[0]
    extra = g.N - plain.N
    assert (extra > 0).any() and (extra == 0).any(), "the scene must exercise both branches"
    check(g, gr, o, orr)


def test_serial_render_example3(gpu):
    """The reference's default scene (Example.example3: AdaptiveSamples 32, FireflySamples 64) through
    Render rather than RenderParallel; 48x32, 2 passes, against the oracle."""
    s, c, smp = scenes.example3()
    g, gr, o, orr = render_both(s, c, smp, 48, 32, spp=4, passes=2, seed=5, engine=_abi.ENGINE_WAVEFRONT,
                                adaptive=32, firefly=64, serial=True)
    check(g, gr, o, orr)


def test_extra_phases_unsupported_on_megakernel(gpu):
    s, c, smp = scenes.gopher3()
    with pytest.raises(_abi.PTError):
        render_gpu(s, c, smp, 32, 32, spp=1, engine=_abi.ENGINE_MEGAKERNEL, adaptive=1)


def test_rccl_gather_single_rank(gpu):
    """pt_comm_unique_id / pt_comm_init / pt_comm_gather (the RCCL ncclReduce of M, V, N that
    assembles a multi-GPU frame) on a one-rank communicator: the gathered Buffer is the
    rendered one, bit for bit.  A 1-GPU box cannot host two RCCL ranks; the N-rank sum
    itself is covered by test_distributed.py (gloo) and test_tiles_shard_equals_full."""
    from ptsharp_amd import Renderer
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 3
    w, h = 80, 70
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    try:
        r.SamplesPerPixel = 2
        r.Seed = 31
        r.Tiles = tiles_for_rank(w, h, 0, 2)   # a rank's share: the other tiles stay zero
        r.RenderParallel()
        before = r.ReadBuffer()
        M, V, N = before.M.copy(), before.V.copy(), before.N.copy()
        assert (N > 0).any() and (N == 0).any()
        r.CommInit(1, 0, Renderer.CommUniqueId())
        r.Gather(0)
        after = r.ReadBuffer()
        assert np.array_equal(after.N, N)
        assert np.array_equal(after.M, M)
        assert np.array_equal(after.V, V)
        r.RenderParallel()   # the context keeps rendering after a gather
        assert (r.ReadBuffer().N == 2 * N).all()
    finally:
        r.close()


@pytest.mark.parametrize("form", ["direct", "scan"])
@pytest.mark.parametrize("name", ["mesh", "gopher3", "gopher3_env", "textured"])
def test_shade_forms(gpu, monkeypatch, form, name):
    """Both forms of k_wf_shade forced at every depth (PT_SHADE_FORM): the direct form and
    the SCAN form (claim 8 x 256 slots, list the ones with work, shade the list) agree
    with the oracle, on a black environment (misses dropped from the list), a constant
    coloured one and a textured one (misses listed and shaded)."""
    from ptsharp_amd import Colour
    monkeypatch.setenv("PT_SHADE_FORM", form)
    if name == "mesh":
        s, c, smp = scenes.bunny_frame(4000, seed=9)
    elif name == "textured":
        s, c, smp = scenes.textured()
    else:
        s, c, smp = scenes.gopher3()
        smp.MaxBounces = 4
        if name == "gopher3_env":
            s.Color = Colour(0.3, 0.5, 0.7)
    g, gr, o, orr = render_both(s, c, smp, 64, 48, spp=2, passes=2, seed=41, engine=_abi.ENGINE_WAVEFRONT)
    check(g, gr, o, orr)


@pytest.mark.parametrize("name", ["mesh", "gopher3", "textured"])
def test_refill_kernels_match_lockstep(gpu, monkeypatch, name):
    """The per-lane refill traversal kernels (k_wf_trace_lanes / k_wf_shadow_lanes, PT_LANES=1)
    and the lockstep ones (PT_LANES=0) visit the same nodes in the same order: the same
    rays and the same Buffer bits; and the refill kernels agree with the oracle where they are
    not the default (gopher3)."""
    def scene():
        if name == "mesh":
            return scenes.bunny_frame(4000, seed=9)
        if name == "textured":
            return scenes.textured()
        s, c, smp = scenes.gopher3()
        smp.MaxBounces = 4
        return s, c, smp
    out = {}
    for lanes in ("0", "1"):
        monkeypatch.setenv("PT_LANES", lanes)
        s, c, smp = scene()
        out[lanes] = render_gpu(s, c, smp, 64, 48, spp=2, passes=2, seed=43, engine=_abi.ENGINE_WAVEFRONT)
    (a, ra), (b, rb) = out["0"], out["1"]
    assert ra == rb
    same_buffer(a, b)
    if name == "gopher3":
        s, c, smp = scene()
        o, orr = O.render(O.OracleScene(s), c, smp, 64, 48, 2, passes=2, seed=43)
        check(b, rb, o, orr)


# ---- pass batches (pt_pass_params.passes): K passes in one call == K calls, bit for bit
def _batched_vs_separate(s, c, smp, w, h, spp, k, tiles=None, engine=_abi.ENGINE_WAVEFRONT, **kw):
    from ptsharp_amd import Renderer
    out = []
    for batched in (False, True):
        r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
        try:
            r.SamplesPerPixel, r.Seed, r.Tiles, r.Engine = spp, 97, tiles, engine
            for name, v in kw.items():
                setattr(r, name, v)
            r.RenderParallel()   # one plain pass first: the batch continues the pass numbering
            rays = r.Stats().rays
            if batched:
                r.RenderPasses(k)
                rays += r.Stats().rays
            else:
                for _ in range(k):
                    r.RenderParallel()
                    rays += r.Stats().rays
            b = r.ReadBuffer()
            out.append((b.M.copy(), b.V.copy(), b.N.copy(), rays, r.Stats().passes))
        finally:
            r.close()
    (m0, v0, n0, r0, p0), (m1, v1, n1, r1, p1) = out
    assert r0 == r1 and p0 == p1 == k + 1
    assert np.array_equal(n0, n1) and np.array_equal(m0, m1) and np.array_equal(v0, v1)
    return n1


def test_pass_batch_equals_separate_passes(gpu):
    s, c, smp = scenes.bunny_frame(4000, seed=9)
    smp.MaxBounces = 3
    n = _batched_vs_separate(s, c, smp, 160, 120, 4, 5)
    assert (n == 6).all()


def test_pass_batch_tile_share_and_oracle(gpu):
    """One rank's eighth of a frame, 8 passes as one batch: the separate passes' bits, and the
    oracle's Buffer (the pass numbering of the batch is the reference's pass loop, Renderer.cs:709)."""
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 4
    w, h = 96, 64
    tiles = tiles_for_rank(w, h, 3, 8)
    _batched_vs_separate(s, c, smp, w, h, 1, 8, tiles=tiles)
    from parity import check
    from ptsharp_amd import Renderer
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    try:
        r.SamplesPerPixel, r.Seed, r.Tiles, r.Engine = 1, 5, tiles, _abi.ENGINE_WAVEFRONT
        r.RenderPasses(3)
        rays = r.Stats().rays
        g = r.ReadBuffer()
    finally:
        r.close()
    o, orays = O.render(O.OracleScene(s), c, smp, w, h, 1, passes=3, seed=5, tiles=tiles)
    check(g, rays, o, orays)


def test_pass_batch_many_chunks(gpu, monkeypatch):
    """A batch larger than the queues: several chunks, each holding parts of several passes."""
    monkeypatch.setenv("PT_WF_MAX_CAP", str(1 << 20))
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 2
    _batched_vs_separate(s, c, smp, 320, 180, 4, 6)


def test_pass_batch_split_by_memory_budget(gpu, monkeypatch):
    """A batch whose accumulator sets exceed the memory budget runs as consecutive sub-batches (here
    forced to 2 passes per launch sequence: 7 = 2 + 2 + 2 + 1), still the separate passes' bits and the
    ray count summed over all 7 (a large K used to ask for K full-frame accumulator sets)."""
    monkeypatch.setenv("PT_BATCH_MAX_PASSES", "2")
    s, c, smp = scenes.bunny_frame(4000, seed=9)
    smp.MaxBounces = 2
    n = _batched_vs_separate(s, c, smp, 96, 64, 2, 7)
    assert (n == 8).all()


@pytest.mark.parametrize("case", ["megakernel", "stratified", "adaptive", "firefly"])
def test_pass_batch_fallbacks(gpu, case):
    """Passes that cannot share one batch (megakernel engine, stratified, adaptive / firefly phases)
    run one by one inside the call: still the separate calls' bits."""
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 3
    kw, engine, spp = {}, _abi.ENGINE_WAVEFRONT, 2
    if case == "megakernel":
        engine = _abi.ENGINE_MEGAKERNEL
    elif case == "stratified":
        kw, spp = {"StratifiedSampling": True}, 4
    elif case == "adaptive":
        kw = {"AdaptiveSamples": 2}
    else:
        kw = {"FireflySamples": 3}
    _batched_vs_separate(s, c, smp, 64, 48, spp, 3, engine=engine, **kw)


def _render_stats(s, c, smp, w, h, spp, seed, tiles=None):
    """One wavefront RenderParallel: (Buffer copy, rays, tail hand-offs of the pass)."""
    from ptsharp_amd import Renderer
    from ptsharp_amd.renderer import Buffer
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    try:
        r.SamplesPerPixel, r.Seed, r.Tiles, r.Engine = spp, seed, tiles, _abi.ENGINE_WAVEFRONT
        r.RenderParallel()
        st = r.Stats()
        b = r.ReadBuffer()
        out = Buffer(w, h)
        out.M, out.V, out.N = b.M.copy(), b.V.copy(), b.N.copy()
        return out, int(st.rays), int(st.tail_handoffs)
    finally:
        r.close()


@pytest.mark.parametrize("name", ["mesh1m", "mixed4k"])
def test_shadow_tail_handoffs_forced(gpu, monkeypatch, name):
    """The shadow refill kernel's tail (idle lanes take stack entries of busy lanes' rays) forced to run
    all pass long (PT_SHADOW_TAIL=early: a wave refills only when every lane is idle and hands off from
    its first claim on).  mixed4k is the routed split (C5's 1M-triangle mesh + SDF + Volume at 4K, the
    scene where round 4's helper read the borrowed ray for the heavy-box test): the hand-off count is
    non-zero, and the Buffer equals the default tail's and the lockstep kernels' (PT_LANES=0) bit for
    bit and the oracle's within the parity bar.  mesh1m: the lean instantiation on the C4 frame."""
    if name == "mixed4k":
        s, c, smp = scenes.mixed(1_000_000)
        w, h, tiles = 3840, 2160, tiles_for_rank(3840, 2160, 5, 1024)
    else:
        s, c, smp = scenes.bunny_frame(1_000_000)
        w, h, tiles = 1920, 1080, tiles_for_rank(1920, 1080, 9, 256)
    monkeypatch.setenv("PT_SHADOW_TAIL", "early")
    e, re_, he = _render_stats(s, c, smp, w, h, 2, 4242, tiles)
    assert he > 0, "the forced tail handed nothing off"
    monkeypatch.delenv("PT_SHADOW_TAIL")
    d, rd, hd = _render_stats(s, c, smp, w, h, 2, 4242, tiles)
    assert re_ == rd
    same_buffer(e, d)
    if name == "mixed4k":
        monkeypatch.setenv("PT_LANES", "0")
        l, rl, _ = _render_stats(s, c, smp, w, h, 2, 4242, tiles)
        monkeypatch.delenv("PT_LANES")
        assert rl == re_
        same_buffer(e, l)
        o, orr = O.render(O.OracleScene(s), c, smp, w, h, 2, passes=1, seed=4242, tiles=tiles)
        check(e, re_, o, orr)


@pytest.mark.parametrize("name", ["gopher3", "materialspheres", "simplesphere", "example1"])
def test_linear_kernels_match_lockstep(gpu, monkeypatch, name):
    """The linear kernels (k_wf_trace_linear / k_wf_shadow_linear: a few analytic records and planes, no
    triangles) test the same records in the same order as the lockstep traversal kernels (PT_LINEAR=0): the
    same rays, the same counted-pass counters and the same Buffer bits.  The four scenes cover planes,
    refraction (transparent / clear spheres), a cube light's neighbours, a thin-lens camera and
    SpecularModeFirst."""
    from ptsharp_amd import Renderer
    out = {}
    for lin in ("0", "1"):
        if lin == "0":
            monkeypatch.setenv("PT_LINEAR", "0")
        else:
            monkeypatch.delenv("PT_LINEAR", raising=False)
        s, c, smp = getattr(scenes, name)()
        smp.MaxBounces = min(smp.MaxBounces, 6)
        b, rays, _ = _render_stats(s, c, smp, 64, 48, 2, 41)
        r = Renderer.NewRenderer(s, c, smp, 32, 24, True, device=0)
        try:
            r.SamplesPerPixel, r.Seed, r.Engine = 1, 5, _abi.ENGINE_WAVEFRONT
            ctr = r.RenderCounted()
            counts = (int(ctr.rays), int(ctr.prims_tested), int(ctr.shadow_rays), int(ctr.shadow_prims),
                      int(ctr.lit_shadow_rays))
        finally:
            r.close()
        out[lin] = (b, rays, counts)
    (a, ra, ca), (b, rb, cb) = out["0"], out["1"]
    assert ra == rb and ra > 0
    assert ca == cb
    same_buffer(a, b)
