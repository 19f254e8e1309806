"""Host-side paths of the drop-in on the GPU: resuming from a saved Buffer (pt_write_buffer),
the single-process communicator (pt_comm_init_all / pt_comm_gather_all) and repeated
gathers, and the tile read/write layout.  The world-2 multi-process render lives in
test_zz_gpu_multiprocess.py, which collects last (it spawns processes)."""
import numpy as np
import pytest

from parity import same_buffer
from ptsharp_amd import Renderer, _abi, scenes, tiles_for_rank

pytestmark = pytest.mark.gpu


def _scene():
    s, c, smp = scenes.bunny_frame(4000, seed=9)
    smp.MaxBounces = 3
    return s, c, smp


def _render(w, h, passes, seed=61, tiles=None, spp=2, engine=_abi.ENGINE_WAVEFRONT):
    s, c, smp = _scene()
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    r.SamplesPerPixel, r.Seed, r.Tiles, r.Engine = spp, seed, tiles, engine
    for _ in range(passes):
        r.RenderParallel()
    b = r.ReadBuffer()
    out = (b.M.copy(), b.V.copy(), b.N.copy())
    r.close()
    return out


class _Buf:
    def __init__(self, m, v, n):
        self.M, self.V, self.N = m, v, n


def test_write_buffer_resumes_iterative_render(gpu):
    """3 passes in one go == 2 passes, Buffer saved, a new context loads it and renders pass 3."""
    w, h = 96, 64
    full = _Buf(*_render(w, h, 3))
    m, v, n = _render(w, h, 2)
    s, c, smp = _scene()
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    try:
        r.SamplesPerPixel, r.Seed = 2, 61
        r.LoadBuffer(_Buf(m, v, n), passes_done=2)
        r.RenderParallel()
        b = r.ReadBuffer()
        same_buffer(_Buf(b.M.copy(), b.V.copy(), b.N.copy()), full)
    finally:
        r.close()


def test_comm_init_all_and_repeated_gathers(gpu):
    """pt_comm_init_all over one context (the .NET host's single-process form), gathers after every
    pass, and the root's next pass clearing the pixels outside its tiles: after gather → pass on a
    tile subset, only that subset holds samples, and those are the 2-pass subset render's bits."""
    w, h = 96, 64
    tiles = tiles_for_rank(w, h, 1, 2)
    s, c, smp = _scene()
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    try:
        r.SamplesPerPixel, r.Seed = 2, 61
        Renderer.CommInitAll([r])
        r.Tiles = None
        r.RenderParallel()                 # pass 1 over the whole frame
        Renderer.GatherAll([r], 0)
        assert (r.ReadBuffer().N == 1).all()
        r.Tiles = tiles
        r.RenderParallel()                 # pass 2 on the subset: the rest is cleared first
        Renderer.GatherAll([r], 0)
        b = r.ReadBuffer()
        got = _Buf(b.M.copy(), b.V.copy(), b.N.copy())
    finally:
        r.close()
    ref = _Buf(*_render(w, h, 2, tiles=tiles))
    same_buffer(got, ref)
    assert (got.N == 0).any() and (got.N == 2).any()


def test_read_write_tiles_layout(gpu):
    """pt_read_tiles packs a tile row-major (edge tiles: zeros outside the image); pt_write_tiles
    puts packed tiles back; a render's tiles moved into a fresh context reproduce its Buffer."""
    w, h = 100, 70                       # 4 x 3 tiles, the last column and row partial
    s, c, smp = _scene()
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    q = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    try:
        r.SamplesPerPixel, r.Seed = 2, 5
        r.RenderParallel()
        b = r.ReadBuffer()
        full = _Buf(b.M.copy(), b.V.copy(), b.N.copy())
        tiles = np.array([11, 0, 5, 3], np.int32)
        M, V, N = r.ReadTiles(tiles)
        for k, t in enumerate(tiles):
            x0, y0 = (t % 4) * 32, (t // 4) * 32
            x1, y1 = min(x0 + 32, w), min(y0 + 32, h)
            assert np.array_equal(M[k, :y1 - y0, :x1 - x0], full.M[y0:y1, x0:x1])
            assert np.array_equal(N[k, :y1 - y0, :x1 - x0], full.N[y0:y1, x0:x1])
            assert (N[k, y1 - y0:, :] == 0).all() and (N[k, :, x1 - x0:] == 0).all()
        all_t = np.arange(12, dtype=np.int32)
        q.WriteTiles(all_t, *r.ReadTiles(all_t))
        b2 = q.ReadBuffer()
        same_buffer(_Buf(b2.M.copy(), b2.V.copy(), b2.N.copy()), full)
    finally:
        r.close()
        q.close()


def test_resume_then_firefly_pass_clears_foreign_pixels(gpu):
    """A rank that resumes from the whole checkpoint (LoadBuffer of the full frame) and then runs a
    firefly pass on its tile subset: the other ranks' pixels are cleared before the pass, so the
    firefly snapshot (all-reduced over the communicator) and the Buffer hold each pixel on its owner
    only — the same bits as a rank that rendered its tiles all along (pt_write_buffer
    never marked the Buffer as holding foreign pixels, and the snapshot then counted them twice)."""
    w, h = 64, 48
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 4
    tiles = tiles_for_rank(w, h, 0, 2)

    def ctx():
        r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
        r.SamplesPerPixel, r.Seed, r.Engine = 1, 23, _abi.ENGINE_WAVEFRONT
        return r

    full = ctx()
    try:
        full.RenderParallel()
        full.RenderParallel()
        b = full.ReadBuffer()
        ck = _Buf(b.M.copy(), b.V.copy(), b.N.copy())
    finally:
        full.close()
    out = []
    for resume in (False, True):
        r = ctx()
        try:
            r.Tiles = tiles
            r.CommInit(1, 0, Renderer.CommUniqueId())
            if resume:
                r.LoadBuffer(ck, passes_done=2)
            else:
                r.RenderParallel()
                r.RenderParallel()
            r.FireflySamples = 4
            r.RenderParallel()
            b = r.ReadBuffer()
            out.append(_Buf(b.M.copy(), b.V.copy(), b.N.copy()))
        finally:
            r.close()
    own = np.zeros((h, w), bool)
    for t in tiles:
        own[(t // 2) * 32:(t // 2) * 32 + 32, (t % 2) * 32:(t % 2) * 32 + 32] = True
    assert (out[1].N[~own] == 0).all(), "foreign pixels survived the resume"
    assert (out[0].N[own] > 3).any(), "no firefly samples: the test exercises nothing"
    same_buffer(out[1], out[0])


def test_contexts_driven_from_threads_equal_full_frame(gpu):
    """bench.py's one-process form drives each context from its own host thread (bench._each).  Two
    contexts on device 0 render the two halves of an interleaved tile split concurrently, in pass
    batches of 2; context 0 takes context 1's tiles (pt_read_tiles → pt_write_tiles, the host form of
    the gather) and must hold the single-context full-frame render, bit for bit."""
    import bench
    w, h = 160, 96
    s, c, smp = _scene()
    rs = []
    try:
        for k in range(2):
            r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
            r.SamplesPerPixel, r.Seed, r.Engine = 2, 61, _abi.ENGINE_WAVEFRONT
            r.Tiles = tiles_for_rank(w, h, k, 2)
            rs.append(r)
        bench._each(rs, lambda i, x: x.RenderPasses(2))
        bench._each(rs, lambda i, x: x.Synchronize())
        t1 = tiles_for_rank(w, h, 1, 2)
        rs[0].WriteTiles(t1, *rs[1].ReadTiles(t1))
        b = rs[0].ReadBuffer()
        got = _Buf(b.M.copy(), b.V.copy(), b.N.copy())
    finally:
        for r in rs:
            r.close()
    same_buffer(got, _Buf(*_render(w, h, 2)))


def test_bench_group_form_one_gpu(gpu, tmp_path):
    """`bench.py --group --gpus 1`: the one-process multi-GPU form (pt_comm_init_all, one host thread per
    device, pt_comm_gather_all inside the timed region) on this box's one GPU; the JSON line reports it,
    and the gathered Buffer passes the bit check."""
    import json

    import bench
    out = tmp_path / "b.json"
    bench.main(["--group", "--gpus", "1", "--steps", "2", "--warmup", "1", "--spp", "2", "--cpu-seconds", "0",
                "--no-parity", "--width", "256", "--height", "128", "--tris", "20000", "--mesh-source", "generator",
                "--json-out", str(out)])
    j = json.loads(out.read_text())
    assert j["n_gpus"] == 1 and j["launch"].startswith("one process, one host thread")
    assert j["config"]["gather_check"]["bit_exact"] is True
    assert "pt_comm_gather_all" in j["config"]["parallelism"]
    assert j["value"] > 0


def test_group_pass_equals_plain_pass(gpu):
    """The group form's render (pt_comm_init_all over one context, passes issued from a worker thread,
    pt_comm_gather_all) leaves the Buffer a plain context leaves, bit for bit."""
    import bench
    w, h = 128, 96
    s, c, smp = _scene()
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    try:
        r.SamplesPerPixel, r.Seed, r.Engine = 2, 61, _abi.ENGINE_WAVEFRONT
        Renderer.CommInitAll([r])
        bench._each([r, r], lambda i, x: None)   # (the helper's threaded branch, no work)
        import threading
        t = threading.Thread(target=lambda: (r.RenderParallel(), r.RenderParallel()))
        t.start()
        t.join()
        Renderer.GatherAll([r], 0)
        b = r.ReadBuffer()
        got = _Buf(b.M.copy(), b.V.copy(), b.N.copy())
    finally:
        r.close()
    same_buffer(got, _Buf(*_render(w, h, 2)))


def test_single_context_resume_keeps_restored_pixels(gpu):
    """A lone context (no communicator) that loads a checkpoint and then renders tile subsets one after
    another keeps every restored pixel outside the current subset (pt_write_buffer used to
    mark the whole checkpoint foreign, and the first subset pass cleared the rest of the frame)."""
    w, h = 96, 64
    m, v, n = _render(w, h, 2)
    s, c, smp = _scene()
    r = Renderer.NewRenderer(s, c, smp, w, h, True, device=0)
    try:
        r.SamplesPerPixel, r.Seed, r.Engine = 2, 61, _abi.ENGINE_WAVEFRONT
        r.LoadBuffer(_Buf(m, v, n), passes_done=2)
        for k in range(2):          # pass 3 over the frame's two tile halves, one subset after the other
            r.Tiles = tiles_for_rank(w, h, k, 2)
            r.RenderParallel()
            r._pass -= 1            # both halves are pass 3 of the frame
        r._pass += 1
        b = r.ReadBuffer()
        got = _Buf(b.M.copy(), b.V.copy(), b.N.copy())
    finally:
        r.close()
    same_buffer(got, _Buf(*_render(w, h, 3)))
