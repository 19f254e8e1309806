"""Host-side paths of the drop-in on the GPU: resuming from a saved Buffer (pt_write_buffer),
the single-process communicator (pt_comm_init_all / pt_comm_gather_all) and repeated
gathers, and a world-2 multi-process render through libptsharp_hip (two ranks on the one
GPU of the box, their tile Buffers summed over gloo) that must equal the 1-process render
bit for bit (pixel-keyed random streams + order-independent accumulation)."""
import os
import socket
import tempfile

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


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


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


def _worker(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    os.environ["PT_WF_MAX_CAP"] = str(1 << 22)   # two contexts share the card: small queues
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        W, H = 200, 120
        s, c, smp = _scene()
        r = Renderer.NewRenderer(s, c, smp, W, H, True, device=0)
        try:
            mine = tiles_for_rank(W, H, rank, world)
            r.SamplesPerPixel, r.Seed, r.Tiles = 2, 71, mine
            for _ in range(2):
                r.RenderParallel()
            # pt_comm_gather's protocol over gloo: tile counts, then each rank's packed tiles to
            # the root, which writes them into its Buffer
            cnt = torch.tensor([len(mine)], dtype=torch.int64)
            cnts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(cnts, cnt)
            if rank != 0:
                dist.send(torch.from_numpy(np.ascontiguousarray(mine, np.int32)), dst=0)
                for a in r.ReadTiles(mine):
                    dist.send(torch.from_numpy(a), dst=0)
            else:
                for p in range(1, world):
                    n = int(cnts[p][0])
                    ids = torch.zeros(n, dtype=torch.int32)
                    dist.recv(ids, src=p)
                    parts = [torch.zeros((n, 32, 32, 3), dtype=torch.float64), torch.zeros((n, 32, 32, 3), dtype=torch.float64),
                             torch.zeros((n, 32, 32), dtype=torch.int32)]
                    for x in parts:
                        dist.recv(x, src=p)
                    r.WriteTiles(ids.numpy(), *(x.numpy() for x in parts))
                b = r.ReadBuffer()
                np.savez(os.path.join(outdir, "gathered.npz"), M=b.M, V=b.V, N=b.N)
        finally:
            r.close()
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_gpu_equal_single_render(gpu):
    """World 2: each process renders its interleaved tiles through libptsharp_hip on the box's GPU;
    the root assembles the frame with pt_comm_gather's tile-compacted protocol (counts, then packed
    tiles via pt_read_tiles / pt_write_tiles) over gloo, and the result is the 1-process render's
    Buffer bit for bit."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        g = np.load(os.path.join(d, "gathered.npz"))
        got = _Buf(g["M"], g["V"], g["N"])
    ref = _Buf(*_render(200, 120, 2, seed=71))
    same_buffer(got, ref)
