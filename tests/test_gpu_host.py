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
        M, V, N = _render(W, H, 2, seed=71, tiles=tiles_for_rank(W, H, rank, world))
        t = [torch.from_numpy(a) for a in (M, V, N)]
        for x in t:
            dist.reduce(x, dst=0, op=dist.ReduceOp.SUM)
        if rank == 0:
            np.savez(os.path.join(outdir, "gathered.npz"), M=t[0].numpy(), V=t[1].numpy(), N=t[2].numpy())
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_gpu_equal_single_render(gpu):
    """World 2: each process renders its interleaved tiles through libptsharp_hip on the box's GPU,
    gloo sums the Buffers (the reduce pt_comm_gather does over RCCL between GPUs), and the result
    is the 1-process render's Buffer bit for bit."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        g = np.load(os.path.join(d, "gathered.npz"))
        got = _Buf(g["M"], g["V"], g["N"])
    ref = _Buf(*_render(200, 120, 2, seed=71))
    same_buffer(got, ref)
