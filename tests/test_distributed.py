"""Multi-rank path on CPU (gloo, world_size 2): each rank renders its interleaved
32x32 tiles (ptsharp_amd.tiles_for_rank), the disjoint Welford buffers are
sum-reduced onto rank 0 — the same gather pt_comm_gather performs with RCCL on
the GPUs — and the result is bit-identical to the unsharded render, because
every pixel's random stream is keyed by pixel, not by rank.
The oracle stands in for the per-rank GPU renderer here (no GPU on this host)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP, SEED = 72, 40, 1, 77


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from ptsharp_amd import scenes
    s, c, smp = scenes.gopher3()
    smp.MaxBounces = 3
    return s, c, smp


def _worker(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import oracle_lib as O
    from ptsharp_amd import tiles_for_rank
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        # control plane as bench.py uses it: rank 0's 128-byte communicator id reaches every rank
        uid = [bytes(range(128)) if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        assert uid[0] == bytes(range(128))
        s, c, smp = _scene()
        buf, rays = O.render(O.OracleScene(s), c, smp, W, H, SPP, seed=SEED, tiles=tiles_for_rank(W, H, rank, world),
                             threads=2)
        M, V, N = (torch.from_numpy(a.copy()) for a in (buf.M, buf.V, buf.N))
        for t in (M, V, N):
            dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
        r = torch.tensor([rays], dtype=torch.int64)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        el = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        if rank == 0:
            np.savez(os.path.join(outdir, "gathered.npz"), M=M.numpy(), V=V.numpy(), N=N.numpy(), rays=r.item(),
                     maxel=el.item())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_tile_sharded_gather_equals_full_render(world):
    import oracle_lib as O
    s, c, smp = _scene()
    full, rays = O.render(O.OracleScene(s), c, smp, W, H, SPP, seed=SEED)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        g = np.load(os.path.join(d, "gathered.npz"))
        assert int(g["rays"]) == rays
        assert float(g["maxel"]) == float(world)
        assert np.array_equal(g["N"], full.N)
        assert np.array_equal(g["M"], full.M)
        assert np.array_equal(g["V"], full.V)
