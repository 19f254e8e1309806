"""Shared GPU-vs-oracle comparison helpers and the parity bar (tightened).

The GPU computes colour in fp64 like the reference's Colour (Colour.cs:10-12) and sums
terms in an order-independent fixed-point form (ptsharp_amd/csrc/pt_accum.h), so a GPU
pass differs from the oracle's recursion only in the fp64 rounding order of its colour
arithmetic.  The bar:
  * Scene.Intersect counts equal (integer work is exact);
  * Welford sample counts N equal on every pixel;
  * M and V (Buffer.cs:33-44) within REL_TOL·max(1, |ref|) on >= MIN_FRACTION_OK of the
    pixels (the residue allowed for: a last-bit difference between the GPU's and glibc's
    fp64 transcendentals that sends one sample elsewhere; none is expected);
  * PSNR >= 50 dB on the 8-bit Buffer.Image bytes (north_star's bar).
"""
from __future__ import annotations

import numpy as np

import oracle_lib as O
from ptsharp_amd import Renderer
from ptsharp_amd.renderer import Buffer

REL_TOL = 1e-9
MIN_FRACTION_OK = 0.999
MIN_PSNR_DB = 50.0


def image8(M: np.ndarray) -> np.ndarray:
    """Buffer.Image(ColorChannel) bytes (Buffer.cs:155-160)."""
    b = Buffer(M.shape[1], M.shape[0])
    b.M = M
    return b.Image()


def psnr8(a: np.ndarray, b: np.ndarray) -> float:
    mse = np.mean((image8(a).astype(np.float64) - image8(b).astype(np.float64)) ** 2)
    return float("inf") if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


def within(gpu: np.ndarray, ref: np.ndarray, rel_tol: float = REL_TOL):
    """Fraction of pixels whose three channels are within rel_tol·max(1, |ref|), and the max |error|."""
    err = np.abs(gpu - ref)
    ok = (err <= rel_tol * np.maximum(1.0, np.abs(ref))).all(axis=2)
    return float(ok.mean()), float(err.max())


def compare(gpu_m: np.ndarray, ref_m: np.ndarray, rel_tol: float = REL_TOL):
    frac, maxerr = within(gpu_m, ref_m, rel_tol)
    return frac, maxerr, psnr8(gpu_m, ref_m)


def check(g, grays, o, orays, exact=False):
    """The parity bar (module docstring) for a GPU Buffer g vs an oracle Buffer o."""
    assert grays == orays, f"Scene.Intersect count: gpu {grays} vs oracle {orays}"
    assert np.array_equal(g.N, o.N), f"sample counts N differ on {int((g.N != o.N).sum())} pixels"
    if exact:
        assert np.array_equal(g.M, o.M), f"M max err {np.abs(g.M - o.M).max()}"
        assert np.array_equal(g.V, o.V), f"V max err {np.abs(g.V - o.V).max()}"
        return
    fm, em = within(g.M, o.M)
    fv, ev = within(g.V, o.V)
    assert fm >= MIN_FRACTION_OK, f"M: only {fm:.5f} of pixels within {REL_TOL:g} (max err {em:.3g})"
    assert fv >= MIN_FRACTION_OK, f"V: only {fv:.5f} of pixels within {REL_TOL:g} (max err {ev:.3g})"
    psnr = psnr8(g.M, o.M)
    assert psnr >= MIN_PSNR_DB, f"PSNR {psnr:.2f} dB"


def same_buffer(a, b):
    """Bit-identical Welford state (determinism, shard and engine equality)."""
    assert np.array_equal(a.N, b.N), f"N differs on {int((a.N != b.N).sum())} pixels"
    assert np.array_equal(a.M, b.M), f"M max diff {np.abs(a.M - b.M).max()}"
    assert np.array_equal(a.V, b.V), f"V max diff {np.abs(a.V - b.V).max()}"


def render_gpu(scene, camera, sampler, w, h, spp, passes=1, seed=0, stratified=False, tiles=None, device=0, engine=0,
               adaptive=0, firefly=0, serial=False):
    """`passes` RenderParallel calls (serial: Render calls, the NumCPU == 1 twin)."""
    r = Renderer.NewRenderer(scene, camera, sampler, w, h, not serial, device=device)
    r.SamplesPerPixel = spp
    r.AdaptiveSamples = adaptive
    r.FireflySamples = firefly
    r.StratifiedSampling = stratified
    r.Seed = seed
    r.Tiles = tiles
    r.Engine = engine
    rays = 0
    for _ in range(passes):
        if serial:
            r.Render()
        else:
            r.RenderParallel()
        rays += r.Stats().rays
    buf = r.ReadBuffer()
    out = Buffer(w, h)
    out.M, out.V, out.N = buf.M.copy(), buf.V.copy(), buf.N.copy()
    r.close()
    return out, rays


def render_both(scene, camera, sampler, w, h, spp, passes=1, seed=0, stratified=False, tiles=None, engine=0,
                adaptive=0, firefly=0, serial=False):
    g, grays = render_gpu(scene, camera, sampler, w, h, spp, passes, seed, stratified, tiles, engine=engine,
                          adaptive=adaptive, firefly=firefly, serial=serial)
    o, orays = O.render(O.OracleScene(scene), camera, sampler, w, h, spp, passes=passes, seed=seed,
                        stratified=stratified, tiles=tiles, adaptive=adaptive, firefly=firefly, serial=serial)
    return g, grays, o, orays
