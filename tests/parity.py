"""Shared GPU-vs-oracle comparison helpers (parity bar from SURVEY.md §8c)."""
from __future__ import annotations

import numpy as np

import oracle_lib as O
from ptsharp_amd import Renderer
from ptsharp_amd.renderer import Buffer

# Per-pixel linear tolerance and the fraction of pixels that must meet it; the
# residue is fp32-colour rounding plus rare fp64 transcendental (OCML vs glibc)
# last-bit differences that send a single sample down another path.
REL_TOL = 1e-3
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


def compare(gpu_m: np.ndarray, ref_m: np.ndarray):
    err = np.abs(gpu_m - ref_m)
    ok = (err <= REL_TOL * np.maximum(1.0, np.abs(ref_m))).all(axis=2)
    return float(ok.mean()), float(err.max()), psnr8(gpu_m, ref_m)


def render_gpu(scene, camera, sampler, w, h, spp, passes=1, seed=0, stratified=False, tiles=None, device=0, engine=0,
               adaptive=0, firefly=0):
    r = Renderer.NewRenderer(scene, camera, sampler, w, h, True, device=device)
    r.SamplesPerPixel = spp
    r.AdaptiveSamples = adaptive
    r.FireflySamples = firefly
    r.StratifiedSampling = stratified
    r.Seed = seed
    r.Tiles = tiles
    r.Engine = engine
    rays = 0
    for _ in range(passes):
        r.RenderParallel()
        rays += r.Stats().rays
    buf = r.ReadBuffer()
    out = Buffer(w, h)
    out.M, out.V, out.N = buf.M.copy(), buf.V.copy(), buf.N.copy()
    r.close()
    return out, rays


def render_both(scene, camera, sampler, w, h, spp, passes=1, seed=0, stratified=False, tiles=None, engine=0,
                adaptive=0, firefly=0):
    g, grays = render_gpu(scene, camera, sampler, w, h, spp, passes, seed, stratified, tiles, engine=engine,
                          adaptive=adaptive, firefly=firefly)
    o, orays = O.render(O.OracleScene(scene), camera, sampler, w, h, spp, passes=passes, seed=seed,
                        stratified=stratified, tiles=tiles, adaptive=adaptive, firefly=firefly)
    return g, grays, o, orays
