#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the CPU oracle (oracle/pt_oracle.cpp).

The reference ships no golden vectors and cannot run here
(C#/.NET 9, unseedable Random.Shared), so these fixtures pin the oracle's own
outputs: the RNG stream that replaces Random.Shared, primitive intersect tables,
and small seeded renders of the config scenes.  tests/test_golden.py checks the
oracle (CPU) and the GPU path against them.

Usage: python tools/make_golden.py   (rewrites tests/golden/golden_v1.npz)
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_lib as O  # noqa: E402
from ptsharp_amd import scenes  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "golden_v1.npz")

# (name, builder, overrides, width, height, spp, passes, seed)
RENDERS = [
    ("furnace", lambda: scenes.furnace(0.5), {}, 40, 30, 2, 2, 101),
    ("emitter16", lambda: scenes.emitter(16), {}, 40, 30, 1, 1, 102),
    ("emitter8", lambda: scenes.emitter(8), {}, 40, 30, 1, 1, 103),
    ("gopher3", scenes.gopher3, {"MaxBounces": 3}, 40, 30, 2, 2, 104),
    ("materialspheres", scenes.materialspheres, {"FirstHitSamples": 4, "MaxBounces": 3}, 40, 30, 2, 1, 105),
    ("simplesphere", scenes.simplesphere, {}, 40, 30, 2, 2, 106),
    ("example1", scenes.example1, {"MaxBounces": 3}, 40, 30, 2, 1, 107),
    ("bunny2k", lambda: scenes.bunny_frame(2000, seed=5), {}, 40, 30, 2, 1, 108),
]


def build(name, builder, overrides):
    s, c, smp = builder()
    for k, v in overrides.items():
        setattr(smp, k, v)
    return s, c, smp


def main():
    L = O.lib()
    out = {}
    # RNG stream
    rng = np.random.default_rng(0)
    n = 64
    seeds = rng.integers(0, 2**63, n, dtype=np.uint64)
    passes = rng.integers(0, 1000, n).astype(np.uint32)
    pixels = rng.integers(0, 1920 * 1080, n).astype(np.uint64)
    samples = rng.integers(0, 1024, n).astype(np.uint32)
    keys = np.array([L.or_camera_key(int(a), int(b), int(c), int(d)) for a, b, c, d in zip(seeds, passes, pixels, samples)],
                    dtype=np.uint64)
    draws = np.array([[L.or_draw(int(k), d) for d in range(12)] for k in keys])
    child = np.array([[L.or_child_key(int(k), c) for c in range(8)] for k in keys], dtype=np.uint64)
    light = np.array([[L.or_light_key(int(k), c) for c in range(3)] for k in keys], dtype=np.uint64)
    out.update(rng_seed=seeds, rng_pass=passes, rng_pixel=pixels, rng_sample=samples, rng_key=keys, rng_draws=draws,
               rng_child=child, rng_light=light)
    # primitive intersect table
    m = 256
    o = rng.uniform(-3, 3, (m, 3)).astype(np.float32)
    d = rng.normal(size=(m, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    prims = {
        "tri": (3, (-1, -1, 0), (1, -1, 0.2), (0, 1, -0.1), 0.0),
        "sphere": (0, (0.2, -0.1, 0.3), (0, 0, 0), (0, 0, 0), 1.3),
        "cube": (1, (-1, -0.5, -1.5), (0.8, 1.2, 0.5), (0, 0, 0), 0.0),
        "plane": (2, (0, 0.25, 0), (0, 1, 0), (0, 0, 0), 0.0),
    }
    for name, (kind, a, b, c, r) in prims.items():
        out[f"kat_{name}_t"] = np.array([L.or_prim_intersect(kind, O.f3(a), O.f3(b), O.f3(c), r, O.f3(oo), O.f3(dd))
                                         for oo, dd in zip(o, d)])
    out["kat_origin"], out["kat_dir"] = o, d
    # renders
    for name, builder, overrides, w, h, spp, npass, seed in RENDERS:
        s, c, smp = build(name, builder, overrides)
        buf, rays = O.render(O.OracleScene(s), c, smp, w, h, spp, passes=npass, seed=seed)
        out[f"render_{name}_M"] = buf.M
        out[f"render_{name}_V"] = buf.V
        out[f"render_{name}_N"] = buf.N
        out[f"render_{name}_rays"] = np.array(rays)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes)")


if __name__ == "__main__":
    main()
