#!/usr/bin/env python3
"""Parity diagnostics for one scene: GPU vs oracle rays, N, M and V for a few pass settings.
Usage: python tools/debug_parity.py example3 64 48 4 "0,0 32,0 0,64 32,64" [engine]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
from parity import render_gpu, within  # noqa: E402
from ptsharp_amd import scenes  # noqa: E402

name, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
settings = [tuple(int(x) for x in s.split(",")) for s in sys.argv[5].split()]
engine = int(sys.argv[6]) if len(sys.argv) > 6 else 2
for ad, ff in settings:
    s, c, smp = scenes.SCENES[name]()
    g, gr = render_gpu(s, c, smp, w, h, spp, passes=1, seed=3, engine=engine, adaptive=ad, firefly=ff)
    o, orr = O.render(O.OracleScene(s), c, smp, w, h, spp, passes=1, seed=3, adaptive=ad, firefly=ff)
    dn = g.N != o.N
    fm, em = within(g.M, o.M)
    print(f"adaptive={ad} firefly={ff}: rays gpu {gr} oracle {orr} (diff {gr - orr}); N differ on {int(dn.sum())} px "
          f"(gpu N sum {int(g.N.sum())}, oracle {int(o.N.sum())}); M within 1e-9 on {fm:.5f}, max err {em:.3g}", flush=True)
    if dn.any():
        ys, xs = np.nonzero(dn)
        for y, x in list(zip(ys, xs))[:5]:
            print(f"   px ({x},{y}): N gpu {g.N[y, x]} oracle {o.N[y, x]}  M gpu {g.M[y, x]} oracle {o.M[y, x]}")
