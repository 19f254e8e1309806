"""Writes the C4 frame's triangles (Example.bunny's scene around the seeded 1M-triangle mesh, after
SmoothNormals / FitInside) and its camera basis for tools/bvh_quality.cpp:
int32 n; float32 v1[n][3], v2[n][3], v3[n][3]; camera p, u, v, w [3] and m.
usage: python tools/dump_c4_mesh.py OUT.bin [triangles]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ptsharp_amd import scenes  # noqa: E402


def main():
    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    scene, camera, _ = scenes.bunny_frame(n)
    fl = scene.Compile()
    with open(out, "wb") as f:
        f.write(np.int32(len(fl.tri_v1) // 3 if fl.tri_v1.ndim == 1 else len(fl.tri_v1)).tobytes())
        for a in (fl.tri_v1, fl.tri_v2, fl.tri_v3):
            f.write(np.ascontiguousarray(a, np.float32).tobytes())
        c = camera.to_c()
        for v in (c.p, c.u, c.v, c.w):
            f.write(np.array(list(v), np.float32).tobytes())
        f.write(np.float32(c.m).tobytes())


if __name__ == "__main__":
    main()
