"""Throughput of the wavefront engine on the named scenes (ptsharp_amd.scenes.SCENES) at one
resolution: Mrays/s and per-kernel ms per pass.  A profiling aid beside bench.py (which
measures the BASELINE workload only).
usage: python tools/bench_scenes.py [--width 1920 --height 1080 --spp 4 --passes 3] [names...]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from ptsharp_amd import Renderer, _abi, scenes  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("names", nargs="*", default=["gopher3", "bunny70k", "textured", "sdf_zoo", "volume",
                                                 "transformed", "instances"])
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=4)
    p.add_argument("--passes", type=int, default=3)
    a = p.parse_args()
    for name in a.names:
        s, c, smp = scenes.SCENES[name]()
        r = Renderer.NewRenderer(s, c, smp, a.width, a.height, True)
        r.SamplesPerPixel = a.spp
        r.Seed = 1234
        r.Engine = _abi.ENGINE_WAVEFRONT
        r.RenderParallel()  # scene upload + warm-up
        r.Flags = _abi.PASS_KERNEL_TIMING
        r.Synchronize()
        t0 = time.perf_counter()
        rays = 0
        kms = np.zeros(_abi.K_SLOTS)
        for _ in range(a.passes):
            r.RenderParallel()
            st = r.Stats()
            rays += st.rays
            kms += np.array(st.kernel_ms[:])
        r.Synchronize()
        dt = time.perf_counter() - t0
        names = ["camera", "trace", "shade", "shadow", "finalize", "mega", "accum", "-"]
        print(json.dumps({"scene": name, "Mrays_per_s": round(rays / dt / 1e6, 1),
                          "rays_per_pass": rays // a.passes,
                          "ms_per_pass": {names[k]: round(kms[k] / a.passes, 3) for k in range(_abi.K_SLOTS) if kms[k]}}),
              flush=True)
        r.close()


if __name__ == "__main__":
    main()
