"""Per-depth cost of the wavefront kernels on C4: render with MaxBounces = 0..4 and
print the increments of kernel time and closest-hit / shadow ray counts per added depth."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from ptsharp_amd import Renderer, _abi, scenes  # noqa: E402

scene, camera, sampler = scenes.bunny_frame(1_000_000, seed=1234)
scene.Compile()
out = []
for mb in range(0, 5):
    sampler.MaxBounces = mb
    r = Renderer.NewRenderer(scene, camera, sampler, 1920, 1080, True)
    r.SamplesPerPixel = 4
    r.Seed = 1234
    r.Engine = _abi.ENGINE_WAVEFRONT
    r.RenderParallel()  # warm-up
    r.Flags = _abi.PASS_KERNEL_TIMING
    ms = np.zeros(_abi.K_SLOTS)
    rays = shadow = 0
    for _ in range(3):
        r.RenderParallel()
        st = r.Stats()
        ms += np.array(st.kernel_ms[:])
        rays += st.rays - st.shadow_rays
        shadow += st.shadow_rays
    r.close()
    out.append({"mb": mb, "trace_ms": ms[1] / 3, "shade_ms": ms[2] / 3, "shadow_ms": ms[3] / 3,
                "rays": rays / 3, "shadow_rays": shadow / 3})
prev = None
for o in out:
    line = dict(o)
    if prev:
        dr, ds = o["rays"] - prev["rays"], o["shadow_rays"] - prev["shadow_rays"]
        line["depth_trace_ns_per_ray"] = (o["trace_ms"] - prev["trace_ms"]) * 1e6 / max(dr, 1)
        line["depth_shadow_ns_per_ray"] = (o["shadow_ms"] - prev["shadow_ms"]) * 1e6 / max(ds, 1)
    else:
        line["depth_trace_ns_per_ray"] = o["trace_ms"] * 1e6 / max(o["rays"], 1)
        line["depth_shadow_ns_per_ray"] = o["shadow_ms"] * 1e6 / max(o["shadow_rays"], 1)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in line.items()}))
    prev = o
