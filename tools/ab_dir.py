"""One line per bench JSON of an A/B directory: workload, variant, Mrays/s, ms/step, per-kernel ms.
usage: python tools/ab_dir.py gpurun_out/ab_xx"""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f))
    w, v = os.path.basename(f)[:-5].split("_", 1)
    k = d["config"].get("kernel_ms_per_step") or {}
    print(f"{w:8s} {v:8s} {d['value']:9.1f} Mrays/s {d['ms_per_step']:9.3f} ms/step  " +
          " ".join(f"{n.split('<')[0].replace('k_wf_', '')}={t:.2f}" for n, t in k.items()))
