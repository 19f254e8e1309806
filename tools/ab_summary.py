"""Summary of a tools/gpu_ab.sh run: per variant and bench, Mrays/s and the per-kernel ms per step.
usage: python tools/ab_summary.py gpurun_out/TAG"""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    j = json.load(open(f))
    k = j["config"].get("kernel_ms_per_step", {})
    ks = "  ".join(f"{n.split('<')[0].replace('k_wf_', '')}={v:.2f}" for n, v in k.items())
    rf = j.get("roofline", {})
    print(f"{os.path.basename(f):24s} {j['value']:10.1f} Mrays/s  {j['ms_per_step']:8.2f} ms/step  "
          f"nodes/ray {rf.get('nodes_per_ray')}  {ks}")
