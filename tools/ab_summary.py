"""Print value and per-kernel ms of each gpurun_out/ab/*.json."""
import glob
import json
import os

for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    d = json.load(open(f))
    k = {n.split("<")[0].replace("k_wf_", ""): v for n, v in d["config"]["kernel_ms_per_step"].items()}
    print(f"{os.path.basename(f)[:-5]:12s} {d['value']:9.1f}  " + "  ".join(f"{n}={v:.1f}" for n, v in k.items()))
