#!/usr/bin/env python3
"""Whole-pass L2-fabric traffic of a workload priced in flops (C2, C5: roofline kernel "whole pass"):
the FETCH_SIZE and WRITE_SIZE passes of tools/gpu_pmc_whole.sh summed over every dispatch of the run,
corrected per MI355X_MICROARCH.md §HBM ((2·FETCH_SIZE + WRITE_SIZE)·1024 bytes), divided by the rays
the run traced (its warm-up passes, the counted pass and the timed steps, each a whole pass of the
workload).  Writes profiles/pmc_traffic_<workload>.json, which bench.py reads for roofline.traffic.
usage: python tools/pmc_whole.py gpurun_out/TAG WORKLOAD TAG"""
import csv
import glob
import json
import os
import sys

src, wl, tag = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def total(sub, counter):
    (path,) = glob.glob(os.path.join(src, sub, "*counter_collection.csv"))
    return sum(float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter)


fetch_kb, write_kb = total(f"fetch_{wl}", "FETCH_SIZE"), total(f"write_{wl}", "WRITE_SIZE")
bench = json.load(open(os.path.join(src, f"bench_{wl}_fetch.json")))
rays_per_pass = bench["value"] * 1e6 * bench["ms_per_step"] * 1e-3
passes = bench["warmup"] + 1 + bench["steps"]   # warm-up, the counted pass, the timed steps
out = {
    "workload": wl, "tag": tag, "source": src, "library": bench.get("library"),
    "fetch_kb": fetch_kb, "write_kb": write_kb,
    "traffic_bytes_total": (2 * fetch_kb + write_kb) * 1024,
    "passes": passes, "rays_per_pass": round(rays_per_pass),
    "traffic_bytes_per_ray": (2 * fetch_kb + write_kb) * 1024 / (rays_per_pass * passes),
    "note": "whole run, every kernel: traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md §HBM; "
            "FETCH/WRITE passes are separate runs of the same command",
}
json.dump(out, open(os.path.join(root, "profiles", f"pmc_traffic_{wl}.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
