#!/usr/bin/env python3
"""Turn a tools/gpu_configs.sh output directory into committed C3 / C2 evidence under profiles/:
<tag>_c3_kernel_stats.csv, <tag>_c2_kernel_stats.csv (rocprofv3 --stats), <tag>_bench_c3.json,
<tag>_bench_c2.json, pmc_traffic_c3.json (L2-fabric bytes per ray of C3's dominant kernel) and
pmc_valu_c2.json (VALU issue fraction of every C2 / C3 kernel).

Traffic (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KB at the L2 fabric side; gfx950
FETCH_SIZE reports half of the bytes of 16-B-per-lane reads: (2·FETCH_SIZE + WRITE_SIZE)·1024.
VALU issue fraction: a SIMD issues one wave64 VALU instruction per 2 cycles, 1024 SIMDs;
cycles per XCD = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs, MI355X_MICROARCH.md 'DVFS
give-back'): frac = 2·SQ_INSTS_VALU / (1024 · GRBM_GUI_ACTIVE / 8).  fp64 VALU issues at half
rate, so for fp64-heavy kernels (shade) the fraction understates the pipe's occupancy.
usage: python tools/pmc_configs.py gpurun_out/TAG TAG"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")


def short(name):
    name = name.replace("void ", "")
    if name.startswith("pt::"):
        name = name[4:]
    return name.split("(")[0]


def sums(path, counters):
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] in counters:
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r["Dispatch_Id"])
    return acc, {k: len(v) for k, v in calls.items()}


def find(d, suffix):
    for f in os.listdir(d):
        if f.endswith(suffix):
            return os.path.join(d, f)
    raise FileNotFoundError(f"{d}/*{suffix}")


for w in ("c3", "c2"):
    shutil.copy(find(f"{src}/trace_{w}", "kernel_stats.csv"), f"{prof}/{tag}_{w}_kernel_stats.csv")
    shutil.copy(f"{src}/bench_{w}.json", f"{prof}/{tag}_bench_{w}.json")

# C3 traffic of the dominant kernel
bench = json.load(open(f"{src}/bench_c3.json"))
kernel = bench["roofline"]["kernel"]
f, _ = sums(find(f"{src}/fetch_c3", "counter_collection.csv"), {"FETCH_SIZE"})
wr, _ = sums(find(f"{src}/write_c3", "counter_collection.csv"), {"WRITE_SIZE"})
fetch, write = f[kernel]["FETCH_SIZE"], wr[kernel]["WRITE_SIZE"]
cfg = bench["config"]
rays_per_step = bench["value"] * 1e6 * bench["ms_per_step"] / 1e3
kind = (1 - cfg["shadow_ray_fraction"]) if "trace" in kernel else (cfg["shadow_ray_fraction"] if "shadow" in kernel else 1.0)
rays_in_kernel = rays_per_step * kind * (bench["steps"] + bench["warmup"])
stats = {short(r["Name"]): r for r in csv.DictReader(open(find(f"{src}/trace_c3", "kernel_stats.csv")))}
c3 = {
    "kernel": kernel, "workload_tris": cfg["triangles"], "source": src, "tag": tag,
    "fetch_kb": fetch, "write_kb": write,
    "traffic_bytes_per_ray": (2 * fetch + write) * 1024 / rays_in_kernel,
    "algorithmic_bytes_per_ray": bench["roofline"]["bytes_per_ray"],
    "rocprof_avg_ns": float(stats[kernel]["AverageNs"]) if kernel in stats else None,
    "bench_avg_launch_ms": bench["roofline"]["avg_launch_ms"],
    "note": "traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md §HBM; separate runs of the same command",
}
json.dump(c3, open(f"{prof}/pmc_traffic_c3.json", "w"), indent=1)

# VALU issue fractions
valu = {"tag": tag, "source": src, "formula": "2*SQ_INSTS_VALU / (1024 * GRBM_GUI_ACTIVE / 8)", "workloads": {}}
for w in ("c2", "c3"):
    acc, calls = sums(find(f"{src}/valu_{w}", "counter_collection.csv"),
                      {"SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVES", "SQ_BUSY_CYCLES"})
    ks = {}
    for k, v in acc.items():
        if v["GRBM_GUI_ACTIVE"] > 0:
            ks[k] = {"valu_issue_frac": round(2 * v["SQ_INSTS_VALU"] / (1024 * v["GRBM_GUI_ACTIVE"] / 8), 4),
                     "valu_insts_per_dispatch": v["SQ_INSTS_VALU"] / max(calls[k], 1),
                     "dispatches": calls[k]}
    valu["workloads"][w] = ks
# bench.py reads the C2 dominant kernel's fraction from "kernels" (bench.py names: shade class with '*')
valu["kernels"] = {}
for k, v in valu["workloads"]["c2"].items():
    key = k
    if k.startswith("k_wf_shade<"):
        key = k.rsplit(",", 1)[0] + ", *>"
        prev = valu["kernels"].get(key)
        if prev and prev["valu_insts_per_dispatch"] * prev["dispatches"] > v["valu_insts_per_dispatch"] * v["dispatches"]:
            continue
    valu["kernels"][key] = v
json.dump(valu, open(f"{prof}/pmc_valu_c2.json", "w"), indent=1)
print(json.dumps({"c3": c3, "valu": valu}, indent=1))
