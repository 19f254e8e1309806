#!/usr/bin/env python3
"""Turn a tools/gpu_evidence.sh output directory into committed evidence under profiles/:
<tag>_kernel_stats.csv (rocprofv3 --stats), <tag>_bench_under_rocprof.json, and
profiles/pmc_traffic.json: FETCH/WRITE traffic per closest-hit ray of the dominant kernel.

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KB at the L2 fabric
side (Infinity-Cache hits included); gfx950 FETCH_SIZE reports half of the bytes of
16-B-per-lane reads, so traffic = (2·FETCH_SIZE + WRITE_SIZE)·1024.
"""
import csv, json, shutil, sys, os

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")
os.makedirs(prof, exist_ok=True)
shutil.copy(f"{src}/trace/trace_kernel_stats.csv", f"{prof}/{tag}_kernel_stats.csv")
bench = json.load(open(f"{src}/bench_trace.json"))
shutil.copy(f"{src}/bench_trace.json", f"{prof}/{tag}_bench_under_rocprof.json")
kernel = bench["roofline"]["kernel"]

def per_launch(path, counter):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if r["Kernel_Name"].startswith("void pt::" + kernel) and r["Counter_Name"] == counter]
    return sum(v), len(v)

fetch, nf = per_launch(f"{src}/fetch/fetch_counter_collection.csv", "FETCH_SIZE")
write, nw = per_launch(f"{src}/write/write_counter_collection.csv", "WRITE_SIZE")
# kernel-trace average duration of the same kernel (must agree with the bench's hipEvent average)
stats = {r["Name"]: r for r in csv.DictReader(open(f"{src}/trace/trace_kernel_stats.csv"))}
row = next(v for k, v in stats.items() if k.startswith("void pt::" + kernel))
cfg = bench["config"]
passes = bench["steps"] + bench["warmup"] + 1   # timed + warmup + the final parity-free pass count
rays_per_step = bench["value"] * 1e6 * bench["ms_per_step"] / 1e3
kind_frac = (1 - cfg["shadow_ray_fraction"]) if "trace" in kernel else (cfg["shadow_ray_fraction"] if "shadow" in kernel else 1.0)
rays_in_kernel = rays_per_step * kind_frac * (bench["steps"] + bench["warmup"])
out = {
    "kernel": kernel, "workload_tris": cfg["triangles"], "source": src, "tag": tag, "library": bench.get("library"),
    "fetch_kb": fetch, "write_kb": write, "launches": [nf, nw],
    "traffic_bytes_total": (2 * fetch + write) * 1024,
    "traffic_bytes_per_ray": (2 * fetch + write) * 1024 / rays_in_kernel,
    "uncorrected_bytes_per_ray": (fetch + write) * 1024 / rays_in_kernel,
    "algorithmic_bytes_per_ray": bench["roofline"]["bytes_per_ray"],
    "rocprof_avg_ns": float(row["AverageNs"]), "rocprof_calls": int(row["Calls"]),
    "bench_avg_launch_ms": bench["roofline"]["avg_launch_ms"],
    "note": "traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md §HBM; FETCH/WRITE passes are separate runs of the same command",
}
json.dump(out, open(f"{prof}/pmc_traffic.json", "w"), indent=1)
json.dump(out, open(f"{prof}/{tag}_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
