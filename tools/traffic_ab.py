"""L2-fabric traffic of the closest-hit kernel from a tools/gpu_counters_ab.sh variant directory:
(2·FETCH_SIZE + WRITE_SIZE)·1024 bytes (MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE halves 16-B reads)
per launch and per ray, beside the bench's compulsory bytes per launch.
usage: python tools/traffic_ab.py gpurun_out/<tag>_<variant>"""
import csv
import glob
import json
import sys

d = sys.argv[1]
K = "k_wf_trace_lanes<false, false>"


def total(p, counter):
    f = glob.glob(f"{d}/{p}/*counter_collection.csv")[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
         if r["Kernel_Name"].startswith("void pt::" + K) and r["Counter_Name"] == counter]
    return sum(v), len(v)


fetch, n = total("fetch", "FETCH_SIZE")
write, _ = total("write", "WRITE_SIZE")
b = json.load(open(f"{d}/bench_fetch.json"))
r = b["roofline"]
traffic = (2 * fetch + write) * 1024 / max(n, 1)
print(f"{K}: {n} launches, L2-fabric traffic {traffic / 1e9:.2f} GB per launch, "
      f"{traffic / r['rays_per_launch']:.1f} B per ray, compulsory {r['compulsory_bytes_per_launch'] / 1e9:.2f} GB per launch, "
      f"traffic / compulsory {traffic / r['compulsory_bytes_per_launch']:.2f}; bench under the fetch pass {b['value']} Mrays/s")
