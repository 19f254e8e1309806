"""Per-depth kernel times from a rocprofv3 kernel-trace CSV of the C4 bench.

Each C4 pass launches, per depth d = 0..MaxBounces, one closest-hit kernel, the two shade forms (one of
them returns at once), one shadow kernel and one light-term accumulation, in depth order.  For every
kernel name this prints the mean duration at each position of that per-pass sequence, so position d is
depth d.  usage: python tools/depth_split.py <kernel_trace.csv> [depths=5] [skip_passes=1]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    depths = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    runs = defaultdict(list)
    with open(path) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        name = r["Kernel_Name"].replace("void ", "").replace("pt::", "").split("(")[0]
        runs[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for name, ds in sorted(runs.items()):
        if not name.startswith("k_wf_") or len(ds) % depths:
            continue
        passes = len(ds) // depths
        if passes <= skip:
            continue
        per = [0.0] * depths
        for p in range(skip, passes):
            for d in range(depths):
                per[d] += ds[p * depths + d]
        per = [x / (passes - skip) for x in per]
        print(f"{name:44s} passes {passes - skip:3d}  " + "  ".join(f"d{d} {x:7.3f}" for d, x in enumerate(per))
              + f"  sum {sum(per):8.3f} ms")


if __name__ == "__main__":
    main()
