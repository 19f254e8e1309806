"""Summary of tools/gpu_envab.sh results: value and ms/step per variant, full frame and 1/8 share,
and the share's per-rank efficiency (8 x share rate / full rate ... i.e. share value / full value).
usage: python tools/envab_summary.py TAG"""
import glob, json, os, sys

tag = sys.argv[1]
rows = {}
for f in sorted(glob.glob(f"gpurun_out/envab/{tag}_*_*.json")):
    name, kind = os.path.basename(f)[len(tag) + 1:-5].rsplit("_", 1)
    rows.setdefault(name, {})[kind] = json.load(open(f))
for name, r in rows.items():
    full, sh = r.get("full"), r.get("shard8")
    line = f"{name:12s}"
    if full:
        line += f" full {full['value']:8.1f} ({full['ms_per_step']:.2f} ms)"
    if sh:
        line += f"  1/8 {sh['value']:8.1f} ({sh['ms_per_step']:.3f} ms)"
    if full and sh:
        line += f"  eff {sh['value'] / full['value']:.3f}"
    print(line)
