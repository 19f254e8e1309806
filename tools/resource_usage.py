#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / spill / occupancy table from `make -C ptsharp_amd/csrc resource-usage`."""
import re
import subprocess
import sys

out = subprocess.run(["make", "-s", "-C", "ptsharp_amd/csrc", "resource-usage"], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (?:Function Name: (\S+)|\s*([A-Za-z /\[\]]+?)(?: \[[\w/]+\])?: (\d+))", line)
    if not m:
        continue
    if m.group(1):
        cur = {"name": subprocess.run(["c++filt"], input=m.group(1), capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[m.group(2).strip()] = int(m.group(3))
pat = sys.argv[1] if len(sys.argv) > 1 else ""
print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'vspill':>6s} {'scratch':>7s} {'waves':>5s} {'LDS':>6s}")
for r in rows:
    if pat in r["name"]:
        name = re.sub(r"\(.*", "", r["name"]).replace("pt::", "")
        print(f"{name:70s} {r.get('VGPRs',0):5d} {r.get('AGPRs',0):5d} {r.get('VGPRs Spill',0):6d} "
              f"{r.get('ScratchSize',0):7d} {r.get('Occupancy',0):5d} {r.get('LDS Size',0):6d}")
