"""Kernel durations and the idle gaps between consecutive kernels of the last pass in a
rocprofv3 kernel-trace CSV (both streams merged in start order)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "k_wf" in r["Kernel_Name"]]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 17
rows = rows[-n:]
prev_end = None
busy = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pt::", "")
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print(f"{name:28s} start+{(s - int(rows[0]['Start_Timestamp'])) / 1e6:8.3f} ms  dur {(e - s) / 1e6:7.3f} ms  gap {gap:8.1f} us")
    prev_end = max(prev_end or 0, e)
span = (max(int(r["End_Timestamp"]) for r in rows) - int(rows[0]["Start_Timestamp"])) / 1e6
print(f"span {span:.3f} ms")
