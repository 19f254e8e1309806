"""Summarise rocprofv3 kernel-trace + counter CSVs per kernel (sums over dispatches)."""
import collections
import csv
import sys

d = sys.argv[1]
def kname(n):
    return n.split("(")[0].replace("void ", "").replace("pt::", "")
st = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(f"{d}/trace/t_kernel_trace.csv")):
    k = kname(r["Kernel_Name"])
    st[k][0] += 1
    st[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
print("kernel time (ms, all dispatches):")
for k, (n, ms) in sorted(st.items(), key=lambda x: -x[1][1]):
    print(f"  {k:28s} calls={n:4d} ms={ms:9.2f}")
cnt = collections.defaultdict(lambda: collections.defaultdict(float))
for p in sys.argv[2:] or ["p1", "p2"]:
    try:
        for r in csv.DictReader(open(f"{d}/{p}/p_counter_collection.csv")):
            cnt[kname(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    except FileNotFoundError:
        pass
for k, c in sorted(cnt.items()):
    if "rocclr" in k:
        continue
    print(k)
    for n, v in sorted(c.items()):
        print(f"    {n:28s} {v:16.4g}")
    if c.get("SQ_WAVES"):
        w = c["SQ_WAVES"]
        print(f"    VALU/wave {c.get('SQ_INSTS_VALU',0)/w:9.1f}  VMEM/wave {c.get('SQ_INSTS_VMEM',0)/w:7.1f}  "
              f"LDS/wave {c.get('SQ_INSTS_LDS',0)/w:7.1f}  SALU/wave {c.get('SQ_INSTS_SALU',0)/w:7.1f}")
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        print(f"    wait_any/wave_cycles {c.get('SQ_WAIT_ANY',0)/wc:6.3f}  wait_inst {c.get('SQ_WAIT_INST_ANY',0)/wc:6.3f}  "
              f"active_inst {c.get('SQ_ACTIVE_INST_ANY',0)/wc:6.3f}")
