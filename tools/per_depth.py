"""Per-depth kernel time of the last wavefront pass in a rocprofv3 kernel-trace CSV."""
import collections, csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_wf" in r["Kernel_Name"] and "<true>" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].replace("void pt::", "").replace("pt::", ""),
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in rows]
fin = [i for i, s in enumerate(seq) if s[0] == "k_wf_finalize"]
start = fin[-2] + 1 if len(fin) > 1 else 0
agg = collections.defaultdict(float); d = 0
for name, ms in seq[start:fin[-1] + 1]:
    if name == "k_wf_camera": d = -1
    if name.startswith("k_wf_trace"): d += 1
    agg[(name, d)] += ms
for k in sorted(agg): print(f"{k[0]:22s} depth {k[1]:2d} {agg[k]:8.2f} ms")
print("total", round(sum(agg.values()), 2))
