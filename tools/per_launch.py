"""Per-launch kernel durations from a rocprofv3 kernel-trace CSV (one pass = camera, then
trace/shade/shadow per depth, then finalize)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pt::", ""),
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in rows]
seq = [s for s in seq if s[0].startswith("k_wf")]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 17
for name, ms in seq[-n:]:
    print(f"{name:28s} {ms:8.3f} ms")
