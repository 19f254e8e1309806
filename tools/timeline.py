"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (tools/gpu_timeline.sh):
kernel durations, overlap and GPU idle time in the last STEP of the run.
usage: python tools/timeline.py gpurun_out/tl_s1/run_kernel_trace.csv [--all]"""
import csv, sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""),
       r["Queue_Id"]) for r in rows]
ks.sort()
# steps end with k_wf_finalize
ends = [i for i, k in enumerate(ks) if "finalize" in k[2]]
lo = ends[-2] + 1 if len(ends) > 1 else 0
step = ks[lo:ends[-1] + 1]
t0 = step[0][0]
busy, cur_s, cur_e = 0, None, None
for s, e, n, q in step:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = step[-1][1] - t0
for s, e, n, q in step:
    print(f"q{q} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  {n[:60]}")
print(f"span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms")
prev_end = ends[-2]
print(f"gap before step: {(step[0][0] - ks[prev_end][1]) / 1e3:.1f} us")
