"""Per-kernel residency / issue / cache figures from tools/gpu_evidence.sh output.

usage: python tools/residency.py gpurun_out/ev_<tag> [label]   (tools/gpu_evidence.sh)
p4: SQ_WAVE_CYCLES, SQ_INSTS_VALU, GRBM_GUI_ACTIVE; p5: TA / TCP stalls; p6: L2 hit and the
fabric read-request level (Little's law latency).  cycles = GRBM_GUI_ACTIVE / 8 (the counter
sums over the 8 XCDs); per-SIMD ratios divide by 1024 SIMDs, per-CU ratios by 256 CUs."""
import collections
import csv
import glob
import sys

# every wavefront kernel of the run (the counted pass' instantiations included, under their own names),
# listed by time; kernels under 1 ms in all are left out


def load(d, p):
    f = glob.glob(f"{d}/{p}/*counter_collection.csv")[0]
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void pt::", "").replace("pt::", "")
        if not name.startswith("k_wf_"):
            continue
        by[name][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[name][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return by, {k: sum(v.values()) for k, v in dur.items()}


d = sys.argv[1]
label = sys.argv[2] if len(sys.argv) > 2 else d
p4, t4 = load(d, "p4")
p5, t5 = load(d, "p5")
p6, _ = load(d, "p6")
print(f"# rocprofv3 --pmc passes (kernel-trace only) of one bench command (tools/gpu_evidence.sh: `bench.py --steps 2 --warmup 1 --spp 16`, "
      f"the bench configuration; tools/gpu_residency.sh: any workload), {label}.")
KERNELS = [k for k in sorted(t4, key=lambda k: -t4[k]) if t4[k] >= 1e-3]
print("# SQ_WAVE_CYCLES counts quad-cycles; cycles = GRBM_GUI_ACTIVE / 8 (sum over XCDs). Per-CU ratios divide by 256 CUs.")
for k in KERNELS:
    if k not in p4 or t4.get(k, 0) <= 0:
        continue
    c = p4[k]
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    clock = cyc / t4[k]
    print(f"{k}: {t4[k] * 1e3:.1f} ms over all dispatches, clock {clock / 1e9:.2f} GHz")
    print(f"  resident waves per SIMD (SQ_WAVE_CYCLES*4/cycles/1024): {c['SQ_WAVE_CYCLES'] * 4 / cyc / 1024:.2f}")
    print(f"  VALU instructions per SIMD-cycle: {c['SQ_INSTS_VALU'] / cyc / 1024:.3f}")
    if k in p5 and t5.get(k, 0) > 0:
        q = p5[k]
        cyc5 = clock * t5[k]
        print(f"  TA busy per CU: {q['TA_TA_BUSY_sum'] / cyc5 / 256:.3f}   "
              f"TCP pending-stall per CU: {q['TCP_PENDING_STALL_CYCLES_sum'] / cyc5 / 256:.3f}   "
              f"TCP tag-conflict stall per CU: {q['TCP_READ_TAGCONFLICT_STALL_CYCLES_sum'] / cyc5 / 256:.3f}")
for k in KERNELS:
    if k not in p6:
        continue
    q = p6[k]
    hit = q["TCC_HIT_sum"] / max(q["TCC_HIT_sum"] + q["TCC_MISS_sum"], 1)
    lat = q["TCC_EA0_RDREQ_LEVEL_sum"] / max(q["TCC_EA0_RDREQ_sum"], 1)
    print(f"{k}: L2 hit rate {hit:.3f}   mean EA read latency (TCC_EA0_RDREQ_LEVEL/RDREQ, cycles) {lat:.0f}")
