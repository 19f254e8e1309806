"""Per-kernel wave-state split from one rocprofv3 --pmc pass of SQ wave-state counters (tools/gpu_r06q.sh):
the share of wave time parked at s_waitcnt / barriers (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY) and
issuing (SQ_ACTIVE_INST_ANY; by kind VALU / VMEM / LDS / SALU), per MI355X_MICROARCH.md's SQ table (the three
are disjoint and sum to SQ_WAVE_CYCLES).  usage: python tools/wave_states.py DIR [DIR ...]"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    for d in sys.argv[1:]:
        f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        if not f:
            print(d, "no counter file")
            continue
        acc = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f[0])):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        print(f"== {d}")
        tot = sum(v.get("SQ_WAVE_CYCLES", 0) for v in acc.values())
        for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
            wc = v.get("SQ_WAVE_CYCLES", 0)
            if wc < 0.01 * tot:
                continue
            sh = {n: v.get(c, 0) / wc for n, c in (("wait", "SQ_WAIT_ANY"), ("stall", "SQ_WAIT_INST_ANY"),
                                                  ("active", "SQ_ACTIVE_INST_ANY"), ("valu", "SQ_ACTIVE_INST_VALU"),
                                                  ("vmem", "SQ_ACTIVE_INST_VMEM"), ("lds", "SQ_ACTIVE_INST_LDS"),
                                                  ("salu", "SQ_ACTIVE_INST_SCA"))}
            print(f"  {k[:58]:58s} {wc / tot:6.1%} of wave time  " + "  ".join(f"{n} {x:.3f}" for n, x in sh.items()))


if __name__ == "__main__":
    main()
