#!/usr/bin/env python3
"""Summarise tools/gpu_valu_mix.sh's counter passes into profiles/pmc_valu_mix_<workload>.json, the
VALU-issue roofline of the C2 and C5 bench lines (bench.py reads it).

Per kernel and summed over the pass (every kernel of one step plus bench.py's counted pass):
  * wave-instructions by kind: SQ_INSTS_VALU, the fp64 ADD / MUL / FMA / TRANS, the fp32 ADD / MUL / FMA /
    TRANS, INT32, INT64, CVT;
  * VALU issue cycles, MI355X_MICROARCH.md's issue costs: a wave64 VALU instruction holds its SIMD 2
    cycles, an fp64 one 4 (the FP64 vector rate is half the FP32 rate); transcendentals (quarter rate) 8,
    fp64 transcendentals 16;
  * the FLOP counters SQ_INSTS_VALU_FLOPS_FP32 / _FP64 (+ _TRANS), scaled per the calibration below;
  * GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs): the kernels' busy cycles under the counters.
Calibration of the FLOPS counters: their ratio to (ADD + MUL + 2·FMA) of the same precision, reported
as flops_per_counted_op; 64 means they count per lane of a full wave.
Normalised per Scene.Intersect call with the bench line's rays per pass × the passes the profiled run
rendered (one step + the counted pass).
usage: python tools/pmc_valu_mix.py gpurun_out/TAG TAG [workloads...]"""
import csv
import json
import os
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
wls = sys.argv[3:] or ["c2", "c5"]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("void ", "")
    if name.startswith("pt::"):
        name = name[4:]
    return name.split("(")[0]


def find(d, suffix):
    for dp, _, fs in os.walk(d):
        for f in fs:
            if f.endswith(suffix):
                return os.path.join(dp, f)
    raise FileNotFoundError(f"{d}/**/*{suffix}")


def sums(path):
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
    return acc, {k: len(v) for k, v in calls.items()}


ISSUE = {"other": 2, "f64": 4, "trans32": 8, "trans64": 16}
for w in wls:
    bench = json.load(open(f"{src}/bench_{w}.json"))
    a, ca = sums(find(f"{src}/{w}_a", "counter_collection.csv"))
    b, _ = sums(find(f"{src}/{w}_b", "counter_collection.csv"))
    rays_per_pass = bench["value"] * 1e6 * bench["ms_per_step"] / 1e3 / bench["config"].get("passes_per_call", 1)
    passes = bench["steps"] + bench["warmup"] + 1   # the timed steps, the warm-up, the counted pass
    rays = rays_per_pass * passes
    kernels, tot = {}, defaultdict(float)
    for k in sorted(set(a) | set(b)):
        v = dict(a.get(k, {}))
        v.update({n: x for n, x in b.get(k, {}).items() if n != "GRBM_GUI_ACTIVE"})
        f64 = v.get("SQ_INSTS_VALU_ADD_F64", 0) + v.get("SQ_INSTS_VALU_MUL_F64", 0) + v.get("SQ_INSTS_VALU_FMA_F64", 0)
        t32, t64 = v.get("SQ_INSTS_VALU_TRANS_F32", 0), v.get("SQ_INSTS_VALU_TRANS_F64", 0)
        other = max(v.get("SQ_INSTS_VALU", 0) - f64 - t32 - t64, 0.0)
        cyc = ISSUE["other"] * other + ISSUE["f64"] * f64 + ISSUE["trans32"] * t32 + ISSUE["trans64"] * t64
        grbm = v.get("GRBM_GUI_ACTIVE", 0) / 8
        row = {n.replace("SQ_INSTS_", "").lower(): x for n, x in v.items() if n.startswith("SQ_INSTS_")}
        row.update({"dispatches": ca.get(k, 0), "valu_issue_cycles": cyc, "busy_cycles_per_xcd": grbm,
                    "valu_issue_frac": round(cyc / (1024 * grbm), 4) if grbm > 0 else None})
        kernels[k] = row
        for n, x in row.items():
            if isinstance(x, (int, float)) and n not in ("valu_issue_frac",):
                tot[n] += x
    fp32_ops = tot.get("valu_add_f32", 0) + tot.get("valu_mul_f32", 0) + 2 * tot.get("valu_fma_f32", 0)
    fp64_ops = tot.get("valu_add_f64", 0) + tot.get("valu_mul_f64", 0) + 2 * tot.get("valu_fma_f64", 0)
    cal32 = tot.get("valu_flops_fp32", 0) / fp32_ops if fp32_ops else None
    cal64 = tot.get("valu_flops_fp64", 0) / fp64_ops if fp64_ops else None
    lanes = 64 if (cal64 or cal32 or 64) < 8 else 1   # counters per wave-instruction -> per lane
    out = {
        "tag": tag, "source": src, "workload": w, "bench_line": f"{src}/bench_{w}.json",
        "library": bench.get("library"),   # bench.py flags the mix when the library it prices differs
        "rays_per_pass": rays_per_pass, "passes_profiled": passes, "rays_profiled": rays,
        "issue_cycles_model": ISSUE,
        "flops_per_counted_op": {"fp32": cal32, "fp64": cal64}, "flop_counter_lane_factor": lanes,
        "per_ray": {
            "valu_insts": tot["valu"] / rays,
            "valu_issue_cycles": tot["valu_issue_cycles"] / rays,
            "f64_insts": (tot.get("valu_add_f64", 0) + tot.get("valu_mul_f64", 0) + tot.get("valu_fma_f64", 0)) / rays,
            "fp32_flops": lanes * (tot.get("valu_flops_fp32", 0) + tot.get("valu_flops_fp32_trans", 0)) / rays,
            "fp64_flops": lanes * (tot.get("valu_flops_fp64", 0) + tot.get("valu_flops_fp64_trans", 0)) / rays,
        },
        "pass_valu_issue_frac_under_counters": round(tot["valu_issue_cycles"] / (1024 * tot["busy_cycles_per_xcd"]), 4)
        if tot["busy_cycles_per_xcd"] else None,
        "kernels": kernels,
    }
    json.dump(out, open(os.path.join(root, "profiles", f"pmc_valu_mix_{w}.json"), "w"), indent=1)
    print(w, json.dumps(out["per_ray"]), out["pass_valu_issue_frac_under_counters"], out["flops_per_counted_op"])
