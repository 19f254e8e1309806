# VALU instruction mix and FLOP counters of every kernel of a C2 / C5 / C4 pass (two --pmc passes per
# workload, kernel trace only, each under its own time limit), for the VALU-issue roofline of the C2 and
# C5 lines (tools/pmc_valu_mix.py -> profiles/pmc_valu_mix_<workload>.json, read by bench.py).
# One step, no warm-up: the profiled run renders that step and the counted pass (bench.py's counters).
# usage: bash tools/gpu_valu_mix.sh TAG [workloads...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-valumix}; shift
WL=${@:-c2 c5}
D=gpurun_out/$T; mkdir -p $D
PA="SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
for W in $WL; do
  A="--workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-parity"
  [ "$W" = c2 ] && A="$A --spp 16"
  timeout -k 10 400 python3 bench.py $A --json-out $D/bench_$W.json > $D/bench_$W.log 2>&1 || exit 1
  timeout -s KILL 400 rocprofv3 --pmc $PA --kernel-trace -d $D/${W}_a -o p --output-format csv -- python3 bench.py $A --json-out $D/bench_${W}_a.json > $D/${W}_a.log 2>&1 || exit 1
  timeout -s KILL 400 rocprofv3 --pmc $PB --kernel-trace -d $D/${W}_b -o p --output-format csv -- python3 bench.py $A --json-out $D/bench_${W}_b.json > $D/${W}_b.log 2>&1 || exit 1
done
exit 0
