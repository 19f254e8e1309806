# Residency / cache counters (tools/residency.py's three --pmc passes, kernel trace only, each a run of its own)
# of any bench workload.   usage: bash tools/gpu_residency.sh TAG [bench.py arguments]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-res}; shift
D=gpurun_out/$TAG; mkdir -p $D
ARGS=${@:---steps 2 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity}
pmc() { P=$1; shift; timeout -s KILL 400 rocprofv3 --pmc "$@" --kernel-trace -d $D/$P -o p --output-format csv -- python3 bench.py $ARGS > $D/$P.log 2>&1; }
pmc p4 SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU && \
pmc p5 TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_TA_BUSY_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum TCP_PERF_SEL_TOTAL_MISS_LRU_READ_sum && \
pmc p6 TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum && \
python tools/residency.py $D $TAG > $D/residency.txt 2>&1
