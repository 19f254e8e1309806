# latency / residency / cache-stall counters (Little's law), separate passes, kernel-trace only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-lat}
D=gpurun_out/$TAG
mkdir -p $D
ARGS="--steps 2 --warmup 1 --spp 4 --cpu-seconds 0 --no-parity --engine wave"
run() { timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d $D/$P -o p --output-format csv -- python3 bench.py $ARGS > $D/$P.log 2>&1; }
P=trace; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o t --output-format csv -- python3 bench.py $ARGS > $D/trace.log 2>&1 && \
P=p4; run SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU && \
P=p5; run TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_TA_BUSY_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum TCP_PERF_SEL_TOTAL_MISS_LRU_READ_sum && \
P=p6; run TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum
