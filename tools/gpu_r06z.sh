# Round-6 evidence on the final tree, part 1: the GPU suite, smoke, rocprof kernel trace + FETCH/WRITE passes of the
# C4 bench (profiles/pmc_traffic.json), the default bench, residency counters (tools/gpu_evidence.sh's steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_evidence.sh r06z quick || exit 1
D=gpurun_out/ev_r06z
CTR="--steps 2 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
pmc() { P=$1; shift; timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d $D/$P -o p --output-format csv -- python3 bench.py $CTR > $D/$P.log 2>&1; }
pmc p4 SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU && \
pmc p5 TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_TA_BUSY_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum TCP_PERF_SEL_TOTAL_MISS_LRU_READ_sum && \
pmc p6 TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum
