# Kernel-trace stats and the residency / cache counter passes (tools/gpu_evidence.sh's p4-p6) of the C4
# bench for a prebuilt library (an A/B build), then tools/residency.py; the current build is restored.
# usage: bash tools/gpu_lib_evidence.sh TAG ab/lib_X.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ev_$1; mkdir -p $D
CUR=ptsharp_amd/libptsharp_hip.so
cp $CUR $D/.cur.so && cp $2 $CUR || exit 1
restore() { cp $D/.cur.so $CUR; rm -f $D/.cur.so; }
CTR="--steps 2 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
pmc() { P=$1; shift; timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d $D/$P -o p --output-format csv -- python3 bench.py $CTR > $D/$P.log 2>&1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- python3 bench.py --steps 4 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity --json-out $D/bench_trace.json > $D/trace.log 2>&1 && \
pmc p4 SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU && \
pmc p5 TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_TA_BUSY_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum TCP_PERF_SEL_TOTAL_MISS_LRU_READ_sum && \
pmc p6 TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum && \
python tools/residency.py $D $1 > $D/residency.txt 2>&1
rc=$?
restore
exit $rc
