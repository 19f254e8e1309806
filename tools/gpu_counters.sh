# per-kernel trace + SQ / cache counter passes (separate runs, no sys/runtime trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cnt}
D=gpurun_out/$TAG
mkdir -p $D
ARGS="--steps 2 --warmup 1 --spp 4 --cpu-seconds 0 --no-parity --engine ${ENGINE:-wave}"
timeout -k 10 120 rocprofv3 -L > $D/avail.txt 2>&1 ; \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o t --output-format csv -- python3 bench.py $ARGS > $D/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $D/p1 -o p --output-format csv -- python3 bench.py $ARGS > $D/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_FLAT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace -d $D/p2 -o p --output-format csv -- python3 bench.py $ARGS > $D/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -d $D/p3 -o p --output-format csv -- python3 bench.py $ARGS > $D/p3.log 2>&1
