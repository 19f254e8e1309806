# C5 instruction-mix counters of the FULL and split kernels (separate --pmc passes, kernel trace only).
# usage: bash tools/gpu_c5_pmc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-c5pmc}; mkdir -p $D
C5="--workload c5 --steps 1 --warmup 0 --cpu-seconds 0 --no-parity"
timeout -s KILL 60 rocprofv3 -L > $D/counters_list.txt 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $D/pa -o p --output-format csv -- python3 bench.py $C5 > $D/pa.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace -d $D/pb -o p --output-format csv -- python3 bench.py $C5 > $D/pb.log 2>&1
