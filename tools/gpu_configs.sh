# C3 / C2 evidence (bench.py --workload c3|c2): bench lines, kernel-trace stats, and PMC passes
# (C3: FETCH_SIZE, WRITE_SIZE for the L2-fabric traffic; C2: VALU issue counters), each pass a
# run of its own under a time limit.  Then tools/pmc_configs.py writes profiles/.
# usage: bash tools/gpu_configs.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-cfg}
D=gpurun_out/$T
mkdir -p $D
C3="--workload c3 --steps 8 --warmup 1 --cpu-seconds 0 --no-parity"
C2="--workload c2 --steps 4 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
timeout -k 10 300 python bench.py $C3 --json-out $D/bench_c3.json > $D/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py $C2 --json-out $D/bench_c2.json > $D/bench_c2.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $D/trace_c3 -o t --output-format csv -- python3 bench.py $C3 --json-out $D/bench_c3_trace.json > $D/trace_c3.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $D/trace_c2 -o t --output-format csv -- python3 bench.py $C2 --json-out $D/bench_c2_trace.json > $D/trace_c2.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch_c3 -o p --output-format csv -- python3 bench.py $C3 > $D/fetch_c3.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write_c3 -o p --output-format csv -- python3 bench.py $C3 > $D/write_c3.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d $D/valu_c2 -o p --output-format csv -- python3 bench.py $C2 > $D/valu_c2.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d $D/valu_c3 -o p --output-format csv -- python3 bench.py $C3 > $D/valu_c3.log 2>&1
