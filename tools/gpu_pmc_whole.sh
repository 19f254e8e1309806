# FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel trace only) of the C2 and C5 bench workloads,
# for tools/pmc_whole.py.   usage: bash tools/gpu_pmc_whole.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-whole}; mkdir -p $D
C2="--workload c2 --steps 4 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
C5="--workload c5 --steps 1 --warmup 0 --cpu-seconds 0 --no-parity"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch_c2 -o p --output-format csv -- python3 bench.py $C2 --json-out $D/bench_c2_fetch.json > $D/fetch_c2.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write_c2 -o p --output-format csv -- python3 bench.py $C2 > $D/write_c2.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch_c5 -o p --output-format csv -- python3 bench.py $C5 --json-out $D/bench_c5_fetch.json > $D/fetch_c5.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write_c5 -o p --output-format csv -- python3 bench.py $C5 > $D/write_c5.log 2>&1
