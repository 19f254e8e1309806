# rocprofv3 evidence for the bench workload: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE in their own runs; no sys/runtime trace with --pmc).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS="--steps ${STEPS:-4} --warmup 1 --spp ${SPP:-16} --cpu-seconds 0 --no-parity --engine ${ENGINE:-auto}"
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- python3 bench.py $ARGS --json-out $D/bench_trace.json > $D/trace.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch -o fetch --output-format csv -- python3 bench.py $ARGS --json-out $D/bench_fetch.json > $D/fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write -o write --output-format csv -- python3 bench.py $ARGS --json-out $D/bench_write.json > $D/write.log 2>&1
