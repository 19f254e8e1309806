# rocprofv3 evidence for the bench workload: kernel trace + stats, then separate PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS="--steps ${STEPS:-4} --warmup 1 --spp ${SPP:-4} --cpu-seconds 0 --no-parity"
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o trace --output-format csv -- python3 bench.py $ARGS --json-out gpurun_out/prof_$TAG/bench_trace.json > gpurun_out/prof_$TAG/trace.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof_$TAG/fetch -o fetch --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG/fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof_$TAG/write -o write --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG/write.log 2>&1
