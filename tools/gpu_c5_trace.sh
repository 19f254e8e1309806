# C5 kernel-trace stats of the current build (rocprofv3 --kernel-trace --stats, one step after one warm-up step).
# usage: bash tools/gpu_c5_trace.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-c5trace}; mkdir -p $D
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o kt -- python3 bench.py --workload c5 --steps 1 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c5_trace.json > $D/kt.log 2>&1
