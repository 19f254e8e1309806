# rocprofv3 kernel trace of the C2 bench (per-launch durations by depth); time-limited.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-c2trace}; mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- python3 bench.py --workload c2 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/bench.json > $D/trace.log 2>&1 || exit 1
