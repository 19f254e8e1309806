# Measurements: per-rank shares with pass batching; C2 with the side stream off (each kernel's own
# time, not its overlap with the main stream); a rocprofv3 kernel trace of the C4 bench (per-launch
# durations: the closest-hit pass by depth).  Each step time-limited; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r03c}; mkdir -p $D
for S in 0/2 0/4 3/8 7/8; do
  F=shard_${S%/*}of${S#*/}
  timeout -k 10 300 python bench.py --shard $S --steps 32 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/$F.json > $D/$F.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --workload c2 --steps 8 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c2_side.json > $D/c2_side.log 2>&1 || exit 1
PT_SIDE_STREAM=0 timeout -k 10 300 python bench.py --workload c2 --steps 8 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c2_noside.json > $D/c2_noside.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- python3 bench.py --steps 4 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/bench_trace.json > $D/trace.log 2>&1 || exit 1
