# GPU tests, then the default bench with one stream and with the side stream, and one rank's
# share (--shard 0/8) of the frame.   usage: bash tools/gpu_side.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-side}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 1
for S in 0 1; do
  PT_SIDE_STREAM=$S timeout -k 10 300 python bench.py --steps 8 --warmup 1 --cpu-seconds 0 --no-parity --json-out gpurun_out/${T}_full_s$S.json > gpurun_out/${T}_full_s$S.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 32 --warmup 2 --cpu-seconds 0 --no-parity --shard 0/8 --json-out gpurun_out/${T}_shard8.json > gpurun_out/${T}_shard8.log 2>&1 || exit 1
exit 0
