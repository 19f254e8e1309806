# Kernel timeline (rocprofv3 kernel trace, CSV) of one rank's share of the C4 frame, with one
# stream and with the side stream.   usage: bash tools/gpu_timeline.sh TAG [SHARD]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-tl}; SH=${2:-0/8}
for S in 0 1; do
  PT_SIDE_STREAM=$S timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_s$S -o run -- python3 bench.py --steps 6 --warmup 1 --cpu-seconds 0 --no-parity --shard $SH > gpurun_out/${T}_s$S.log 2>&1 || exit 1
done
exit 0
