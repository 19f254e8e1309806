# Kernel timelines (rocprofv3 kernel trace, CSV) of one rank's share of the C4 frame under
# environment variants.   usage: VARIANTS="s0:PT_SIDE_STREAM=0|s1:PT_SIDE_STREAM=1" bash tools/gpu_timeline.sh TAG [SHARD]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-tl}; SH=${2:-0/8}
IFS='|' read -ra VS <<< "${VARIANTS:-s0:PT_SIDE_STREAM=0|s1:PT_SIDE_STREAM=1}"
for V in "${VS[@]}"; do
  NAME=${V%%:*}; ENVS=${V#*:}
  for kv in $ENVS; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_$NAME -o run -- python3 bench.py --steps 6 --warmup 1 --cpu-seconds 0 --no-parity --shard $SH > gpurun_out/${T}_$NAME.log 2>&1 || exit 1
  for kv in $ENVS; do unset "${kv%%=*}"; done
done
exit 0
