# A/B of run-time (environment) variants on one build: the GPU tests, then per variant a short
# bench of the full C4 frame and of one rank's share (--shard 0/8).
# usage: VARIANTS="p1:PT_PIPES=1|p2:PT_PIPES=2" bash tools/gpu_envab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/envab
T=${1:-e}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/envab/${T}_tests.log 2>&1 || exit 1
fi
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
for V in "${VS[@]}"; do
  NAME=${V%%:*}; ENVS=${V#*:}
  env $ENVS timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 1 --cpu-seconds 0 --no-parity --json-out gpurun_out/envab/${T}_${NAME}_full.json > gpurun_out/envab/${T}_${NAME}_full.log 2>&1 || exit 1
  env $ENVS timeout -k 10 300 python bench.py --steps 32 --warmup 2 --cpu-seconds 0 --no-parity --shard 0/8 --json-out gpurun_out/envab/${T}_${NAME}_shard8.json > gpurun_out/envab/${T}_${NAME}_shard8.log 2>&1 || exit 1
done
exit 0
