# A/B of runtime env settings (e.g. PT_SORT) on one box: parity tests under the first, then a short bench each.
# usage: SETTINGS="base:|t1s0:PT_SORT=t1s0" bash tools/gpu_ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
IFS='|' read -ra VS <<< "${SETTINGS:-base:}"
first=1
for V in "${VS[@]}"; do
  NAME=${V%%:*}; ENVS=${V#*:}
  if [ $first = 1 ]; then
    env $ENVS timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/ab/tests_$NAME.log 2>&1 || exit 1
    first=0
  fi
  env $ENVS timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 1 --spp ${SPP:-16} --cpu-seconds 0 --no-parity --engine wave --json-out gpurun_out/ab/$NAME.json > gpurun_out/ab/$NAME.log 2>&1 || exit 1
done
