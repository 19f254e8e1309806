# C4 bench under environment variants on the current build (no rebuild): VARIANTS="name:VAR=value ..|..".
# usage: VARIANTS="base:|side:PT_SIDE_STREAM=1" bash tools/gpu_c4_env_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-envab}; mkdir -p $D
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
for V in "${VS[@]}"; do
  NAME=${V%%:*}; ENVS=${V#*:}
  echo "== $NAME ($ENVS)" >> $D/progress.log
  env $ENVS timeout -k 10 300 python -u bench.py --steps ${STEPS:-16} --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/c4_$NAME.json > $D/c4_$NAME.log 2>&1 || exit 1
done
