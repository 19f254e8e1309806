# C4 (or WORKLOAD=c5 ...) bench under environment variants on the current build (no rebuild):
# VARIANTS="name:VAR=value ..|..", ROUNDS rounds alternating.
# usage: VARIANTS="base:|side:PT_SIDE_STREAM=1" [WORKLOAD=c5] [ROUNDS=2] bash tools/gpu_c4_env_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-envab}; mkdir -p $D
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
W=${WORKLOAD:-c4}
if [ "$W" = c4 ]; then A="--steps ${STEPS:-16} --warmup 2"; else A="--workload $W --steps 1 --warmup 1"; fi
for r in $(seq 1 ${ROUNDS:-1}); do
  for V in "${VS[@]}"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    echo "== $NAME ($ENVS) round $r" >> $D/progress.log
    env $ENVS timeout -k 10 400 python -u bench.py $A --cpu-seconds 0 --no-parity --json-out $D/${W}_${NAME}_$r.json > $D/${W}_${NAME}_$r.log 2>&1 || exit 1
    echo "$NAME round $r: $(python -c "import json;j=json.load(open('$D/${W}_${NAME}_$r.json'));print(j['value'],j['config']['kernel_ms_per_step'])")" >> $D/summary.txt
  done
done
