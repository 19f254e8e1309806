# A/B of compile-time variants: the GPU test suite on the first variant, then per variant the C4 bench,
# the C2 bench (NO_C2=1 skips it) and the 1/8 share (bench.py --shard 0/8).  usage: VARIANTS="a:|b:-DFLAG=0" bash tools/gpu_ab2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-ab2}; mkdir -p $D
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
first=1
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > $D/build_$NAME.log 2>&1 || exit 1
  if [ $first = 1 ] && [ -z "$NO_TESTS" ]; then
    timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $D/tests_$NAME.log 2>&1 || exit 1
  fi
  first=0
  timeout -k 10 300 python bench.py --steps ${STEPS:-16} --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/c4_$NAME.json > $D/c4_$NAME.log 2>&1 || exit 1
  [ -z "$NO_C2" ] && { timeout -k 10 300 python bench.py --workload c2 --steps 6 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c2_$NAME.json > $D/c2_$NAME.log 2>&1 || exit 1; }
  timeout -k 10 300 python bench.py --shard 0/8 --steps 32 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/shard8_$NAME.json > $D/shard8_$NAME.log 2>&1 || exit 1
done
