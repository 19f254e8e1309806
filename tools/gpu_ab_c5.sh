# A/B of compile-time variants on C5 (bench.py --workload c5): the row-4 / mixed-scene GPU tests on the
# first variant (TESTS: pytest selection, default the shape-extension file and the baseline file),
# then per variant one C5 step.  usage: VARIANTS="a:|b:-DFLAG=0" bash tools/gpu_ab_c5.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-abc5}; mkdir -p $D
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
first=1
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > $D/build_$NAME.log 2>&1 || exit 1
  if [ $first = 1 ] && [ -z "$NO_TESTS" ]; then
    timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_shapes_ext.py tests/test_00_gpu_baseline.py} -x -v -m gpu --timeout 300 --timeout-method thread > $D/tests_$NAME.log 2>&1 || exit 1
    echo "tests ok"
  fi
  first=0
  timeout -k 10 300 python -u bench.py --workload c5 --steps ${STEPS:-1} --warmup 1 --json-out $D/c5_$NAME.json > $D/c5_$NAME.log 2>&1 || exit 1
  echo "$NAME: $(python -c "import json;d=json.load(open('$D/c5_$NAME.json'));print(d['value'], {k: v for k, v in d['config']['kernel_ms_per_step'].items()})")"
done
