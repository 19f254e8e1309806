# A/B of compile-time variants: parity tests on the first, then a short bench per variant.
# usage: VARIANTS="base:|static:-DPT_TRACE_STATIC" bash tools/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
first=1
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > gpurun_out/ab/build_$NAME.log 2>&1 || exit 1
  if [ $first = 1 ] || [ -n "$TESTS_ALL" ]; then
    timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/ab/tests_$NAME.log 2>&1 || exit 1
    first=0
  fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --spp ${SPP:-16} --cpu-seconds 0 --no-parity --engine wave --json-out gpurun_out/ab/$NAME.json > gpurun_out/ab/$NAME.log 2>&1 || exit 1
done
