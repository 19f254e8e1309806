# A/B of compile-time variants: the GPU tests on the first variant, then a short bench per variant
# (and tools/bench_scenes.py on SCENES, bench.py --shard SHARD, if set).  usage: VARIANTS="base:|w6:-DPT_RAYS_WAVES=6" bash tools/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
first=1
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > gpurun_out/ab/build_$NAME.log 2>&1 || exit 1
  if [ $first = 1 ] || [ -n "$TESTS_ALL" ]; then
    timeout -k 10 900 python -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab/tests_$NAME.log 2>&1 || exit 1
    first=0
  fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 1 --spp ${SPP:-16} --cpu-seconds 0 --no-parity --json-out gpurun_out/ab/$NAME.json > gpurun_out/ab/$NAME.log 2>&1 || exit 1
  if [ -n "$SHARD" ]; then
    timeout -k 10 300 python bench.py --steps 32 --warmup 2 --cpu-seconds 0 --no-parity --shard $SHARD --json-out gpurun_out/ab/shard_$NAME.json > gpurun_out/ab/shard_$NAME.log 2>&1 || exit 1
  fi
  if [ -n "$SCENES" ]; then
    timeout -k 10 300 python tools/bench_scenes.py $SCENES > gpurun_out/ab/scenes_$NAME.jsonl 2> gpurun_out/ab/scenes_$NAME.log || exit 1
  fi
done
