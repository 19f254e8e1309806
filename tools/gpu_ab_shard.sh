# A/B of compile-time variants on the full frame and on one rank's share of an 8-way split
# (bench.py --shard 0/8): the per-launch fill/drain overheads weigh most there.
# usage: VARIANTS="base:|x:-DFOO" bash tools/gpu_ab_shard.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > gpurun_out/ab/build_$NAME.log 2>&1 || exit 1
  timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/ab/tests_$NAME.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-parity --json-out gpurun_out/ab/$NAME.json > gpurun_out/ab/$NAME.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --cpu-seconds 0 --no-parity --shard 0/8 --json-out gpurun_out/ab/${NAME}_s8.json > gpurun_out/ab/${NAME}_s8.log 2>&1 || exit 1
done
