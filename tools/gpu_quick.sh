# GPU tests (verbose, per-test durations), the default bench, and optionally tools/bench_scenes.py on
# SCENES; each step time-limited, stops at the first crash.   usage: bash tools/gpu_quick.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-q}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --durations=15 ${PYTEST_ARGS:-} > gpurun_out/${T}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --cpu-seconds 5 --json-out gpurun_out/${T}_bench.json > gpurun_out/${T}_bench.log 2>&1 || exit 1
[ -n "$SCENES" ] && timeout -k 10 600 python tools/bench_scenes.py $SCENES > gpurun_out/${T}_scenes.jsonl 2> gpurun_out/${T}_scenes.log
exit 0
