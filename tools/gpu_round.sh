# The driver's round-end GPU steps, rehearsed: the -m gpu suite (collection order as the driver's),
# smoke(), and the default bench; each step time-limited, stops at the first crash.
# usage: bash tools/gpu_round.sh TAG [pytest args]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-round}; shift
D=gpurun_out/$T
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --durations=20 "$@" > $D/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $D/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1 || exit 1
exit 0
