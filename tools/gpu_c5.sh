# C5 (BASELINE.json configs[4]) on one GPU: the row-4 shape tests, then the c5 bench line and its
# rocprofv3 kernel trace; each step time-limited, stops at the first failure.
# usage: bash tools/gpu_c5.sh TAG [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-c5}; shift
D=gpurun_out/$T; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_shapes_ext.py -v -m gpu --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit 1
echo "tests ok"
timeout -k 10 400 python -u bench.py --workload c5 --json-out $D/bench_c5.json "$@" > $D/bench_c5.log 2>&1 || exit 1
echo "bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- python3 bench.py --workload c5 --steps 1 --warmup 1 --json-out $D/bench_c5_rocprof.json "$@" > $D/trace.log 2>&1 || exit 1
echo "trace ok"
