# The whole -m gpu suite on the current tree, then the C4 and C5 bench lines (each step time-limited,
# stops at the first failure).   usage: bash tools/gpu_suite.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-suite}; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 16 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/c4.json > $D/c4.log 2>&1 && \
timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c5.json > $D/c5.log 2>&1
