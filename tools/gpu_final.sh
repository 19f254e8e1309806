# End-of-round bench lines on the final tree: the whole -m gpu suite, smoke, the default C4 bench and the
# C2 / C3 / C5 lines (each step time-limited; stops at the first failure).   usage: bash tools/gpu_final.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-final}; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 && \
timeout -k 10 900 python -u bench.py --json-out $D/bench_default.json > $D/bench_default.log 2>&1 && \
timeout -k 10 400 python -u bench.py --workload c5 --json-out $D/bench_c5.json > $D/bench_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --steps 16 --warmup 2 --cpu-seconds 0 --json-out $D/bench_c3.json > $D/bench_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c2 --steps 8 --warmup 1 --cpu-seconds 0 --json-out $D/bench_c2.json > $D/bench_c2.log 2>&1
