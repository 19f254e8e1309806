# smoke + all GPU tests + default bench; each GPU step time-limited, stops at first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 && \
timeout -k 10 600 python -u bench.py --json-out gpurun_out/bench_default.json > gpurun_out/bench_default.log 2>&1
