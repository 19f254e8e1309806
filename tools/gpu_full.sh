# full round check: all GPU tests, smoke, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_all.log 2>&1; echo "rc=$?" >> gpurun_out/gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python bench.py --json-out gpurun_out/bench_default.json > gpurun_out/bench_default.log 2>&1
