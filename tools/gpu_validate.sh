set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/val_gpu_all.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val_smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --json-out gpurun_out/val_bench.json > gpurun_out/val_bench.log 2>&1
