# row-4 parity + full GPU suite + quick bench; each step time-limited, stops at first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes_ext.py tests/test_gpu_textures.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_row4.log 2>&1
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
timeout -k 10 300 python -u bench.py --steps 8 --warmup 1 --cpu-seconds 0 --no-parity --json-out gpurun_out/quick.json > gpurun_out/quick.log 2>&1
