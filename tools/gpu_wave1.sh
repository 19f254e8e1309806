set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --spp 4 --cpu-seconds 0 --no-parity --engine wave --json-out gpurun_out/wave.json > gpurun_out/wave.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --spp 4 --cpu-seconds 0 --no-parity --engine mega --json-out gpurun_out/mega.json > gpurun_out/mega.log 2>&1
