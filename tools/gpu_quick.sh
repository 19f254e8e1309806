# parity tests + wavefront bench (short); stops at the first failing GPU step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --spp ${SPP:-16} --cpu-seconds 0 --no-parity --engine ${ENGINE:-wave} --json-out gpurun_out/quick.json > gpurun_out/quick.log 2>&1
