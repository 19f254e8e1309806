# parity tests + wavefront bench (short)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --spp 4 --cpu-seconds 0 --no-parity --engine ${ENGINE:-wave} --json-out gpurun_out/quick.json > gpurun_out/quick.log 2>&1
