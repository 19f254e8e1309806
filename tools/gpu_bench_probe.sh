set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --spp 1 --cpu-seconds 5 --json-out gpurun_out/probe1.json > gpurun_out/probe1.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --spp 8 --cpu-seconds 0 --no-parity --json-out gpurun_out/probe8.json > gpurun_out/probe8.log 2>&1
