set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03b; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_parity.py -v -m gpu -k "gather or comm or resume or write or tiles" --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1 || exit 1
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/bench_w2.json > $D/bench_w2.log 2>&1 || exit 1
