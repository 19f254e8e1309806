# Round-3 checks: the gather / resume / batch GPU tests, the default bench (C4 from OBJ), a 2-rank
# rehearsal of the N-GPU bench path (two ranks share the box's one GPU: gloo gather + its bit check),
# and the 1/8 share with and without pass batching.  Each step time-limited; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r03b}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_parity.py -v -m gpu -k "gather or comm or resume or write or tiles or batch" --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --shard 0/8 --passes-per-call 1 --steps 32 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/shard8_k1.json > $D/shard8_k1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --shard 0/8 --steps 32 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/shard8_k8.json > $D/shard8_k8.log 2>&1 || exit 1
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/bench_w2.json > $D/bench_w2.log 2>&1 || exit 1
