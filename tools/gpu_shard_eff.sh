# Per-rank workload of an N-GPU run measured on one GPU (bench.py --shard 0/N), N = 2, 4, 8.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/shard
for N in 2 4 8; do
  timeout -k 10 300 python bench.py --shard 0/$N --steps 16 --warmup 2 --cpu-seconds 0 --no-parity --json-out gpurun_out/shard/s$N.json > gpurun_out/shard/s$N.log 2>&1 || exit 1
done
