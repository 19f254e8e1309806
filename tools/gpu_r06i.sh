# C4 with Example.bunny's FireflySamples 32 (Example.cs:1100): the firefly phase at the 1M-triangle frame's scale;
# then C2 and C3 on the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06i; mkdir -p $D
timeout -k 10 600 python -u bench.py --firefly 32 --steps 16 --warmup 2 --cpu-seconds 5 --json-out $D/bench_c4_firefly32.json > $D/bench_c4_firefly32.log 2>&1 &&
timeout -k 10 600 python -u bench.py --workload c2 --steps 8 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/bench_c2.json > $D/bench_c2.log 2>&1 &&
timeout -k 10 600 python -u bench.py --workload c3 --steps 16 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/bench_c3.json > $D/bench_c3.log 2>&1
