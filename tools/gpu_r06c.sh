# Region sort of the deep queues (PT_REGION_SORT=1): bit-identity tests, then a same-box C4 A/B and counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06c; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "region_sort" --timeout 300 --timeout-method thread > $D/tests.log 2>&1 &&
VARIANTS="base:|sort:PT_REGION_SORT=1" ROUNDS=2 bash tools/gpu_c4_env_ab.sh r06c/ab &&
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $D/trace_sort -o t --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity > $D/trace_base.log 2>&1 &&
PT_REGION_SORT=1 timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $D/pmc_sort -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity > $D/pmc_sort.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $D/pmc_base -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity > $D/pmc_base.log 2>&1
