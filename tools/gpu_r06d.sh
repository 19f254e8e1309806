# Region sort, diagnosis: whole regions per XCD partition (1) against every region spread over the partitions (2:
# balanced by construction, every XCD on the same region at the same time), same box, with L2 counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06d; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "region_sort" --timeout 300 --timeout-method thread > $D/tests.log 2>&1 &&
VARIANTS="base:|sort1:PT_REGION_SORT=1|sort2:PT_REGION_SORT=2" ROUNDS=1 bash tools/gpu_c4_env_ab.sh r06d/ab &&
PT_REGION_SORT=2 timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $D/pmc_sort2 -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity > $D/pmc_sort2.log 2>&1
