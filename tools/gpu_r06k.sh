# Exact power-of-two stratum division (pt_math.h div_strata): parity subset, then same-box A/B against the
# previous build on C2 (16 children per camera hit) and C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06k; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gopher3 or c2 or example3 or serial or furnace or c4_mesh1m" > $D/tests.log 2>&1 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06k/c2 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06k/c4 || exit 1
