# k_wf_nee_accum with four rows of a window in flight (PT_NEE_AHEAD): parity subset, same-box A/B on C2 and C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06t; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gopher3 or c2 or example3 or serial or c4_mesh1m or accum or firefly or adaptive" > $D/tests.log 2>&1 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06t/c2 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06t/c4 || exit 1
