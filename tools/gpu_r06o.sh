# k_wf_trace / k_wf_shadow (the lockstep kernels: C2's analytic scene, C5's analytic halves): a ray's two queue
# loads issued together (one round trip): parity subset, then same-box A/B on C2 and C5 against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06o; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gopher3 or c2 or example3 or serial or furnace or shapes_ext or c5 or volume or lockstep" > $D/tests.log 2>&1 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" C5=all bash tools/gpu_ab_lib.sh r06o/c2 || exit 1
