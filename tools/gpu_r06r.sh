# k_wf_trace_linear / k_wf_shadow_linear (a few analytic records and planes, no triangles: C2): the whole GPU suite
# on the in-tree build, then same-box C2 A/B against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06r; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06r/c2 || exit 1
