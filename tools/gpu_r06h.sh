# 64-B BVH8 node units (the current build) against the 128-B node (ab/lib_node128.so): the parity tests that
# traverse the triangle BVH first, then a same-box C4 A/B and C5 once per library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06h; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_gpu_parity.py tests/test_gpu_volume_march.py -x -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || exit 1
LIBS="node128:ab/lib_node128.so" ROUNDS=2 C5=all bash tools/gpu_ab_lib.sh r06h/ab
