# Queues for 2^29 entries within half the device (one shadow set on one stream; C2's pass in one chunk of 17
# depths instead of two): the whole GPU suite, then same-box A/B on C2 and C4 against the last library, C5 once each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06y; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06y/c2 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 C5=all bash tools/gpu_ab_lib.sh r06y/c4 || exit 1
