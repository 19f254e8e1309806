# Shade: the triangle record loaded beside the queue entry in the SCAN form (current) against after it (ab/lib_nopre.so):
# parity of the shade and baseline tests, then C4 / C3 / C5 same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06j; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || exit 1
LIBS="nopre:ab/lib_nopre.so" ROUNDS=2 C5=all bash tools/gpu_ab_lib.sh r06j/ab
