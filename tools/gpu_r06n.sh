# k_wf_nee_accum: a row's weights loaded with its flag and the next row's loads ahead of this row's sums:
# parity subset on the in-tree build, then same-box A/B on C2 and C4 against the previous build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06n; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gopher3 or c2 or example3 or serial or furnace or c4_mesh1m or textures or accum" > $D/tests.log 2>&1 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06n/c2 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06n/c4 || exit 1
