# Shade: a few analytic records and planes staged in the block's LDS with the materials and lights (a sphere / cube
# hit's record read there in hit_info): parity subset, then same-box A/B on C2 and C4 against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06s; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gopher3 or c2 or example3 or serial or furnace or c4_mesh1m or textures or shapes_ext" > $D/tests.log 2>&1 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06s/c2 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06s/c4 || exit 1
