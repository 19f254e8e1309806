# Shade: materials and lights staged in LDS (stage_shading) and child 0's key reused: parity subset on the
# in-tree build (both), then same-box A/B on C4 and C2: cur (both) / lds (staging only) / base (HEAD).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06l; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gopher3 or c2 or example3 or serial or furnace or c4_mesh1m or textures or shapes_ext" > $D/tests.log 2>&1 || exit 1
LIBS="lds:ab/lib_lds.so base:ab/lib_base.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06l/c4 || exit 1
LIBS="lds:ab/lib_lds.so base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06l/c2 || exit 1
