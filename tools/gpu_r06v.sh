# SCAN shade rows per claim (PT_SHADE_SCAN 6 / 4 against 8) and the light-term window (PT_ACC_WIN 8 / 32 against 16):
# same box, alternating, C4 then C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIBS="sc6:ab/lib_sc6.so sc4:ab/lib_sc4.so aw8:ab/lib_aw8.so aw32:ab/lib_aw32.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06v/c4 || exit 1
LIBS="sc6:ab/lib_sc6.so aw8:ab/lib_aw8.so aw32:ab/lib_aw32.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06v/c2 || exit 1
