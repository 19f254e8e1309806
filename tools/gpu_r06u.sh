# Refill thresholds re-checked on the BVH8 kernels: closest hit PT_REFILL_IDLE 32 / 48 and shadow
# PT_SHADOW_REFILL_IDLE 24 / 40 against the kept 40 / 32 (cur), same box, C4, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIBS="ri32:ab/lib_ri32.so ri48:ab/lib_ri48.so si24:ab/lib_si24.so si40:ab/lib_si40.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06u || exit 1
