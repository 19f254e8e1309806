# Timing probe: inner triangle-BVH nodes read 4 of their 8 pieces (wrong boxes; ab/lib_probe_half.so) against the
# current build, C4 bench with counted nodes per ray: does the step loop's time follow its load instructions?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIBS="half:ab/lib_probe_half.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06b
