# Fresnel reflectance with one division (rPar² == rOrth² exactly): parity subset, same-box A/B on C2 and C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06w; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gopher3 or c2 or materialspheres or example1 or c4_mesh1m or serial or linear" > $D/tests.log 2>&1 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 STEPS=8 BARGS="--workload c2" bash tools/gpu_ab_lib.sh r06w/c2 || exit 1
LIBS="base:ab/lib_base.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06w/c4 || exit 1
