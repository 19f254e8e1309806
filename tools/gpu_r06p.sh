# k_wf_shade_miss (C5's textured-environment misses): hit record and queue entry loaded together, next row
# prefetched: parity subset, then same-box C5 A/B (two runs each) against the previous build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06p; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "textures or c5 or shapes_ext or env" > $D/tests.log 2>&1 || exit 1
for r in 1 2; do
LIBS="base:ab/lib_base.so" ROUNDS=0 C5=all bash tools/gpu_ab_lib.sh r06p/c5_$r || exit 1
done
