# C5: the adaptive phase's chunks up to 64M / 128M camera samples (PT_EXTRA_CHUNK_MAX) against 32M, now that the
# queues hold 2^29 entries: same box, C5 twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
LIBS="ec64:ab/lib_ec64.so ec128:ab/lib_ec128.so" ROUNDS=0 C5=all bash tools/gpu_ab_lib.sh r06ec/c5_$r || exit 1
done
