# The GPU test suite under every scheduling override at once per line (each must leave the
# Buffers bit-identical to the oracle's parity bar): side stream forced on / off, per-lane
# refill kernels forced on / off, each shade form forced, small queues (many chunks).
# usage: bash tools/gpu_matrix.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/matrix
T=${1:-m}
run() {
  NAME=$1; shift
  env "$@" timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/matrix/${T}_$NAME.log 2>&1
  rc=$?
  echo "$NAME rc=$rc $(tail -1 gpurun_out/matrix/${T}_$NAME.log)" >> gpurun_out/matrix/${T}_summary.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ]
}
run side1 PT_SIDE_STREAM=1 && \
run side0 PT_SIDE_STREAM=0 && \
run lanes1 PT_LANES=1 && \
run lanes0 PT_LANES=0 && \
run direct PT_SHADE_FORM=direct && \
run scan PT_SHADE_FORM=scan && \
run smallq PT_WF_MAX_CAP=4194304
