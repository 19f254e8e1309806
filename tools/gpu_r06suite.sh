# The whole GPU suite on the round's final library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ev_r06suite; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || exit 1
