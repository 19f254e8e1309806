# The library with 64M-sample extra-phase chunks: the GPU tests of the extra phases and C5, smoke, the VALU
# instruction mixes of C4 / C2 / C5 on it, and the C5 and C4 lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ev_r06final; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c5 or adaptive or firefly or extra or serial or example3 or volume or shapes_ext" > $D/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
bash tools/gpu_valu_mix.sh r06finalvm c4 c2 c5 || exit 1
timeout -k 10 400 python -u bench.py --workload c5 --json-out $D/bench_c5.json > $D/bench_c5.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --json-out $D/bench_default.json > $D/bench_default.log 2>&1 || exit 1
