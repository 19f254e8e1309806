# Round-6 last library: the whole GPU suite (with the linear-vs-lockstep test) and the VALU instruction mixes of
# C4 / C2 / C5 (bench.py's shade line, C4's VALU-issue view, the C2 / C5 rooflines).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ev_r06g2; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
bash tools/gpu_valu_mix.sh r06gvm c4 c2 c5 || exit 1
