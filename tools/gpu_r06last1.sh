# Round-6 last library, evidence part 1: the VALU instruction mixes of C4 / C2 / C5 on it (bench.py's shade line,
# C4's VALU-issue view, the C2 / C5 rooflines).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_valu_mix.sh r06lastvm c4 c2 c5 || exit 1
