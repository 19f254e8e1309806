# Round-6 final tree, part A: the VALU instruction mix of C4 / C2 / C5 (bench.py's shade line and the C2 / C5
# VALU-issue rooflines) and the C2 / C5 whole-pass FETCH / WRITE passes (tools/gpu_valu_mix.sh, gpu_pmc_whole.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_valu_mix.sh r06fvm c4 c2 c5 || exit 1
bash tools/gpu_pmc_whole.sh r06fw || exit 1
