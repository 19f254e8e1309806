# Round-6 final tree, part B: tools/gpu_evidence.sh (GPU suite, smoke, rocprof kernel trace + FETCH / WRITE passes
# of the C4 bench, the default bench line, residency counters, per-rank shard workloads, the other scenes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_evidence.sh r06f || exit 1
