# VERDICT r05 #7b: the instanced-mesh scene on the round-4 tree (ab/r04, its own code) and the current tree,
# same box, one stream (PT_SIDE_STREAM=0: every kernel's time its own), alternated, then a kernel trace of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06e; mkdir -p $D
for r in 1 2; do
  (cd ab/r04 && PT_SIDE_STREAM=0 timeout -k 10 200 python -u tools/bench_scenes.py instances > ../../$D/r04_$r.jsonl 2> ../../$D/r04_$r.log) || exit 1
  PT_SIDE_STREAM=0 timeout -k 10 200 python -u tools/bench_scenes.py instances > $D/cur_$r.jsonl 2> $D/cur_$r.log || exit 1
done
(cd ab/r04 && PT_SIDE_STREAM=0 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d ../../$D/trace_r04 -o t --output-format csv -- python3 tools/bench_scenes.py instances > ../../$D/trace_r04.log 2>&1) || exit 1
PT_SIDE_STREAM=0 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $D/trace_cur -o t --output-format csv -- python3 tools/bench_scenes.py instances > $D/trace_cur.log 2>&1
