# Per-launch kernel trace of tools/bench_scenes.py on one scene (per-depth breakdown via tools/per_depth.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=${1:-gopher3}
D=gpurun_out/scene_depth_$S
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace -d $D -o kt --output-format csv -- python3 tools/bench_scenes.py --passes 2 $S > $D/log 2>&1 && \
python3 tools/per_depth.py $(find $D -name '*kernel_trace.csv' | head -1) > $D/per_depth.txt
