# Per-launch kernel trace of a short default bench (for per-depth time breakdown).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/depth_${1:-x}
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace -d $D -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/bench.json > $D/log 2>&1 && \
python3 tools/per_depth.py $(find $D -name '*kernel_trace.csv' | head -1) > $D/per_depth.txt
