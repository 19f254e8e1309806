# Round evidence for the current engine: GPU tests, smoke, rocprofv3 kernel trace + FETCH/WRITE
# passes, PMC summary (profiles/pmc_traffic.json, read by the bench), the default bench, then
# the residency/latency counter passes.  Each GPU step is time-limited; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r01d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
bash tools/gpu_profile.sh $TAG && \
python tools/pmc_summary.py gpurun_out/prof_$TAG $TAG > gpurun_out/pmc_summary_$TAG.log 2>&1 && \
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_$TAG.json && \
timeout -k 10 900 python -u bench.py --json-out gpurun_out/bench_default.json > gpurun_out/bench_default.log 2>&1 && \
bash tools/gpu_counters2.sh lat_$TAG
