# The bench's parity leg on C2 and C3 (the oracle against the full frame at the timed spp), and on C4 with a
# 60-s CPU budget (a larger pixel sample), on the last library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06x; mkdir -p $D
timeout -k 10 600 python -u bench.py --workload c2 --steps 8 --warmup 1 --cpu-seconds 30 --json-out $D/bench_c2_parity.json > $D/bench_c2_parity.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --workload c3 --steps 16 --warmup 2 --cpu-seconds 30 --json-out $D/bench_c3_parity.json > $D/bench_c3_parity.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --cpu-seconds 60 --json-out $D/bench_c4_parity60.json > $D/bench_c4_parity60.log 2>&1 || exit 1
