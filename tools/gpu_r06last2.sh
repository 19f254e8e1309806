# Round-6 last library, evidence part 2: the C4 rocprof kernel trace + FETCH / WRITE passes (profiles/pmc_traffic.json on
# this library), the default C4 line (after the VALU mixes: its shade line and VALU-issue view priced), C5 (line and
# one-stream kernel times), C3 and C2 lines with kernel stats, and a two-rank torch.distributed.run rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ev_r06last; mkdir -p $D
PROF="--steps 4 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- python3 bench.py $PROF --json-out $D/bench_trace.json > $D/trace.log 2>&1 || exit 1
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch -o fetch --output-format csv -- python3 bench.py $PROF --json-out $D/bench_fetch.json > $D/fetch.log 2>&1 || exit 1
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write -o write --output-format csv -- python3 bench.py $PROF --json-out $D/bench_write.json > $D/write.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --json-out $D/bench_default.json > $D/bench_default.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload c5 --json-out $D/bench_c5.json > $D/bench_c5.log 2>&1 || exit 1
PT_SIDE_STREAM=0 timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c5one -o kt -- python3 bench.py --workload c5 --steps 1 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c5_one_stream_bench.json > $D/c5one.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c3 --steps 16 --warmup 2 --cpu-seconds 30 --json-out $D/bench_c3.json > $D/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c2 --steps 8 --warmup 1 --cpu-seconds 30 --json-out $D/bench_c2.json > $D/bench_c2.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c2 -o kt -- python3 bench.py --workload c2 --steps 4 --warmup 1 --cpu-seconds 0 --no-parity > $D/c2_trace.log 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 8 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/bench_w2_rehearsal.json > $D/bench_w2_rehearsal.log 2>&1 || exit 1
