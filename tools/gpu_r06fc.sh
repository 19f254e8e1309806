# Round-6 final tree, part C: the default C4 line again (with the roofline's VALU-issue view), C5 (its line and its one-stream kernel times), C3 and C2 lines with kernel stats, and a
# two-rank torch.distributed.run rehearsal on one GPU (gloo gather; the per-rank scale_detail over gloo).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ev_r06fc; mkdir -p $D
timeout -k 10 600 python -u bench.py --json-out $D/bench_default.json > $D/bench_default.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload c5 --json-out $D/bench_c5.json > $D/bench_c5.log 2>&1 || exit 1
PT_SIDE_STREAM=0 timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c5one -o kt -- python3 bench.py --workload c5 --steps 1 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c5_one_stream_bench.json > $D/c5one.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c3 --steps 16 --warmup 2 --cpu-seconds 0 --json-out $D/bench_c3.json > $D/bench_c3.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c3 -o kt -- python3 bench.py --workload c3 --steps 4 --warmup 1 --cpu-seconds 0 --no-parity > $D/c3_trace.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c2 --steps 8 --warmup 1 --cpu-seconds 0 --json-out $D/bench_c2.json > $D/bench_c2.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c2 -o kt -- python3 bench.py --workload c2 --steps 4 --warmup 1 --cpu-seconds 0 --no-parity > $D/c2_trace.log 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 8 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/bench_w2_rehearsal.json > $D/bench_w2_rehearsal.log 2>&1 || exit 1
