# Round evidence, second call (tools/gpu_evidence.sh TAG quick is the first): residency / cache
# counters of the bench workload (separate --pmc passes, kernel trace only), per-rank shard
# workloads (N = 2, 4, 8), the C3 / C2 / C5 bench lines, and the scene table.  Each GPU step
# time-limited; stops at the first failure.   usage: bash tools/gpu_evidence_rest.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}
D=gpurun_out/ev_$TAG
mkdir -p $D
CTR="--steps 2 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
pmc() { P=$1; shift; timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d $D/$P -o p --output-format csv -- python3 bench.py $CTR > $D/$P.log 2>&1; }
pmc p4 SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU && \
pmc p5 TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_TA_BUSY_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum TCP_PERF_SEL_TOTAL_MISS_LRU_READ_sum && \
pmc p6 TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum && \
python tools/residency.py $D $TAG > $D/residency.txt 2>&1 || exit 1
echo "counters ok"
for S in 0/2 0/4 0/8 3/8 7/8; do
  F=shard_${S%/*}of${S#*/}
  timeout -k 10 300 python bench.py --shard $S --steps 16 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/$F.json > $D/$F.log 2>&1 || exit 1
done
echo "shards ok"
timeout -k 10 300 python bench.py --workload c3 --steps 16 --warmup 2 --cpu-seconds 0 --json-out $D/bench_c3.json > $D/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 8 --warmup 1 --cpu-seconds 0 --json-out $D/bench_c2.json > $D/bench_c2.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c5 --json-out $D/bench_c5.json > $D/bench_c5.log 2>&1 || exit 1
echo "configs ok"
timeout -k 10 600 python tools/bench_scenes.py > $D/scenes.jsonl 2> $D/scenes.log
