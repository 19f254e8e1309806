# Round evidence, one gpurun call (each GPU step time-limited; stops at the first failure):
#   GPU tests + smoke; rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE passes of the
#   bench workload (separate runs, no sys/runtime trace with --pmc) -> profiles/<tag>_* and
#   profiles/pmc_traffic.json; the default bench; residency / cache counters at the bench's own
#   configuration (C4, 16 spp, one full pass per step); per-rank shard workloads (N = 2, 4, 8).
# usage: bash tools/gpu_evidence.sh r02a [quick]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
D=gpurun_out/ev_$TAG
mkdir -p $D
PROF="--steps 4 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
CTR="--steps 2 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
pmc() { P=$1; shift; timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d $D/$P -o p --output-format csv -- python3 bench.py $CTR > $D/$P.log 2>&1; }
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- python3 bench.py $PROF --json-out $D/bench_trace.json > $D/trace.log 2>&1 && \
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch -o fetch --output-format csv -- python3 bench.py $PROF --json-out $D/bench_fetch.json > $D/fetch.log 2>&1 && \
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write -o write --output-format csv -- python3 bench.py $PROF --json-out $D/bench_write.json > $D/write.log 2>&1 && \
python tools/pmc_summary.py $D $TAG > $D/pmc_summary.log 2>&1 && \
timeout -k 10 900 python -u bench.py --json-out $D/bench_default.json > $D/bench_default.log 2>&1 || exit 1
[ "$2" = quick ] && exit 0
pmc p4 SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU && \
pmc p5 TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_TA_BUSY_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum TCP_PERF_SEL_TOTAL_MISS_LRU_READ_sum && \
pmc p6 TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum && \
python tools/residency.py $D $TAG > $D/residency.txt 2>&1 || exit 1
for S in 0/2 0/4 0/8 3/8 7/8; do
  F=shard_${S%/*}of${S#*/}
  timeout -k 10 300 python bench.py --shard $S --steps 16 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/$F.json > $D/$F.log 2>&1 || exit 1
done
timeout -k 10 600 python tools/bench_scenes.py > $D/scenes.jsonl 2> $D/scenes.log
